"""BASELINE config 5: the rule set the Intel IPU VSP programs, replayed onto the GPU pipeline.

The reference's Intel VSP never forwards a frame itself: it writes P4 entries into the IPU's FXP
(`p4rt-ctl add-entry br0 linux_networking_control.<table> <match>,action=...`).  Here the same entry
strings go through this repo's P4Runtime (dataplane/p4rt.py), which compiles them onto the GPU
tables, and synthetic traffic of the kinds that rule set exists for runs through the fused kernel:

  * Init (`lifecycleservice.go` doInit): phy-port, LAG and primary-network rules, and the
    peer-to-peer VSI loopbacks of every host-VF pair (`AddPeerToPeerP4Rules`, O(n^2):
    p4rtclient.go:903-920);
  * one bridge port per host VF (`AddHostVfP4Rules`: 5 entries per VF, p4rtclient.go:647-731);
  * one network function (`AddNFP4Rules`: the NF ports' representor rules and a VSI loopback for
    every host VF x {NF in, NF out}, p4rtclient.go:819-859).

Traffic (every frame a 64-B IPv4 / UDP frame of a 1M-5-tuple pool, so hashing sees as many flows
as the headline):
  * VF -> VF    (dst MAC of another host VF: K3 vsi_to_vsi_loopback);
  * VF -> NF    (dst MAC of the NF's ingress port: K3, the loopbacks AddNFP4Rules installs);
  * NF -> wire  (the NF's egress port to an external MAC: K4 source_port_to_pr_map, its representor
    on the ACC bridge - the way out to the wire);
  * VF -> other (unknown dst MAC: K4 to the VF's own representor, the OvS side).

`build()` programs a data plane through `IntelIpuVsp` + `InProcessP4rtClient` (the reference call
path: VSP -> p4rt client -> P4Runtime), `traffic()` makes a batch and the egress port each frame
must leave on.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..ops import packets as P

N_VFS = 8


@dataclass
class P4IpuScenario:
    vf_macs: list
    acc_macs: list
    vf_pr_macs: list        # each host VF's ACC representor (AddHostVfP4Rules accMac)
    nf_in: str
    nf_out: str
    nf_out_pr: str
    rules: dict             # table -> entries installed
    n_entries: int


def _mac(b1: int, tail: int) -> str:
    return f"00:{b1:02x}:00:00:{(tail >> 8) & 0xFF:02x}:{tail & 0xFF:02x}"


def build(dp, n_vfs: int = N_VFS) -> P4IpuScenario:
    """Program `dp` (a DataPlane) with the Intel VSP's rule set for `n_vfs` host VFs and one NF."""
    from ..dataplane.p4rt import P4Runtime
    from ..dataplane.p4server import InProcessP4rtClient, program_rules
    from ..vsp import intel_ipu as ipu

    rt = P4Runtime(dp)
    client = InProcessP4rtClient({"br0": rt})
    acc = [_mac(0x10 + i, i) for i in range(16)]          # the ACC's APF netdevs (enp0s1f0d*)
    vfs = [_mac(0x30 + i, 0x0314) for i in range(n_vfs)]   # host VF MACs (VSI = MAC byte 1)
    vf_prs = [_mac(0x50 + i, 0x0315) for i in range(n_vfs)]
    nf_in, nf_out = _mac(0x28, 1), _mac(0x29, 1)
    vsp = ipu.IntelIpuVsp(client, acc, vf_mac_list=lambda: vfs)
    vsp.init(True, "")                                    # phy port, peer-to-peer (n^2), LAG, primary network
    failed = []
    for vf, pr in zip(vfs, vf_prs):                       # AddHostVfP4Rules per host VF
        failed += program_rules(client, ipu.host_vf_rules(vf, pr))
    vsp.create_network_function(nf_in, nf_out)            # AddNFP4Rules
    failed += vsp.failed
    if failed:
        raise RuntimeError(f"{len(failed)} IPU rules refused: {failed[:2]}")
    dp.commit(full=True)
    counts = {name.split(".")[-1]: len(rows) for name, rows in rt.entries.items() if rows}
    return P4IpuScenario(vfs, acc, vf_prs, nf_in, nf_out, acc[ipu.NF_OUT_PR_INTF_INDEX], counts,
                         int(sum(counts.values())))


MIX = (("vf_to_vf", 0.4), ("vf_to_nf", 0.3), ("nf_to_wire", 0.2), ("vf_to_ovs", 0.1))


def traffic(sc: P4IpuScenario, n: int, seed: int = 0, flows: int = 1 << 20):
    """n frames of the four kinds (MIX).  Returns (slots [n,64] u8, inmeta [n] u32, expected egress
    port [n] i64, kind [n] u8 index into MIX)."""
    from ..dataplane.p4rt import vport_for_vsi

    rng = np.random.default_rng(seed)
    nv = len(sc.vf_macs)
    kind = rng.choice(len(MIX), size=n, p=[w for _, w in MIX]).astype(np.uint8)
    src_vf = rng.integers(0, nv, n)
    dst_vf = (src_vf + 1 + rng.integers(0, nv - 1, n)) % nv
    mb = lambda m: np.frombuffer(bytes(int(x, 16) for x in m.split(":")), np.uint8)  # noqa: E731
    vf_b = np.stack([mb(m) for m in sc.vf_macs])
    smac = vf_b[src_vf].copy()
    dmac = vf_b[dst_vf].copy()
    vsi = lambda m: int(m.split(":")[1], 16)  # noqa: E731
    vf_port = np.array([vport_for_vsi(vsi(m)) for m in sc.vf_macs])
    pr_port = np.array([vport_for_vsi(vsi(m)) for m in sc.vf_pr_macs])
    in_port = vf_port[src_vf].copy()
    exp = vf_port[dst_vf].copy()
    k = kind == 1                                          # VF -> NF ingress
    dmac[k] = mb(sc.nf_in)
    exp[k] = vport_for_vsi(vsi(sc.nf_in))
    k = kind == 2                                          # NF egress -> its representor (wire side)
    smac[k] = mb(sc.nf_out)
    ext = np.zeros((int(k.sum()), 6), np.uint8)
    ext[:, 0], ext[:, 1], ext[:, 5] = 0x02, 0xEE, rng.integers(1, 255, int(k.sum()))
    dmac[k] = ext
    in_port[k] = vport_for_vsi(vsi(sc.nf_out))
    exp[k] = vport_for_vsi(vsi(sc.nf_out_pr))
    k = kind == 3                                          # VF -> unknown MAC: its own representor
    ext = np.zeros((int(k.sum()), 6), np.uint8)
    ext[:, 0], ext[:, 1], ext[:, 5] = 0x02, 0xDD, rng.integers(1, 255, int(k.sum()))
    dmac[k] = ext
    exp[k] = pr_port[src_vf[k]]
    f = rng.integers(0, flows, n)                          # 5-tuples from a 1M-flow pool
    slots, lens = P.craft(n, dmac=dmac, smac=smac, src_ip=(0x0A000000 | (f >> 4)).astype(np.uint32),
                          dst_ip=(0x0A800000 | (f & 0xFFFF)).astype(np.uint32), sport=(1024 + (f & 0x7FFF)),
                          dport=(2000 + ((f >> 15) & 0x1F)))
    return slots, P.inmeta(in_port, lens), exp.astype(np.int64), kind
