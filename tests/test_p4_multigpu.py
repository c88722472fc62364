"""The Intel-IPU-equivalent P4 pipeline across several GPUs (BASELINE config 5): the reference's
AddHostVfP4Rules / AddNFP4Rules / peer-to-peer / primary-network / LAG entry strings
(ipuplugin p4rtclient.go:647-731,819-859, rebuilt by vsp/intel_ipu.py) replayed through the p4rt-ctl
CLI into a pipeline server whose bridge spans 2-3 data planes (MultiDataPlane: compiled once,
replicated by every commit), then frames forwarded across the planes - batch split by RSS owner,
and live through the native I/O engine - with results equal to ONE plane fed the same rules.
CPU oracle planes here; the same code drives one plane per MI355X."""
import io
import shutil
import tempfile
import time
from contextlib import redirect_stderr, redirect_stdout
from pathlib import Path

import numpy as np
import pytest

from dpu_operator_amd.cmd import p4rt_ctl
from dpu_operator_amd.cmd.p4rt_server import build_dataplane
from dpu_operator_amd.dataplane.multi import MultiDataPlane
from dpu_operator_amd.dataplane.p4rt import PHY_BASE, P4Runtime
from dpu_operator_amd.dataplane.p4server import P4rtServer
from dpu_operator_amd.ops import packets as P
from dpu_operator_amd.vsp import intel_ipu as ipu

VFS = [f"00:{0x08 + i:02x}:00:00:03:14" for i in range(4)]
ACCS = [f"00:{0x10 + i:02x}:00:00:03:15" for i in range(4)]
NF_IN, NF_OUT, PR_IN, PR_OUT = "00:20:00:00:00:01", "00:21:00:00:00:01", "00:22:00:00:00:01", "00:23:00:00:00:01"


def _rules():
    rules = []
    for vf, acc in zip(VFS, ACCS):
        rules += ipu.host_vf_rules(vf, acc)
    rules += ipu.peer_to_peer_rules(VFS)
    rules += ipu.nf_rules(VFS[:2], NF_IN, NF_OUT, PR_IN, PR_OUT)
    rules += ipu.primary_network_rules("00:0d:00:00:00:04", "00:0e:00:00:00:01")
    rules += ipu.lag_rules()
    return rules


def _program_via_cli(dp, lag=None):
    """Start a pipeline server on `dp` and replay every rule with the p4rt-ctl CLI."""
    rt = P4Runtime(dp, lag_ports=lag or {0: PHY_BASE, 1: PHY_BASE + 1})
    srv = P4rtServer({"br0": rt}).start()
    addr = f"127.0.0.1:{srv.port}"
    try:
        for r in _rules():
            o, e = io.StringIO(), io.StringIO()
            with redirect_stdout(o), redirect_stderr(e):
                rc = p4rt_ctl.main(["-g", addr, r.verb, r.bridge, r.table, r.entry])
            assert rc == 0, (r, o.getvalue(), e.getvalue())
    finally:
        srv.stop()
    dp.commit()
    return rt


def _traffic(n=3000, seed=0):
    """Frames from every VF / representor / NF port toward every known MAC (and unknown ones)."""
    rng = np.random.default_rng(seed)
    srcs = [(8 + i + 16, VFS[i]) for i in range(4)] + [(0x10 + i + 16, ACCS[i]) for i in range(4)] + \
        [(0x20 + 16, NF_IN), (0x21 + 16, NF_OUT), (PHY_BASE, "02:00:00:00:00:07")]
    dsts = VFS + ACCS + [NF_IN, NF_OUT, "00:0e:00:00:00:01", "02:00:00:00:00:99", "ff:ff:ff:ff:ff:ff"]
    frames, lens, ports = [], [], []
    for k in range(n):
        port, smac = srcs[rng.integers(len(srcs))]
        f, ln = P.craft(1, dmac=dsts[rng.integers(len(dsts))], smac=smac, src_ip=0x0A000001 + int(rng.integers(1 << 16)),
                        dst_ip=0x0A100000 + int(rng.integers(1 << 16)), sport=int(rng.integers(1, 65535)), dport=80)
        frames.append(f[0])
        lens.append(int(ln[0]))
        ports.append(port)
    fr = np.stack(frames)
    ln = np.array(lens, np.uint32)
    return P.header_slots(fr, ln), P.inmeta(np.array(ports), ln)


@pytest.mark.parametrize("n", [2, 3])
def test_p4_rules_replicated_over_planes_match_one_plane(n):
    m = build_dataplane("cpu", str(n), flow_buckets=1 << 10)
    assert isinstance(m, MultiDataPlane) and len(m.planes) == n
    one = build_dataplane("cpu", "1", flow_buckets=1 << 10)
    rt_m, rt_1 = _program_via_cli(m), _program_via_cli(one)
    assert rt_m.stats["compiles"] == rt_1.stats["compiles"]            # compiled once per write, not per plane
    # the compiled tables are the same objects on every plane, uploaded to each
    for p in m.planes[1:]:
        assert p.ports is m.planes[0].ports and p.macs is m.planes[0].macs
        assert p._versions["ports"] == m.planes[0].ports.version
    slots, im = _traffic()
    r, r1 = m.run(slots, im), one.run(slots, im)
    assert np.array_equal(r.meta, r1.meta) and np.array_equal(r.out, r1.out)
    assert len(np.unique(r.extra["owner"])) == n                        # the planes all carried traffic
    op, _, rs = P.meta_fields(r.meta)
    assert (rs == 0).mean() > 0.3 and len(np.unique(op[rs == 0])) >= 6   # K2 / K3 / K4 / NF / wire egresses
    assert np.array_equal(m.port_counters(), one.port_counters())


@pytest.fixture
def shm():
    from dpu_operator_amd.dataplane.native_io import memif_dir

    d = Path(tempfile.mkdtemp(prefix="dpu-p4mg-", dir=memif_dir()))
    yield d
    shutil.rmtree(d, ignore_errors=True)


def test_p4_pipeline_live_over_planes(shm):
    """The same pipeline, live: memif ports on the VF / representor vports, the native engine
    (2 rx queues) steering every frame to its owner plane; what every port receives equals the
    one-plane batch result."""
    from dpu_operator_amd.dataplane.native_io import MemifVport, NativeLivePath
    from dpu_operator_amd.native import nfdp

    nf = nfdp()
    m = build_dataplane("cpu", "3", flow_buckets=1 << 10)
    one = build_dataplane("cpu", "1", flow_buckets=1 << 10)
    _program_via_cli(m)
    _program_via_cli(one)
    slots, im = _traffic(1500, seed=3)
    ports = sorted({int(x) for x in (im & 0xFFFF)} | {int(p) for p in P.meta_fields(one.run(slots, im).meta)[0]
                                                       if int(p) < 4000})
    r1 = one.run(slots, im)
    op, _, rs = P.meta_fields(r1.meta)
    exp: dict[int, list[bytes]] = {}
    for i in np.nonzero(rs == 0)[0]:
        exp.setdefault(int(op[i]), []).append(P.assemble(r1.out[i], int(r1.meta[i]), slots[i], int(im[i] >> 16)))
    side = one.side_result()                 # K9 mirror copies (side pass replicas) go out too
    rp, _, rr = P.meta_fields(side["rep_meta"])
    for k in np.nonzero(rr == 0)[0]:
        s_ = int(side["rep_src"][k])
        exp.setdefault(int(rp[k]), []).append(P.assemble(side["rep_hdr"][k], int(side["rep_meta"][k]), slots[s_],
                                                         int(im[s_] >> 16)))
    paths = {p: str(shm / f"p{p}") for p in ports}
    live = NativeLivePath(m, {p: MemifVport(paths[p], ring_size=4096) for p in ports}, queues=2).start()
    try:
        eps = {p: nf.MemifEndpoint(paths[p]) for p in ports}
        src = im & 0xFFFF
        for p in ports:
            fr = [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == p)[0]]
            assert eps[p].send(fr) == len(fr)
        got = {p: [] for p in ports}
        want = sum(len(v) for k, v in exp.items() if k in paths)
        t_end = time.monotonic() + 10
        while sum(map(len, got.values())) < want and time.monotonic() < t_end:
            for p, e in eps.items():
                got[p] += e.recv()
            time.sleep(0.002)
        for p, frames in exp.items():
            if p in paths:
                assert sorted(got[p]) == sorted(frames), p
        assert live.error is None
    finally:
        live.stop()
