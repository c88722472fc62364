"""Benchmark / test scenarios: pods on VF ports, an SFC, 1M flows, synthetic 64-B traffic.

The default chain mirrors what the reference realises with one NF pod per chain
(``examples/sfc.yaml``; ``marvell/main.go:490-563`` steering) but with the NFs executed on the GPU:

    pod VF (tagged vlan = vf+2, spoof-checked)  ->  ACL (TCAM, R rules)  ->  SNAT  ->
    L2 steer to the destination pod's VF (MAC rewrite, egress tag = its vlan)

Flows are random pod->pod 5-tuples; the key zone is the ingress bridge.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..ops import packets as P
from . import tables as T

POD_NET = 0x0A800000       # 10.128.0.0/16 pod addresses
NAT_NET = 0xC6336400       # 198.51.100.0/24 SNAT pool
GW_MAC = "02:00:00:00:ff:01"


def pod_mac(i: int) -> bytes:
    return bytes([0x02, 0xAA, (i >> 24) & 0xFF, (i >> 16) & 0xFF, (i >> 8) & 0xFF, i & 0xFF])


def vf_mac(i: int) -> bytes:
    return bytes([0x02, 0xBB, (i >> 24) & 0xFF, (i >> 16) & 0xFF, (i >> 8) & 0xFF, i & 0xFF])


@dataclass
class Scenario:
    n_pods: int
    pod_port: np.ndarray      # pod -> vport
    pod_gpu: np.ndarray       # pod -> owning GPU (egress side)
    keys: np.ndarray          # [F,4] flow keys
    actions: np.ndarray       # [F,4]
    flow_src_pod: np.ndarray  # [F]
    flow_dst_pod: np.ndarray  # [F]
    flow_sport: np.ndarray
    flow_dport: np.ndarray
    chain_id: int
    bridge: int = 1


def build_sfc(
    dp,
    n_pods: int = 8,
    n_flows: int = 1 << 20,
    n_acl: int = 256,
    seed: int = 0,
    hops=("acl", "nat", "l2fwd"),
    pod_gpu: np.ndarray | None = None,
    port_base: int = 0,
    install_flows: bool = True,
    flow_filter=None,
) -> Scenario:
    """Program `dp` (a DataPlane or anything with ports/chains/acl/flows) with the scenario.

    ``flow_filter(keys, hashes) -> bool mask`` selects which flows this table installs (flow
    sharding); all flows are still returned so traffic can be generated for any of them."""
    rng = np.random.default_rng(seed)
    bridge = 1
    pod_port = port_base + np.arange(n_pods, dtype=np.int64)
    if pod_gpu is None:
        pod_gpu = np.zeros(n_pods, np.int64)
    for i in range(n_pods):
        dp.ports.set(
            int(pod_port[i]),
            flags=T.PORT_VALID | T.PORT_SPOOFCHK | T.PORT_VLAN_ISOLATE | T.PORT_TAG_EGRESS,
            vlan=(i % 4094) + 2,
            bridge_id=bridge,
            mac=pod_mac(i),          # spoofchk: the pod's own MAC (what the VF was given)
            peer_mac=pod_mac(i),
            gpu=int(pod_gpu[i]),
        )
    # L2 table: pod MACs (used on flow miss, e.g. ARP / non-IP)
    for i in range(n_pods):
        dp.macs.insert(bridge, pod_mac(i), int(pod_port[i]))
    chain_id = dp.chains.add(list(hops))
    # ACL: R rules.  R-1 rules deny traffic to unused 192.168.x.0/24 subnets or to one rarely
    # used destination-port; the last rule permits the pod network.
    for r in range(max(n_acl - 1, 0)):
        if r % 8 == 7:
            dp.acl.add(permit=False, dport=int(rng.integers(1, 1024)), proto=17)
        else:
            dp.acl.add(permit=False, dst=f"192.168.{r % 256}.0/24", dport=int(1000 + r))
    if n_acl:
        dp.acl.add(permit=True, src="10.128.0.0/16")
    # flows
    src = rng.integers(0, n_pods, n_flows)
    dst = (src + rng.integers(1, max(n_pods, 2), n_flows)) % n_pods if n_pods > 1 else src
    sport = rng.integers(1024, 65536, n_flows)
    dport = rng.integers(1024, 65536, n_flows)
    keys = T.flow_key(POD_NET + src, POD_NET + dst, sport, dport, 17, bridge)
    # make keys unique (collisions are astronomically rare, but dedupe to be exact)
    _, uniq = np.unique(keys.view(np.dtype((np.void, 16))), return_index=True)
    if len(uniq) != n_flows:
        keep = np.sort(uniq)
        keys, src, dst, sport, dport = keys[keep], src[keep], dst[keep], sport[keep], dport[keep]
    F = len(keys)
    actions = T.flow_action(
        chain_id=chain_id,
        out_port=pod_port[dst],
        nat_ip=NAT_NET + (np.arange(F) % 250) + 1,
        nat_port=1024 + (np.arange(F) % 60000),
        vlan=0,
        flow_id=np.arange(F),
    )
    sc = Scenario(n_pods, pod_port, np.asarray(pod_gpu), keys, actions, src, dst, sport, dport, chain_id, bridge)
    if install_flows:
        sel = np.ones(F, bool)
        if flow_filter is not None:
            from ..native import nfdp

            sel = flow_filter(keys, nfdp().toeplitz(keys, dp.flows.rss_key))
        dp.flows.insert_many(keys[sel], actions[sel])
    return sc


def traffic(sc: Scenario, n: int, seed: int = 1, flows: np.ndarray | None = None, frame_len: int = 60,
            src_pods: np.ndarray | None = None) -> tuple[np.ndarray, np.ndarray]:
    """n packets of uniformly random flows (optionally restricted to `flows` indices, or to flows
    whose source pod is in `src_pods`): tagged 64-B frames from the source pod's VF.
    Returns (slots uint8[n,64], inmeta uint32[n])."""
    rng = np.random.default_rng(seed)
    pool = flows
    if src_pods is not None:
        pool = np.where(np.isin(sc.flow_src_pod, src_pods))[0]
    f = rng.integers(0, len(sc.keys), n) if pool is None else pool[rng.integers(0, len(pool), n)]
    s, d = sc.flow_src_pod[f], sc.flow_dst_pod[f]
    smac = np.frombuffer(b"".join(pod_mac(int(i)) for i in range(sc.n_pods)), np.uint8).reshape(-1, 6)[s]
    slots, lens = P.craft(
        n,
        dmac=GW_MAC,
        smac=smac,
        src_ip=POD_NET + s,
        dst_ip=POD_NET + d,
        sport=sc.flow_sport[f],
        dport=sc.flow_dport[f],
        proto=17,
        vlan=(s % 4094) + 2,
        frame_len=frame_len,
        payload_seed=seed,
    )
    return slots, P.inmeta(sc.pod_port[s], lens)
