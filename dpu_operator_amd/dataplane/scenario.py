"""Benchmark / test scenarios: pods on VF ports, an SFC, 1M flows, synthetic 64-B traffic.

The default chain mirrors what the reference realises with one NF pod per chain
(``examples/sfc.yaml``; ``marvell/main.go:490-563`` steering) but with the NFs executed on the GPU:

    pod VF (tagged vlan = vf+2, spoof-checked)  ->  ACL (TCAM, R rules)  ->  SNAT  ->
    L2 steer to the destination pod's VF (MAC rewrite, egress tag = its vlan)

Flows are random pod->pod 5-tuples; the key zone is the ingress bridge.
"""
from __future__ import annotations

from dataclasses import dataclass

import ipaddress

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
            src_pods: np.ndarray | None = None, return_flows: bool = False):
    """n packets of uniformly random flows (optionally restricted to `flows` indices, or to flows
    whose source pod is in `src_pods`): tagged 64-B frames from the source pod's VF.
    Returns (slots uint8[n,64], inmeta uint32[n]) [, flow index per packet]."""
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
    if return_flows:
        return slots, P.inmeta(sc.pod_port[s], lens), f
    return slots, P.inmeta(sc.pod_port[s], lens)


# Simple IMIX (7 x 64 B, 4 x 576 B, 1 x 1500 B wire packets, FCS included) and the jumbo size.
IMIX_SIMPLE = ((64, 7), (576, 4), (1500, 1))
IMIX_JUMBO = ((64, 7), (576, 4), (1500, 1), (9000, 1))


def imix_sizes(n: int, mix=IMIX_SIMPLE, seed: int = 0) -> np.ndarray:
    """Per-packet wire sizes (FCS included) drawn from a weighted mix."""
    sizes = np.array([sz for sz, _ in mix])
    w = np.array([wt for _, wt in mix], np.float64)
    return np.random.default_rng(seed).choice(sizes, n, p=w / w.sum())


def traffic_frames(sc: Scenario, n: int, sizes: np.ndarray, seed: int = 1, flows: np.ndarray | None = None):
    """Like ``traffic`` with per-packet sizes (64..9600: the tagged frame in memory = the untagged
    frame + FCS on the wire, the bench's 64-B convention): returns (header slots uint8[n,64], inmeta, frames uint8[n, max_len], lens).  The frames
    are what the I/O layer holds; the data plane reads only the header slots."""
    rng = np.random.default_rng(seed)
    f = rng.integers(0, len(sc.keys), n) if flows is None else flows[rng.integers(0, len(flows), n)]
    sizes = np.asarray(sizes, np.int64)
    lens = np.zeros(n, np.uint32)
    width = int(sizes.max())
    frames = np.zeros((n, max(width, 64)), np.uint8)
    for sz in np.unique(sizes):
        idx = np.where(sizes == sz)[0]
        s, d = sc.flow_src_pod[f[idx]], sc.flow_dst_pod[f[idx]]
        smac = np.frombuffer(b"".join(pod_mac(int(i)) for i in range(sc.n_pods)), np.uint8).reshape(-1, 6)[s]
        fr, ln = P.craft_full(len(idx), dmac=GW_MAC, smac=smac, src_ip=POD_NET + s, dst_ip=POD_NET + d,
                              sport=sc.flow_sport[f[idx]], dport=sc.flow_dport[f[idx]], proto=17,
                              vlan=(s % 4094) + 2, frame_len=int(sz) - 4, payload_seed=seed + int(sz))
        frames[idx, : fr.shape[1]] = fr[:, : frames.shape[1]]
        lens[idx] = ln
    src = sc.flow_src_pod[f]
    return P.header_slots(frames, lens), P.inmeta(sc.pod_port[src], lens), frames, lens


def install_deny_flows(dp, sc: Scenario, k: int = 4096, seed: int = 11) -> dict:
    """Flows the ACL hop denies: dst 192.168.(r % 256).x, dport 1000 + r for deny rule r of
    build_sfc's ACL (r % 8 != 7), from random pods, on the scenario's chain."""
    from . import tables as T2

    rng = np.random.default_rng(seed)
    n_rules = max(len(dp.acl.rules) - 1, 1)
    r = rng.integers(0, n_rules, 4 * k)
    r = r[r % 8 != 7][:k]
    src = rng.integers(0, sc.n_pods, len(r))
    dst_ip = 0xC0A80000 + ((r % 256) << 8) + rng.integers(1, 255, len(r))
    sport = rng.integers(1024, 65536, len(r))
    dport = 1000 + r
    keys = T2.flow_key(POD_NET + src, dst_ip, sport, dport, 17, sc.bridge)
    acts = T2.flow_action(chain_id=sc.chain_id, out_port=sc.pod_port[(src + 1) % sc.n_pods], nat_ip=NAT_NET + 1,
                          nat_port=2000, vlan=0, flow_id=0)
    dp.flows.insert_many(keys, acts)
    return {"src": src, "dst_ip": dst_ip, "sport": sport, "dport": dport}


def traffic_mixed(sc: Scenario, deny: dict, n: int, seed: int = 1, miss: float = 0.05, deny_frac: float = 0.02,
                  malformed: float = 0.001, src_pods: np.ndarray | None = None):
    """The bench's realistic mix: `miss` of the packets hit no flow (random source port -> L2
    fallback -> slow-path punt), `deny_frac` hit flows the ACL denies, `malformed` carry an
    impossible length; the rest are the headline's forwarded pod->pod flows."""
    pk, im = traffic(sc, n, seed=seed, src_pods=src_pods)
    rng = np.random.default_rng(seed + 101)
    u = rng.random(n)
    mi = np.where(u < miss)[0]
    pk[mi, 38:40] = rng.integers(0, 256, (len(mi), 2), dtype=np.uint8)   # sport bytes (tagged: L4 at 38)
    di = np.where((u >= miss) & (u < miss + deny_frac))[0]
    if len(di):
        j = rng.integers(0, len(deny["src"]), len(di))
        s = deny["src"][j]
        smac = np.frombuffer(b"".join(pod_mac(int(i)) for i in range(sc.n_pods)), np.uint8).reshape(-1, 6)[s]
        dpk, dl = P.craft(len(di), dmac=GW_MAC, smac=smac, src_ip=POD_NET + s, dst_ip=deny["dst_ip"][j],
                          sport=deny["sport"][j], dport=deny["dport"][j], proto=17, vlan=(s % 4094) + 2)
        pk[di] = dpk
        im[di] = P.inmeta(sc.pod_port[s], dl)
    bi = np.where((u >= miss + deny_frac) & (u < miss + deny_frac + malformed))[0]
    im[bi] = (im[bi] & 0xFFFF) | (10 << 16)
    return pk, im


def with_sizes(pk: np.ndarray, im: np.ndarray, sizes: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Turn 64-B tagged header slots into the headers of frames of `sizes` bytes (the payload
    beyond the slot is the I/O layer's and never read): IPv4 / UDP lengths and the IPv4 header
    checksum follow the size; the UDP checksum is set to 0 (none)."""
    pk = pk.copy()
    sizes = np.asarray(sizes, np.uint32)
    tot = sizes - 18                     # tagged: 14 + 4 tag
    pk[:, 20] = (tot >> 8) & 0xFF
    pk[:, 21] = tot & 0xFF
    pk[:, 42] = ((tot - 20) >> 8) & 0xFF
    pk[:, 43] = (tot - 20) & 0xFF
    pk[:, 44:46] = 0
    pk[:, 28:30] = 0
    w = (pk[:, 18:38:2].astype(np.uint32) << 8) | pk[:, 19:38:2]
    c = w.sum(axis=1)
    c = (c & 0xFFFF) + (c >> 16)
    c = (c & 0xFFFF) + (c >> 16)
    c = ~c & 0xFFFF
    pk[:, 28] = (c >> 8) & 0xFF
    pk[:, 29] = c & 0xFF
    return pk, (im & 0xFFFF) | (sizes << 16)


def add_acl_rules(dp, total: int, seed: int = 5) -> None:
    """Grow build_sfc's ACL to `total` rules (more deny rules before the final permit)."""
    rng = np.random.default_rng(seed)
    final = dp.acl.rules.pop()
    r = len(dp.acl.rules)
    while len(dp.acl.rules) < total - 1:
        if r % 8 == 7:
            dp.acl.add(permit=False, dport=int(rng.integers(1, 1024)), proto=17)
        else:
            dp.acl.add(permit=False, dst=f"192.168.{r % 256}.0/24", dport=int(1000 + r))
        r += 1
    dp.acl.rules.append(final)
    dp.acl.version += 1


WELL_KNOWN_PORTS = (20, 21, 22, 23, 25, 53, 67, 69, 80, 110, 123, 137, 161, 179, 389, 443, 445, 500, 514, 636,
                    993, 1433, 1521, 1812, 2049, 3306, 3389, 4500, 5060, 5432, 6379, 8080, 8443, 9090)


def acl_wild_rules(n_rules: int = 1024, seed: int = 21, max_entries: int = 4000) -> list[dict]:
    """A ClassBench-style ACL (the shape of the public "acl1" seed filters): 5-tuple rules with
    overlapping, nested source / destination prefixes of every length (a third wildcard), TCP /
    UDP / wildcard protocols, wildcard, exact and range ports (ranges expand into several ternary
    entries).  Some prefixes sit inside the pod network, so traffic meets partial matches all
    through the list and no tile prefilter can skip most of it.  Returns `acl.add` keyword dicts,
    highest priority first; their expansion stays within `max_entries` ternary entries."""
    rng = np.random.default_rng(seed)

    def seeds(k, inside):
        out = []
        for _ in range(k):
            ln = int(rng.choice([8, 12, 16, 20, 24, 28, 32]))
            base = (POD_NET | int(rng.integers(0, 1 << 16))) if inside and ln >= 16 else int(rng.integers(1, 224)) << 24 | int(rng.integers(0, 1 << 24))
            net = ipaddress.IPv4Network((base & ~((1 << (32 - ln)) - 1) & 0xFFFFFFFF, ln))
            out.append(net)
        return out

    pool = seeds(48, True) + seeds(144, False)
    # nesting: narrower children of some pool prefixes (overlap in both directions)
    for net in list(pool[:64]):
        if net.prefixlen <= 24:
            sub = list(net.subnets(new_prefix=min(32, net.prefixlen + int(rng.integers(2, 9)))))
            pool.append(sub[int(rng.integers(0, len(sub)))])

    def pfx():
        return None if rng.random() < 0.33 else str(pool[int(rng.integers(0, len(pool)))])

    def port(kind_p):
        u = rng.random()
        if u < kind_p[0]:
            return None
        if u < kind_p[0] + kind_p[1]:
            return int(rng.choice(WELL_KNOWN_PORTS)) if rng.random() < 0.7 else int(rng.integers(1024, 65536))
        if u < kind_p[0] + kind_p[1] + kind_p[2]:
            return (1024, 65535) if rng.random() < 0.6 else (0, 1023)
        lo = int(rng.integers(1024, 60000))
        return (lo, lo + int(rng.integers(3, 200)))

    rules, entries = [], 0
    while len(rules) < n_rules:
        r = dict(permit=bool(rng.random() < 0.25), src=pfx(), dst=pfx(),
                 proto=[6, 17, None][int(rng.choice(3, p=[0.45, 0.35, 0.20]))],
                 sport=port((0.78, 0.08, 0.12)), dport=port((0.30, 0.42, 0.18)))
        ns = 1 if not isinstance(r["sport"], tuple) else len(T.range_to_prefixes(*r["sport"]))
        nd = 1 if not isinstance(r["dport"], tuple) else len(T.range_to_prefixes(*r["dport"]))
        if entries + ns * nd > max_entries - (n_rules - len(rules) - 1):
            r["sport"] = None if ns > 1 else r["sport"]
            r["dport"] = int(rng.choice(WELL_KNOWN_PORTS)) if nd > 1 else r["dport"]
            ns = nd = 1
        rules.append(r)
        entries += ns * nd
    return rules


def install_acl_wild(dp, n_rules: int = 1024, seed: int = 21) -> dict:
    """Replace the ACL with `acl_wild_rules` + build_sfc's final pod-network permit.  Returns the
    previous rules (restore with ``dp.acl.rules = info["saved"]; dp.acl.version += 1``) and sizes."""
    saved = list(dp.acl.rules)
    final = saved[-1] if saved else None
    dp.acl.rules = []
    for r in acl_wild_rules(n_rules, seed):
        dp.acl.add(**r)
    if final is not None:
        dp.acl.rules.append(final)
    dp.acl.version += 1
    return {"saved": saved, "rules": n_rules + (final is not None), "entries": len(dp.acl.rules)}


ROUTER_MAC = "02:00:00:00:fe:01"


def install_l3_routes(dp, sc: Scenario, n_background: int = 100_000, seed: int = 13) -> dict:
    """Turn the SFC into an L3-routed SFC: the chain becomes acl -> nat -> route, every pod IP is a
    /32 route through an 8-way ECMP group of nexthops whose members all reach that pod (one
    neighbour MAC per member), and `n_background` random prefixes (/8 - /28, outside the pod
    network) fill the DIR-24-8 table like a real FIB.  Returns what was installed; the caller
    restores the chain with `dp.chains.set(sc.chain_id, hops)`."""
    rng = np.random.default_rng(seed)
    nh = 0
    for d in range(sc.n_pods):
        members = []
        for w in range(8):
            mac = bytes([0x02, 0x60, 0, 0, d & 0xFF, w])
            dp.nexthops.set(nh, int(sc.pod_port[d]), dmac=mac, smac=ROUTER_MAC)
            members.append(nh)
            nh += 1
        dp.ecmp.set_group(d, members)
        dp.routes.add(f"{ipaddress.IPv4Address(POD_NET + d)}/32", ecmp_group=d)
    sink = nh
    dp.nexthops.set(sink, int(sc.pod_port[0]), dmac=bytes([0x02, 0x60, 0, 0, 0xFF, 0xFF]), smac=ROUTER_MAC)
    plen = rng.integers(8, 29, n_background)
    base = rng.integers(0x0B000000, 0xDF000000, n_background, dtype=np.int64)
    added = 0
    for b, pl in zip(base.tolist(), plen.tolist()):
        net = b & ~((1 << (32 - pl)) - 1) & 0xFFFFFFFF
        if (net >> 16) == (POD_NET >> 16) or (net >> 24) == (POD_NET >> 24):
            continue
        dp.routes.add(f"{ipaddress.IPv4Address(net)}/{pl}", nexthop=sink)
        added += 1
    dp.chains.set(sc.chain_id, ["acl", "nat", "route"])
    return {"pod_routes": sc.n_pods, "ecmp_ways": 8, "background_prefixes": added, "nexthops": nh + 1}


# ---- dual stack: IPv6 pod flows next to the IPv4 SFC (bench value_ipv6) ----
POD6_NET = 0xFD00_0000_0000_0000_0000_0000_0A80_0000   # fd00::10.128.0.0/112-style pod addresses


def install_ipv6(dp, sc: Scenario, n_flows: int = 1 << 16, n_rules: int = 64, seed: int = 17) -> dict:
    """IPv6 flows between the scenario's pods (same chain: the NAT hop leaves IPv6 alone) and an
    IPv6 ACL of `n_rules` rules: /48 denies of unused fd01:: prefixes and dport denies, then a
    pod-network permit.  Vectorized: folded keys via tables.fold6's numpy twin, one insert_many.
    Returns the flows (for traffic_ipv6)."""
    rng = np.random.default_rng(seed)
    src = rng.integers(0, sc.n_pods, n_flows)
    dst = (src + rng.integers(1, max(sc.n_pods, 2), n_flows)) % sc.n_pods
    sport = rng.integers(1024, 65536, n_flows)
    dport = rng.integers(1024, 65536, n_flows)
    # addresses: POD6_NET + pod, unique per pod; words are the raw little-endian loads
    w_src = np.stack([T.ip6_raw(POD6_NET + int(p)) for p in range(sc.n_pods)])[src]
    w_dst = np.stack([T.ip6_raw(POD6_NET + int(p)) for p in range(sc.n_pods)])[dst]

    def fold(w):
        h = T.fmix32(w[:, 3] ^ np.uint32(0x6B43A9B5))
        for k in (2, 1, 0):
            h = T.fmix32(w[:, k] ^ h)
        return h

    keys = np.zeros((n_flows, 4), np.uint32)
    keys[:, 0], keys[:, 1] = fold(w_src), fold(w_dst)
    keys[:, 2] = P.port_raw(sport) | (P.port_raw(dport) << np.uint32(16))
    keys[:, 3] = 17 | T.KEY_V6 | (sc.bridge << 16)
    _, uniq = np.unique(keys.view(np.dtype((np.void, 16))), return_index=True)
    keep = np.sort(uniq)
    keys, src, dst, sport, dport = keys[keep], src[keep], dst[keep], sport[keep], dport[keep]
    w_src, w_dst = w_src[keep], w_dst[keep]
    actions = T.flow_action(chain_id=sc.chain_id, out_port=sc.pod_port[dst], flow_id=np.arange(len(keys)))
    dp.flows.insert_many(keys, actions)
    addrs = np.concatenate([w_src, w_dst], axis=1).astype(np.uint32)
    for k, a in zip(map(tuple, keys.tolist()), addrs):
        dp.flows6[k] = a
    if not dp._flow6_on:
        dp._flow6_on = True
        dp._flow6_full = True
    for r in range(max(n_rules - 1, 0)):
        if r % 8 == 7:
            dp.acl.add(permit=False, dport=int(rng.integers(1, 1024)), proto=17, family=6)
        else:
            dp.acl.add(permit=False, dst=f"fd01:{r:x}::/48", dport=int(1000 + r))
    if n_rules:
        dp.acl.add(permit=True, src="fd00::/96")
    return {"src": src, "dst": dst, "sport": sport, "dport": dport, "flows": len(keys), "rules": n_rules}


def traffic_ipv6(sc: Scenario, info: dict, n: int, seed: int = 1, frame_len: int = 62) -> tuple[np.ndarray, np.ndarray]:
    """n tagged IPv6 / UDP frames of random installed IPv6 flows from the source pod's VF
    (frame_len: untagged, no FCS; 62 = the smallest IPv6 / UDP frame).  (slots, inmeta)."""
    rng = np.random.default_rng(seed)
    f = rng.integers(0, len(info["src"]), n)
    s, d = info["src"][f], info["dst"][f]
    smac = np.frombuffer(b"".join(pod_mac(int(i)) for i in range(sc.n_pods)), np.uint8).reshape(-1, 6)[s]
    fr, ln = P.craft6_full(n, dmac=GW_MAC, smac=smac, src6=[POD6_NET + int(x) for x in s],
                           dst6=[POD6_NET + int(x) for x in d], sport=info["sport"][f], dport=info["dport"][f],
                           frame_len=frame_len, payload_seed=seed)
    tagged = np.zeros((n, frame_len + 4), np.uint8)
    tagged[:, :12] = fr[:, :12]
    tagged[:, 12], tagged[:, 13] = 0x81, 0x00
    vid = (s % 4094) + 2
    tagged[:, 14], tagged[:, 15] = (vid >> 8) & 0xFF, vid & 0xFF
    tagged[:, 16:] = fr[:, 12:]
    lens = ln + 4
    return P.header_slots(tagged, lens), P.inmeta(sc.pod_port[s], lens)


# ---- overlay: the SFC's traffic arriving VXLAN-encapsulated on a VTEP port (bench value_vxlan) ----
LOCAL_VTEP, REMOTE_VTEP, VXLAN_VNI = 0xC0000201, 0xC0000202, 5000   # 192.0.2.1 / .2
VTEP_MAC, UNDERLAY_GW_MAC, REMOTE_POD_MAC = "02:00:00:00:0e:01", "02:00:00:00:0e:02", "02:00:00:00:bb:01"


def install_vxlan(dp, sc: Scenario) -> dict:
    """An underlay VTEP port (local VTEP 192.0.2.1) and a tunnel port on the scenario's bridge whose
    (remote VTEP 192.0.2.2, VNI 5000) frames are terminated in one pass (wide header pairs) and run
    through the SFC as received on the tunnel port.  Returns the two ports."""
    vtep = int(sc.pod_port.max()) + 1
    tun = vtep + 1
    dp.ports.set(vtep, flags=T.PORT_VALID | T.PORT_VTEP, mac=VTEP_MAC)
    dp.ports.a[vtep]["ext"] = int(P.ip_raw(np.uint32(LOCAL_VTEP)))
    dp.ports.set(tun, flags=T.PORT_VALID | T.PORT_TUNNEL, bridge_id=sc.bridge)
    dp.ports.a[tun]["lag"] = 0
    dp.tunnels.set(0, src=str(ipaddress.IPv4Address(LOCAL_VTEP)), dst=str(ipaddress.IPv4Address(REMOTE_VTEP)),
                   vni=VXLAN_VNI, out_port=vtep, smac=VTEP_MAC, dmac=UNDERLAY_GW_MAC)
    dp.terms.insert(str(ipaddress.IPv4Address(REMOTE_VTEP)), VXLAN_VNI, tun)
    dp.ports.version += 1
    return {"vtep": vtep, "tunnel": tun}


def traffic_vxlan(sc: Scenario, ports: dict, n: int, seed: int = 1, inner_len: int = 60):
    """n VXLAN frames on the VTEP port: each inner frame (inner_len B, untagged, no FCS) is a packet
    of a random installed flow, from a remote MAC to the gateway.  Every frame is longer than 64 B,
    so it arrives as a wide header pair: returns (slots [2n, 64], inmeta [2n]) and the inner
    frames' flow indices."""
    rng = np.random.default_rng(seed)
    f = rng.integers(0, len(sc.keys), n)
    s, d = sc.flow_src_pod[f], sc.flow_dst_pod[f]
    inner, ilen = P.craft_full(n, dmac=GW_MAC, smac=REMOTE_POD_MAC, src_ip=POD_NET + s, dst_ip=POD_NET + d,
                               sport=sc.flow_sport[f], dport=sc.flow_dport[f], proto=17, frame_len=inner_len,
                               payload_seed=seed)
    L = 50 + inner_len
    fr = np.zeros((n, max(L, 128)), np.uint8)
    fr[:, 0:6] = P.mac_bytes(VTEP_MAC)
    fr[:, 6:12] = P.mac_bytes(UNDERLAY_GW_MAC)
    fr[:, 12], fr[:, 13] = 0x08, 0x00
    ip = np.zeros(20, np.uint8)
    ip[0], ip[8], ip[9] = 0x45, 64, 17
    ip[2:4] = np.frombuffer((20 + 8 + 8 + inner_len).to_bytes(2, "big"), np.uint8)
    ip[6] = 0x40
    ip[12:16] = np.frombuffer(REMOTE_VTEP.to_bytes(4, "big"), np.uint8)
    ip[16:20] = np.frombuffer(LOCAL_VTEP.to_bytes(4, "big"), np.uint8)
    c = int(sum(int.from_bytes(bytes(ip[k:k + 2]), "big") for k in range(0, 20, 2)))
    while c >> 16:
        c = (c & 0xFFFF) + (c >> 16)
    ip[10:12] = np.frombuffer((~c & 0xFFFF).to_bytes(2, "big"), np.uint8)
    fr[:, 14:34] = ip
    sport = 0xC000 | (rng.integers(0, 0x4000, n))
    fr[:, 34], fr[:, 35] = (sport >> 8) & 0xFF, sport & 0xFF
    fr[:, 36], fr[:, 37] = 4789 >> 8, 4789 & 0xFF
    fr[:, 38], fr[:, 39] = ((8 + 8 + inner_len) >> 8) & 0xFF, (8 + 8 + inner_len) & 0xFF
    fr[:, 42] = 0x08
    fr[:, 46:49] = np.frombuffer(VXLAN_VNI.to_bytes(3, "big"), np.uint8)
    fr[:, 50:50 + inner_len] = inner[:, :inner_len]
    lens = np.full(n, L, np.uint32)
    slots, im, _ = P.wide_slots(fr, lens, ports["vtep"], wide_ports={ports["vtep"]})
    return slots, im, f


def install_vxlan_egress(dp, sc: Scenario) -> dict:
    """Every pod's VF becomes a VXLAN tunnel port (tunnel 0: local VTEP 192.0.2.1 -> remote
    192.0.2.2, VNI 5000, out of an underlay VTEP port): the headline's traffic then leaves
    encapsulated, so each forwarded packet also gets its outer-header record from the side pass.
    Returns the underlay port."""
    vtep = int(sc.pod_port.max()) + 1
    dp.ports.set(vtep, flags=T.PORT_VALID, mac=VTEP_MAC)
    dp.tunnels.set(0, src=str(ipaddress.IPv4Address(LOCAL_VTEP)), dst=str(ipaddress.IPv4Address(REMOTE_VTEP)),
                   vni=VXLAN_VNI, out_port=vtep, smac=VTEP_MAC, dmac=UNDERLAY_GW_MAC)
    for p in sc.pod_port:
        dp.ports.a[int(p)]["flags"] |= np.uint32(T.PORT_TUNNEL)
        dp.ports.a[int(p)]["lag"] = 0
    dp.ports.version += 1
    return {"underlay": vtep}
