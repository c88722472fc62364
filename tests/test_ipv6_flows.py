"""IPv6 flow state: exact 5-tuple flows and the IPv6 ACL (TCAM over src6 / dst6 / ports / next
header / zone), VERDICT r2 missing #6.

Expectations come from an independent model: a Python dict keyed by the full 5-tuple (no
folding), first-match ACL evaluation with the `ipaddress` module, and the chain's MAC rewrite
spelled out field by field.  The data plane folds each IPv6 address into one FlowKey word
(nfdp.h fold6) and checks the slot's side entry on every hit, so a packet whose folded key
collides with an installed flow must miss: the test crafts such an address by inverting fmix32.
The GPU tests hold the fused kernel (v6_kernel pre-pass + the V6 instances) and the ring kernel to
the C++ oracle bit for bit."""
import ipaddress

import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P

POD_MAC = {101: "02:00:00:00:00:01", 102: "02:00:00:00:00:02", 103: "02:00:00:00:00:03", 104: "02:00:00:00:00:04"}
PEER_MAC = {101: "0a:00:00:00:00:01", 102: "0a:00:00:00:00:02", 103: "0a:00:00:00:00:03", 104: "0a:00:00:00:00:04"}
BRIDGE = 7
SRCS = ["2001:db8:a::1", "2001:db8:a::2", "fd00:1::5", "2001:db8:b:c::9"]
DSTS = ["2001:db8:f::1", "fd00:bad::7", "2001:db8:f::2", "2600::1"]


def _inv_fmix32(h: int) -> int:
    """Inverse of nfdp.h fmix32 (each step is a bijection on 32 bits)."""
    def unxorshift(x, s):
        r = x
        for _ in range(32 // s + 1):
            r = x ^ (r >> s)
        return r & 0xFFFFFFFF

    h = unxorshift(h, 16)
    h = (h * pow(0xC2B2AE35, -1, 1 << 32)) & 0xFFFFFFFF
    h = unxorshift(h, 13)
    h = (h * pow(0x85EBCA6B, -1, 1 << 32)) & 0xFFFFFFFF
    return unxorshift(h, 16)


def _colliding_addr(addr: str) -> str:
    """Another IPv6 address with the same fold6 value as `addr` (different low words, first word solved)."""
    w = [int(x) for x in T.ip6_raw(addr)]
    target = T.fold6(w)
    w2 = [0, w[1] ^ 0x01000000, w[2], w[3] ^ 0x00FF0000]
    h = int(T.fmix32(np.uint32(w2[3]) ^ np.uint32(0x6B43A9B5)))
    h = int(T.fmix32(np.uint32(w2[2]) ^ np.uint32(h)))
    h = int(T.fmix32(np.uint32(w2[1]) ^ np.uint32(h)))
    w2[0] = _inv_fmix32(target) ^ h
    assert T.fold6(w2) == target and w2 != w
    return str(ipaddress.IPv6Address(np.array(w2, "<u4").tobytes()))


def _plane(device, nflows=64, seed=0, hops=("acl", "l2fwd")):
    dp = DataPlane(device=device, flow_buckets=1 << 10)
    for p in POD_MAC:
        dp.ports.set(p, flags=T.PORT_VALID, bridge_id=BRIDGE, mac=POD_MAC[p], peer_mac=PEER_MAC[p])
    chain = dp.chains.add(list(hops))
    # IPv6 ACL: deny one /32, deny TCP dport 22, permit the rest of fd00::/8 explicitly
    dp.acl.add(permit=False, dst="fd00:bad::/32")
    dp.acl.add(permit=False, proto=6, dport=22, family=6)
    dp.acl.add(permit=True, src="fd00::/8")
    dp.acl.add(permit=False, dst="10.9.0.0/16")            # an IPv4 rule: never applies to IPv6
    rng = np.random.default_rng(seed)
    flows = {}
    for i in range(nflows):
        s, d = SRCS[i % len(SRCS)], DSTS[(i // 2) % len(DSTS)]
        sport, dport = int(rng.integers(1024, 60000)), [22, 80, 443, 53][i % 4]
        proto = 6 if i % 3 == 0 else 17
        out = 101 + (i % 4)
        dp.add_flow6(s, d, sport, dport, proto, BRIDGE, T.flow_action(chain_id=chain, out_port=out, flow_id=i)[0])
        flows[(s, d, sport, dport, proto)] = out
    dp.commit(full=True)
    return dp, flows


def _model_acl(dp, src, dst, sport, dport, proto):
    """First-match over the IPv6 rules with ipaddress semantics (rules re-derived from their words)."""
    for r in dp.acl.rules6:
        def words_net(base):
            v = np.array(r.value[base:base + 4], "<u4").tobytes()
            m = np.array(r.mask[base:base + 4], "<u4").tobytes()
            return int.from_bytes(v, "big"), int.from_bytes(m, "big")
        ok = True
        for base, a in ((0, src), (4, dst)):
            v, m = words_net(base)
            ok &= (int(ipaddress.IPv6Address(a)) & m) == v
        pv = (int(r.value[8]) & int(r.mask[8]))
        pw = (int(P.port_raw(np.uint32(sport))) | (int(P.port_raw(np.uint32(dport))) << 16)) if proto in (6, 17) else 0
        ok &= (pw & int(r.mask[8])) == pv
        ok &= ((proto | (BRIDGE << 16)) & int(r.mask[9])) == int(r.value[9])
        if ok:
            return r.permit
    return dp.acl.default_permit


def _trace(flows, n=1024, seed=1):
    rng = np.random.default_rng(seed)
    keys = list(flows)
    coll = _colliding_addr(keys[0][0])
    pk = []
    for j in range(n):
        k = keys[int(rng.integers(0, len(keys)))]
        kind = j % 8
        if kind == 5:            # unknown 5-tuple (sport off by one): a miss
            k = (k[0], k[1], k[2] + 1, k[3], k[4])
        elif kind == 6:          # the folded key of flow 0 from another source address: must miss
            k = (coll, keys[0][1], keys[0][2], keys[0][3], keys[0][4])
        pk.append(k)
    frames, lens, inp = [], [], []
    for (s, d, sp, dp_, pr) in pk:
        fr, ln = P.craft6_full(1, dmac="0e:00:00:00:00:99", smac=PEER_MAC[101], src6=s, dst6=d, sport=sp, dport=dp_,
                               frame_len=90)
        fr[0, 20] = pr
        frames.append(fr[0]); lens.append(ln[0]); inp.append(101)
    fr = np.stack(frames)
    ln = np.array(lens, np.uint32)
    return P.header_slots(fr, ln), P.inmeta(np.array(inp), ln), pk


def _expect(dp, flows, pk):
    exp = []
    for k in pk:
        out = flows.get(k)
        if out is None:
            exp.append((5, None))   # no flow, no MAC entry: punted (no_route)
        elif not _model_acl(dp, *k):
            exp.append((4, None))
        else:
            exp.append((0, out))
    return exp


def test_flow_key6_fold_matches_native():
    from dpu_operator_amd.native import nfdp

    w = [int(x) for x in T.ip6_raw("2001:db8::1234:5678")]
    assert T.fold6(w) == int(nfdp().fold6(*w))
    key, addrs = T.flow_key6("2001:db8::1", "fd00::2", 1000, 443, 6, 3)
    assert int(key[3]) == 6 | T.KEY_V6 | (3 << 16) and len(addrs) == 8
    assert _colliding_addr("2001:db8:a::1") != "2001:db8:a::1"


def test_ipv6_flows_oracle_vs_independent_model():
    dp, flows = _plane("cpu")
    slots, im, pk = _trace(flows)
    r = dp.run(slots, im)
    port, olen, reason = P.meta_fields(r.meta)
    exp = _expect(dp, flows, pk)
    for j, (er, eport) in enumerate(exp):
        assert int(reason[j]) == er, (j, pk[j], int(reason[j]), er)
        if er == 0:
            assert int(port[j]) == eport
            o = r.out[j].tobytes()
            assert o[0:6] == P.mac_bytes(PEER_MAC[eport]).tobytes() and o[6:12] == P.mac_bytes(POD_MAC[eport]).tobytes()
            assert o[12:] == slots[j].tobytes()[12:]            # only the MACs change for IPv6
    # the colliding address missed although its folded key is installed
    assert sum(1 for k in pk if k[0] not in SRCS) > 0
    # per-flow counters: every hit counted on its flow
    dp.harvest()
    hits = sum(1 for e in exp if e[0] != 5)
    assert int(dp.flow_totals[:, 0].sum()) == hits


def test_ipv6_flow_remove_and_rules_dont_leak_to_ipv4():
    dp, flows = _plane("cpu", nflows=8)
    k = next(iter(flows))
    assert dp.remove_flow6(*k[:4], k[4], BRIDGE)
    dp.commit()
    slots, im, _ = _trace({k: 101}, n=8)
    r = dp.run(slots, im)
    _, _, reason = P.meta_fields(r.meta)
    assert int(reason[0]) == 5     # removed: the flow stage misses, L2 punts
    # an IPv4 packet is classified by the IPv4 rules only (10.9/16 denied, nothing else)
    assert len(dp.acl.rules6) == 3 and len(dp.acl.rules) == 1


def test_ipv6_flow_collision_is_refused():
    dp = DataPlane(device="cpu", flow_buckets=1 << 8)
    dp.add_flow6("2001:db8:a::1", "2001:db8:f::1", 5, 6, 17)
    with pytest.raises(ValueError):
        dp.add_flow6(_colliding_addr("2001:db8:a::1"), "2001:db8:f::1", 5, 6, 17)
    # removing the never-installed colliding 5-tuple leaves the installed flow alone
    assert not dp.remove_flow6(_colliding_addr("2001:db8:a::1"), "2001:db8:f::1", 5, 6, 17)
    assert len(dp.flows) == 1 and len(dp.flows6) == 1
    assert dp.remove_flow6("2001:db8:a::1", "2001:db8:f::1", 5, 6, 17)
    assert len(dp.flows) == 0 and not dp.flows6


@pytest.mark.gpu
def test_ipv6_flows_gpu_bit_exact():
    import torch

    (c, flows), (g, _) = _plane("cpu"), _plane("cuda")
    slots, im, pk = _trace(flows, n=8192, seed=4)
    rc = c.run(slots, im)
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert c.drop_counters() == g.drop_counters()
    c.harvest(); g.harvest()
    assert np.array_equal(c.flow_totals, g.flow_totals)


@pytest.mark.gpu
def test_ipv6_flows_mixed_with_ipv4_gpu_bit_exact():
    """IPv6 flows + rules and the IPv4 headline scenario's traffic in one batch (V6 instances)."""
    import torch

    from dpu_operator_amd.dataplane import scenario

    def build(dev):
        dp = DataPlane(device=dev, flow_buckets=1 << 13)
        sc = scenario.build_sfc(dp, n_pods=8, n_flows=1 << 14, n_acl=64, seed=3)
        for p in POD_MAC:
            dp.ports.set(p, flags=T.PORT_VALID, bridge_id=BRIDGE, mac=POD_MAC[p], peer_mac=PEER_MAC[p])
        chain = dp.chains.add(["acl", "l2fwd"])
        dp.acl.add(permit=False, dst="fd00:bad::/32")
        for i, s in enumerate(SRCS):
            dp.add_flow6(s, DSTS[i], 1000 + i, 80, 17, BRIDGE, T.flow_action(chain_id=chain, out_port=101 + i)[0])
        dp.commit(full=True)
        return dp, sc

    (c, sc), (g, _) = build("cpu"), build("cuda")
    s4, i4 = scenario.traffic(sc, 4096, seed=9)
    fl = {(SRCS[i], DSTS[i], 1000 + i, 80, 17): 101 + i for i in range(4)}
    s6, i6, _ = _trace(fl, n=4096, seed=2)
    slots = np.concatenate([s4, s6]); im = np.concatenate([i4, i6])
    perm = np.random.default_rng(0).permutation(len(slots))
    slots, im = np.ascontiguousarray(slots[perm]), np.ascontiguousarray(im[perm])
    rc = c.run(slots, im)
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)


def test_dual_stack_scenario_forwards_everything():
    """bench.py's value_ipv6 traffic on the oracle: every IPv6 packet hits its flow and is forwarded
    to the destination pod (and tagged by the egress port), IPv4 unchanged."""
    from dpu_operator_amd.dataplane import scenario as S

    dp = DataPlane(device="cpu", flow_buckets=1 << 12)
    sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 11, n_acl=16, seed=1)
    info = S.install_ipv6(dp, sc, 1 << 10, 16)
    dp.commit(full=True)
    pk6, im6 = S.traffic_ipv6(sc, info, 512, seed=3)
    pk4, im4 = S.traffic(sc, 512, seed=4)
    r = dp.run(np.concatenate([pk4, pk6]), np.concatenate([im4, im6]))
    port, _, reason = P.meta_fields(r.meta)
    assert np.all(reason == 0)
    rng = np.random.default_rng(3)
    f = rng.integers(0, len(info["src"]), 512)
    assert np.array_equal(port[512:], sc.pod_port[info["dst"][f]])
    dp.harvest()
    assert int(dp.flow_totals[:, 0].sum()) == 1024


@pytest.mark.gpu
@pytest.mark.parametrize("n_acl", [256, 1024])
def test_ipv6_flows_big_batch_gpu_bit_exact(n_acl):
    """More packets than one grid-stride pass of v6_kernel and of the fused kernel (the IPv6 key
    hand-over through the out slots must address whole slots), on the 4-wave and the early-fetch
    V6 instances."""
    import torch

    from dpu_operator_amd.dataplane import scenario as S

    def build(dev):
        dp = DataPlane(device=dev, flow_buckets=1 << 16, hash_mode="lds", acl_mode="mfma")
        sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 16, n_acl=n_acl, seed=0)
        info6 = S.install_ipv6(dp, sc, 1 << 14, 64)
        dp.commit(full=True)
        return dp, sc, info6

    (g, sc, info6), (c, _, _) = build("cuda"), build("cpu")
    pk6, im6 = S.traffic_ipv6(sc, info6, 1 << 19, seed=5)
    pk4, im4 = S.traffic(sc, 1 << 19, seed=6)
    perm = np.random.default_rng(1).permutation(1 << 20)
    pk, im = np.ascontiguousarray(np.concatenate([pk4, pk6])[perm]), np.ascontiguousarray(np.concatenate([im4, im6])[perm])
    rc = c.run(pk, im)
    r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    m = r.meta.cpu().numpy().view(np.uint32)
    assert np.array_equal(m, rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert (P.meta_fields(m)[2] == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("coop", [True, False])
def test_ipv6_flows_ring_kernel_bit_exact(coop):
    """The persistent ring kernel's V6 instances (inline fold, scalar IPv6 TCAM, side check) on a
    dual-stack trace, against the oracle."""
    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.ring import RingPath

    cap = 1 << 14

    def build(dev):
        dp = DataPlane(device=dev, flow_buckets=1 << 14, hash_mode="lds", acl_mode="mfma")
        sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 14, n_acl=64, seed=0)
        info6 = S.install_ipv6(dp, sc, 1 << 12, 16)
        dp.commit(full=True)
        return dp, sc, info6

    (g, sc, info6), (c, _, _) = build("cuda"), build("cpu")
    pk6, im6 = S.traffic_ipv6(sc, info6, cap // 2, seed=5)
    pk4, im4 = S.traffic(sc, cap // 2, seed=6)
    perm = np.random.default_rng(2).permutation(cap)
    pk, im = np.ascontiguousarray(np.concatenate([pk4, pk6])[perm]), np.ascontiguousarray(np.concatenate([im4, im6])[perm])
    ring = RingPath(g, capacity=cap, deadline_s=30.0, coop=coop)
    try:
        ring.stage(pk, im)
        ring.start()
        for _ in range(4):
            end = ring.publish(cap // 4)
        ring.wait(end, 10.0)
        ring.stop()
        out, meta = ring.results()
    finally:
        ring.close()
    rc = c.run(pk, im)
    assert np.array_equal(meta, rc.meta)
    assert np.array_equal(out, rc.out)
    assert (P.meta_fields(meta)[2] == 0).all()
    g.harvest()
    c.harvest()
    assert np.array_equal(g.flow_totals, c.flow_totals)


def _hop_limits(slots, every=5):
    s = slots.copy()
    s[::every, 21] = 1          # (UDP checksum does not cover the hop limit)
    return s


def test_ipv6_ttl_hop_decrements_hop_limit():
    """The chain's ttl hop on an IPv6 flow: hop limit - 1, or ttl_expired at 1."""
    dp, flows = _plane("cpu", hops=("acl", "ttl", "l2fwd"))
    slots, im, pk = _trace(flows, n=256)
    slots = _hop_limits(slots)
    r = dp.run(slots, im)
    port, _, reason = P.meta_fields(r.meta)
    exp = _expect(dp, flows, pk)
    for j, (er, _) in enumerate(exp):
        if er != 0:
            continue
        if slots[j, 21] == 1:
            assert int(reason[j]) == 8
        else:
            assert int(reason[j]) == 0 and r.out[j, 21] == slots[j, 21] - 1


@pytest.mark.gpu
def test_ipv6_ttl_hop_gpu_bit_exact():
    import torch

    (c, flows), (g, _) = _plane("cpu", hops=("acl", "ttl", "l2fwd")), _plane("cuda", hops=("acl", "ttl", "l2fwd"))
    slots, im, _ = _trace(flows, n=4096, seed=6)
    slots = _hop_limits(slots)
    rc = c.run(slots, im)
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert (P.meta_fields(rc.meta)[2] == 8).sum() > 100
