"""IPv6 on the data plane: routed interfaces over the IPv6 FIB (P4 ipv6_table: LPM, nexthops,
8-way ECMP, hop limit), and IPv6 bridged by MAC on L2 ports.

Expectations are independent of the kernels: a Python longest-prefix match over the route set
(`Route6Table.lookup`, the `ipaddress` module) and field-by-field frame checks; the UDP checksum
is verified over the IPv6 pseudo-header after forwarding (the hop limit is not covered by it, so a
routed frame's L4 checksum stays valid).  The GPU test holds the HIP kernel to the oracle bit for
bit."""
import ipaddress

import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P

RMAC = ["02:40:00:00:00:0a", "02:40:00:00:00:0b", "02:40:00:00:00:0c", "02:40:00:00:00:0d"]
NBR = ["02:50:00:00:00:0a", "02:50:00:00:00:0b", "02:50:00:00:00:0c", "02:50:00:00:00:0d"]
POOL = ["2001:db8:9::1", "2001:db8:1:7::5", "2001:db8:1:2::77", "2001:db8:1:2::99", "2001:db8:1:2:ffff::1",
        "2600::1", "2001:db8:ffff::2", "fd00::1"]


def _router(device):
    dp = DataPlane(device=device, flow_buckets=1 << 10)
    for i in range(4):
        dp.ports.set(10 + i, flags=T.PORT_VALID | T.PORT_ROUTED, mac=RMAC[i], bridge_id=20 + i)
        dp.nexthops.set(i + 1, 10 + i, dmac=NBR[i], smac=RMAC[i])
    dp.ecmp.set_group(0, [2, 3])
    dp.routes6.add("::/0", nexthop=1)
    dp.routes6.add("2001:db8::/32", nexthop=2)
    dp.routes6.add("2001:db8:1::/48", nexthop=3)
    dp.routes6.add("2001:db8:1:2::/64", ecmp_group=0)
    dp.routes6.add("2001:db8:1:2::99/128", nexthop=4)
    dp.routes6.add("fd00::/8", nexthop=4)
    dp.commit(full=True)
    return dp


def _trace(n=512, seed=0):
    rng = np.random.default_rng(seed)
    dsts = [POOL[i] for i in rng.integers(0, len(POOL), n)]
    hl = np.where(rng.random(n) < 0.05, 1, 64).astype(np.uint8)
    sizes = np.where(np.arange(n) % 3 == 0, 1500, 90)
    full = np.zeros((n, 1500), np.uint8)
    lens = np.zeros(n, np.uint32)
    for sz in (90, 1500):
        idx = np.where(sizes == sz)[0]
        fr, ln = P.craft6_full(len(idx), dmac=RMAC[0], smac=NBR[0], src6="2001:db8:77::1",
                               dst6=[dsts[i] for i in idx], sport=rng.integers(1024, 65535, len(idx)), dport=53,
                               hop_limit=hl[idx], frame_len=sz, payload_seed=sz)
        full[idx, :sz] = fr
        lens[idx] = ln
    return P.header_slots(full, lens), P.inmeta(np.full(n, 10), lens), full, lens, dsts, hl


def _udp6_ok(o: bytes) -> bool:
    fr = np.frombuffer(o, np.uint8)
    seg = fr[54:].astype(np.uint64)
    if len(seg) & 1:
        seg = np.append(seg, 0)
    w = (seg[0::2] << 8) | seg[1::2]
    ps = fr[22:54].astype(np.uint64)
    c = int(w.sum() + ((ps[0::2] << 8) | ps[1::2]).sum() + (len(fr) - 54) + 17)
    while c >> 16:
        c = (c & 0xFFFF) + (c >> 16)
    return c == 0xFFFF


def test_lpm6_reference_and_build():
    t = T.Route6Table()
    t.add("2001:db8::/32", nexthop=1)
    t.add("2001:db8:1::/48", nexthop=2)
    t.add("::/0", ecmp_group=3)
    assert t.lookup("2001:db8:1::5") == T.ROUTE_NH | 2
    assert t.lookup("2001:db8:2::5") == T.ROUTE_NH | 1
    assert t.lookup("::1") == T.ROUTE_ECMP | 3
    tab, lens, nl = t.build()
    assert list(lens[:nl]) == [48, 32, 0] and tab.shape[1] == 8 and tab.shape[0] >= 6


def test_ipv6_routing_oracle_model():
    dp = _router("cpu")
    slots, im, frames, lens, dsts, hl = _trace()
    r = dp.run(slots, im)
    port, olen, reason = P.meta_fields(r.meta)
    ecmp_used = set()
    for i in range(len(dsts)):
        res = dp.routes6.lookup(dsts[i])
        if hl[i] == 1:
            assert reason[i] == 8  # hop limit exceeded
            continue
        if res & T.ROUTE_ECMP:
            # member chosen by a hash of the IPv6 addresses / ports: any member of the group
            nh = int(port[i]) - 9
            assert nh in set(int(x) for x in dp.ecmp.a[(res & 0xFFFF) * 8:(res & 0xFFFF) * 8 + 8]), (i, dsts[i])
            ecmp_used.add(nh)
        else:
            nh = res & 0xFFFF
        assert (reason[i], port[i]) == (0, 9 + nh), (i, dsts[i], hex(res))
        o = P.assemble(r.out[i], int(r.meta[i]), frames[i], int(lens[i]))
        assert len(o) == lens[i]
        assert o[0:6] == bytes.fromhex(NBR[nh - 1].replace(":", "")) and o[6:12] == bytes.fromhex(RMAC[nh - 1].replace(":", ""))
        assert o[21] == hl[i] - 1
        assert o[22:] == bytes(frames[i, 22:int(lens[i])])   # addresses + L4 untouched
        assert _udp6_ok(o)
    assert ecmp_used == {2, 3}


def test_ipv6_no_route_and_l2_bridging():
    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    dp.ports.set(1, flags=T.PORT_VALID | T.PORT_ROUTED, mac=RMAC[0], bridge_id=3)
    dp.ports.set(2, flags=T.PORT_VALID, bridge_id=3)
    dp.ports.set(3, flags=T.PORT_VALID, bridge_id=3)
    dp.macs.insert(3, NBR[2], 3)
    dp.routes6.add("2001:db8::/32", nexthop=0)
    dp.nexthops.set(0, 2, dmac=NBR[1], smac=RMAC[0])
    dp.commit(full=True)
    fr, ln = P.craft6_full(3, dmac=np.stack([P.mac_bytes(m) for m in (RMAC[0], RMAC[0], NBR[2])]), smac=NBR[0],
                           src6="2001:db8::1",
                           dst6=["2001:db8::2", "2600::1", "2001:db8::3"], sport=1, dport=2)
    r = dp.run(P.header_slots(fr, ln), P.inmeta(np.array([1, 1, 2]), ln))
    port, _, reason = P.meta_fields(r.meta)
    assert (int(reason[0]), int(port[0])) == (0, 2)          # routed
    assert int(reason[1]) == 5 and int(port[1]) == T.PORT_PUNT  # no route: punted
    assert (int(reason[2]), int(port[2])) == (0, 3)          # not to the router MAC: bridged by MAC


@pytest.mark.gpu
def test_ipv6_routing_gpu_bit_exact():
    import torch

    c, g = _router("cpu"), _router("cuda")
    slots, im, _, _, _, _ = _trace(4096, seed=3)
    rc = c.run(slots, im)
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert c.drop_counters() == g.drop_counters()
