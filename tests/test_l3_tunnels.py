"""L3 routing (P4 ipv4_table LPM, nexthop_table, ecmp_hash_table, rif_mod_table) and VXLAN /
GENEVE tunnels (encap on tunnel ports, termination + recirculation) on the data plane.

Expectations are computed independently: a Python longest-prefix match over the route set,
field-by-field frame models, full IPv4 / UDP checksum verification of the assembled frames.
The GPU tests hold the HIP kernels to the oracle bit for bit (outer-header records included)."""
import ipaddress

import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P

RMAC = ["02:40:00:00:00:0a", "02:40:00:00:00:0b", "02:40:00:00:00:0c", "02:40:00:00:00:0d"]
NBR = ["02:50:00:00:00:0a", "02:50:00:00:00:0b", "02:50:00:00:00:0c", "02:50:00:00:00:0d"]


VM_DST = {"10.1.2.5": "02:66:00:00:00:05", "10.1.2.200": "02:66:00:00:00:c8"}   # vm_dst_ip4_mac_map
VM_SRC = {"10.9.0.1": "02:77:00:00:00:01"}                                        # vm_src_ip4_mac_map


def _router(device, vmmac=False):
    dp = DataPlane(device=device, flow_buckets=1 << 10)
    if vmmac:
        for ip, mac in VM_DST.items():
            dp.vmmac.set(ip, T.VMMAC_DST, mac)
        for ip, mac in VM_SRC.items():
            dp.vmmac.set(ip, T.VMMAC_SRC, mac)
    for i in range(4):
        dp.ports.set(10 + i, flags=T.PORT_VALID | T.PORT_ROUTED, mac=RMAC[i], bridge_id=20 + i)
        dp.nexthops.set(i + 1, 10 + i, dmac=NBR[i], smac=RMAC[i])
    dp.ecmp.set_group(0, [2, 3])
    dp.routes.add("10.1.0.0/16", nexthop=2)
    dp.routes.add("10.1.2.0/24", nexthop=3)
    dp.routes.add("10.1.2.128/25", ecmp_group=0)
    dp.routes.add("10.1.2.200/32", nexthop=4)
    dp.routes.add("0.0.0.0/0", nexthop=1)
    dp.commit(full=True)
    return dp


def _l3_trace(n=512, seed=0):
    rng = np.random.default_rng(seed)
    pool = ["10.1.9.9", "10.1.2.5", "10.1.2.129", "10.1.2.250", "10.1.2.200", "8.8.8.8", "10.2.0.1"]
    dsts = np.array([int(ipaddress.IPv4Address(pool[i])) for i in rng.integers(0, len(pool), n)], np.uint32)
    ttl = np.where(rng.random(n) < 0.05, 1, 64)
    frames, lens = [], []
    for sz in (64, 1500):
        idx = np.arange(n)[(np.arange(n) % 2) == (sz == 1500)]
        fr, ln = P.craft_full(len(idx), dmac=RMAC[0], smac=NBR[0], src_ip=0x0A090001, dst_ip=dsts[idx],
                              sport=rng.integers(1024, 65535, len(idx)), dport=80, proto=17, frame_len=sz - 4)
        frames.append((idx, fr, ln))
    full = np.zeros((n, 1500), np.uint8)
    lens = np.zeros(n, np.uint32)
    for idx, fr, ln in frames:
        full[idx, : fr.shape[1]] = fr[:, :1500]
        lens[idx] = ln
    full[ttl == 1, 22] = 1
    # TTL change needs the IPv4 checksum redone for those
    for i in np.where(ttl == 1)[0]:
        full[i, 24:26] = 0
        w = (full[i, 14:34:2].astype(np.uint32) << 8) | full[i, 15:34:2]
        c = int(w.sum())
        c = (c & 0xFFFF) + (c >> 16)
        c = (c & 0xFFFF) + (c >> 16)
        full[i, 24], full[i, 25] = (~c >> 8) & 0xFF, ~c & 0xFF
    return P.header_slots(full, lens), P.inmeta(np.full(n, 10), lens), full, lens, dsts, ttl


def test_routing_oracle_model():
    dp = _router("cpu")
    slots, im, frames, lens, dsts, ttl = _l3_trace()
    r = dp.run(slots, im)
    port, olen, reason = P.meta_fields(r.meta)
    h = r.extra["hash"]
    for i in range(len(dsts)):
        res = dp.routes.lookup(int(dsts[i]))
        if ttl[i] == 1:
            assert reason[i] == 8  # ttl_expired
            continue
        nh = res & 0xFFFF if res & T.ROUTE_NH else int(dp.ecmp.a[(res & 0xFFFF) * 8 + (int(h[i]) & 7)])
        assert (reason[i], port[i]) == (0, 9 + nh), (i, hex(res))
        o = P.assemble(r.out[i], int(r.meta[i]), frames[i], int(lens[i]))
        assert o[0:6] == bytes.fromhex(NBR[nh - 1].replace(":", "")) and o[6:12] == bytes.fromhex(RMAC[nh - 1].replace(":", ""))
        assert o[22] == 63 and len(o) == lens[i]
        assert P.check_csums(np.frombuffer(o, np.uint8)[None], np.array([len(o)]))[0]
    ecmp_nh = {int(dp.ecmp.a[(int(h[i]) & 7)]) for i in range(len(dsts))
               if ttl[i] != 1 and dp.routes.lookup(int(dsts[i])) & T.ROUTE_ECMP}
    assert ecmp_nh == {2, 3}  # both ECMP members used


def test_vm_mac_maps_oracle_model():
    """VM IPv4 -> MAC maps on routed traffic: mapped destinations get the map's dmac, the mapped
    source (every packet of the trace) the map's smac; port, TTL and checksums as without maps."""
    dp = _router("cpu", vmmac=True)
    slots, im, frames, lens, dsts, ttl = _l3_trace()
    r = dp.run(slots, im)
    port, olen, reason = P.meta_fields(r.meta)
    for i in range(len(dsts)):
        if ttl[i] == 1:
            continue
        assert reason[i] == 0
        o = P.assemble(r.out[i], int(r.meta[i]), frames[i], int(lens[i]))
        d = str(ipaddress.IPv4Address(int(dsts[i])))
        if d in VM_DST:
            assert o[0:6] == bytes.fromhex(VM_DST[d].replace(":", ""))
        else:
            assert o[0:6] == bytes.fromhex(NBR[int(port[i]) - 10].replace(":", ""))
        assert o[6:12] == bytes.fromhex(VM_SRC["10.9.0.1"].replace(":", ""))
        assert P.check_csums(np.frombuffer(o, np.uint8)[None], np.array([len(o)]))[0]


def test_route_hop_in_a_chain_and_no_route():
    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    dp.ports.set(1, flags=T.PORT_VALID, mac="02:00:00:00:00:01")
    dp.ports.set(2, flags=T.PORT_VALID, mac="02:00:00:00:00:02")
    dp.nexthops.set(0, 2, dmac=NBR[1], smac=RMAC[1])
    dp.routes.add("192.0.2.0/24", nexthop=0)
    cid = dp.chains.add(["nat", "route"])
    keys = T.flow_key([0x0A000001, 0x0A000001], [0xC0000205, 0xC6336405], [5, 5], [7, 7], 17, 0)
    dp.flows.insert_many(keys, np.repeat(T.flow_action(chain_id=cid, out_port=1, nat_ip=0xC6336401, nat_port=999), 2, axis=0))
    dp.commit(full=True)
    fr, ln = P.craft(2, dmac="02:00:00:00:00:01", smac="02:00:00:00:00:99", src_ip=0x0A000001,
                     dst_ip=np.array([0xC0000205, 0xC6336405], np.uint32), sport=5, dport=7)
    r = dp.run(fr, P.inmeta(np.array([1, 1]), ln))
    port, _, reason = P.meta_fields(r.meta)
    assert (int(port[0]), int(reason[0])) == (2, 0)                 # SNAT then routed
    assert (int(port[1]), int(reason[1])) == (T.PORT_PUNT, 5)       # no route -> slow path
    assert bytes(r.out[0][26:30]) == bytes([198, 51, 100, 1]) and r.out[0][22] == 63


LOCAL_VTEP, REMOTE_VTEP = "192.0.2.1", "192.0.2.2"
POD_MAC, REMOTE_MAC = "02:00:00:00:aa:01", "02:00:00:00:bb:01"


def _overlay(device, kind=T.TUN_VXLAN):
    """Pod port 1 on bridge 3; tunnel port 20 -> underlay port 30 (VTEP 192.0.2.1); remote MAC behind
    the tunnel (l2_to_tunnel_v4); (192.0.2.2, vni 5000) terminates onto port 20."""
    dp = DataPlane(device=device, flow_buckets=1 << 10)
    dp.ports.set(1, flags=T.PORT_VALID, bridge_id=3, mac=POD_MAC)
    dp.ports.set(20, flags=T.PORT_VALID | T.PORT_TUNNEL, bridge_id=3)
    dp.ports.set_lag(20, None)
    dp.ports.a[20]["lag"] = 0
    dp.ports.a[20]["flags"] |= T.PORT_TUNNEL
    dp.ports.set(30, flags=T.PORT_VALID | T.PORT_VTEP, mac="02:00:00:00:0e:01")
    dp.ports.a[30]["ext"] = int(P.ip_raw(np.uint32(int(ipaddress.IPv4Address(LOCAL_VTEP)))))
    dp.tunnels.set(0, src=LOCAL_VTEP, dst=REMOTE_VTEP, vni=5000, out_port=30, smac="02:00:00:00:0e:01",
                   dmac="02:00:00:00:0e:02", kind=kind)
    dp.terms.insert(REMOTE_VTEP, 5000, 20)
    dp.macs.insert(3, REMOTE_MAC, 20)
    dp.macs.insert(3, POD_MAC, 1)
    dp.ports.version += 1
    dp.commit(full=True)
    return dp


def _encap_trace():
    frames, lens = [], []
    for sz in (64, 700, 1400):
        f, ln = P.craft_full(1, dmac=REMOTE_MAC, smac=POD_MAC, src_ip=0x0A000001, dst_ip=0x0A000002, sport=1234,
                             dport=80, frame_len=sz - 4)
        frames.append(f[0, : ln[0]])
        lens.append(int(ln[0]))
    arena = np.zeros((3, 1500), np.uint8)
    for i, f in enumerate(frames):
        arena[i, : len(f)] = f
    return P.header_slots(arena, np.array(lens)), P.inmeta(np.ones(3), np.array(lens)), arena, np.array(lens, np.uint32)


def _check_outer(o: bytes, inner: bytes, kind) -> None:
    assert o[12:14] == b"\x08\x00" and o[14] == 0x45 and o[23] == 17
    w = np.frombuffer(o[14:34], ">u2").astype(np.uint32)
    c = int(w.sum())
    assert ((c & 0xFFFF) + (c >> 16)) & 0xFFFF == 0xFFFF                         # IPv4 header checksum
    assert int.from_bytes(o[16:18], "big") == len(o) - 14                        # total length
    assert o[26:30] == ipaddress.IPv4Address(LOCAL_VTEP).packed and o[30:34] == ipaddress.IPv4Address(REMOTE_VTEP).packed
    assert int.from_bytes(o[36:38], "big") == (4789 if kind == T.TUN_VXLAN else 6081)
    assert int.from_bytes(o[34:36], "big") >= 0xC000                             # entropy source port
    assert int.from_bytes(o[38:40], "big") == len(o) - 34
    assert o[42] == (0x08 if kind == T.TUN_VXLAN else 0x00) and int.from_bytes(o[46:49], "big") == 5000
    if kind == T.TUN_GENEVE:
        assert o[44:46] == b"\x65\x58"
    assert o[50:] == inner


@pytest.mark.parametrize("kind", [T.TUN_VXLAN, T.TUN_GENEVE])
def test_encap_terminate_recirculate_oracle(kind):
    dp = _overlay("cpu", kind)
    slots, im, arena, lens = _encap_trace()
    r = dp.run(slots, im)
    side = dp.side_result()
    port, olen, reason = P.meta_fields(r.meta)
    assert (port == 20).all() and (reason == 0).all() and (olen == lens + 50).all()
    assert P.meta_xhdr(r.meta).all()
    outs = [P.assemble(r.out[i], int(r.meta[i]), arena[i], int(lens[i]), side["xhdr"][i]) for i in range(3)]
    for i, o in enumerate(outs):
        _check_outer(o, bytes(arena[i, : lens[i]]), kind)
    # the reverse direction: the remote VTEP's encapsulation arrives on the underlay port
    back = []
    for o in outs:
        b = bytearray(o)
        b[26:30], b[30:34] = o[30:34], o[26:30]  # remote -> local
        inner = bytearray(b[50:])
        inner[0:6], inner[6:12] = inner[6:12], inner[0:6]  # reply to the pod
        b[50:] = inner
        back.append(bytes(b))
    bl = np.array([len(b) for b in back], np.uint32)
    barena = np.zeros((3, 1500), np.uint8)
    for i, b in enumerate(back):
        barena[i, : len(b)] = np.frombuffer(b, np.uint8)
    r2 = dp.run(P.header_slots(barena, bl), P.inmeta(np.full(3, 30), bl))
    p2, l2, rs2 = P.meta_fields(r2.meta)
    assert (rs2 == 13).all() and (p2 == 20).all() and (l2 == bl - 50).all()   # terminated -> recirculate
    # recirculation: the inner frame re-enters on the tunnel port and is bridged to the pod
    inner = np.zeros((3, 1500), np.uint8)
    for i in range(3):
        inner[i, : l2[i]] = barena[i, 50: 50 + l2[i]]
    r3 = dp.run(P.header_slots(inner, l2), P.inmeta(np.full(3, 20), l2))
    p3, l3, rs3 = P.meta_fields(r3.meta)
    assert (rs3 == 0).all() and (p3 == 1).all() and (l3 == l2).all()
    assert dp.drop_counters().get("recirc") == 3


def test_unknown_vni_is_not_terminated():
    dp = _overlay("cpu")
    slots, im, arena, lens = _encap_trace()
    r = dp.run(slots, im)
    o = bytearray(P.assemble(r.out[0], int(r.meta[0]), arena[0], int(lens[0]), dp.side_result()["xhdr"][0]))
    o[26:30], o[30:34] = o[30:34], o[26:30]
    o[48] ^= 1  # other VNI
    fr = np.frombuffer(bytes(o), np.uint8)[None]
    r2 = dp.run(P.header_slots(fr, np.array([len(o)])), P.inmeta(np.array([30]), np.array([len(o)])))
    assert P.meta_fields(r2.meta)[2][0] == 5  # no_route (punted), not recirculated


@pytest.mark.gpu
@pytest.mark.parametrize("vmmac", [False, True])
def test_routing_gpu_bit_exact(vmmac):
    import torch

    c, g = _router("cpu", vmmac), _router("cuda", vmmac)
    slots, im, *_ = _l3_trace(4096, seed=3)
    rc = c.run(slots, im)
    rg = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(rg.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(rg.out.cpu().numpy(), rc.out)
    assert np.array_equal(g.port_counters(), c.port_counters())


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [T.TUN_VXLAN, T.TUN_GENEVE])
def test_tunnels_gpu_bit_exact(kind):
    import torch

    c, g = _overlay("cpu", kind), _overlay("cuda", kind)
    slots, im, arena, lens = _encap_trace()
    rc = c.run(slots, im)
    sc = c.side_result()
    rg = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    sg = g.side_result()
    assert np.array_equal(rg.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(rg.out.cpu().numpy(), rc.out)
    assert np.array_equal(sg["xhdr"][:3], sc["xhdr"][:3])


def test_l3_routed_sfc_scenario():
    """The bench's L3-routed SFC variant (scenario.install_l3_routes): acl -> nat -> route with
    pod /32s through 8-way ECMP over 100K background prefixes.  Checked against the flows' own
    destinations: egress = the destination pod's port, dst MAC = one of that pod's 8 neighbours
    (hash-selected), src MAC = the router's, TTL - 1 with a valid checksum, SNAT applied."""
    from dpu_operator_amd.dataplane import scenario as S

    dp = DataPlane(device="cpu", flow_buckets=1 << 12)
    sc = S.build_sfc(dp, n_pods=8, n_flows=4000, n_acl=32)
    dp.commit(full=True)
    info = S.install_l3_routes(dp, sc, n_background=20_000)
    dp.commit()
    assert info["background_prefixes"] > 19_000
    pk, im, fl = S.traffic(sc, 2048, seed=4, return_flows=True)
    r = dp.run(pk, im)
    port, _, reason = P.meta_fields(r.meta)
    assert (reason == 0).all()
    dst = sc.flow_dst_pod[fl]
    assert np.array_equal(port, sc.pod_port[dst])
    lens = im >> 16
    for i in range(0, 2048, 7):
        o = P.assemble(r.out[i], int(r.meta[i]), pk[i], int(lens[i]))
        u = o[:12] + o[16:] if o[12:14] == b"\x81\x00" else o
        assert u[0:4] == bytes([0x02, 0x60, 0, 0]) and u[4] == int(dst[i])     # one of the pod's neighbours
        assert u[6:12] == bytes.fromhex(S.ROUTER_MAC.replace(":", ""))
        assert u[22] == 63                                                        # TTL 64 -> 63
        assert u[26:30] == int(sc.actions[fl[i], 1]).to_bytes(4, "little")       # SNAT source
        assert P.check_csums(np.frombuffer(u, np.uint8)[None], np.array([len(u)]))[0]
    assert len({int(r.out[i, 5]) for i in range(2048)}) == 8                     # all ECMP members used


# ---- IPv6 underlay (P4 vxlan / geneve_encap_v6_mod_table, l2_to_tunnel_v6, ipv6_tunnel_term_table) ----
LOCAL6, REMOTE6, TRANSIT6 = "2001:db8:f::1", "2001:db8:f::2", "2001:db8:f::99"


def _overlay6(device, kind=T.TUN_VXLAN):
    """As _overlay, over an IPv6 underlay: tunnel port 21 (tunnels6[0]) -> underlay port 30 whose
    local VTEP is 2001:db8:f::1; (2001:db8:f::2, vni 7000) terminates onto port 21."""
    dp = DataPlane(device=device, flow_buckets=1 << 10)
    dp.ports.set(1, flags=T.PORT_VALID, bridge_id=3, mac=POD_MAC)
    dp.ports.set(21, flags=T.PORT_VALID | T.PORT_TUNNEL | T.PORT_TUNNEL6, bridge_id=3)
    dp.ports.a[21]["lag"] = 0
    dp.ports.set(30, flags=T.PORT_VALID | T.PORT_VTEP, mac="02:00:00:00:0e:01")
    dp.tunnels6.set(0, src=LOCAL6, dst=REMOTE6, vni=7000, out_port=30, smac="02:00:00:00:0e:01",
                    dmac="02:00:00:00:0e:02", kind=kind, traffic_class=0x28)
    dp.vtep6.set(LOCAL6)
    dp.terms6.insert(REMOTE6, 7000, 21)
    dp.macs.insert(3, REMOTE_MAC, 21)
    dp.macs.insert(3, POD_MAC, 1)
    dp.ports.version += 1
    dp.commit(full=True)
    return dp


def _check_outer6(o: bytes, inner: bytes, kind) -> None:
    assert o[12:14] == b"\x86\xdd"
    vtf = int.from_bytes(o[14:18], "big")
    assert vtf >> 28 == 6 and (vtf >> 20) & 0xFF == 0x28 and vtf & 0xFFFFF               # version, class, label
    assert int.from_bytes(o[18:20], "big") == len(o) - 54 and o[20] == 17 and o[21] == 64  # payload, UDP, hops
    assert o[22:38] == ipaddress.IPv6Address(LOCAL6).packed and o[38:54] == ipaddress.IPv6Address(REMOTE6).packed
    assert int.from_bytes(o[54:56], "big") >= 0xC000
    assert int.from_bytes(o[56:58], "big") == (4789 if kind == T.TUN_VXLAN else 6081)
    assert int.from_bytes(o[58:60], "big") == len(o) - 54 and o[60:62] == b"\0\0"        # RFC 6935 zero csum
    assert o[62] == (0x08 if kind == T.TUN_VXLAN else 0x00) and int.from_bytes(o[66:69], "big") == 7000
    if kind == T.TUN_GENEVE:
        assert o[64:66] == b"\x65\x58"
    assert o[70:] == inner


def _reverse6(outs):
    back = []
    for o in outs:
        b = bytearray(o)
        b[22:38], b[38:54] = o[38:54], o[22:38]  # remote -> local
        inner = bytearray(b[70:])
        inner[0:6], inner[6:12] = inner[6:12], inner[0:6]
        b[70:] = inner
        back.append(bytes(b))
    bl = np.array([len(b) for b in back], np.uint32)
    arena = np.zeros((len(back), 1600), np.uint8)
    for i, b in enumerate(back):
        arena[i, : len(b)] = np.frombuffer(b, np.uint8)
    return back, arena, bl


@pytest.mark.parametrize("kind", [T.TUN_VXLAN, T.TUN_GENEVE])
def test_ipv6_underlay_encap_terminate_recirculate(kind):
    dp = _overlay6("cpu", kind)
    slots, im, arena, lens = _encap_trace()
    r = dp.run(slots, im)
    side = dp.side_result()
    port, olen, reason = P.meta_fields(r.meta)
    assert (port == 21).all() and (reason == 0).all() and (olen == lens + 70).all() and P.meta_xhdr(r.meta).all()
    outs = [P.assemble(r.out[i], int(r.meta[i]), arena[i], int(lens[i]), side["xhdr"][i]) for i in range(3)]
    for i, o in enumerate(outs):
        _check_outer6(o, bytes(arena[i, : lens[i]]), kind)
    back, barena, bl = _reverse6(outs)
    r2 = dp.run(P.header_slots(barena, bl), P.inmeta(np.full(3, 30), bl))
    p2, l2, rs2 = P.meta_fields(r2.meta)
    assert (rs2 == 14).all() and (p2 == T.PORT_NONE).all() and (l2 == bl - 70).all()   # recirc6
    for i in range(3):
        tp, inner = dp.resolve_recirc6(back[i])
        assert tp == 21 and inner == back[i][70:]
        r3 = dp.run(P.header_slots(np.frombuffer(inner, np.uint8)[None], np.array([len(inner)])),
                    P.inmeta(np.array([21]), np.array([len(inner)])))
        p3, l3, rs3 = P.meta_fields(r3.meta)
        assert (int(rs3[0]), int(p3[0]), int(l3[0])) == (0, 1, len(inner))           # bridged to the pod
    assert dp.drop_counters().get("recirc6") == 3


def test_ipv6_underlay_unknown_vni_and_transit():
    dp = _overlay6("cpu")
    slots, im, arena, lens = _encap_trace()
    r = dp.run(slots, im)
    o = P.assemble(r.out[1], int(r.meta[1]), arena[1], int(lens[1]), dp.side_result()["xhdr"][1])
    back, barena, bl = _reverse6([o])
    wrong_vni = bytearray(back[0])
    wrong_vni[68] ^= 1
    assert dp.resolve_recirc6(bytes(wrong_vni)) is None                  # no (source, VNI) entry: slow path
    transit = bytearray(back[0])
    transit[38:54] = ipaddress.IPv6Address(TRANSIT6).packed               # not to this VTEP
    fr = np.frombuffer(bytes(transit), np.uint8)[None]
    r2 = dp.run(P.header_slots(fr, bl), P.inmeta(np.array([30]), bl))
    assert P.meta_fields(r2.meta)[2][0] != 14                            # bridged / punted, not terminated
    assert dp.resolve_recirc6(bytes(transit)) is None


def test_ipv6_outer_header_binding_matches_model():
    """The native make_outer (64-B entry) against _check_outer6's field model."""
    dp = _overlay6("cpu")
    inner = bytes(range(60))
    x = dp.nf.make_outer(dp.tunnels6.bytes_of(0), len(inner), 0x12345)
    assert len(x) == 70
    _check_outer6(x + inner, inner, T.TUN_VXLAN)
    assert int.from_bytes(x[15:18], "big") & 0xFFFFF == 0x12345 & 0xFFFFF          # hash-derived flow label


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [T.TUN_VXLAN, T.TUN_GENEVE])
def test_ipv6_tunnels_gpu_bit_exact(kind):
    import torch

    c, g = _overlay6("cpu", kind), _overlay6("cuda", kind)
    slots, im, arena, lens = _encap_trace()
    rc = c.run(slots, im)
    sc = c.side_result()
    rg = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    sg = g.side_result()
    assert np.array_equal(rg.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(rg.out.cpu().numpy(), rc.out)
    assert np.array_equal(sg["xhdr"][:3], sc["xhdr"][:3])
    outs = [P.assemble(rc.out[i], int(rc.meta[i]), arena[i], int(lens[i]), sc["xhdr"][i]) for i in range(3)]
    _, barena, bl = _reverse6(outs)
    s2, i2 = P.header_slots(barena, bl), P.inmeta(np.full(3, 30), bl)
    r2c = c.run(s2, i2)
    r2g = g.run(torch.from_numpy(s2).cuda(), torch.from_numpy(i2.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r2g.meta.cpu().numpy().view(np.uint32), r2c.meta)
    assert (P.meta_fields(r2c.meta)[2] == 14).all()


# ---- single-pass termination: wide header pairs (pipeline.h decap_pair, kernels.hip pair_kernel) ----
def _tag(frames: list[bytes], vid: int = 0) -> list[bytes]:
    """The same frames with an outer 802.1Q tag (vid 0: priority tag, passes VLAN isolation)."""
    return [f[:12] + bytes([0x81, 0x00, vid >> 8, vid & 0xFF]) + f[12:] for f in frames]


def _arena(frames: list[bytes]):
    ln = np.array([len(f) for f in frames], np.uint32)
    ar = np.zeros((len(frames), max(int(ln.max()), 128)), np.uint8)
    for i, f in enumerate(frames):
        ar[i, : len(f)] = np.frombuffer(f, np.uint8)
    return ar, ln


def _two_pass(dp, frame: bytes, enc: int) -> tuple[int, int, bytes]:
    """The recirculation path for one terminated frame: the inner frame re-entered on the tunnel
    port as a 64-B slot.  (egress port, reason, assembled frame)."""
    tp = 20 if enc == 50 else 21
    inner = frame[enc:]
    ia, il = _arena([inner])
    r = dp.run(P.header_slots(ia, il), P.inmeta(np.array([tp]), il))
    port, _, reason = P.meta_fields(r.meta)
    out = P.assemble(r.out[0], int(r.meta[0]), ia[0], int(il[0])) if int(reason[0]) == 0 else b""
    return int(port[0]), int(reason[0]), out


def _reverse_v4(outs):
    back = []
    for o in outs:
        b = bytearray(o)
        b[26:30], b[30:34] = o[30:34], o[26:30]
        inner = bytearray(b[50:])
        inner[0:6], inner[6:12] = inner[6:12], inner[0:6]
        b[50:] = inner
        back.append(bytes(b))
    return back


def _underlay_frames(dp, v6: bool):
    slots, im, arena, lens = _encap_trace()
    r = dp.run(slots, im)
    side = dp.side_result()
    outs = [P.assemble(r.out[i], int(r.meta[i]), arena[i], int(lens[i]), side["xhdr"][i]) for i in range(3)]
    return _reverse6(outs)[0] if v6 else _reverse_v4(outs)


@pytest.mark.parametrize("v6", [False, True])
@pytest.mark.parametrize("tagged", [False, True])
@pytest.mark.parametrize("kind", [T.TUN_VXLAN, T.TUN_GENEVE])
def test_single_pass_termination_equals_recirculation(v6, tagged, kind):
    """A tunnel frame that arrives as a wide header pair is terminated in ONE pass (IPv4 and IPv6
    underlays, outer tag or not, VXLAN and GENEVE): the head's egress is the inner frame bridged to
    the pod, byte for byte what the two-pass path (recirculate the inner frame on the tunnel port)
    delivers; the continuation's meta carries strip / valid bytes; rx is counted on the VTEP port
    (outer) and the tunnel port (inner); nothing is recirculated."""
    dp = (_overlay6 if v6 else _overlay)("cpu", kind)
    frames = _underlay_frames(dp, v6)
    if tagged:
        frames = _tag(frames)
    enc = (70 if v6 else 50) + (4 if tagged else 0)
    ar, ln = _arena(frames)
    slots, im, pos = P.wide_slots(ar, ln, 30, wide_ports={30})
    assert len(slots) == 6                                  # every frame is longer than 64 B: a pair
    dp.reset_counters()
    r = dp.run(slots, im)
    port, olen, reason = P.meta_fields(r.meta)
    for i, f in enumerate(frames):
        h = int(pos[i])
        assert int(reason[h + 1]) == 15 and P.cont_info(int(r.meta[h + 1])) == (enc, min(64, 128 - enc))
        assert (int(port[h]), int(reason[h]), int(olen[h])) == (1, 0, len(f) - enc)
        got = P.assemble(r.out[h], int(r.meta[h]), ar[i], int(ln[i]), cont_meta=int(r.meta[h + 1]))
        ref = _two_pass(_overlay6("cpu", kind) if v6 else _overlay("cpu", kind), f if not tagged else
                        f[:12] + f[16:], enc - (4 if tagged else 0))
        assert ref[:2] == (1, 0) and got == ref[2]
    pc = dp.port_counters()
    assert int(pc[30, 0]) == 3 and int(pc[20 if not v6 else 21, 0]) == 3 and int(pc[1, 2]) == 3
    assert int(pc[30, 1]) == sum(len(f) for f in frames)
    d = dp.drop_counters()
    assert d.get("cont") == 3 and not d.get("recirc") and not d.get("recirc6") and not d.get("bad_port")


def test_single_pass_unknown_vni_falls_back():
    """A pair whose (source, VNI) has no termination entry goes through the pipeline as received,
    exactly like a 64-B slot of the same frame (here: IPv4 punted to the slow path, IPv6 recirc6);
    the continuation then says strip 0 / 64 valid bytes."""
    for v6 in (False, True):
        dp = (_overlay6 if v6 else _overlay)("cpu")
        frames = _underlay_frames(dp, v6)
        b = bytearray(frames[1])
        b[68 if v6 else 48] ^= 1
        ar, ln = _arena([bytes(b)])
        slots, im, pos = P.wide_slots(ar, ln, 30, wide_ports={30})
        r = dp.run(slots, im)
        r1 = dp.run(P.header_slots(ar, ln), P.inmeta(np.array([30]), ln))
        assert int(r.meta[0]) == int(r1.meta[0]) and np.array_equal(r.out[0], r1.out[0])
        assert P.cont_info(int(r.meta[1])) == (0, 64)


@pytest.mark.gpu
@pytest.mark.parametrize("v6", [False, True])
def test_single_pass_termination_gpu_bit_exact(v6):
    """pair_kernel + fused kernel + pair_fix on the GPU = the oracle, bit for bit (metas, out slots,
    port / drop counters), on a mix of pairs (tagged / untagged, known / unknown VNI) and plain
    pod traffic; running the same (rewritten-in-place) batch again gives the same metas / slots."""
    import torch

    c, g = (_overlay6 if v6 else _overlay)("cpu"), (_overlay6 if v6 else _overlay)("cuda")
    frames = _underlay_frames(c, v6)
    frames = frames + _tag(frames)
    bad = bytearray(frames[0])
    bad[68 if v6 else 48] ^= 1
    frames.append(bytes(bad))
    pod, pl = P.craft(4, dmac=REMOTE_MAC, smac=POD_MAC, src_ip=0x0A000001, dst_ip=0x0A000002, sport=5, dport=6)
    mix = frames[:3] + [bytes(pod[k, : pl[k]]) for k in range(4)] + frames[3:]
    ports = [30, 30, 30, 1, 1, 1, 1] + [30] * (len(frames) - 3)
    ar, ln = _arena(mix)
    slots, im, pos = P.wide_slots(ar, ln, np.array(ports), wide_ports={30})
    c.reset_counters()
    g.reset_counters()
    rc = c.run(slots, im)
    ts, ti = torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda()
    for rnd in range(2):
        rg = g.run(ts, ti)
        torch.cuda.synchronize()
        assert np.array_equal(rg.meta.cpu().numpy().view(np.uint32), rc.meta), rnd
        assert np.array_equal(rg.out.cpu().numpy(), rc.out), rnd
        if rnd == 0:   # (a rerun finds the heads already rewritten: the outer rx is not counted again)
            assert np.array_equal(g.port_counters(), c.port_counters())
            assert g.drop_counters() == c.drop_counters()
