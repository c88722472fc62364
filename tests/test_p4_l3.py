"""P4Runtime entry strings for the L3 / tunnel / LAG-rx / smac / ARP-trap tables of the
linux_networking pipeline (fxp-net_linux-networking.p4info.txt:168-1110), compiled onto the
GPU tables and checked with packets."""
import ipaddress

import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.p4rt import PHY_BASE, TUNNEL_PORT_BASE, P4Error, P4Runtime
from dpu_operator_amd.ops import packets as P

C = "linux_networking_control."


@pytest.fixture
def rt():
    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    return P4Runtime(dp)


def _send(dp, port, dmac, dst, smac="02:00:00:00:00:99", ttl=64):
    fr, ln = P.craft(1, dmac=dmac, smac=smac, src_ip=0x0A000001, dst_ip=int(ipaddress.IPv4Address(dst)), sport=9,
                     dport=80, ttl=ttl)
    dp.commit()
    r = dp.run(fr, P.inmeta(np.array([port]), ln))
    op, ln2, rs = P.meta_fields(r.meta)
    return int(op[0]), int(rs[0]), r.out[0]


def test_l3_entries_route_packets(rt):
    dp = rt.dp
    add = rt.add_entry
    add(C + "rif_mod_table_start", "rif_mod_map_id0=5,action=linux_networking_control.set_src_mac_start(0x0240)")
    add(C + "rif_mod_table_mid", "rif_mod_map_id1=5,action=linux_networking_control.set_src_mac_mid(0x0000)")
    add(C + "rif_mod_table_last", "rif_mod_map_id2=5,action=linux_networking_control.set_src_mac_last(0x0001)")
    add(C + "nexthop_table", "user_meta.cmeta.nexthop_id=1,bit16_zeros=0,"
        "action=linux_networking_control.set_nexthop_info_dmac(5,1,0x0250,0x00000001)")
    add(C + "nexthop_table", "user_meta.cmeta.nexthop_id=2,bit16_zeros=0,"
        "action=linux_networking_control.set_nexthop_info_dmac(5,2,0x0250,0x00000002)")
    add(C + "ipv4_table", "ipv4_table_lpm_root=0,ipv4_dst_match=10.20.0.0/16,"
        "action=linux_networking_control.ipv4_set_nexthop_id(1)")
    add(C + "ipv4_table", "ipv4_table_lpm_root=0,ipv4_dst_match=10.20.30.0/24,"
        "action=linux_networking_control.ecmp_hash_action(3)")
    for h in range(8):
        add(C + "ecmp_hash_table", f"flex=3,hash={h},priority=10,"
            f"action=linux_networking_control.set_nexthop_id({1 + (h & 1)})")
    with pytest.raises(P4Error):  # LPM prefix length beyond 32 bits
        add(C + "ipv4_table", "ipv4_table_lpm_root=0,ipv4_dst_match=10.0.0.0/33,action=linux_networking_control.NoAction()")
    assert len(dp.routes) == 2 and dp.nexthops.a[1]["valid"] and dp.ecmp.n == 4
    # router interface: port 4001 (physical 1) routes IPv4 sent to its MAC
    dp.ports.set(PHY_BASE + 1, flags=T.PORT_VALID | T.PORT_ROUTED, mac="02:40:00:00:00:01")
    op, rs, out = _send(dp, PHY_BASE + 1, "02:40:00:00:00:01", "10.20.1.1")
    assert (op, rs) == (PHY_BASE + 1, 0) and bytes(out[0:6]) == bytes.fromhex("025000000001")
    assert bytes(out[6:12]) == bytes.fromhex("024000000001") and out[22] == 63
    seen = {_send(dp, PHY_BASE + 1, "02:40:00:00:00:01", f"10.20.30.{k}")[0] for k in range(1, 40)}
    assert seen == {PHY_BASE + 1, PHY_BASE + 2}  # ECMP spread over both nexthops
    assert _send(dp, PHY_BASE + 1, "02:40:00:00:00:01", "10.99.0.1")[1] == 5  # no route
    rt.del_entry(C + "ipv4_table", "ipv4_table_lpm_root=0,ipv4_dst_match=10.20.0.0/16")
    assert len(dp.routes) == 1


def test_vxlan_entries_encap_and_terminate(rt):
    dp = rt.dp
    add = rt.add_entry
    add(C + "vxlan_encap_mod_table", "vmeta.common.mod_blob_ptr=7,"
        "action=linux_networking_control.vxlan_encap(192.0.2.1,192.0.2.2,0,4789,7000)")
    add(C + "l2_to_tunnel_v4", "hdrs.mac[vmeta.common.depth].da=02:00:00:00:bb:01,"
        "action=linux_networking_control.set_tunnel_v4(192.0.2.2)")
    add(C + "ipv4_tunnel_term_table", "ipv4_src=192.0.2.2,vni=7000,action=linux_networking_control.set_vxlan_decap_outer_hdr(1)")
    add(C + "rx_ipv4_tunnel_source_port", "ipv4_src=192.0.2.2,vni=7000,action=linux_networking_control.set_source_port(40)")
    dp.ports.set(1, flags=T.PORT_VALID, bridge_id=0)
    tport = TUNNEL_PORT_BASE
    assert dp.ports.a[tport]["flags"] & T.PORT_TUNNEL and dp.tunnels.n == 1
    assert dp.terms.n == 1 and dp.ports.a[PHY_BASE]["flags"] & T.PORT_VTEP
    op, rs, out = _send(dp, 1, "02:00:00:00:bb:01", "10.0.0.2")
    assert (op, rs) == (tport, 0)
    xh = dp.side_result()["xhdr"][0]
    assert bytes(xh[30:34]) == ipaddress.IPv4Address("192.0.2.2").packed and int.from_bytes(bytes(xh[46:49]), "big") == 7000


def test_lag_rx_smac_and_arp_trap_tables(rt):
    dp = rt.dp
    rt.add_entry(C + "rx_lag_table", "vmeta.common.port_id=2,user_meta.cmeta.lag_group_id=1,"
                 "action=linux_networking_control.fwd_to_vsi(30)")
    assert int(dp.ports.a[PHY_BASE + 2]["default_out"]) == 30
    rt.add_entry(C + "tx_acc_vsi", "vmeta.common.vsi=5,zero_padding=0,action=linux_networking_control.l2_fwd_and_bypass_bridge(40)")
    rt.add_entry(C + "l2_fwd_smac_table", "hdrs.mac[vmeta.common.depth].sa=02:00:00:00:00:01,user_meta.pmeta.bridge_id=0,"
                 "action=linux_networking_control.NoAction()")
    rt.add_entry(C + "always_trap_arp_table", "hdrs.inval.data=0x806,hdrs.inval.data=0,action=linux_networking_control.do_trap_enable()")
    owned = [p for p in range(len(dp.ports.a)) if dp.ports.a[p]["flags"] & T.PORT_ARP_TRAP]
    assert owned and all(dp.ports.a[p]["flags"] & T.PORT_VALID for p in owned)
    assert any(dp.ports.a[p]["flags"] & T.PORT_LEARN for p in owned)


def test_pipeline_table_count():
    from dpu_operator_amd.dataplane.p4info import MI355X_P4INFO

    # the reference's 55 linux_networking tables + the 5 older-pipeline tables its IPU VSP programs
    assert len(MI355X_P4INFO.tables) >= 60


def test_ipv6_table_entries_route_packets(rt):
    """ipv6_table (p4info.txt:871: ipv6_table_lpm_root exact + ipv6_dst_match LPM /128) with
    ipv6_set_nexthop_id and ecmp_v6_hash_action, compiled onto the IPv6 FIB; the root LUT is
    accepted (the GPU FIB needs no root split)."""
    dp = rt.dp
    add = rt.add_entry
    add(C + "ipv6_lpm_root_lut", "user_meta.cmeta.bit16_zeros=0/0,priority=1,"
        "action=linux_networking_control.ipv6_lpm_root_lut_action(0)")
    for nh in (1, 2):
        add(C + "nexthop_table", f"user_meta.cmeta.nexthop_id={nh},bit16_zeros=0,"
            f"action=linux_networking_control.set_nexthop_info_dmac(5,{nh},0x0250,0x0000000{nh})")
    add(C + "ipv6_table", "ipv6_table_lpm_root=0,ipv6_dst_match=2001:db8::/32,"
        "action=linux_networking_control.ipv6_set_nexthop_id(1)")
    add(C + "ipv6_table", "ipv6_table_lpm_root=0,ipv6_dst_match=2001:db8:5::/48,"
        "action=linux_networking_control.ecmp_v6_hash_action(4)")
    for h in range(8):
        add(C + "ecmp_hash_table", f"flex=4,hash={h},priority=10,"
            f"action=linux_networking_control.set_nexthop_id({1 + (h & 1)})")
    with pytest.raises(P4Error):  # beyond 128 bits
        add(C + "ipv6_table", "ipv6_table_lpm_root=0,ipv6_dst_match=2001:db8::/129,"
            "action=linux_networking_control.NoAction()")
    assert len(dp.routes6) == 2
    assert dp.routes6.lookup("2001:db8:5::1") == T.ROUTE_ECMP | 4
    dp.ports.set(PHY_BASE + 1, flags=T.PORT_VALID | T.PORT_ROUTED, mac="02:40:00:00:00:01")
    dp.commit()

    def send6(dst, sport=9):
        fr, ln = P.craft6_full(1, dmac="02:40:00:00:00:01", smac="02:00:00:00:00:99", src6="2001:db8:9::1",
                               dst6=dst, sport=sport, dport=80)
        r = dp.run(P.header_slots(fr, ln), P.inmeta(np.array([PHY_BASE + 1]), ln))
        op, _, rs = P.meta_fields(r.meta)
        return int(op[0]), int(rs[0]), r.out[0]

    op, rs, out = send6("2001:db8:1::1")
    assert (op, rs) == (PHY_BASE + 1, 0) and bytes(out[0:6]) == bytes.fromhex("025000000001") and out[21] == 63
    assert {send6("2001:db8:5::7", sport=s)[0] for s in range(1, 40)} == {PHY_BASE + 1, PHY_BASE + 2}
    assert send6("2600::1")[1] == 5  # no route
    rt.del_entry(C + "ipv6_table", "ipv6_table_lpm_root=0,ipv6_dst_match=2001:db8::/32")
    assert len(dp.routes6) == 1


def test_geneve_vlan_pop_encap_and_decap_push_vlan(rt):
    """geneve_encap_vlan_pop_mod_table (GENEVE encap of the untagged inner frame) and
    set_geneve_decap_outer_and_push_vlan + geneve_decap_and_push_vlan_mod_table: the terminated
    inner frame leaves its tunnel's port with the mod entry's vid pushed."""
    dp = rt.dp
    add = rt.add_entry
    add(C + "geneve_encap_vlan_pop_mod_table", "vmeta.common.mod_blob_ptr=9,"
        "action=linux_networking_control.geneve_encap_vlan_pop(192.0.2.1,192.0.2.3,0,6081,9000)")
    add(C + "l2_to_tunnel_v4", "hdrs.mac[vmeta.common.depth].da=02:00:00:00:cc:01,"
        "action=linux_networking_control.set_tunnel_v4(192.0.2.3)")
    add(C + "geneve_decap_and_push_vlan_mod_table", "vmeta.common.mod_blob_ptr=2,"
        "action=linux_networking_control.geneve_decap_and_push_vlan(0,0,321)")
    add(C + "ipv4_tunnel_term_table", "ipv4_src=192.0.2.3,vni=9000,"
        "action=linux_networking_control.set_geneve_decap_outer_and_push_vlan(2)")
    assert dp.tunnels.n == 1 and int(dp.tunnels.a[0]["type"]) == T.TUN_GENEVE
    tp = TUNNEL_PORT_BASE + 128 + 2
    assert dp.ports.a[tp]["flags"] & T.PORT_INGRESS_TAG and int(dp.ports.a[tp]["ext"]) & 0xFFF == 321
    # an inner frame re-entering on the termination port leaves tagged with vid 321
    dp.ports.update(tp, bridge_id=0, default_out=5)
    dp.ports.set(5, flags=T.PORT_VALID, bridge_id=0)
    op, rs, out = _send(dp, tp, "02:00:00:00:00:05", "10.0.0.9")
    assert (op, rs) == (5, 0) and bytes(out[12:16]) == b"\x81\x00" + (321).to_bytes(2, "big")


def test_ipv6_underlay_tunnel_tables(rt):
    """l2_to_tunnel_v6 + vxlan_encap_v6_mod_table (p4info.txt: set_tunnel_v6 ipv6_1..4, the encap's
    128-bit addresses, ds / ecn / flow label / hop limit), ipv6_tunnel_term_table and
    rx_ipv6_tunnel_source_port: the IPv6 encap leaves on the tunnel's port with a 70-B outer header,
    and the reverse direction is recognised on the underlay port (recirc6) and resolved to the
    termination port, whose source-port bridge mapping applies."""
    dp = rt.dp
    add = rt.add_entry
    add(C + "vxlan_encap_v6_mod_table", "vmeta.common.mod_blob_ptr=11,action=linux_networking_control.vxlan_encap_v6("
        "2001:db8:f::1,2001:db8:f::2,10,0,0xabcde,32,0,4789,7100)")
    add(C + "l2_to_tunnel_v6", "hdrs.mac[vmeta.common.depth].da=02:00:00:00:dd:01,"
        "action=linux_networking_control.set_tunnel_v6(0x20010db8,0x000f0000,0x00000000,0x00000002)")
    add(C + "ipv6_tunnel_term_table", "ipv6_src=2001:db8:f::2,vni=7100,action=linux_networking_control.set_vxlan_decap_outer_hdr(3)")
    add(C + "rx_ipv6_tunnel_source_port", "ipv6_src=2001:db8:f::2,vni=7100,action=linux_networking_control.set_source_port(44)")
    add(C + "source_port_to_bridge_map", "user_meta.cmeta.source_port=44/0xffff,hdrs.vlan_ext[vmeta.common.depth].hdr.vid=0/0,"
        "priority=1,action=linux_networking_control.set_bridge_id(6)")
    tport = TUNNEL_PORT_BASE + 64
    assert dp.tunnels6.n == 1 and dp.ports.a[tport]["flags"] & T.PORT_TUNNEL6
    e = dp.tunnels6.a[0]
    assert int(e["tc_flow"]) == ((10 << 2) << 20 | 0xABCDE) and int(e["hop_limit"]) == 32
    assert dp.vtep6.active and dp.ports.a[PHY_BASE]["flags"] & T.PORT_VTEP and len(dp.terms6) == 1
    dp.ports.set(1, flags=T.PORT_VALID, bridge_id=0)
    fr, ln = P.craft(1, dmac="02:00:00:00:dd:01", smac="02:00:00:00:00:77", src_ip=0x0A000001, dst_ip=0x0A000002,
                     sport=9, dport=80)
    dp.commit()
    r = dp.run(fr, P.inmeta(np.array([1]), ln))
    op, olen, rs = P.meta_fields(r.meta)
    assert (int(op[0]), int(rs[0]), int(olen[0])) == (tport, 0, int(ln[0]) + 70)
    o = P.assemble(r.out[0], int(r.meta[0]), fr[0], int(ln[0]), dp.side_result()["xhdr"][0])
    assert o[12:14] == b"\x86\xdd" and o[38:54] == ipaddress.IPv6Address("2001:db8:f::2").packed
    assert int.from_bytes(o[14:18], "big") & 0xFFFFF == 0xABCDE and o[21] == 32
    assert int.from_bytes(o[66:69], "big") == 7100
    # reverse: from the remote VTEP to the local one, on the underlay port
    b = bytearray(o)
    b[22:38], b[38:54] = o[38:54], o[22:38]
    arr = np.frombuffer(bytes(b), np.uint8)[None]
    r2 = dp.run(P.header_slots(arr, np.array([len(b)])), P.inmeta(np.array([PHY_BASE]), np.array([len(b)])))
    assert int(P.meta_fields(r2.meta)[2][0]) == 14
    tp, inner = dp.resolve_recirc6(bytes(b))
    assert tp == TUNNEL_PORT_BASE + 128 + 3 and inner == bytes(b[70:])
    assert int(dp.ports.a[tp]["bridge_id"]) == 6
    rt.del_entry(C + "ipv6_tunnel_term_table", "ipv6_src=2001:db8:f::2,vni=7100")
    assert len(dp.terms6) == 0 and not dp.vtep6.active


def test_keyless_lem_tables_accept_noaction(rt):
    """lem_exception / lem_clear (keyless, NoAction only in the p4info): one entry each is
    accepted, a second is ALREADY_EXISTS, and nothing in the data plane changes."""
    before = rt.dp.ports.a.copy()
    for t in ("lem_exception", "lem_clear"):
        rt.add_entry(C + t, "action=linux_networking_control.NoAction()")
        with pytest.raises(P4Error):
            rt.add_entry(C + t, "action=linux_networking_control.NoAction()")
    assert (rt.dp.ports.a == before).all()


def _l3_one_nexthop(rt):
    add = rt.add_entry
    for part, v in (("start", 0x0240), ("mid", 0x0000), ("last", 0x0001)):
        add(C + f"rif_mod_table_{part}", f"rif_mod_map_id{('start', 'mid', 'last').index(part)}=5,"
            f"action=linux_networking_control.set_src_mac_{part}({v:#06x})")
    add(C + "nexthop_table", "user_meta.cmeta.nexthop_id=1,bit16_zeros=0,"
        "action=linux_networking_control.set_nexthop_info_dmac(5,1,0x0250,0x00000001)")
    add(C + "ipv4_table", "ipv4_table_lpm_root=0,ipv4_dst_match=10.20.0.0/16,"
        "action=linux_networking_control.ipv4_set_nexthop_id(1)")
    rt.dp.ports.set(PHY_BASE + 1, flags=T.PORT_VALID | T.PORT_ROUTED, mac="02:40:00:00:00:01")


def test_vm_ip4_mac_map_tables_rewrite_routed_macs(rt):
    """vm_dst_ip4_mac_map_table / vm_src_ip4_mac_map_table (p4info.txt:1393-1440): a routed packet
    to a mapped destination leaves with the mapped dmac instead of the nexthop's, one from a
    mapped source with the mapped smac instead of the router interface's; others are unchanged.
    Expected bytes are written out by hand here (independent of the oracle)."""
    dp = rt.dp
    _l3_one_nexthop(rt)
    rt.add_entry(C + "vm_dst_ip4_mac_map_table", "ipv4_dst=10.20.7.7,"
                 "action=linux_networking_control.vm_dst_ip4_mac_map_action(0x0266,0x7788,0x99aa)")
    rt.add_entry(C + "vm_src_ip4_mac_map_table", "ipv4_src=10.0.0.1,"
                 "action=linux_networking_control.vm_src_ip4_mac_map_action(0x02ab,0xcdef,0x0102)")
    assert dp.vmmac.n == 2
    op, rs, out = _send(dp, PHY_BASE + 1, "02:40:00:00:00:01", "10.20.7.7")   # src 10.0.0.1 (mapped)
    assert (op, rs) == (PHY_BASE + 1, 0)
    assert bytes(out[0:6]) == bytes.fromhex("0266778899aa")
    assert bytes(out[6:12]) == bytes.fromhex("02abcdef0102") and out[22] == 63
    op, rs, out = _send(dp, PHY_BASE + 1, "02:40:00:00:00:01", "10.20.7.8")   # unmapped destination
    assert bytes(out[0:6]) == bytes.fromhex("025000000001") and bytes(out[6:12]) == bytes.fromhex("02abcdef0102")
    rt.del_entry(C + "vm_src_ip4_mac_map_table", "ipv4_src=10.0.0.1")
    op, rs, out = _send(dp, PHY_BASE + 1, "02:40:00:00:00:01", "10.20.7.7")
    assert bytes(out[0:6]) == bytes.fromhex("0266778899aa") and bytes(out[6:12]) == bytes.fromhex("024000000001")
    rt.del_entry(C + "vm_dst_ip4_mac_map_table", "ipv4_dst=10.20.7.7")
    assert dp.vmmac.n == 0 and dp.tables_ptrs()["vmmac"] == 0
    op, rs, out = _send(dp, PHY_BASE + 1, "02:40:00:00:00:01", "10.20.7.7")
    assert bytes(out[0:6]) == bytes.fromhex("025000000001")


def test_vmmac_table_probe_and_twin():
    t = T.VmMacTable(slots=16)
    for k in range(10):
        t.set(f"10.1.0.{k}", T.VMMAC_DST, f"02:00:00:00:01:{k:02x}")
    t.set("10.1.0.3", T.VMMAC_SRC, "02:00:00:00:02:03")
    t.set("10.1.0.3", T.VMMAC_DST, "02:00:00:00:03:03")   # overwrite in place
    assert t.n == 11
    assert t.lookup("10.1.0.3", T.VMMAC_DST) == T.mac_raw("02:00:00:00:03:03")
    assert t.lookup("10.1.0.3", T.VMMAC_SRC) == T.mac_raw("02:00:00:00:02:03")
    assert t.lookup("10.1.0.99", T.VMMAC_SRC) is None
    with pytest.raises(ValueError):
        t.set("10.1.0.1", 3, "02:00:00:00:00:01")


def test_always_recirculate_table_accepts_entries(rt):
    before = rt.dp.ports.a.copy()
    rt.add_entry(C + "always_recirculate_table", "hdrs.inval.data=1,hdrs.inval.data=0,"
                 "action=linux_networking_control.do_recirculate()")
    assert (rt.dp.ports.a == before).all()


def test_all_reference_tables_compiled():
    """Every table of the reference's linux_networking p4info has a definition here."""
    from dpu_operator_amd.dataplane.p4info import TABLES, P4Info

    from test_p4 import REF_P4INFO

    if not REF_P4INFO.exists():
        pytest.skip("reference P4Info not mounted")
    ref = P4Info.from_text(REF_P4INFO.read_text())
    names = {t.name.split(".")[-1] for t in ref.tables.values()}
    assert names <= {t[0].split(".")[-1] for t in TABLES} and len(names) == 55
