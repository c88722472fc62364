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

    assert len(MI355X_P4INFO.tables) >= 38
