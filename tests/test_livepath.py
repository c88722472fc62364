"""Live packet path (dataplane/netio.py): real TAP netdevs in real network namespaces, frames
moved through the data plane (oracle here; the same LivePath drives the HIP kernels on a GPU).

Two endpoints ping each other through a learning, flooding bridge: the first echo request needs
ARP (broadcast -> flooded to the other port, ARP copy trapped to the slow path), the reply is
unicast to a MAC the data plane learned.  A second test sends 1400-B and 4000-B pings through a
VF-style port pair with VLAN isolation to cover frames beyond the 64-B header slot.
Skipped without CAP_NET_ADMIN / CAP_SYS_ADMIN (namespaces, TAP)."""
import os

import numpy as np
import pytest

from dpu_operator_amd.testutils import netns as NS

pytestmark = pytest.mark.skipif(not NS.privileged(), reason="needs CAP_NET_ADMIN + CAP_SYS_ADMIN (netns, TAP)")


def _setup(tag: str, mtu: int = 1500):
    from dpu_operator_amd.cni.netlink import RtNetlink
    from dpu_operator_amd.dataplane import tables as T
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.dataplane.netio import LivePath, TapPort

    nl = RtNetlink()
    taps = [TapPort(f"lp{tag}{i}") for i in range(2)]
    if mtu != 1500:
        for t in taps:
            nl.link_set_mtu(t.name, mtu)
    eps = [NS.Endpoint(f"lp{tag}-ns{i}", taps[i].name, f"10.93.{ord(tag[0]) % 200}.{i + 1}/24", nl) for i in range(2)]
    if mtu != 1500:
        for e in eps:
            nl.link_set_mtu(e.ifname, mtu, e.ns)
    dp = DataPlane(device="cpu", flow_buckets=1 << 10, mac_slots=1 << 10)
    for i in range(2):
        dp.ports.set(i, flags=T.PORT_VALID | T.PORT_LEARN | T.PORT_ARP_TRAP, bridge_id=7)
    dp.flood.set_members(7, [0, 1])
    dp.commit(full=True)
    punts = []
    live = LivePath(dp, {0: taps[0], 1: taps[1]}, on_punt=lambda f, p, r: punts.append((p, r))).start()
    return dp, taps, eps, live, punts


def _teardown(taps, eps, live):
    live.stop()
    for e in eps:
        e.close()
    for t in taps:
        t.close()


def test_ping_between_namespaces_through_the_data_plane():
    dp, taps, eps, live, punts = _setup("a")
    try:
        rtt = NS.ping(eps[0].ns, eps[1].nl.addr_list(eps[1].ifname, eps[1].ns)[0].split("/")[0])
        assert rtt is not None, (live.stats, live.error)
        assert live.error is None
        assert live.stats["replicas"] == 0 or live.stats["rx"] >= 3
        assert any(r == 12 for _, r in punts)          # the ARP request was copied to the slow path
        dp.pull_learned()
        learned = {(b, m) for b, m, _ in dp.macs.learned()}
        assert (7, eps[0].mac) in learned and (7, eps[1].mac) in learned
        pc = dp.port_counters()
        assert pc[0, 0] >= 2 and pc[1, 0] >= 2         # rx on both ports
        stages = dict(dp.latency.items())                # per-stage latency of every live batch
        assert {"rx", "pipeline", "side", "tx", "batch"} <= set(stages)
        assert abs(stages["batch"].count - live.stats["batches"]) <= 1   # the loop thread may be mid-cycle
        assert stages["batch"].quantile(0.5) < 0.5
    finally:
        _teardown(taps, eps, live)


def test_jumbo_pings_cross_the_data_plane():
    dp, taps, eps, live, punts = _setup("b", mtu=9000)
    try:
        dst = eps[1].nl.addr_list(eps[1].ifname, eps[1].ns)[0].split("/")[0]
        for size in (1400, 4000, 8900):
            assert NS.ping(eps[0].ns, dst, payload=os.urandom(size), seq=size & 0xFFFF) is not None, size
        pc = dp.port_counters()
        assert pc[0, 1] > 8900 and pc[1, 3] > 8900     # byte counters saw the jumbo frames
    finally:
        _teardown(taps, eps, live)


def test_gpu_vsp_live_vports_carry_pod_traffic():
    """The VSP end to end: SetNumVfs creates TAP vports, CreateBridgePort programs the pods' VFs,
    the vports move into two pod namespaces, and the pods ping each other through the VSP's data
    plane (no NF: one L2 bridge with flooding for ARP)."""
    from dpu_operator_amd.cni.netlink import RtNetlink
    from dpu_operator_amd.vsp.gpu import GpuVsp

    nl = RtNetlink()
    vsp = GpuVsp(device="cpu", nl=nl, flow_buckets=1 << 10, vport_prefix="lvp", live=True)
    eps = []
    try:
        vsp.init(True, "")
        vsp.set_num_vfs(2)
        for i in range(2):
            mac = f"02:5e:00:00:00:{i + 1:02x}"
            nl.link_set_hw_addr(f"lvp{i}", mac)
            vsp.create_bridge_port(f"host0-{i}", bytes(int(x, 16) for x in mac.split(":")), 1, [str(2 + i)])
            eps.append(NS.Endpoint(f"lvp-pod{i}", f"lvp{i}", f"10.94.0.{i + 1}/24", nl))
        assert NS.ping(eps[0].ns, "10.94.0.2") is not None, (vsp.livepath.stats, vsp.livepath.error)
        assert NS.ping(eps[1].ns, "10.94.0.1") is not None
        st = vsp.livepath.stats
        assert st["rx"] >= 4 and st["tx"] >= 4
    finally:
        vsp.stop_live()
        for e in eps:
            e.close()


def test_gpu_vsp_sfc_pod_to_external_through_the_nf():
    """The reference e2e's NF scenario (e2e_test.go: pod <-> NF <-> external) on live netdevs:
    a pod VF, an NF pod with ingress / egress vports (a bump-in-the-wire forwarder in its own
    namespace) and the uplink to an "external" host.  CreateNetworkFunction steers
    VF -> NF-in and NF-out -> wire; replies come back wire -> NF-out -> NF -> NF-in -> VF by the
    pod's MAC (OvS K11-K13 rules, GPU tables here).  The pod pings the external host, and every
    packet crosses the NF."""
    from dpu_operator_amd.cni.netlink import RtNetlink
    from dpu_operator_amd.dataplane.netio import TapPort
    from dpu_operator_amd.vsp.gpu import GpuVsp

    nl = RtNetlink()
    wire = TapPort("lvwire")
    nl.link_set_up("lvwire")
    vsp = GpuVsp(device="cpu", nl=nl, flow_buckets=1 << 10, vport_prefix="lvn", live=True, uplink=wire)
    eps, nf = [], None
    try:
        vsp.init(True, "")
        vsp.set_num_vfs(3)
        pod_mac = "02:5e:00:00:01:01"
        nl.link_set_hw_addr("lvn0", pod_mac)
        vsp.create_bridge_port("host0-0", bytes(int(x, 16) for x in pod_mac.split(":")), 1, ["2"])
        eps.append(NS.Endpoint("lvn-pod", "lvn0", "10.95.0.1/24", nl))
        eps.append(NS.Endpoint("lvn-ext", "lvwire", "10.95.0.100/24", nl))
        nf = NS.WireNF("lvn-nf", "lvn1", "lvn2", nl)
        vsp.create_network_function(nf.macs[0], nf.macs[1])
        assert NS.ping(eps[0].ns, "10.95.0.100", timeout=5) is not None, (vsp.livepath.stats, vsp.livepath.error)
        assert NS.ping(eps[1].ns, "10.95.0.1", timeout=5) is not None
        assert nf.forwarded >= 4                      # ARP + echo both ways went through the NF
        assert vsp.livepath.error is None
    finally:
        if nf is not None:
            nf.close()
        vsp.stop_live()
        for e in eps:
            e.close()
        wire.close()
