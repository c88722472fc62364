"""Closed control loops: node agent <-> GPU port table, data-plane metrics in the running VSP.

The reference's octep_cp_agent applies host ctrl-net requests (SET_MTU, LINK_STATUS, RX_STATE,
DEV_REMOVE) to the SoC interface (marvell/.../octep_cp_agent/loop.c:107-288); here they land in
the GPU port table through cpagent.AgentBridge.  Expectations come from that protocol: a link-down
or removed function neither receives nor sends, RX off stops delivery to it, the MTU bounds the
L3 size of frames delivered to it.  The stats direction (data-plane port counters -> the
agent's GET_IF_STATS answer) and the VSP's /metrics (counters + latency histograms) are checked too.
"""
from __future__ import annotations

import http.client
import os
import shutil
import tempfile
import threading
import time

import numpy as np
import pytest

from dpu_operator_amd import cpagent
from dpu_operator_amd.cpagent import H2F, SET, Reply
from dpu_operator_amd.daemon.deviceplugin import wait_until
from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.ops import packets as P
from dpu_operator_amd.utils.latency import LatencyHist, LatencyStats
from dpu_operator_amd.utils.paths import PathManager

A = cpagent.native()
POD = {1: "0a:00:00:00:00:01", 2: "0a:00:00:00:00:02"}


@pytest.fixture
def node():
    """GPU VSP (oracle data plane) with two bridged VFs + the node agent attached to it."""
    from dpu_operator_amd.cni.netlink import FakeNetlink
    from dpu_operator_amd.vsp.gpu import GpuVsp

    d = tempfile.mkdtemp(prefix="cl", dir="/tmp")
    vsp = GpuVsp(PathManager(d), device="cpu", nl=FakeNetlink(), flow_buckets=1 << 8)
    vsp.init(True, "x")
    vsp.set_num_vfs(4)
    for vf, mac in POD.items():
        vsp.create_bridge_port(f"host0-{vf}", bytes.fromhex(mac.replace(":", "")), 0, [100 + vf])
    mbox = os.path.join(d, "mbox")
    ag = A.Agent(mbox, cpagent.default_config(n_vfs=4))
    ag.start()
    bridge = vsp.attach_agent(ag, state_period_s=0.01, stats_period_s=0.05)
    host = A.HostCtrl(mbox)
    assert host.wait_ready(2000)
    yield vsp, ag, host, bridge
    vsp.stop()
    ag.stop()
    shutil.rmtree(d, ignore_errors=True)


def _send(vsp, src_vf, dst_vf, frame_len=100, n=4):
    slots, lens = P.craft(n, dmac=POD[dst_vf], smac=POD[src_vf], src_ip=0x0A000001, dst_ip=0x0A000002,
                          sport=1000, dport=2000, frame_len=frame_len)
    with vsp._lock:
        r = vsp.dp.run(slots, P.inmeta(np.full(n, src_vf, np.uint32), lens))
    port, _, reason = P.meta_fields(r.meta)
    return int(port[0]), T.REASONS[int(reason[0])]


def _until_applied(bridge, port, st):
    assert wait_until(lambda: bridge.state.applied.get(port) == st, 3), bridge.state.applied.get(port)


def test_agent_mtu_link_rx_reach_gpu_port_flags(node):
    vsp, ag, host, bridge = node
    assert _send(vsp, 1, 2) == (2, "ok")
    _until_applied(bridge, 2, (True, True, 1500))                 # config defaults applied at attach
    assert _send(vsp, 1, 2, frame_len=1514) == (2, "ok")          # L3 1500 = MTU
    assert _send(vsp, 1, 2, frame_len=1515)[1] == "too_big"

    assert host.request(0, 0, 2, H2F.MTU, SET, 9000)["reply"] == Reply.OK
    _until_applied(bridge, 2, (True, True, 9000))
    assert _send(vsp, 1, 2, frame_len=9014) == (2, "ok")

    assert host.request(0, 0, 2, H2F.LINK_STATUS, SET, 0)["reply"] == Reply.OK
    _until_applied(bridge, 2, (False, True, 9000))
    assert vsp.dp.ports.a[2]["flags"] & T.PORT_LINK_DOWN
    assert _send(vsp, 1, 2)[1] == "bad_port"                       # no delivery to a down link
    assert _send(vsp, 2, 1)[1] == "bad_port"                       # nor transmission from it
    assert host.request(0, 0, 2, H2F.LINK_STATUS, SET, 1)["reply"] == Reply.OK
    _until_applied(bridge, 2, (True, True, 9000))
    assert _send(vsp, 1, 2) == (2, "ok")

    assert host.request(0, 0, 2, H2F.RX_STATE, SET, 0)["reply"] == Reply.OK
    _until_applied(bridge, 2, (True, False, 9000))
    assert _send(vsp, 1, 2)[1] == "bad_port"                       # RX off: nothing delivered
    assert _send(vsp, 2, 1) == (1, "ok")                           # but it still transmits

    # the VSP re-programs its ports on every steering change: agent state survives that
    vsp.create_bridge_port("host0-3", bytes.fromhex("0a0000000003"), 0, [103])
    assert vsp.dp.ports.a[2]["flags"] & T.PORT_RX_OFF and vsp.dp.ports.a[2]["mtu"] == 9000

    assert host.request(0, 0, 2, H2F.DEV_REMOVE)["reply"] == Reply.OK
    _until_applied(bridge, 2, (False, False, 9000))
    assert _send(vsp, 2, 1)[1] == "bad_port"
    assert bridge.errors == 0


def test_agent_stats_come_from_the_dataplane(node):
    vsp, ag, host, bridge = node
    _send(vsp, 1, 2, frame_len=200, n=7)
    assert wait_until(lambda: host.request(0, 0, 1, H2F.GET_IF_STATS)["rx"]["pkts"] == 7, 3)
    st = host.request(0, 0, 2, H2F.GET_IF_STATS)
    assert st["tx"]["pkts"] == 7 and st["tx"]["octets"] >= 7 * 200


def test_dataplane_ports_target_without_vsp():
    from dpu_operator_amd.dataplane.engine import DataPlane

    dp = DataPlane(device="cpu", flow_buckets=1 << 6)
    dp.ports.set(5, flags=T.PORT_VALID)
    dp.commit(full=True)
    cpagent.DataPlanePorts(dp).set_port_state(5, False, True, 1400)
    a = dp.ports.a[5]
    assert a["flags"] & T.PORT_LINK_DOWN and a["flags"] & T.PORT_VALID and a["mtu"] == 1400


def test_latency_histogram_buckets_and_quantiles():
    h = LatencyHist()
    h.observe_many(np.array([1e-6] * 90 + [1e-3] * 10))
    h.observe(2e-3)
    assert h.count == 101 and abs(h.sum - (90e-6 + 10e-3 + 2e-3)) < 1e-9
    assert 1e-6 <= h.quantile(0.5) < 2.1e-6 and 1e-3 <= h.quantile(0.99) < 2.1e-3
    b, _ = h.buckets()
    cum = [c for _, c in b]
    assert cum == sorted(cum) and b[-1] == ("+Inf", 101.0)
    s = LatencyStats()
    s.observe("rx", 1e-5)
    assert [k for k, _ in s.items()] == ["rx"]


def _get(port, path):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    c.request("GET", path)
    r = c.getresponse()
    out = r.status, r.read().decode()
    c.close()
    return out


def test_vsp_command_serves_dataplane_metrics_and_runs_the_agent():
    """`vsp --vendor amd-gpu --metrics-bind-address ... --agent-mbox ...`: the running VSP exports
    its data plane (counters, port states, latency histograms) and closes the agent loops."""
    from dpu_operator_amd.cmd import vsp as vsp_cmd
    from dpu_operator_amd.daemon.plugin import GrpcPlugin

    root = tempfile.mkdtemp(prefix="vm", dir="/tmp")
    mbox = os.path.join(root, "mbox")
    stop = threading.Event()
    holder = {}
    orig = vsp_cmd._extras

    def spy(a, vsp):
        holder["vsp"] = vsp
        return orig(a, vsp)

    vsp_cmd._extras = spy
    t = threading.Thread(target=vsp_cmd.main, kwargs={"stop": stop, "argv": [
        "--vendor", "amd-gpu", "--root", root, "--device", "cpu", "--flow-buckets", "256",
        "--metrics-bind-address", "127.0.0.1:0", "--agent-mbox", mbox, "--agent-vfs", "4"]}, daemon=True)
    t.start()
    try:
        assert wait_until(lambda: "vsp" in holder and getattr(holder["vsp"], "metrics", None) is not None, 10)
        vsp = holder["vsp"]
        assert _get(vsp.metrics.port, "/metrics")[0] == 200      # before Init: no data plane yet
        plugin = GrpcPlugin(True, path_manager=PathManager(root), start_timeout=5)
        plugin.start()
        plugin.set_num_vfs(2)
        host = A.HostCtrl(mbox)
        assert host.wait_ready(2000)
        assert host.request(0, 0, 1, H2F.LINK_STATUS, SET, 0)["reply"] == Reply.OK
        assert wait_until(lambda: bool(vsp.dp.ports.a[1]["flags"] & T.PORT_LINK_DOWN), 3)
        vsp.dp.latency.observe("pipeline", 3e-5)
        code, text = _get(vsp.metrics.port, "/metrics")
        assert code == 200
        assert 'dpu_ports_down{dataplane="gpu0",state="link_down"} 1.0' in text
        assert 'dpu_packet_latency_seconds_count{dataplane="gpu0",stage="pipeline"} 1.0' in text
        plugin.close()
    finally:
        vsp_cmd._extras = orig
        stop.set()
        t.join(10)
        shutil.rmtree(root, ignore_errors=True)
