"""Entry points and manager plumbing: operator (metrics, probes, leader election, webhook),
admission endpoint, VSP launcher, pipeline server, example CNI server, Prometheus exporter."""
from __future__ import annotations

import http.client
import json
import shutil
import socket
import ssl
import subprocess
import tempfile
import threading
import time

import numpy as np
import pytest

from dpu_operator_amd import vars as V
from dpu_operator_amd.api.v1 import KIND_DPU_OPERATOR_CONFIG
from dpu_operator_amd.cmd import cniserver_example, operator as op_cmd, p4rt_server, vsp as vsp_cmd
from dpu_operator_amd.controller.webhook_server import VALIDATE_PATH, WebhookServer, review_response
from dpu_operator_amd.daemon.deviceplugin import wait_until
from dpu_operator_amd.k8s.apiserver import ApiServer, Forbidden
from dpu_operator_amd.k8s.leader import LeaderElector
from dpu_operator_amd.utils.metrics import MetricsServer, register_dataplane
from dpu_operator_amd.utils.paths import PathManager


def _get(port, path):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
    c.request("GET", path)
    r = c.getresponse()
    out = r.status, r.read()
    c.close()
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(mode="host", name=V.DPU_OPERATOR_CONFIG_NAME):
    return {"apiVersion": "config.openshift.io/v1", "kind": KIND_DPU_OPERATOR_CONFIG, "metadata": {"name": name},
            "spec": {"mode": mode}}


def test_operator_main_reconciles_and_serves_probes():
    api = ApiServer()
    api.create({"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                "metadata": {"name": "clusterversions.config.openshift.io"}})  # an OpenShift cluster
    args = op_cmd.build_parser().parse_args(["--metrics-bind-address", "127.0.0.1:0",
                                             "--health-probe-bind-address", "127.0.0.1:0", "--cert-dir", "/nonexistent"])
    from dpu_operator_amd.images import DummyImageManager

    op = op_cmd.Operator(args, api, image_manager=DummyImageManager()).start()
    try:
        assert _get(op.probes.port, "/healthz")[0] == 200
        assert wait_until(lambda: _get(op.probes.port, "/readyz")[0] == 200, 5)
        with pytest.raises(Forbidden):
            api.create(_cfg(name="wrong"))
        api.create(_cfg("host"))
        assert wait_until(lambda: api.try_get("DaemonSet", "dpu-daemon", V.NAMESPACE) is not None, 5)
        code, body = _get(op.metrics.port, "/metrics")
        assert code == 200 and b"dpu_reconcile_total" in body
    finally:
        op.stop()


def test_leader_election_single_leader_and_failover():
    api = ApiServer()
    events = []
    a = LeaderElector(api, "lock", V.NAMESPACE, "a", lease_duration=0.3, renew=0.05,
                      on_started=lambda: events.append("a+"), on_stopped=lambda: events.append("a-")).start()
    assert wait_until(lambda: a.leader, 2)
    b = LeaderElector(api, "lock", V.NAMESPACE, "b", lease_duration=0.3, renew=0.05,
                      on_started=lambda: events.append("b+"), release_on_cancel=False).start()
    time.sleep(0.4)
    assert a.leader and not b.leader
    a._stop.set()          # a dies without releasing: b takes over after the lease expires
    a._t.join(2)
    assert wait_until(lambda: b.leader, 3)
    lease = api.get("Lease", "lock", V.NAMESPACE)
    assert lease["spec"]["holderIdentity"] == "b" and lease["spec"]["leaseTransitions"] == 1
    b.stop()
    assert events[:2] == ["a+", "b+"]


def test_leader_survives_transient_errors_and_steps_down_at_renew_deadline():
    """API errors never kill the election thread; a leader whose renews keep failing gives up
    leadership at the renew deadline, before its lease could expire."""
    api = ApiServer()
    events = []
    a = LeaderElector(api, "lock2", V.NAMESPACE, "a", lease_duration=0.6, renew=0.05, renew_deadline=0.3,
                      on_started=lambda: events.append("+"), on_stopped=lambda: events.append("-")).start()
    assert wait_until(lambda: a.leader, 2)
    real = api.update
    fails = {"n": 0}

    def flaky(obj):
        if fails["n"] < 2:        # two transport errors: shorter than the deadline -> still leader
            fails["n"] += 1
            raise OSError("connection reset")
        return real(obj)

    api.update = flaky
    time.sleep(0.25)
    assert a.leader and a._t.is_alive() and a.errors == 2
    api.update = lambda obj: (_ for _ in ()).throw(OSError("apiserver down"))
    t0 = time.monotonic()
    assert wait_until(lambda: not a.leader, 2)
    assert time.monotonic() - t0 < 0.6 and a._t.is_alive()   # stepped down before lease expiry
    api.update = real
    assert wait_until(lambda: a.leader, 2)                     # and re-acquires once healthy
    a.stop()
    assert events[:3] == ["+", "-", "+"]


def test_admission_endpoint():
    ok = review_response({"request": {"uid": "1", "operation": "CREATE", "object": _cfg("dpu")}})
    assert ok["response"]["allowed"]
    bad = review_response({"request": {"uid": "2", "operation": "UPDATE", "object": _cfg("fast")}})
    assert not bad["response"]["allowed"] and bad["response"]["status"]["message"] == "Invalid mode"
    assert review_response({"request": {"uid": "3", "operation": "DELETE", "object": _cfg(name="x")}})["response"]["allowed"]
    if not shutil.which("openssl"):
        pytest.skip("openssl not available")
    d = tempfile.mkdtemp(prefix="wh", dir="/tmp")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=wh",
                    "-keyout", f"{d}/tls.key", "-out", f"{d}/tls.crt"], check=True, capture_output=True)
    from dpu_operator_amd.nri.server import KeyPairReloader

    srv = WebhookServer(KeyPairReloader(f"{d}/tls.crt", f"{d}/tls.key", insecure=True), "127.0.0.1", 0).start()
    try:
        ctx = ssl.create_default_context()
        ctx.check_hostname, ctx.verify_mode = False, ssl.CERT_NONE
        c = http.client.HTTPSConnection("127.0.0.1", srv.port, context=ctx, timeout=5)
        c.request("POST", VALIDATE_PATH, body=json.dumps({"request": {"uid": "9", "operation": "CREATE",
                                                                       "object": _cfg(name="nope")}}))
        resp = json.loads(c.getresponse().read())["response"]
        assert resp["uid"] == "9" and not resp["allowed"]
        c.close()
    finally:
        srv.stop()
        shutil.rmtree(d, ignore_errors=True)


def test_vsp_launcher_mock():
    root = tempfile.mkdtemp(prefix="vl", dir="/tmp")
    stop = threading.Event()
    t = threading.Thread(target=vsp_cmd.main, args=(["--vendor", "mock", "--root", root],), kwargs={"stop": stop},
                         daemon=True)
    t.start()
    try:
        from dpu_operator_amd.daemon.plugin import GrpcPlugin

        plugin = GrpcPlugin(True, path_manager=PathManager(root), start_timeout=5)
        assert plugin.start() == ("127.0.0.1", 50051)
        assert len(plugin.get_devices().devices) == 4
        plugin.close()
    finally:
        stop.set()
        t.join(5)
        shutil.rmtree(root, ignore_errors=True)


def test_pipeline_server_entry():
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.dataplane.p4server import GrpcP4rtClient

    dp = DataPlane(device="cpu", flow_buckets=1 << 6)
    dp.commit(full=True)
    port = _free_port()
    stop = threading.Event()
    t = threading.Thread(target=p4rt_server.main, args=([f"--address=127.0.0.1:{port}", "--lag", "0:4093"],),
                         kwargs={"stop": stop, "dataplane": dp}, daemon=True)
    t.start()
    try:
        c = GrpcP4rtClient(f"127.0.0.1:{port}")
        assert wait_until(lambda: c.run("add-entry", "br0", "linux_networking_control.tx_acc_vsi",
                                        "vmeta.common.vsi=5,zero_padding=0,"
                                        "action=linux_networking_control.l2_fwd_and_bypass_bridge(40)").ok, 5)
        assert dp.ports.a[21]["default_out"] == 40
        c.close()
    finally:
        stop.set()
        t.join(5)


def test_example_cni_server():
    from dpu_operator_amd.cni.netlink import FakeNetlink, Link
    from dpu_operator_amd.testutils.kubelet import cni_call

    root = tempfile.mkdtemp(prefix="ce", dir="/tmp")
    nl = FakeNetlink()
    nl.add_link(Link(name="dp_interface0", mac="02:00:00:00:00:01"))
    nl.add_netns("/var/run/netns/x")
    sock = f"{root}/cni.sock"
    stop = threading.Event()
    t = threading.Thread(target=cniserver_example.main, args=([f"--socket={sock}", f"--root={root}"],),
                         kwargs={"nl": nl, "stop": stop}, daemon=True)
    t.start()
    try:
        assert wait_until(lambda: __import__("os").path.exists(sock), 5)
        res = cni_call(sock, "ADD", {"cniVersion": "0.4.0", "name": "n", "type": "dpu-cni", "deviceID": "dp_interface0"},
                       netns="/var/run/netns/x", ifname="net1")
        assert res["interfaces"][0]["mac"] == "02:00:00:00:00:01"
        assert nl.link_by_name("net1", "/var/run/netns/x").alias == "dp_interface0"
    finally:
        stop.set()
        t.join(5)
        shutil.rmtree(root, ignore_errors=True)


def test_dataplane_metrics_exporter():
    from prometheus_client import CollectorRegistry

    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane

    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    sc = S.build_sfc(dp, n_pods=4, n_flows=512, n_acl=8)
    dp.commit(full=True)
    pk, im = S.traffic(sc, 1000)
    dp.run(pk, im)
    dp.harvest()
    reg = CollectorRegistry()
    register_dataplane(dp, "gpu0", reg)
    srv = MetricsServer("127.0.0.1:0", reg).start()
    try:
        code, body = _get(srv.port, "/metrics")
        text = body.decode()
        assert code == 200
        assert 'dpu_flows_installed{dataplane="gpu0"} 512.0' in text
        assert 'dpu_table_entries{dataplane="gpu0",table="flows"} 512.0' in text
        assert 'dpu_table_entries{dataplane="gpu0",table="macs_static"} 4.0' in text
        assert 'dpu_table_entries{dataplane="gpu0",table="acl_rules"} 8.0' in text
        rx = sum(float(line.split()[-1]) for line in text.splitlines() if line.startswith("dpu_port_rx_packets_total"))
        assert rx == 1000
        assert 'dpu_flow_lookups_total{dataplane="gpu0",result="hit"} 1000.0' in text
        assert 'dpu_flow_lookups_total{dataplane="gpu0",result="miss"} 0.0' in text
        assert _get(srv.port, "/other")[0] == 404
    finally:
        srv.stop()
