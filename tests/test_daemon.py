"""Node-daemon tests: side managers, device plugin + kubelet registration, the full daemon loop.

Mirrors internal/daemon/{hostsidemanager,dpusidemanager,daemon}_test.go: a CNI ADD through the
host-side CNI server must reach the device side as an OPI CreateBridgePort; the device side with
the mock VSP must make `openshift.io/dpu` allocatable on the node; the full daemon on a fake
platform must detect the engine and bring the VSP up.  The colocated MI355X path is then driven
end to end: NF pod + workload pod CNI calls program the GPU data plane (CPU oracle here), and a
packet from the workload VF is steered into the NF.
"""
from __future__ import annotations

import os
import shutil
import tempfile
import threading
from concurrent import futures

import grpc
import numpy as np
import pytest

from dpu_operator_amd import vars as V
from dpu_operator_amd.cni.netlink import FakeNetlink
from dpu_operator_amd.cni.sriov import SriovManagerStub
from dpu_operator_amd.cni.types import CNIError
from dpu_operator_amd.daemon.daemon import Daemon
from dpu_operator_amd.daemon.deviceplugin import wait_until
from dpu_operator_amd.daemon.managers import DpuSideManager, HostSideManager
from dpu_operator_amd.daemon.plugin import GrpcPlugin
from dpu_operator_amd.k8s.apiserver import ApiServer
from dpu_operator_amd.platform.platform import FakePlatform, PciDevice
from dpu_operator_amd.proto import GoogleEmpty, opi, vendor
from dpu_operator_amd.proto.grpcutil import service_handler
from dpu_operator_amd.testutils.kubelet import FakeKubelet, cni_call
from dpu_operator_amd.utils.fileutils import touch
from dpu_operator_amd.utils.paths import PathManager
from dpu_operator_amd.vsp import MockVsp


@pytest.fixture
def pm():
    root = tempfile.mkdtemp(prefix="dpu", dir="/tmp")  # short: unix socket paths are <= 108 bytes
    yield PathManager(root)
    shutil.rmtree(root, ignore_errors=True)


class DummyPlugin:
    """hostsidemanager_test.go DummyPlugin: Start -> the dummy DPU daemon's address."""

    def __init__(self, port):
        self.port = port

    def start(self):
        return "127.0.0.1", self.port

    def close(self):
        pass

    def create_bridge_port(self, req):
        return opi.BridgePort()

    def delete_bridge_port(self, req):
        pass

    def create_network_function(self, i, o):
        pass

    def delete_network_function(self, i, o):
        pass

    def get_devices(self):
        return vendor.DeviceListResponse()

    def set_num_vfs(self, n):
        return vendor.VfCount(vf_cnt=n)


class DummyDpuDaemon:
    def __init__(self):
        self.bridge_ports = 0
        self.names = []
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        self.server.add_generic_rpc_handlers((service_handler(opi, "BridgePortService", self),))
        self.port = self.server.add_insecure_port("127.0.0.1:0")
        self.server.start()

    def CreateBridgePort(self, req, ctx):
        self.bridge_ports += 1
        self.names.append(req.bridge_port.name)
        return opi.BridgePort()

    def DeleteBridgePort(self, req, ctx):
        self.bridge_ports -= 1
        return GoogleEmpty()

    def stop(self):
        self.server.stop(grace=0)


CONF = {"cniVersion": "0.4.0", "name": "dpucni", "type": "dpucni",
        "OrigVfState": {"EffectiveMac": "00:11:22:33:44:55"}, "vlan": 7}


def test_host_side_cni_add_del_reaches_device_side(pm):
    dpu = DummyDpuDaemon()
    host = HostSideManager(DummyPlugin(dpu.port), SriovManagerStub(), path_manager=pm, register_device_plugin=False,
                           dp_poll=0.05)
    try:
        host.start_vsp()
        host.setup_devices()
        host.listen()
        host.serve()
        res = cni_call(pm.cni_server_path(), "ADD", CONF)
        assert res["cniVersion"] == "0.4.0"
        assert dpu.bridge_ports == 1 and dpu.names == ["host0-0"]
        cni_call(pm.cni_server_path(), "DEL", CONF)
        assert dpu.bridge_ports == 0
    finally:
        host.stop()
        dpu.stop()


def test_cni_server_rejects_bad_requests(pm):
    dpu = DummyDpuDaemon()
    host = HostSideManager(DummyPlugin(dpu.port), SriovManagerStub(), path_manager=pm, register_device_plugin=False)
    try:
        host.start_vsp()
        host.setup_devices()
        host.listen()
        host.serve()
        from dpu_operator_amd.cni.server import post_unix
        from dpu_operator_amd.cni.types import Request

        env = {"CNI_COMMAND": "ADD", "CNI_CONTAINERID": "c", "CNI_PATH": "/p", "CNI_ARGS": "K8S_POD_NAMESPACE=x;K8S_POD_NAME=y"}
        code, body = post_unix(pm.cni_server_path(), "/cni", Request(env=env, config=b"{}").to_json())
        assert code == 400 and b"CNI_NETNS" in body
        env["CNI_NETNS"], env["CNI_ARGS"] = "/n", "K8S_POD_NAMESPACE=x"
        with pytest.raises(CNIError, match="K8S_POD_NAME"):
            from dpu_operator_amd.cni.shim import Plugin

            Plugin(pm.cni_server_path()).post_request(env, b"{}")

        code, body = post_unix(pm.cni_server_path(), "/cni", b"{}", method="GET")
        assert code == 405
        code, body = post_unix(pm.cni_server_path(), "/cni", b'{"env": {}}')
        assert code == 400 and b"CNI_COMMAND" in body
    finally:
        host.stop()
        dpu.stop()


def _serve_vsp(vsp, pm):
    vsp.pm = pm
    return vsp.start()


def test_dpu_side_mock_vsp_device_plugin_allocatable(pm):
    api = ApiServer()
    kubelet = FakeKubelet(pm, api).start()
    vsp = _serve_vsp(MockVsp(), pm)
    plugin = GrpcPlugin(True, path_manager=pm)
    dsm = DpuSideManager(plugin, FakeNetlink(), api, pm, dp_poll=0.05)
    try:
        dsm.start_vsp()
        assert dsm.port == 50051  # what the VSP's Init returned
        dsm.port = 0              # tests bind an ephemeral port for the OPI server
        dsm.setup_devices()
        dsm.listen()
        dsm.serve()
        assert wait_until(lambda: kubelet.allocatable() == 4, 5)
        node = api.get("Node", "worker-0")
        assert node["status"]["allocatable"][V.RESOURCE_NAME] == "4"
        assert kubelet.registrations[0].resource_name == V.RESOURCE_NAME
        assert kubelet.registrations[0].endpoint == "dpuNet.sock"
        r = kubelet.allocate(["ens5f0", "ens5f1"])
        assert r.container_responses[0].envs["NF-DEV"] == "ens5f0,ens5f1,"
        with pytest.raises(grpc.RpcError) as ei:
            kubelet.allocate(["nope"])
        assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
        names = [c[0] for c in vsp.calls]
        assert names[0] == "Init" and "SetNumVfs" in names
        assert vsp.num_vfs == 8
    finally:
        dsm.stop()
        kubelet.stop()
        vsp.stop()


def test_full_daemon_detects_ipu_and_starts_vsp(pm):
    touch(pm.wrap("/dpu-cni"))
    api = ApiServer()
    vsp = _serve_vsp(MockVsp(opi_port=0), pm)
    d = Daemon(FakePlatform("IPU Adapter E2100-CCQDA2"), "dpu", api, None, pm, tick=0.05,
               manager_kw={"register_device_plugin": False, "dp_poll": 0.05})
    d.prepare()
    out = {}
    t = threading.Thread(target=lambda: out.setdefault("err", d.serve()), daemon=True)
    t.start()
    try:
        assert wait_until(lambda: any(c[0] == "SetNumVfs" for c in vsp.calls), 5)
        assert len(d.managers) == 1 and isinstance(d.managers[0], DpuSideManager)
        import os

        assert os.access(pm.cni_path(), os.X_OK)
    finally:
        d.stop_event.set()
        t.join(5)
        vsp.stop()
    assert out.get("err") is None


def test_daemon_no_platform_keeps_scanning(pm):
    touch(pm.wrap("/dpu-cni"))
    d = Daemon(FakePlatform("plain server"), "auto", None, None, pm, tick=0.02)
    t = threading.Thread(target=d.serve, daemon=True)
    t.start()
    threading.Event().wait(0.2)
    assert d.managers == []
    d.stop_event.set()
    t.join(5)


def test_daemon_side_manager_failure_stops_serve(pm):
    touch(pm.wrap("/dpu-cni"))

    class Broken(DummyPlugin):
        def start(self):
            raise RuntimeError("vsp never came up")

    d = Daemon(FakePlatform("IPU Adapter E2100-CCQDA2"), "dpu", None, None, pm, tick=0.02,
               plugin_factory=lambda spec: Broken(0), manager_kw={"register_device_plugin": False})
    err = d.serve()
    assert isinstance(err, RuntimeError) and "never came up" in str(err)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_colocated_gpu_node_end_to_end(pm, device):
    """MI355X node: daemon -> ColocatedSideManager -> GPU VSP -> steering verified, on the C++
    oracle (cpu) and on the HIP kernels (cuda): CNI ADDs and OPI CreateBridgePort program the
    tables, then frames go through the data plane."""
    from dpu_operator_amd.ops import packets as P
    from dpu_operator_amd.vsp.gpu import WIRE_PORT, GpuVsp

    touch(pm.wrap("/dpu-cni"))
    api = ApiServer()
    nl = FakeNetlink()
    kubelet = FakeKubelet(pm, api).start()
    gvsp = GpuVsp(path_manager=pm, device=device, nl=nl, flow_buckets=1 << 8)
    gvsp.start()
    plat = FakePlatform("AMD server", [PciDevice("0000:05:00.0", "1002", "75a3", class_code=0x120000)])
    d = Daemon(plat, "auto", api, None, pm, nl=nl, tick=0.05, manager_kw={"dp_poll": 0.05})
    t = threading.Thread(target=d.serve, daemon=True)
    t.start()
    try:
        assert wait_until(lambda: kubelet.allocatable() == 8, 10), kubelet.devices
        mgr = d.managers[0]
        assert mgr.kind == "colocated"
        sock = pm.cni_server_path()
        # NF pod: two vports moved into its netns -> CreateNetworkFunction(mac0, mac1)
        nl.add_netns("/var/run/netns/nf")
        for i, dev in enumerate(("dpuvp6", "dpuvp7")):
            cni_call(sock, "ADD", {"cniVersion": "0.4.0", "name": V.NF_NAD_NAME, "type": "dpu-cni", "deviceID": dev},
                     netns="/var/run/netns/nf", ifname=f"net{i + 1}", pod_ns=V.NAMESPACE, pod_name="nf")
        assert len(gvsp.nfs) == 1
        nf = gvsp.nfs[0]
        assert (nf["in"], nf["out"]) == (6, 7)
        # workload pod on VF 0 (host side -> OPI CreateBridgePort host0-0 over loopback)
        wl = dict(CONF, VFID=0)
        cni_call(sock, "ADD", wl, pod_ns="default", pod_name="client")
        assert wait_until(lambda: "host0-0" in gvsp.bridge_ports, 5)
        port0 = gvsp.dp.ports.a[0]
        assert port0["vlan"] == 2  # logical bridge = vf + 2
        # a frame from the workload pod goes to the NF ingress vport, tagged toward... NF-in is untagged
        pod_mac = "00:11:22:33:44:55"
        frames, lens = P.craft(1, dmac="02:00:00:00:ff:01", smac=pod_mac, src_ip=0x0A000002, dst_ip=0x08080808,
                               sport=1234, dport=53)
        out, meta = gvsp.process(frames, [0])
        op, _, reason = P.meta_fields(meta)
        assert int(reason[0]) == 0 and int(op[0]) == 6
        # spoofed source MAC is dropped at the VF
        frames2, _ = P.craft(1, dmac="02:00:00:00:ff:01", smac="00:de:ad:be:ef:00", src_ip=0x0A000002,
                             dst_ip=0x08080808, sport=1, dport=2)
        _, meta2 = gvsp.process(frames2, [0])
        assert int(P.meta_fields(meta2)[2][0]) == 3  # spoof
        # the NF's egress vport forwards to the wire; the wire comes back in through NF-out
        _, meta3 = gvsp.process(frames, [7])
        assert int(P.meta_fields(meta3)[0][0]) == WIRE_PORT
        reply, _ = P.craft(1, dmac=pod_mac, smac="02:00:00:00:ff:01", src_ip=0x08080808, dst_ip=0x0A000002,
                           sport=53, dport=1234)
        _, meta4 = gvsp.process(reply, [WIRE_PORT])
        assert int(P.meta_fields(meta4)[0][0]) == 7
        # NF ingress side, dst = pod MAC -> the pod's VF, tagged with its VLAN
        out5, meta5 = gvsp.process(reply, [6])
        op5, len5, r5 = P.meta_fields(meta5)
        assert int(op5[0]) == 0 and int(r5[0]) == 0
        assert out5[0, 12] == 0x81 and out5[0, 15] == 2
        # hairpin: NF egress side, dst = pod MAC -> back into NF-out
        _, meta6 = gvsp.process(reply, [7])
        assert int(P.meta_fields(meta6)[0][0]) == 7
        # teardown
        cni_call(sock, "DEL", wl, pod_ns="default", pod_name="client")
        assert wait_until(lambda: "host0-0" not in gvsp.bridge_ports, 5)
        for i, dev in enumerate(("dpuvp6", "dpuvp7")):
            cni_call(sock, "DEL", {"cniVersion": "0.4.0", "name": V.NF_NAD_NAME, "type": "dpu-cni", "deviceID": dev},
                     netns="/var/run/netns/nf", ifname=f"net{i + 1}", pod_ns=V.NAMESPACE, pod_name="nf")
        assert gvsp.nfs == []
        assert np.all(gvsp.dp.ports.a[0]["vlan"] == 0)
    finally:
        d.stop_event.set()
        t.join(10)
        kubelet.stop()
        gvsp.stop()


def test_device_plugin_mounts_memif_vports_into_the_pod(pm):
    """GPU VSP with shared-memory vports: Allocate hands the pod its region (a bind mount of
    <memif_dir>/<vport>.memif at PathManager.memif_container_path, listed in NF-MEMIF), like the
    memif / vhost-user device plugins; the region the pod gets is the one the engine serves."""
    from dpu_operator_amd.native import nfdp
    from dpu_operator_amd.vsp.gpu import GpuVsp

    touch(pm.wrap("/dpu-cni"))
    api = ApiServer()
    kubelet = FakeKubelet(pm, api).start()
    gvsp = GpuVsp(path_manager=pm, device="cpu", nl=FakeNetlink(), flow_buckets=1 << 8, live=True,
                  vport_kind="memif")
    assert gvsp.memif_dir == pm.memif_dir() and gvsp.live_engine == "native"
    gvsp.start()
    plat = FakePlatform("AMD server", [PciDevice("0000:05:00.0", "1002", "75a3", class_code=0x120000)])
    d = Daemon(plat, "auto", api, None, pm, nl=FakeNetlink(), tick=0.05, manager_kw={"dp_poll": 0.05})
    t = threading.Thread(target=d.serve, daemon=True)
    t.start()
    try:
        assert wait_until(lambda: kubelet.allocatable() == 8, 10), kubelet.devices
        resp = kubelet.allocate(["dpuvp2", "dpuvp3"])
        cr = resp.container_responses[0]
        assert cr.envs["NF-DEV"] == "dpuvp2,dpuvp3,"
        mounts = {m.container_path: m.host_path for m in cr.mounts}
        assert mounts == {pm.memif_container_path(f"dpuvp{i}"): f"{pm.memif_dir()}/dpuvp{i}.memif" for i in (2, 3)}
        assert cr.envs["NF-MEMIF"].split(",") == [pm.memif_container_path("dpuvp2"), pm.memif_container_path("dpuvp3")]
        assert all(os.path.exists(h) for h in mounts.values())
        nfdp().MemifEndpoint(mounts[pm.memif_container_path("dpuvp2")])   # a valid region the pod can attach to
    finally:
        kubelet.stop()
        gvsp.stop_live()
