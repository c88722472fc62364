"""Control-plane unit and integration tests mirroring the reference's suites:
webhook validation, CNI netconf parsing, CNI logging labels, filesystem mode / cluster flavour
detection, controller DaemonSet + NADs for both modes with owner-reference GC, SFC reconciler
(NF pods with 2 DPU resources, N+1 chains -> last Pending until one is deleted), strict template
rendering, CNI server dispatch, GARP / unsolicited-NA frames, PCI allocator, wire round trips."""
from __future__ import annotations

import json
import os
import shutil
import struct
import tempfile

import pytest

from dpu_operator_amd import render
from dpu_operator_amd import vars as V
from dpu_operator_amd.api import v1
from dpu_operator_amd.k8s.apiserver import ApiServer, Forbidden, make_node
from dpu_operator_amd.k8s.manager import Request
from dpu_operator_amd.utils.paths import FilesystemMode, Flavour, PathManager


# ------------------------------------------------------------------------------ API / webhook (A1-A3)
@pytest.mark.parametrize("mode", ["host", "dpu", "auto"])
def test_webhook_accepts_valid_modes(mode):
    # the webhook allows auto (dpuoperatorconfig_webhook.go:55-58); the reconciler rejects it later
    assert v1.validate_dpu_operator_config({"metadata": {"name": V.DPU_OPERATOR_CONFIG_NAME},
                                            "spec": {"mode": mode}}) == []


@pytest.mark.parametrize("obj", [
    {"metadata": {"name": "not-the-standard-name"}, "spec": {"mode": "host"}},
    {"metadata": {"name": V.DPU_OPERATOR_CONFIG_NAME}, "spec": {"mode": "bogus"}},
])
def test_webhook_rejects(obj):
    with pytest.raises(v1.ValidationError):
        v1.validate_dpu_operator_config(obj)


def test_typed_round_trip():
    cfg = v1.DpuOperatorConfig(spec=v1.DpuOperatorConfigSpec(mode="dpu", logLevel=2))
    back = v1.DpuOperatorConfig.from_obj(cfg.to_obj())
    assert back.spec == cfg.spec and back.name == V.DPU_OPERATOR_CONFIG_NAME
    sfc = v1.ServiceFunctionChain("chain", network_functions=[v1.NetworkFunction("nf1", "img")])
    assert v1.ServiceFunctionChain.from_obj(sfc.to_obj()).network_functions == sfc.network_functions


# ------------------------------------------------------------------------------ CNI helpers (C3-C5)
def test_netconf_parsing():
    from dpu_operator_amd.cni.helper import read_cni_config

    conf = read_cni_config(json.dumps({
        "cniVersion": "0.4.0", "name": "dpunfcni-conf", "type": "dpu-cni", "deviceID": "0000:05:00.2",
        "vlan": 4, "spoofchk": "on", "ipam": {"type": "host-local"}, "logLevel": "debug",
        "OrigVfState": {"HostIFName": "ens1f0v2", "EffectiveMAC": "00:11:22:33:44:55"}}).encode())
    assert conf.name == "dpunfcni-conf" and conf.deviceID == "0000:05:00.2" and conf.vlan == 4
    assert conf.spoofchk == "on" and conf.ipam["type"] == "host-local" and conf.logLevel == "debug"
    assert conf.OrigVfState.HostIFName == "ens1f0v2"
    with pytest.raises(ValueError):
        read_cni_config(b"{not json")
    with pytest.raises(ValueError):
        read_cni_config(b"[1, 2]")


def test_cni_logging_prepends_labels(tmp_path):
    from dpu_operator_amd.cni import logging as clog

    log_file = tmp_path / "cni.log"
    clog.init("debug", str(log_file))
    clog.set_labels("dpu-cni", "cid-1", "/var/run/netns/x", "net1")
    clog.info("attached", vf=3)
    clog.debug("detail")
    clog.init("error", str(log_file))
    clog.info("suppressed")
    text = log_file.read_text()
    assert 'attached cniName="dpu-cni" containerID="cid-1" netns="/var/run/netns/x" ifname="net1" vf="3"' in text
    assert "detail" in text and "suppressed" not in text


# ------------------------------------------------------------------------------ environment (U1-U2)
def test_filesystem_mode_detector(tmp_path):
    from dpu_operator_amd.utils.environment import FilesystemModeDetector

    assert FilesystemModeDetector(str(tmp_path)).detect_mode() == FilesystemMode.PACKAGE
    (tmp_path / "run").mkdir()
    (tmp_path / "run" / "ostree-booted").write_text("")
    assert FilesystemModeDetector(str(tmp_path)).detect_mode() == FilesystemMode.IMAGE

    def eperm(_p):
        raise PermissionError(1, "Operation not permitted")

    assert FilesystemModeDetector("/", stat_fn=eperm).detect_mode() == FilesystemMode.IMAGE  # EPERM = present


def test_cluster_flavour():
    from dpu_operator_amd.utils.environment import ClusterEnvironment

    api = ApiServer()
    assert ClusterEnvironment(api).flavour() == Flavour.UNKNOWN
    node = make_node("kind-control-plane")
    node["status"]["images"] = [{"names": ["docker.io/kindest/node@sha256:1"]}]
    api.create(node)
    assert ClusterEnvironment(api).flavour() == Flavour.KIND
    api.create({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "microshift-version",
                                                                       "namespace": "kube-public"}})
    assert ClusterEnvironment(api).flavour() == Flavour.MICROSHIFT


# ------------------------------------------------------------------------------ operator (O2, R1)
def _operator(mode):
    from dpu_operator_amd.controller.operator import DpuOperatorConfigReconciler, install_webhook
    from dpu_operator_amd.images import DummyImageManager

    api = ApiServer(scheduler=False)
    api.create({"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                "metadata": {"name": "clusterversions.config.openshift.io"}})
    install_webhook(api)
    rec = DpuOperatorConfigReconciler(api, DummyImageManager())
    api.create({"apiVersion": v1.API_VERSION, "kind": v1.KIND_DPU_OPERATOR_CONFIG,
                "metadata": {"name": V.DPU_OPERATOR_CONFIG_NAME}, "spec": {"mode": mode}})
    rec.reconcile(Request("", V.DPU_OPERATOR_CONFIG_NAME))
    return api, rec


@pytest.mark.parametrize("mode", ["host", "dpu"])
def test_controller_daemonset_and_nads(mode):
    api, _ = _operator(mode)
    ds = api.get("DaemonSet", "dpu-daemon", V.NAMESPACE)
    args = ds["spec"]["template"]["spec"]["containers"][0]["args"]
    assert args[0] == "--mode" and args[1] == "auto"  # dpuoperatorconfig_controller_test.go:81-171
    nads = api.list("NetworkAttachmentDefinition")
    assert [n["metadata"]["name"] for n in nads] == [V.NF_NAD_NAME if mode == "dpu" else "default-sriov-net"]
    cfg = json.loads(nads[0]["spec"]["config"])
    assert cfg["type"] == "dpu-cni"
    # owner references: deleting the CR garbage-collects everything it rendered
    api.delete(v1.KIND_DPU_OPERATOR_CONFIG, V.DPU_OPERATOR_CONFIG_NAME)
    assert api.try_get("DaemonSet", "dpu-daemon", V.NAMESPACE) is None and not api.list("NetworkAttachmentDefinition")


def test_controller_rejects_auto_for_nads():
    from dpu_operator_amd.k8s.apiserver import BadRequest

    with pytest.raises(BadRequest):
        _operator("auto")


def test_webhook_blocks_bad_update():
    api, _ = _operator("host")
    cur = api.get(v1.KIND_DPU_OPERATOR_CONFIG, V.DPU_OPERATOR_CONFIG_NAME)
    cur["spec"]["mode"] = "bogus"
    with pytest.raises(Forbidden):
        api.update(cur)


def test_render_is_strict():
    with pytest.raises(render.TemplateError):
        render.apply_template("image: {{.Missing}}", {"Present": 1})
    assert render.apply_template("ns: {{.Namespace}}", {"Namespace": "x"}) == "ns: x"


# ------------------------------------------------------------------------------ SFC reconciler (SFC1)
def test_sfc_nf_pods_and_resource_exhaustion():
    """Each NF pod asks for 2 DPU devices; with 8 allocatable, the 5th single-NF chain stays
    Pending until one chain is deleted (e2e_test.go:525-592)."""
    from dpu_operator_amd.daemon.sfc import SfcReconciler

    api = ApiServer()
    api.create(make_node("worker-0", allocatable={V.RESOURCE_NAME: "8"}))
    rec = SfcReconciler(api)
    for k in range(5):
        sfc = v1.ServiceFunctionChain(f"sfc{k}", network_functions=[v1.NetworkFunction(f"nf{k}", "quay.io/nf:1")])
        api.create(sfc.to_obj())
        rec.reconcile(Request(V.NAMESPACE, f"sfc{k}"))
    pods = {p["metadata"]["name"]: p for p in api.list("Pod", V.NAMESPACE)}
    assert len(pods) == 5
    req = pods["nf0"]["spec"]["containers"][0]["resources"]["requests"]
    assert req[V.RESOURCE_NAME] == "2"
    assert pods["nf0"]["metadata"]["annotations"]["k8s.v1.cni.cncf.io/networks"].count(V.NF_NAD_NAME) == 2
    phases = [pods[f"nf{k}"]["status"]["phase"] for k in range(5)]
    assert phases == ["Running"] * 4 + ["Pending"]
    api.delete(v1.KIND_SFC, "sfc0", V.NAMESPACE)  # GC removes nf0 -> nf4 gets scheduled
    assert api.try_get("Pod", "nf0", V.NAMESPACE) is None
    assert api.get("Pod", "nf4", V.NAMESPACE)["status"]["phase"] == "Running"


def test_sfc_gpu_functions_go_to_the_chain_table():
    from dpu_operator_amd.daemon.sfc import SfcReconciler

    api = ApiServer()
    seen = []
    rec = SfcReconciler(api, on_gpu_chain=lambda name, kinds: seen.append((name, kinds)))
    sfc = v1.ServiceFunctionChain("g", network_functions=[v1.NetworkFunction("fw", "gpu-nf://acl,nat"),
                                                          v1.NetworkFunction("rt", "gpu-nf://ttl")])
    api.create(sfc.to_obj())
    rec.reconcile(Request(V.NAMESPACE, "g"))
    assert seen == [("g", ["acl", "nat", "ttl"])] and api.list("Pod", V.NAMESPACE) == []
    assert api.get(v1.KIND_SFC, "g", V.NAMESPACE)["status"]["gpuHops"] == ["acl", "nat", "ttl"]


# ------------------------------------------------------------------------------ CNI server (S4)
def test_cni_server_dispatch():
    from dpu_operator_amd.cni.server import Server
    from dpu_operator_amd.testutils.kubelet import cni_call

    root = tempfile.mkdtemp(prefix="dpuc", dir="/tmp")
    calls = []
    try:
        srv = Server(lambda r: calls.append(("ADD", r.pod_name, r.ifname)) or {"cniVersion": "0.4.0"},
                     lambda r: calls.append(("DEL", r.pod_name, r.ifname)), PathManager(root)).start()
        conf = {"cniVersion": "0.4.0", "name": "n", "type": "dpu-cni"}
        cni_call(srv.socket_path, "ADD", conf, pod_name="p1", ifname="net1")
        cni_call(srv.socket_path, "DEL", conf, pod_name="p1", ifname="net1")
        assert calls == [("ADD", "p1", "net1"), ("DEL", "p1", "net1")] and srv.requests_served == 2
        srv.shutdown()
    finally:
        shutil.rmtree(root, ignore_errors=True)


# ------------------------------------------------------------------------------ SR6 / SR5
def test_garp_and_unsolicited_na_frames():
    from dpu_operator_amd.cni.sriov.packet import garp_frame, unsolicited_na_frame

    g = garp_frame("02:00:00:00:00:01", "10.0.0.5")
    assert g[:6] == b"\xff" * 6 and g[12:14] == b"\x08\x06"
    op = struct.unpack("!H", g[20:22])[0]
    assert op in (1, 2) and g[28:32] == bytes([10, 0, 0, 5]) and g[38:42] == bytes([10, 0, 0, 5])
    na = unsolicited_na_frame("02:00:00:00:00:01", "fd00::5")
    assert na[12:14] == b"\x86\xdd" and na[20] == 58 and na[54] == 136  # ICMPv6 neighbor advertisement
    assert na[0:2] == b"\x33\x33"  # all-nodes multicast


def test_pci_allocator(tmp_path):
    from dpu_operator_amd.cni.sriov.pci_allocator import PCIAllocator

    live = {"/var/run/netns/a"}
    alloc = PCIAllocator(str(tmp_path), netns_exists=lambda ns: ns in live)
    alloc.save_allocated_pci("0000:05:00.2", "/var/run/netns/a")
    assert alloc.is_allocated("0000:05:00.2")
    live.clear()  # the pod's netns is gone: a stale allocation is released
    assert not alloc.is_allocated("0000:05:00.2")
    alloc.save_allocated_pci("0000:05:00.3", "/var/run/netns/b")
    alloc.delete_allocated_pci("0000:05:00.3")
    assert not os.path.exists(os.path.join(str(tmp_path), "0000:05:00.3"))


# ------------------------------------------------------------------------------ wire schemas (V0)
def test_proto_wire_round_trip():
    from dpu_operator_amd.proto import deviceplugin as dp
    from dpu_operator_amd.proto import opi, vendor

    req = opi.CreateBridgePortRequest(bridge_port=opi.BridgePort(
        name="host0-3", spec=opi.BridgePortSpec(ptype=opi.BRIDGE_PORT_TYPE_ACCESS, mac_address=b"\x00\x11\x22\x33\x44\x55",
                                                logical_bridges=["5"])))
    b = req.SerializeToString()
    back = opi.CreateBridgePortRequest.FromString(b)
    assert back.bridge_port.spec.logical_bridges == ["5"] and back.bridge_port.name == "host0-3"
    nf = vendor.NFRequest(input="a", output="b")
    assert vendor.NFRequest.FromString(nf.SerializeToString()) == nf
    # field numbers on the wire (golden bytes): Device{ID=1 "x", health=2 "Healthy"}
    assert dp.Device(ID="x", health="Healthy").SerializeToString() == b"\x0a\x01x\x12\x07Healthy"


# ------------------------------------------------------------------------------ node policy config
def test_node_config_file_env_and_wiring(tmp_path):
    from dpu_operator_amd.config import NodeConfig, node_config, set_node_config
    from dpu_operator_amd.daemon.deviceplugin import DeviceHandler
    from dpu_operator_amd.daemon.sfc import network_function_pod

    d = NodeConfig()
    assert (d.vf_count, d.logical_bridge(3), d.nf_devices_per_pod, d.comm_port) == (8, 5, 2, 8085)
    p = tmp_path / "node.yaml"
    p.write_text("vf_count: 16\nlogical_bridge_offset: 100\nnf_devices_per_pod: 3\n")
    cfg = NodeConfig.load(str(p), env={"DPU_CFG_HASH_MODE": "mfma"})
    assert cfg.vf_count == 16 and cfg.logical_bridge(0) == 100 and cfg.hash_mode == "mfma"
    with pytest.raises(ValueError):
        NodeConfig.load(str(p), env={"DPU_CFG_HASH_MODE": "bogus"})
    bad = tmp_path / "bad.yaml"
    bad.write_text("no_such_key: 1\n")
    with pytest.raises(ValueError):
        NodeConfig.load(str(bad), env={})
    set_node_config(cfg)
    try:
        assert DeviceHandler(None, True).vf_count == 16
        pod = network_function_pod("nf", "img")
        assert pod["spec"]["containers"][0]["resources"]["requests"][V.RESOURCE_NAME] == "3"
        assert pod["metadata"]["annotations"]["k8s.v1.cni.cncf.io/networks"].count(V.NF_NAD_NAME) == 3
        assert node_config() is cfg
    finally:
        set_node_config(None)
