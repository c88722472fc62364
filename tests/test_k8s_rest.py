"""Contract suite for the Kubernetes API surface, run twice: against the in-process ApiServer and
through k8s/rest.py's RestClient talking HTTP to an emulated API endpoint (testutils/kubeapi.py,
bearer-token auth, kubeconfig discovery).  The operator and the daemon's SFC reconciler run over
the REST client end to end (reference cmd/main.go:64-86, dpusidemanager.go:256-292)."""
import base64
import os
import threading
import time

import pytest

from dpu_operator_amd import vars as V
from dpu_operator_amd.api.scheme import SCHEME
from dpu_operator_amd.api.v1 import KIND_DPU_OPERATOR_CONFIG, KIND_SFC, crd_manifests
from dpu_operator_amd.k8s import rest as R
from dpu_operator_amd.k8s.apiserver import (AlreadyExists, ApiServer, Conflict, Forbidden, NotFound,
                                            set_controller_reference)
from dpu_operator_amd.testutils.kubeapi import KubeApiServer


def wait_until(fn, t=5.0):
    end = time.monotonic() + t
    while time.monotonic() < end:
        if fn():
            return True
        time.sleep(0.02)
    return False


@pytest.fixture(params=["inproc", "rest"])
def env(request, tmp_path):
    backing = ApiServer(scheme=SCHEME)
    for crd in crd_manifests():
        backing.create(crd)
    backing.create({"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                    "metadata": {"name": "clusterversions.config.openshift.io"}})  # an OpenShift cluster
    if request.param == "inproc":
        yield backing, backing
        return
    srv = KubeApiServer(backing, token="s3cret").start()
    client = R.RestClient(R.ClusterConfig.from_kubeconfig(srv.kubeconfig(str(tmp_path / "kc.yaml"))))
    yield client, backing
    client.close()
    srv.stop()


def _cm(name, ns="default", labels=None, data=None):
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": ns, "labels": labels or {}},
            "data": data or {}}


def test_crud_conflicts_and_errors(env):
    api, _ = env
    o = api.create(_cm("a", labels={"app": "x"}, data={"k": "1"}))
    assert o["metadata"]["uid"] and o["metadata"]["resourceVersion"]
    with pytest.raises(AlreadyExists):
        api.create(_cm("a"))
    api.create(_cm("b", labels={"app": "y"}))
    api.create(_cm("c", ns="other", labels={"app": "x"}))
    assert [x["metadata"]["name"] for x in api.list("ConfigMap", "default")] == ["a", "b"]
    assert [x["metadata"]["name"] for x in api.list("ConfigMap", labels={"app": "x"})] == ["c", "a"] or \
        sorted(x["metadata"]["name"] for x in api.list("ConfigMap", labels={"app": "x"})) == ["a", "c"]
    g = api.get("ConfigMap", "a", "default")
    g["data"]["k"] = "2"
    u = api.update(g)
    assert u["data"]["k"] == "2" and u["metadata"]["resourceVersion"] != g["metadata"]["resourceVersion"]
    with pytest.raises(Conflict):
        api.update(g)  # stale resourceVersion
    api.delete("ConfigMap", "a", "default")
    with pytest.raises(NotFound):
        api.get("ConfigMap", "a", "default")
    assert api.try_get("ConfigMap", "a", "default") is None
    with pytest.raises(NotFound):
        api.delete("ConfigMap", "a", "default")


def test_cluster_scoped_status_and_apply(env):
    api, _ = env
    cfg = {"apiVersion": "config.openshift.io/v1", "kind": KIND_DPU_OPERATOR_CONFIG,
           "metadata": {"name": V.DPU_OPERATOR_CONFIG_NAME}, "spec": {"mode": "host"}}
    c = api.create(cfg)
    assert "namespace" not in c["metadata"]
    c["status"] = {"conditions": [{"type": "Ready", "status": "True"}]}
    s = api.update_status(c)
    assert s["status"]["conditions"][0]["type"] == "Ready"
    a = api.apply({**cfg, "spec": {"mode": "dpu"}, "metadata": {**cfg["metadata"], "labels": {"x": "1"}}})
    assert a["spec"]["mode"] == "dpu" and a["metadata"]["labels"] == {"x": "1"}
    assert api.get(KIND_DPU_OPERATOR_CONFIG, V.DPU_OPERATOR_CONFIG_NAME)["status"]["conditions"]


def test_watch_events_and_gc(env):
    api, backing = env
    seen = []
    lock = threading.Lock()

    def fn(t, o):
        with lock:
            seen.append((t, o["metadata"]["name"]))

    api.create(_cm("pre"))
    cancel = api.watch("ConfigMap", fn, replay=True, namespace="default")
    try:
        owner = api.create(_cm("owner"))
        dep = set_controller_reference(owner, _cm("dep"))
        api.create(dep)
        d = api.get("ConfigMap", "dep", "default")
        d["data"] = {"z": "9"}
        api.update(d)
        api.delete("ConfigMap", "owner", "default")  # background cascade deletes "dep"
        assert wait_until(lambda: ("DELETED", "dep") in seen, 5), seen
        assert ("ADDED", "pre") in seen and ("ADDED", "owner") in seen and ("MODIFIED", "dep") in seen
        assert api.try_get("ConfigMap", "dep", "default") is None
    finally:
        cancel()
    n = len(seen)
    api.create(_cm("after"))
    time.sleep(0.3)
    assert len(seen) == n  # cancelled


def test_admission_is_server_side(env):
    api, backing = env

    def deny(op, obj, old):
        if obj["metadata"]["name"] != V.DPU_OPERATOR_CONFIG_NAME:
            raise ValueError("name must be " + V.DPU_OPERATOR_CONFIG_NAME)

    backing.register_validating(KIND_DPU_OPERATOR_CONFIG, deny)  # the cluster's webhook
    with pytest.raises(Forbidden):
        api.create({"apiVersion": "config.openshift.io/v1", "kind": KIND_DPU_OPERATOR_CONFIG,
                    "metadata": {"name": "wrong"}, "spec": {"mode": "host"}})


def test_operator_reconciles_over_the_api(env):
    from dpu_operator_amd.cmd import operator as op_cmd
    from dpu_operator_amd.images import DummyImageManager

    api, backing = env
    args = op_cmd.build_parser().parse_args(["--metrics-bind-address", "127.0.0.1:0",
                                             "--health-probe-bind-address", "127.0.0.1:0", "--cert-dir", "/nonexistent"])
    op = op_cmd.Operator(args, api, image_manager=DummyImageManager()).start()
    try:
        api.create({"apiVersion": "config.openshift.io/v1", "kind": KIND_DPU_OPERATOR_CONFIG,
                    "metadata": {"name": V.DPU_OPERATOR_CONFIG_NAME}, "spec": {"mode": "dpu"}})
        assert wait_until(lambda: backing.try_get("DaemonSet", "dpu-daemon", V.NAMESPACE) is not None, 8)
        assert wait_until(lambda: len(backing.list("NetworkAttachmentDefinition", V.NAMESPACE)) > 0, 8)
    finally:
        op.stop()


def test_sfc_reconciler_over_the_api(env):
    from dpu_operator_amd.daemon.sfc import SfcReconciler
    from dpu_operator_amd.k8s.manager import Manager

    api, backing = env
    mgr = Manager(api, namespace=V.NAMESPACE)
    mgr.add("sfc", SfcReconciler(api), KIND_SFC, owns=("Pod",))
    mgr.start()
    try:
        api.create({"apiVersion": "config.openshift.io/v1", "kind": KIND_SFC,
                    "metadata": {"name": "sfc1", "namespace": V.NAMESPACE},
                    "spec": {"networkFunctions": [{"name": "nf1", "image": "quay.io/x/nf:1"}]}})
        assert wait_until(lambda: backing.try_get("Pod", "nf1", V.NAMESPACE) is not None, 8)
        pod = backing.get("Pod", "nf1", V.NAMESPACE)
        assert pod["metadata"]["ownerReferences"][0]["kind"] == KIND_SFC
    finally:
        mgr.stop()


def test_watch_relists_after_410(tmp_path):
    backing = ApiServer()
    backing.create(_cm("x"))
    srv = KubeApiServer(backing).start()
    try:
        c = R.RestClient(R.ClusterConfig(server=srv.url))
        got = []
        w = R._Watch(c, "ConfigMap", lambda t, o: got.append((t, o["metadata"]["name"])), True, None)
        w.rv = "1"  # older than the endpoint's event log -> 410 -> re-list (ADDED replay)
        srv.floor = 10 ** 9
        w.start()
        assert wait_until(lambda: ("ADDED", "x") in got, 5)
        srv.floor = 0
        backing.create(_cm("y"))
        assert wait_until(lambda: ("ADDED", "y") in got, 5)
        w.stop()
    finally:
        srv.stop()


def test_relist_after_gap_emits_deletes_and_modifies(tmp_path):
    """A re-list (after 410 Gone) is a Replace: objects deleted while the watch was down produce
    DELETED with their last known state, known objects MODIFIED, new ones ADDED."""
    backing = ApiServer()
    backing.create(_cm("x"))
    backing.create(_cm("z", data={"k": "last"}))
    srv = KubeApiServer(backing).start()
    try:
        c = R.RestClient(R.ClusterConfig(server=srv.url))
        got = []
        w = R._Watch(c, "ConfigMap", lambda t, o: got.append((t, o["metadata"]["name"], o.get("data"))), True, None)
        w._list(first=True)
        assert sorted((t, n) for t, n, _ in got) == [("ADDED", "x"), ("ADDED", "z")]
        got.clear()
        backing.delete("ConfigMap", "z", "default")      # during the gap
        backing.create(_cm("n"))
        w._list(first=False)
        assert ("DELETED", "z", {"k": "last"}) in got
        assert ("MODIFIED", "x", {}) in got and ("ADDED", "n", {}) in got and len(got) == 3
        assert set(w.known) == {("default", "x"), ("default", "n")}
        # events on the stream keep the known set current
        w._track("DELETED", backing.get("ConfigMap", "n", "default"))
        got.clear()
        w._list(first=False)
        assert ("ADDED", "n", {}) in got
    finally:
        srv.stop()


def test_unauthorized_without_token(tmp_path):
    srv = KubeApiServer(ApiServer(), token="t").start()
    try:
        with pytest.raises(Forbidden):
            R.RestClient(R.ClusterConfig(server=srv.url)).list("ConfigMap")
    finally:
        srv.stop()


def test_config_discovery(tmp_path, monkeypatch):
    sa = tmp_path / "sa"
    sa.mkdir()
    (sa / "token").write_text("tok\n")
    (sa / "ca.crt").write_text("-----BEGIN CERTIFICATE-----\n")
    (sa / "namespace").write_text("openshift-dpu-operator")
    monkeypatch.setattr(R, "SA_DIR", str(sa))
    monkeypatch.delenv("KUBECONFIG", raising=False)
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.0.0.1")
    monkeypatch.setenv("KUBERNETES_SERVICE_PORT", "443")
    cfg = R.ClusterConfig.discover()
    assert cfg.server == "https://10.0.0.1:443" and cfg.token == "tok" and cfg.namespace == "openshift-dpu-operator"
    kc = tmp_path / "kc.yaml"
    kc.write_text(f"""
apiVersion: v1
kind: Config
current-context: c2
clusters:
- name: k
  cluster: {{server: "https://api.example:6443/", certificate-authority-data: "{base64.b64encode(b'PEM').decode()}"}}
users:
- name: u
  user: {{token: abc}}
contexts:
- name: c2
  context: {{cluster: k, user: u, namespace: ns1}}
""")
    monkeypatch.setenv("KUBECONFIG", str(kc))
    cfg = R.ClusterConfig.discover()
    assert cfg.server == "https://api.example:6443" and cfg.token == "abc" and cfg.namespace == "ns1"
    assert open(cfg.ca_file, "rb").read() == b"PEM"
    monkeypatch.delenv("KUBECONFIG")
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST")
    assert R.connect() is None


def test_daemon_entry_needs_a_cluster(monkeypatch):
    from dpu_operator_amd.cmd import daemon as d_cmd

    monkeypatch.delenv("KUBECONFIG", raising=False)
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    assert d_cmd.main(["--root", "/nonexistent-root"]) == 2
