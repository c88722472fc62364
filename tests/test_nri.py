"""Network Resources Injector: selection parsing, resource/node-selector/Downward-API patches,
control switches, the in-process admission hook, and the HTTPS webhook server (TLS, /mutate,
/healthz, key-pair hot reload).  Expectations follow the vendored injector's behaviour
(webhook.go, controlswitches.go)."""
from __future__ import annotations

import base64
import http.client
import json
import os
import shutil
import ssl
import subprocess
import tempfile
import time

import pytest

from dpu_operator_amd import vars as V
from dpu_operator_amd.cmd import nri as nri_cmd
from dpu_operator_amd.k8s.apiserver import ApiServer, Forbidden
from dpu_operator_amd.nri import webhook as W
from dpu_operator_amd.nri.server import InjectorServer, KeyPairReloader

RES = V.RESOURCE_NAME


def nad(name, ns="default", res=RES, node_sel=None):
    ann = {W.DEFAULT_RESOURCE_NAME_KEY: res} if res else {}
    if node_sel:
        ann[W.NODE_SELECTOR_KEY] = node_sel
    return {"apiVersion": "k8s.cni.cncf.io/v1", "kind": "NetworkAttachmentDefinition",
            "metadata": {"name": name, "namespace": ns, "annotations": ann}, "spec": {"config": "{}"}}


def pod(nets, resources=None, ns="default"):
    c = {"name": "c", "image": "x"}
    if resources is not None:
        c["resources"] = resources
    return {"apiVersion": "v1", "kind": "Pod",
            "metadata": {"name": "p", "namespace": ns, "annotations": {W.NETWORKS_ANNOTATION: nets} if nets else {}},
            "spec": {"containers": [c, {"name": "side", "image": "y"}]}}


def cache(*nads):
    d = {(n["metadata"]["namespace"], n["metadata"]["name"]): n for n in nads}
    return W.NadCache(lambda ns, name: d.get((ns, name)))


def test_parse_selections():
    s = W.parse_network_selections("a, other/b@net1", "default")
    assert s == [{"namespace": "default", "name": "a", "interface": ""},
                 {"namespace": "other", "name": "b", "interface": "net1"}]
    j = W.parse_network_selections('[{"name": "a"}, {"name": "b", "namespace": "x", "interface": "eth9"}]', "d")
    assert j[0]["namespace"] == "d" and j[1]["interface"] == "eth9"
    for bad in ("a/b/c", "a@b@c", "Bad_Name"):
        with pytest.raises(ValueError):
            W.parse_network_selections(bad, "default")
    assert W.parse_network_selections("a", "") is None


def test_resource_injection():
    sw = W.ControlSwitches()
    nads = cache(nad("sriov"), nad("plain", res=None), nad("other", res="intel.com/x", node_sel="zone=a"))
    p = W.apply_patch(pod("sriov, sriov, plain, other"), W.mutate_pod(pod("sriov, sriov, plain, other"), nads, sw))
    r = p["spec"]["containers"][0]["resources"]
    assert r["requests"] == {RES: "2", "intel.com/x": "1"} and r["limits"] == r["requests"]
    assert p["spec"]["nodeSelector"] == {"zone": "a"}
    assert "resources" not in p["spec"]["containers"][1]
    # an explicit request wins unless honor-resources is on
    explicit = {"requests": {RES: "3"}, "limits": {RES: "3"}}
    assert W.mutate_pod(pod("sriov", explicit), nads, sw) == []
    sw2 = W.ControlSwitches(honor_resources=True)
    p2 = W.apply_patch(pod("sriov", explicit), W.mutate_pod(pod("sriov", explicit), nads, sw2))
    assert p2["spec"]["containers"][0]["resources"]["requests"][RES] == "4"
    with pytest.raises(ValueError, match="could not find"):
        W.mutate_pod(pod("missing"), nads, sw)
    assert W.mutate_pod(pod(None), nads, sw) == []
    sw3 = W.ControlSwitches(inject_hugepage_down_api=True)
    p3 = W.apply_patch(pod("sriov"), W.mutate_pod(pod("sriov"), nads, sw3))
    assert p3["spec"]["volumes"][0]["name"] == "podnetinfo"
    assert all(c["volumeMounts"][0]["mountPath"] == "/etc/podnetinfo" for c in p3["spec"]["containers"])


def test_control_switches_configmap():
    sw = W.ControlSwitches()
    assert not sw.honor_existing()
    sw.process_configmap({"data": {"features": json.dumps({W.HONOR_EXISTING: True, W.HUGEPAGE_DOWNAPI: True})}})
    assert sw.honor_existing() and sw.hugepage_down_api()
    sw.process_configmap({"data": {"features": "{not json"}})
    assert not sw.honor_existing()  # back to the flag state
    sw.process_configmap(None)
    assert sw.state() == "HugePageInject: false / HonorExistingResources: false / EnableResourceNames: true"


def test_api_admission_hook_sfc_pods():
    api = ApiServer()
    W.api_admission_hook(api)
    api.create(nad(V.NF_NAD_NAME, ns=V.NAMESPACE))
    created = api.create(pod(f"{V.NF_NAD_NAME}, {V.NF_NAD_NAME}", ns=V.NAMESPACE))
    assert created["spec"]["containers"][0]["resources"]["limits"][RES] == "2"
    with pytest.raises(Forbidden, match="could not find"):
        api.create(dict(pod("nope"), metadata={"name": "q", "namespace": "default",
                                                "annotations": {W.NETWORKS_ANNOTATION: "nope"}}))


@pytest.fixture
def certs():
    if not shutil.which("openssl"):
        pytest.skip("openssl not available")
    d = tempfile.mkdtemp(prefix="nri", dir="/tmp")

    def make():
        subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-days", "1", "-subj", "/CN=nri",
                        "-keyout", f"{d}/key.pem", "-out", f"{d}/cert.pem"], check=True, capture_output=True)

    make()
    yield d, make
    shutil.rmtree(d, ignore_errors=True)


def _post(port, body, path="/mutate", method="POST", ctype="application/json"):
    ctx = ssl.create_default_context()
    ctx.check_hostname = False
    ctx.verify_mode = ssl.CERT_NONE
    c = http.client.HTTPSConnection("127.0.0.1", port, context=ctx, timeout=10)
    c.request(method, path, body=body, headers={"Content-Type": ctype})
    r = c.getresponse()
    out = r.status, r.read()
    c.close()
    return out


def test_https_webhook_server(certs):
    d, make = certs
    api = ApiServer()
    api.create(nad("sriov"))
    reloader = KeyPairReloader(f"{d}/cert.pem", f"{d}/key.pem", insecure=True)
    nads = W.NadCache(lambda ns, name: api.try_get("NetworkAttachmentDefinition", name, ns))
    srv = InjectorServer(nads, W.ControlSwitches(), reloader, "127.0.0.1", 0, 0, api=api).start()
    try:
        review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
                  "request": {"uid": "u1", "kind": {"kind": "Pod"}, "namespace": "default", "object": pod("sriov")}}
        code, body = _post(srv.port, json.dumps(review))
        resp = json.loads(body)["response"]
        assert code == 200 and resp["uid"] == "u1" and resp["allowed"] and resp["patchType"] == "JSONPatch"
        patch = json.loads(base64.b64decode(resp["patch"]))
        assert {"op": "add", "path": "/spec/containers/0/resources/requests/openshift.io~1dpu", "value": "1"} in patch
        review["request"]["object"] = pod("missing")
        resp = json.loads(_post(srv.port, json.dumps(review))[1])["response"]
        assert not resp["allowed"] and "could not find" in resp["status"]["message"]
        assert _post(srv.port, None, method="GET")[0] == 405
        assert _post(srv.port, "{}", path="/other")[0] == 404
        assert _post(srv.port, "{}", ctype="text/plain")[0] == 400
        c = http.client.HTTPConnection("127.0.0.1", srv.health_port, timeout=5)
        c.request("GET", "/healthz")
        assert c.getresponse().status == 200
        c.close()
        # key pair hot reload
        n = reloader.reloads
        time.sleep(0.02)
        make()
        os.utime(f"{d}/cert.pem")
        assert _post(srv.port, json.dumps(review))[0] == 200
        assert reloader.reloads == n + 1
        # control switches from the ConfigMap
        api.create({"apiVersion": "v1", "kind": "ConfigMap",
                    "metadata": {"name": W.CONTROL_SWITCHES_CM, "namespace": srv.namespace},
                    "data": {"features": json.dumps({W.HONOR_EXISTING: True})}})
        srv.refresh_switches()
        assert srv.switches.honor_existing()
    finally:
        srv.stop()


def test_cli_validation():
    assert nri_cmd.main(["--port", "80"]) == 1
    assert nri_cmd.main(["--network-resource-name-keys", ""]) == 1
    assert nri_cmd.main(["--health-check-port", "8443"]) == 1
