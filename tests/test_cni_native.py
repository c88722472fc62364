"""The native `dpu-cni` binary (csrc/cni/dpu_cni.cpp) speaks the same protocol as the Python shim
(cni/shim.py, reference dpu-cni/pkgs/cni/cnishim.go): same request the server sees, same ADD
result / error objects, DEL result ignored, CHECK no-op, VERSION list."""
import io
import json
import os
import subprocess

import pytest

from dpu_operator_amd.cni import shim
from dpu_operator_amd.cni.server import Server
from dpu_operator_amd.native import build

CONF = {"cniVersion": "0.4.0", "name": "default-sriov-net", "type": "dpu-cni",
        "deviceID": "0000:03:00.2", "vlan": 2, "ipam": {"type": "host-local", "subnet": "10.56.217.0/24"}}
ENV = {"CNI_CONTAINERID": "cid-1", "CNI_NETNS": "/var/run/netns/x", "CNI_IFNAME": "net1", "CNI_PATH": "/opt/cni/bin",
       "CNI_ARGS": "IgnoreUnknown=1;K8S_POD_NAMESPACE=default;K8S_POD_NAME=my-pod;K8S_POD_UID=u-1"}


@pytest.fixture(scope="module")
def binary():
    return str(build.build_exe("dpu-cni"))


@pytest.fixture()
def server(tmp_path):
    seen = []

    def add(req):
        seen.append(("ADD", req.container_id, req.ifname, req.pod_namespace, req.pod_name, req.cni_conf_bytes()
                     if hasattr(req, "cni_conf_bytes") else None))
        if req.pod_name == "boom":
            raise RuntimeError("no VF available")
        return {"cniVersion": "1.0.0", "interfaces": [{"name": req.ifname, "mac": "02:00:00:00:00:01", "sandbox": req.netns}],
                "ips": [{"address": "10.56.217.5/24", "interface": 0}], "dns": {}}

    def dele(req):
        seen.append(("DEL", req.container_id, req.ifname, req.pod_namespace, req.pod_name, None))
        return {"ignored": True}

    sock = str(tmp_path / "run" / "dpu-cni" / "dpu-cni-server.sock")
    srv = Server(add, dele, socket_path=sock).start()
    try:
        yield sock, seen
    finally:
        srv.shutdown()


def _native(binary, sock, cmd, conf, **env_over):
    env = {"PATH": os.environ.get("PATH", ""), **ENV, "CNI_COMMAND": cmd, "DPU_CNI_SOCKET": sock, **env_over}
    data = conf if isinstance(conf, bytes) else json.dumps(conf).encode()
    r = subprocess.run([binary], input=data, env=env, capture_output=True, timeout=30)
    return r.returncode, r.stdout.decode()


def _python(sock, cmd, conf, **env_over):
    env = {**ENV, "CNI_COMMAND": cmd, **env_over}
    out = io.StringIO()
    data = conf if isinstance(conf, bytes) else json.dumps(conf).encode()
    rc = shim.main(env=env, stdin=data, stdout=out, socket_path=sock)
    return rc, out.getvalue()


def test_add_matches_python_shim(binary, server):
    sock, seen = server
    rc_n, out_n = _native(binary, sock, "ADD", CONF)
    rc_p, out_p = _python(sock, "ADD", CONF)
    assert rc_n == rc_p == 0
    assert json.loads(out_n) == json.loads(out_p)
    assert json.loads(out_n)["cniVersion"] == "0.4.0"      # the config's version wins
    assert seen[0][:5] == seen[1][:5] == ("ADD", "cid-1", "net1", "default", "my-pod")


def test_del_check_version(binary, server):
    sock, seen = server
    assert _native(binary, sock, "DEL", CONF) == (0, "")
    assert _native(binary, sock, "CHECK", CONF) == (0, "")
    assert [s[0] for s in seen] == ["DEL"]                    # CHECK never reaches the daemon
    rc, out = _native(binary, sock, "VERSION", b"")
    assert rc == 0 and json.loads(out) == json.loads(_python(sock, "VERSION", b"")[1])


@pytest.mark.parametrize("case", ["daemon_error", "bad_config", "no_daemon", "bad_command", "missing_args"])
def test_errors_match_python_shim(binary, server, tmp_path, case):
    sock, _ = server
    kw, conf, cmd = {}, CONF, "ADD"
    if case == "daemon_error":
        kw["CNI_ARGS"] = "K8S_POD_NAMESPACE=default;K8S_POD_NAME=boom"
    elif case == "bad_config":
        conf = b"{not json"
    elif case == "no_daemon":
        sock = str(tmp_path / "nothing.sock")
    elif case == "bad_command":
        cmd = "FROB"
    elif case == "missing_args":
        kw["CNI_ARGS"] = "K8S_POD_NAMESPACE=default"
    rc_n, out_n = _native(binary, sock, cmd, conf, **kw)
    rc_p, out_p = _python(sock, cmd, conf, **kw)
    assert rc_n == rc_p == 1
    en, ep = json.loads(out_n), json.loads(out_p)
    assert en["code"] == ep["code"] and en["cniVersion"] == ep["cniVersion"]
    if case in ("daemon_error", "missing_args"):
        assert en["msg"] == ep["msg"]                         # the daemon's message passes through verbatim


def test_binary_is_static(binary):
    out = subprocess.run(["file", binary], capture_output=True, text=True).stdout
    assert "statically linked" in out
