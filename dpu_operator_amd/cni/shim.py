"""`dpu-cni` — the CNI plugin binary kubelet/Multus executes.

Reference: dpu-cni/dpu-cni.go:17-42 and dpu-cni/pkgs/cni/cnishim.go:20-139.  It serialises the
CNI environment + stdin into a Request, POSTs it to the daemon's CNI server over the unix socket
and prints the daemon's Result converted to the requested cniVersion.  DEL ignores the result,
CHECK is a no-op, VERSION prints the supported versions.

Run as ``python -m dpu_operator_amd.cni.shim``.  What the daemon installs on the host is the static
native twin of this module, csrc/cni/dpu_cni.cpp (kubelet execs it outside any container).
"""
from __future__ import annotations

import json
import os
import sys

from .helper import new_cni_request, read_cni_config
from .server import post_unix
from .types import CNI_ADD, CNI_CHECK, CNI_DEL, SERVER_SOCKET_PATH, SUPPORTED_VERSIONS, CNIError


class Plugin:
    def __init__(self, socket_path: str = SERVER_SOCKET_PATH):
        self.socket_path = socket_path

    def post_request(self, env: dict, stdin: bytes) -> dict:
        req = new_cni_request(env, stdin)
        try:
            code, body = post_unix(self.socket_path, "/cni", req.to_json())
        except OSError as e:
            raise CNIError(f"failed to send CNI request: {e}", 11) from e
        if code != 200:
            raise CNIError(f"CNI request failed with status {code}: '{body.decode(errors='replace').strip()}'", 999)
        resp = json.loads(body or b"{}")
        return resp.get("Result") or {}

    def cmd_add(self, env: dict, stdin: bytes) -> dict:
        conf = read_cni_config(stdin)
        result = self.post_request(env, stdin)
        if not result:
            raise CNIError("CNI server returned no result for ADD")
        result["cniVersion"] = conf.cniVersion or result.get("cniVersion", "1.0.0")
        return result

    def cmd_del(self, env: dict, stdin: bytes) -> None:
        self.post_request(env, stdin)  # result ignored

    def cmd_check(self, env: dict, stdin: bytes) -> None:
        return None


def main(argv=None, env=None, stdin=None, stdout=None, socket_path: str | None = None) -> int:
    env = dict(os.environ if env is None else env)
    stdout = stdout or sys.stdout
    data = (stdin if stdin is not None else sys.stdin.buffer.read()) if env.get("CNI_COMMAND") != "VERSION" else b""
    p = Plugin(socket_path or env.get("DPU_CNI_SOCKET", SERVER_SOCKET_PATH))
    cmd = env.get("CNI_COMMAND", "")
    try:
        if cmd == CNI_ADD:
            stdout.write(json.dumps(p.cmd_add(env, data)))
        elif cmd == CNI_DEL:
            p.cmd_del(env, data)
        elif cmd == CNI_CHECK:
            p.cmd_check(env, data)
        elif cmd == "VERSION":
            stdout.write(json.dumps({"cniVersion": "1.0.0", "supportedVersions": SUPPORTED_VERSIONS}))
        else:
            raise CNIError(f"unknown CNI_COMMAND: {cmd}", 4)
    except CNIError as e:
        stdout.write(json.dumps(e.to_json()))
        return 1
    except ValueError as e:
        stdout.write(json.dumps(CNIError(str(e), 6).to_json()))
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
