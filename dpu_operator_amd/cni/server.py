"""CNI server: HTTP/1.1 + JSON over a root-only unix socket, route POST /cni.

Reference: dpu-cni/pkgs/cniserver/cniserver.go:26-313.  Same validation as
cniRequestToPodRequest (:141-231): CNI_COMMAND, CNI_CONTAINERID, CNI_NETNS, CNI_PATH required,
CNI_IFNAME defaults to eth0, CNI_ARGS must be `k=v;...` with K8S_POD_NAMESPACE and K8S_POD_NAME
(K8S_POD_UID optional); the stdin config must parse.  ADD/DEL are dispatched to injected handlers;
any error is a 400 with the message as body; non-POST is 405.  Unlike the reference the process
environment is NOT mutated per request (the reference's os.Setenv is a cross-request race,
SURVEY.md §5): the CNI_* values are passed to handlers inside the PodRequest.
"""
from __future__ import annotations

import json
import os
import socket
import socketserver
import threading
from http.server import BaseHTTPRequestHandler
from typing import Callable

from ..utils.faults import FAULTS
from ..utils.metrics import CONTROL
from ..utils.trace import TRACER
from ..utils.paths import PathManager
from . import logging as clog
from .helper import read_cni_config
from .types import CNI_ADD, CNI_DEL, PodRequest, Request

Handler = Callable[[PodRequest], dict | None]


def gather_cni_args(env: dict) -> dict:
    if "CNI_ARGS" not in env:
        raise ValueError(f"missing CNI_ARGS: '{env}'")
    out = {}
    for arg in env["CNI_ARGS"].split(";"):
        parts = arg.split("=")
        if len(parts) != 2:
            raise ValueError(f"invalid CNI_ARG '{arg}'")
        out[parts[0].strip()] = parts[1].strip()
    return out


def cni_request_to_pod_request(cr: Request) -> PodRequest:
    env = cr.env
    if "CNI_COMMAND" not in env:
        raise ValueError("missing CNI_COMMAND")
    req = PodRequest(command=env["CNI_COMMAND"])
    for attr, key in (("container_id", "CNI_CONTAINERID"), ("netns", "CNI_NETNS")):
        if key not in env:
            raise ValueError(f"missing {key}")
        setattr(req, attr, env[key])
    req.ifname = env.get("CNI_IFNAME", "eth0")
    if "CNI_PATH" not in env:
        raise ValueError("missing CNI_PATH")
    req.path = env["CNI_PATH"]
    args = gather_cni_args(env)
    if "K8S_POD_NAMESPACE" not in args:
        raise ValueError("missing K8S_POD_NAMESPACE")
    if "K8S_POD_NAME" not in args:
        raise ValueError("missing K8S_POD_NAME")
    req.pod_namespace, req.pod_name = args["K8S_POD_NAMESPACE"], args["K8S_POD_NAME"]
    req.pod_uid = args.get("K8S_POD_UID", "")
    try:
        conf = read_cni_config(cr.config)
    except ValueError as e:
        raise ValueError("broken stdin args") from e
    req.net_name = conf.name
    req.cni_conf = conf
    req.device_info = cr.device_info
    req.cni_req = cr
    return req


class _UnixHTTPServer(socketserver.ThreadingMixIn, socketserver.UnixStreamServer):
    daemon_threads = True
    allow_reuse_address = True


class Server:
    def __init__(self, add_handler: Handler, del_handler: Handler, path_manager: PathManager | None = None,
                 socket_path: str | None = None):
        self.add_handler = add_handler
        self.del_handler = del_handler
        self.pm = path_manager or PathManager("/")
        self.socket_path = socket_path or self.pm.cni_server_path()
        self._srv: _UnixHTTPServer | None = None
        self._thread: threading.Thread | None = None
        self.requests_served = 0

    # ------------------------------------------------------------------ request handling
    def handle_cni_request(self, body: bytes) -> bytes:
        cr = Request.from_json(body)
        req = cni_request_to_pod_request(cr)
        clog.set_labels(req.net_name, req.container_id, req.netns, req.ifname)
        result = None
        FAULTS.check(f"cni.{req.command}")
        with TRACER.span(f"cni.{req.command}", pod=f"{req.pod_namespace}/{req.pod_name}", ifname=req.ifname):
            if req.command == CNI_ADD:
                result = self.add_handler(req)
            elif req.command == CNI_DEL:
                result = self.del_handler(req)
        self.requests_served += 1
        return json.dumps({"Result": result}).encode()

    def _make_handler(self):
        server = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.1"

            def log_message(self, fmt, *args):  # noqa: D401 - quiet
                return

            def address_string(self):
                return "unix"

            def _reply(self, code: int, body: bytes, ctype: str = "text/plain; charset=utf-8"):
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_POST(self):
                if self.path != "/cni":
                    return self._reply(404, b"404 page not found\n")
                n = int(self.headers.get("Content-Length", "0") or 0)
                body = self.rfile.read(n)
                cmd = "unknown"
                try:
                    cmd = (json.loads(body or b"{}").get("env") or {}).get("CNI_COMMAND", "unknown")
                except ValueError:
                    pass
                try:
                    out = server.handle_cni_request(body)
                except Exception as e:  # noqa: BLE001 - any failure is a 400 with the message
                    CONTROL.cni_requests.labels(cmd, "error").inc()
                    return self._reply(400, f"{e}\n".encode())
                CONTROL.cni_requests.labels(cmd, "success").inc()
                self._reply(200, out, "application/json")

            def _not_allowed(self):
                if self.path != "/cni":
                    return self._reply(404, b"404 page not found\n")
                self._reply(405, b"Method not allowed\n")

            do_GET = do_PUT = do_DELETE = do_PATCH = _not_allowed

        return H

    # ------------------------------------------------------------------ lifecycle
    def listen(self) -> "Server":
        PathManager.ensure_socket_dir_exists(self.socket_path)
        self._srv = _UnixHTTPServer(self.socket_path, self._make_handler(), bind_and_activate=True)
        os.chmod(self.socket_path, 0o600)
        return self

    def serve(self) -> None:
        assert self._srv is not None
        self._srv.serve_forever(poll_interval=0.05)

    def start(self) -> "Server":
        if self._srv is None:
            self.listen()
        self._thread = threading.Thread(target=self.serve, name="cni-server", daemon=True)
        self._thread.start()
        return self

    def shutdown(self) -> None:
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None
        if self._thread:
            self._thread.join(timeout=5)
        try:
            os.unlink(self.socket_path)
        except FileNotFoundError:
            pass


def post_unix(socket_path: str, path: str, body: bytes, method: str = "POST", timeout: float = 120.0) -> tuple[int, bytes]:
    """Minimal HTTP/1.1 client over a unix socket (what the shim uses)."""
    s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    s.settimeout(timeout)
    try:
        s.connect(socket_path)
        hdr = (f"{method} {path} HTTP/1.1\r\nHost: dummy\r\nContent-Type: application/json\r\n"
               f"Content-Length: {len(body)}\r\nConnection: close\r\n\r\n").encode()
        s.sendall(hdr + body)
        data = b""
        while True:
            chunk = s.recv(65536)
            if not chunk:
                break
            data += chunk
    finally:
        s.close()
    head, _, payload = data.partition(b"\r\n\r\n")
    status = int(head.split(b" ", 2)[1])
    for line in head.split(b"\r\n")[1:]:
        k, _, v = line.partition(b":")
        if k.strip().lower() == b"content-length":
            payload = payload[: int(v.strip())]
    return status, payload
