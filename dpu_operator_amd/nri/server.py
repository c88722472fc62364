"""HTTPS front end of the Network Resources Injector.

Reference: cmd/nri/networkresourcesinjector.go:43-253 and webhook/tlsutils.go — TLS >= 1.2 on
`--bind-address:--port` (8443) serving POST /mutate (other verbs 405, other paths 404), optional
client-CA verification (repeatable --client-ca, disabled with --insecure), certificate hot
reload when the key pair on disk changes (fsnotify there, mtime polling here), a plain-HTTP
/healthz on --health-check-port (8444), and the `nri-control-switches` ConfigMap re-read every
30 s into the control switches.
"""
from __future__ import annotations

import json
import logging
import os
import socket
import ssl
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .webhook import CONTROL_SWITCHES_CM, ControlSwitches, NadCache, admission_response

log = logging.getLogger("dpu.nri.server")


class KeyPairReloader:
    def __init__(self, cert: str, key: str, client_cas: list[str] | None = None, insecure: bool = False):
        self.cert, self.key = cert, key
        self.client_cas = list(client_cas or [])
        self.insecure = insecure
        self._stamp = None
        self._ctx: ssl.SSLContext | None = None
        self._lock = threading.Lock()
        self.reloads = 0

    def _mtimes(self):
        return tuple(os.stat(p).st_mtime_ns for p in (self.cert, self.key))

    def context(self) -> ssl.SSLContext:
        with self._lock:
            stamp = self._mtimes()
            if self._ctx is None or stamp != self._stamp:
                ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
                ctx.minimum_version = ssl.TLSVersion.TLSv1_2
                ctx.load_cert_chain(self.cert, self.key)
                if self.client_cas and not self.insecure:
                    for ca in self.client_cas:
                        ctx.load_verify_locations(ca)
                    ctx.verify_mode = ssl.CERT_REQUIRED
                self._ctx, self._stamp = ctx, stamp
                self.reloads += 1
                log.info("loaded TLS key pair %s (reload #%d)", self.cert, self.reloads)
            return self._ctx


class _TLSServer(ThreadingHTTPServer):
    daemon_threads = True

    def __init__(self, addr, handler, reloader: KeyPairReloader):
        self.reloader = reloader
        super().__init__(addr, handler)

    def get_request(self):
        sock, addr = super().get_request()
        sock.settimeout(10)
        try:
            # the handshake runs on the handler thread (first read), not on the accept loop
            return self.reloader.context().wrap_socket(sock, server_side=True, do_handshake_on_connect=False), addr
        except (ssl.SSLError, OSError):
            sock.close()
            raise


class InjectorServer:
    def __init__(self, nads: NadCache, switches: ControlSwitches, reloader: KeyPairReloader | None,
                 address: str = "0.0.0.0", port: int = 8443, health_port: int = 8444, api=None,
                 namespace: str = "openshift-dpu-operator", cm_poll: float = 30.0):
        self.nads, self.switches = nads, switches
        self.reloader = reloader
        self.address, self.port, self.health_port = address, port, health_port
        self.api, self.namespace, self.cm_poll = api, namespace, cm_poll
        self._srv = None
        self._health = None
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.requests = 0

    def _handler(self):
        outer = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, fmt, *args):
                log.debug(fmt, *args)

            def _send(self, code, body: bytes, ctype="application/json"):
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def do_POST(self):
                if self.path != "/mutate":
                    return self._send(404, b"404 page not found\n", "text/plain")
                if self.headers.get("Content-Type", "") != "application/json":
                    return self._send(400, b"invalid Content-Type, expected application/json\n", "text/plain")
                n = int(self.headers.get("Content-Length", "0") or 0)
                try:
                    review = json.loads(self.rfile.read(n) or b"{}")
                except ValueError as e:
                    return self._send(400, f"error deserializing AdmissionReview: {e}\n".encode(), "text/plain")
                outer.requests += 1
                self._send(200, json.dumps(admission_response(review, outer.nads, outer.switches)).encode())

            def do_GET(self):
                if self.path == "/mutate":
                    return self._send(405, b"Invalid HTTP verb requested\n", "text/plain")
                self._send(404, b"404 page not found\n", "text/plain")

            do_PUT = do_DELETE = do_GET

        return H

    def _health_handler(self):
        class H(BaseHTTPRequestHandler):
            def log_message(self, fmt, *args):
                pass

            def do_GET(self):
                code = 200 if self.path == "/healthz" else 404
                self.send_response(code)
                self.send_header("Content-Length", "0")
                self.end_headers()

        return H

    def _poll_switches(self) -> None:
        while not self._stop.wait(self.cm_poll):
            self.refresh_switches()

    def refresh_switches(self) -> None:
        if self.api is None:
            return
        cm = self.api.try_get("ConfigMap", CONTROL_SWITCHES_CM, self.namespace)
        self.switches.process_configmap(cm)

    def start(self) -> "InjectorServer":
        if self.reloader is None:
            raise ValueError("TLS key pair required")
        self._srv = _TLSServer((self.address, self.port), self._handler(), self.reloader)
        self.port = self._srv.server_address[1]
        self._health = ThreadingHTTPServer((self.address, self.health_port), self._health_handler())
        self._health.daemon_threads = True
        self.health_port = self._health.server_address[1]
        self.refresh_switches()
        for target in (self._srv.serve_forever, self._health.serve_forever, self._poll_switches):
            t = threading.Thread(target=target, daemon=True)
            t.start()
            self._threads.append(t)
        return self

    def stop(self) -> None:
        self._stop.set()
        for s in (self._srv, self._health):
            if s is not None:
                s.shutdown()
                s.server_close()


def valid_port(p: int) -> bool:
    return 1024 <= p <= 65535


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p
