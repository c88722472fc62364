"""In-container Kubernetes REST endpoint over the in-process ``ApiServer`` (envtest stand-in).

Serves the API paths ``k8s/rest.py`` (and any Kubernetes client) uses:

    /api/v1[/namespaces/<ns>]/<plural>[/<name>[/status]]
    /apis/<group>/<version>[/namespaces/<ns>]/<plural>[/<name>[/status]]
    /api/v1, /apis/<group>/<version>          (discovery: resources with kind + namespaced)

with the semantics of a real API server that the contract tests pin: JSON bodies, Status
objects with code / reason on errors (404 NotFound, 409 AlreadyExists / Conflict, 403, 400),
list metadata.resourceVersion, labelSelector, bearer-token auth, and
``?watch=1&resourceVersion=N`` streams of {"type", "object"} lines that resume from N (events
newer than N are replayed from a log) or answer 410 Gone when N predates the log.  Deletions get
a fresh resourceVersion like a real server's.  Used by tests/test_k8s_rest.py to run the same
contract suite against ``ApiServer`` directly and through ``RestClient``, and as a local
stand-in cluster (``python -m dpu_operator_amd.testutils.kubeapi --port 6443``).
"""
from __future__ import annotations

import argparse
import collections
import json
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ..k8s.apiserver import CLUSTER_SCOPED, ApiError, ApiServer, match_labels
from ..k8s.rest import KINDS


def _status(code: int, reason: str, msg: str) -> dict:
    return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure", "message": msg,
            "reason": reason, "code": code}


class KubeApiServer:
    def __init__(self, api: ApiServer | None = None, host: str = "127.0.0.1", port: int = 0, token: str | None = None,
                 log_size: int = 100000):
        self.api = api or ApiServer()
        self.token = token
        self.by_plural = {(av, plural): kind for kind, (av, plural) in KINDS.items()}
        self._cv = threading.Condition()
        self._log: collections.deque = collections.deque(maxlen=log_size)
        self.floor = self._max_rv()
        self.api.watch("*", self._record, replay=False)
        self.httpd = ThreadingHTTPServer((host, port), self._handler())
        self.httpd.daemon_threads = True
        self.port = self.httpd.server_address[1]
        self.url = f"http://{host}:{self.port}"
        self._t = None
        self.stopping = False

    # ------------------------------------------------------------------ event log
    def _max_rv(self) -> int:
        with self.api._lock:
            return max([int(o["metadata"]["resourceVersion"]) for o in self.api._objs.values()] + [0])

    def _record(self, etype: str, obj: dict) -> None:
        if etype == "DELETED":
            obj["metadata"]["resourceVersion"] = str(next(self.api._rv))
        with self._cv:
            self._log.append((int(obj["metadata"]["resourceVersion"]), etype, obj))
            self._cv.notify_all()

    def current_rv(self) -> int:
        with self._cv:
            last = self._log[-1][0] if self._log else 0
        return max(last, self._max_rv())

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "KubeApiServer":
        self._t = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="kubeapi")
        self._t.start()
        return self

    def stop(self) -> None:
        self.stopping = True
        with self._cv:
            self._cv.notify_all()
        self.httpd.shutdown()
        self.httpd.server_close()

    def kubeconfig(self, path: str) -> str:
        import yaml

        user = {"token": self.token} if self.token else {}
        kc = {"apiVersion": "v1", "kind": "Config", "current-context": "emu",
              "clusters": [{"name": "emu", "cluster": {"server": self.url}}],
              "users": [{"name": "emu", "user": user}],
              "contexts": [{"name": "emu", "context": {"cluster": "emu", "user": "emu", "namespace": "default"}}]}
        with open(path, "w") as f:
            yaml.safe_dump(kc, f)
        return path

    # ------------------------------------------------------------------ HTTP
    def _route(self, path: str):
        """-> (kind, namespace, name, sub, api_version) or a discovery tuple ('discovery', av)."""
        seg = [s for s in path.split("/") if s]
        if seg[:2] == ["api", "v1"]:
            av, rest = "v1", seg[2:]
        elif seg[:1] == ["apis"] and len(seg) >= 3:
            av, rest = f"{seg[1]}/{seg[2]}", seg[3:]
        else:
            return None
        if not rest:
            return ("discovery", av)
        ns = None
        if rest[0] == "namespaces" and len(rest) >= 3:
            ns, rest = rest[1], rest[2:]
        plural = rest[0]
        kind = self.by_plural.get((av, plural))
        if kind is None:
            return None
        name = rest[1] if len(rest) > 1 else None
        sub = rest[2] if len(rest) > 2 else None
        return kind, ns, name, sub, av

    def _handler(self):
        srv = self

        class H(BaseHTTPRequestHandler):
            protocol_version = "HTTP/1.0"

            def log_message(self, *a):  # quiet
                pass

            def _send(self, code: int, obj: dict) -> None:
                b = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(b)))
                self.end_headers()
                self.wfile.write(b)

            def _err(self, e: ApiError) -> None:
                self._send(e.code, _status(e.code, e.reason, str(e)))

            def _auth(self) -> bool:
                if srv.token and self.headers.get("Authorization") != f"Bearer {srv.token}":
                    self._send(401, _status(401, "Unauthorized", "Unauthorized"))
                    return False
                return True

            def _body(self) -> dict:
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n)) if n else {}

            def _parse(self):
                u = urllib.parse.urlsplit(self.path)
                q = dict(urllib.parse.parse_qsl(u.query))
                return srv._route(u.path), q

            def do_GET(self):
                if not self._auth():
                    return
                r, q = self._parse()
                if r is None:
                    return self._send(404, _status(404, "NotFound", "the server could not find the requested resource"))
                if r[0] == "discovery":
                    res = [{"name": pl, "kind": k, "namespaced": k not in CLUSTER_SCOPED}
                           for k, (av, pl) in KINDS.items() if av == r[1]]
                    return self._send(200, {"kind": "APIResourceList", "groupVersion": r[1], "resources": res})
                kind, ns, name, sub, av = r
                try:
                    if name:
                        o = srv.api.get(kind, name, ns)
                        return self._send(200, o)
                    sel = None
                    if q.get("labelSelector"):
                        sel = dict(p.split("=", 1) for p in q["labelSelector"].split(",") if "=" in p)
                    if q.get("watch") in ("1", "true"):
                        return self._watch(kind, ns, sel, int(q.get("resourceVersion") or 0),
                                           float(q.get("timeoutSeconds") or 300))
                    rv = srv.current_rv()
                    items = srv.api.list(kind, ns, sel)
                    return self._send(200, {"kind": f"{kind}List", "apiVersion": av,
                                            "metadata": {"resourceVersion": str(rv)}, "items": items})
                except ApiError as e:
                    return self._err(e)

            def _watch(self, kind, ns, sel, rv: int, timeout: float):
                self.send_response(200)
                self.send_header("Content-Type", "application/json")
                self.end_headers()

                def wanted(o):
                    md = o.get("metadata") or {}
                    return (o.get("kind") == kind and (ns is None or kind in CLUSTER_SCOPED or md.get("namespace") == ns)
                            and match_labels(md.get("labels"), sel))

                if rv and rv < srv.floor:
                    st = _status(410, "Expired", f"too old resource version: {rv} ({srv.floor})")
                    self.wfile.write(json.dumps({"type": "ERROR", "object": st}).encode() + b"\n")
                    return
                deadline = time.monotonic() + timeout
                last = rv
                while not srv.stopping and time.monotonic() < deadline:
                    with srv._cv:
                        evs = [e for e in srv._log if e[0] > last]
                        if not evs:
                            srv._cv.wait(timeout=0.5)
                            continue
                    for erv, et, o in evs:
                        last = max(last, erv)
                        if wanted(o):
                            try:
                                self.wfile.write(json.dumps({"type": et, "object": o}).encode() + b"\n")
                                self.wfile.flush()
                            except OSError:
                                return

            def do_POST(self):
                if not self._auth():
                    return
                r, _ = self._parse()
                if r is None or r[0] == "discovery":
                    return self._send(404, _status(404, "NotFound", "no such resource"))
                kind, ns, name, sub, av = r
                try:
                    obj = self._body()
                    obj.setdefault("kind", kind)
                    obj.setdefault("apiVersion", av)
                    if ns and kind not in CLUSTER_SCOPED:
                        obj.setdefault("metadata", {})["namespace"] = ns
                    self._send(201, srv.api.create(obj))
                except ApiError as e:
                    self._err(e)

            def do_PUT(self):
                if not self._auth():
                    return
                r, _ = self._parse()
                if r is None or r[0] == "discovery" or not r[2]:
                    return self._send(404, _status(404, "NotFound", "no such resource"))
                kind, ns, name, sub, av = r
                try:
                    obj = self._body()
                    obj.setdefault("kind", kind)
                    if ns and kind not in CLUSTER_SCOPED:
                        obj.setdefault("metadata", {})["namespace"] = ns
                    self._send(200, srv.api.update(obj, subresource=sub))
                except ApiError as e:
                    self._err(e)

            def do_DELETE(self):
                if not self._auth():
                    return
                r, _ = self._parse()
                if r is None or r[0] == "discovery" or not r[2]:
                    return self._send(404, _status(404, "NotFound", "no such resource"))
                kind, ns, name, sub, av = r
                try:
                    srv.api.delete(kind, name, ns)
                    self._send(200, {"kind": "Status", "apiVersion": "v1", "status": "Success", "code": 200})
                except ApiError as e:
                    self._err(e)

        return H


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(prog="kubeapi-emulator")
    ap.add_argument("--port", type=int, default=6443)
    ap.add_argument("--token", default=None)
    ap.add_argument("--kubeconfig", default="", help="write a kubeconfig for this endpoint here")
    a = ap.parse_args(argv)
    from ..api.scheme import SCHEME

    s = KubeApiServer(ApiServer(scheme=SCHEME), port=a.port, token=a.token).start()
    if a.kubeconfig:
        s.kubeconfig(a.kubeconfig)
    print(f"kube API emulator on {s.url}", flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        s.stop()


if __name__ == "__main__":
    main()
