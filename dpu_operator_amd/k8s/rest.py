"""Kubernetes REST client with the surface of the in-process ``ApiServer``.

The reference builds a controller-runtime manager against the cluster (cmd/main.go:64-86) and
the daemon watches Pods and ServiceFunctionChains through it (hostsidemanager.go:320-346,
dpusidemanager.go:256-292).  ``RestClient`` gives the operator, the daemon, the SFC reconciler,
the leader elector and ``render`` the same calls they make on ``k8s/apiserver.py`` -
get / try_get / list / create / update / update_status / apply / delete / watch - but over the
Kubernetes HTTP API:

* config: in-cluster (service-account token + CA, ``KUBERNETES_SERVICE_HOST/PORT``) or a
  kubeconfig (server, CA / insecure-skip-tls-verify, bearer token or client certificate);
* kinds map to REST paths through a static table of the kinds this framework touches, plus API
  discovery (``/apis/<group>/<version>``) for anything else that carries an apiVersion;
* errors map to the same exceptions (404 NotFound, 409 AlreadyExists / Conflict, 403 Forbidden,
  400 / 422 BadRequest); optimistic concurrency through metadata.resourceVersion;
* watch = list (replayed as ADDED) + a streaming ``?watch=1&resourceVersion=`` request per kind
  on a thread, resumed from the last resourceVersion after a dropped connection and re-listed
  after 410 Gone, like a client-go reflector.

Admission hooks are server-side in a real cluster (the webhooks in config/webhook and the NRI
deployment), so ``register_validating`` / ``register_mutating`` only record the hook.
"""
from __future__ import annotations

import base64
import copy
import http.client
import json
import logging
import os
import ssl
import tempfile
import threading
import time
import urllib.parse
from dataclasses import dataclass, field
from typing import Callable

import yaml

from .apiserver import CLUSTER_SCOPED, AlreadyExists, ApiError, BadRequest, Conflict, Forbidden, NotFound

log = logging.getLogger("dpu.k8s.rest")

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

# kind -> (apiVersion, plural); scope from CLUSTER_SCOPED
KINDS: dict[str, tuple[str, str]] = {
    "Pod": ("v1", "pods"), "Node": ("v1", "nodes"), "Namespace": ("v1", "namespaces"),
    "ConfigMap": ("v1", "configmaps"), "Secret": ("v1", "secrets"), "Service": ("v1", "services"),
    "ServiceAccount": ("v1", "serviceaccounts"), "Event": ("v1", "events"),
    "PersistentVolume": ("v1", "persistentvolumes"),
    "DaemonSet": ("apps/v1", "daemonsets"), "Deployment": ("apps/v1", "deployments"),
    "Lease": ("coordination.k8s.io/v1", "leases"),
    "Role": ("rbac.authorization.k8s.io/v1", "roles"),
    "RoleBinding": ("rbac.authorization.k8s.io/v1", "rolebindings"),
    "ClusterRole": ("rbac.authorization.k8s.io/v1", "clusterroles"),
    "ClusterRoleBinding": ("rbac.authorization.k8s.io/v1", "clusterrolebindings"),
    "CustomResourceDefinition": ("apiextensions.k8s.io/v1", "customresourcedefinitions"),
    "MutatingWebhookConfiguration": ("admissionregistration.k8s.io/v1", "mutatingwebhookconfigurations"),
    "ValidatingWebhookConfiguration": ("admissionregistration.k8s.io/v1", "validatingwebhookconfigurations"),
    "NetworkAttachmentDefinition": ("k8s.cni.cncf.io/v1", "network-attachment-definitions"),
    "DpuOperatorConfig": ("config.openshift.io/v1", "dpuoperatorconfigs"),
    "ServiceFunctionChain": ("config.openshift.io/v1", "servicefunctionchains"),
    "ClusterVersion": ("config.openshift.io/v1", "clusterversions"),
}


@dataclass
class ClusterConfig:
    server: str                        # https://host:port
    token: str | None = None
    ca_file: str | None = None
    insecure: bool = False
    cert_file: str | None = None
    key_file: str | None = None
    namespace: str = "default"
    _tmp: list = field(default_factory=list, repr=False)

    @staticmethod
    def in_cluster() -> "ClusterConfig | None":
        host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
        tok = os.path.join(SA_DIR, "token")
        if not host or not port or not os.path.exists(tok):
            return None
        if ":" in host and not host.startswith("["):
            host = f"[{host}]"
        ns_file = os.path.join(SA_DIR, "namespace")
        return ClusterConfig(server=f"https://{host}:{port}", token=open(tok).read().strip(),
                             ca_file=os.path.join(SA_DIR, "ca.crt"),
                             namespace=open(ns_file).read().strip() if os.path.exists(ns_file) else "default")

    @staticmethod
    def from_kubeconfig(path: str, context: str | None = None) -> "ClusterConfig":
        with open(path) as f:
            kc = yaml.safe_load(f) or {}
        ctx_name = context or kc.get("current-context")
        ctxs = {c["name"]: c.get("context") or {} for c in kc.get("contexts") or []}
        if ctx_name not in ctxs:
            raise ValueError(f"kubeconfig {path}: context {ctx_name!r} not found")
        ctx = ctxs[ctx_name]
        cluster = {c["name"]: c.get("cluster") or {} for c in kc.get("clusters") or []}.get(ctx.get("cluster"))
        user = {u["name"]: u.get("user") or {} for u in kc.get("users") or []}.get(ctx.get("user"), {})
        if not cluster or "server" not in cluster:
            raise ValueError(f"kubeconfig {path}: cluster of context {ctx_name!r} has no server")
        cfg = ClusterConfig(server=cluster["server"].rstrip("/"), namespace=ctx.get("namespace") or "default",
                            insecure=bool(cluster.get("insecure-skip-tls-verify")))
        base = os.path.dirname(os.path.abspath(path))

        def file_or_data(k: str, src: dict) -> str | None:
            if src.get(k + "-data"):
                t = tempfile.NamedTemporaryFile("wb", delete=False, prefix="kc-", suffix=".pem")
                t.write(base64.b64decode(src[k + "-data"]))
                t.close()
                cfg._tmp.append(t.name)
                return t.name
            v = src.get(k)
            return None if not v else (v if os.path.isabs(v) else os.path.join(base, v))

        cfg.ca_file = file_or_data("certificate-authority", cluster)
        cfg.cert_file = file_or_data("client-certificate", user)
        cfg.key_file = file_or_data("client-key", user)
        if user.get("token"):
            cfg.token = user["token"]
        elif user.get("tokenFile"):
            cfg.token = open(user["tokenFile"]).read().strip()
        return cfg

    @staticmethod
    def discover(kubeconfig: str | None = None) -> "ClusterConfig | None":
        """--kubeconfig, then $KUBECONFIG, then in-cluster; None when there is no cluster."""
        path = kubeconfig or os.environ.get("KUBECONFIG")
        if path:
            return ClusterConfig.from_kubeconfig(path)
        return ClusterConfig.in_cluster()


def _raise_for(status: int, body: bytes) -> None:
    try:
        st = json.loads(body or b"{}")
    except ValueError:
        st = {}
    msg = st.get("message") or body[:300].decode(errors="replace")
    reason = st.get("reason", "")
    if status == 404:
        raise NotFound(msg)
    if status == 409:
        raise AlreadyExists(msg) if reason == "AlreadyExists" else Conflict(msg)
    if status in (401, 403):
        raise Forbidden(msg)
    if status in (400, 422):
        raise BadRequest(msg)
    e = ApiError(msg)
    e.code = status
    raise e


class RestClient:
    """HTTP client for the Kubernetes API with the ApiServer call surface."""

    def __init__(self, cfg: ClusterConfig, timeout: float = 30.0):
        self.cfg = cfg
        self.timeout = timeout
        u = urllib.parse.urlsplit(cfg.server)
        self.https = u.scheme == "https"
        self.host = u.hostname
        self.port = u.port or (443 if self.https else 80)
        self.prefix = u.path.rstrip("/")
        self._ssl = None
        if self.https:
            ctx = ssl.create_default_context(cafile=cfg.ca_file) if cfg.ca_file else ssl.create_default_context()
            if cfg.insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            if cfg.cert_file:
                ctx.load_cert_chain(cfg.cert_file, cfg.key_file)
            self._ssl = ctx
        self._kinds = dict(KINDS)
        self._lock = threading.Lock()
        self._watches: list["_Watch"] = []
        self.events: list = []
        self.admission: dict[str, list] = {}

    # ------------------------------------------------------------------ transport
    def _conn(self, timeout: float | None = None):
        t = self.timeout if timeout is None else timeout
        if self.https:
            return http.client.HTTPSConnection(self.host, self.port, context=self._ssl, timeout=t)
        return http.client.HTTPConnection(self.host, self.port, timeout=t)

    def _headers(self, body: bool = False) -> dict:
        h = {"Accept": "application/json", "User-Agent": "dpu-operator-amd"}
        if body:
            h["Content-Type"] = "application/json"
        if self.cfg.token:
            h["Authorization"] = f"Bearer {self.cfg.token}"
        return h

    def request(self, method: str, path: str, body: dict | None = None, query: dict | None = None) -> dict:
        q = ("?" + urllib.parse.urlencode(query)) if query else ""
        c = self._conn()
        try:
            data = json.dumps(body).encode() if body is not None else None
            c.request(method, self.prefix + path + q, body=data, headers=self._headers(data is not None))
            r = c.getresponse()
            raw = r.read()
            if r.status >= 300:
                _raise_for(r.status, raw)
            return json.loads(raw) if raw else {}
        finally:
            c.close()

    # ------------------------------------------------------------------ paths
    def _kind(self, kind: str, api_version: str | None = None) -> tuple[str, str]:
        with self._lock:
            hit = self._kinds.get(kind)
        if hit:
            return hit
        if not api_version:
            raise BadRequest(f"unknown kind {kind!r} (no apiVersion to discover it with)")
        base = "/api/v1" if api_version == "v1" else f"/apis/{api_version}"
        for res in self.request("GET", base).get("resources", []):
            if res.get("kind") == kind and "/" not in res.get("name", ""):
                with self._lock:
                    self._kinds[kind] = (api_version, res["name"])
                return api_version, res["name"]
        raise BadRequest(f"kind {kind!r} not served by {api_version}")

    def path(self, kind: str, name: str | None = None, namespace: str | None = None, api_version: str | None = None,
             sub: str | None = None, all_namespaces: bool = False) -> str:
        av, plural = self._kind(kind, api_version)
        base = "/api/v1" if av == "v1" else f"/apis/{av}"
        p = base
        if kind not in CLUSTER_SCOPED and not all_namespaces:
            p += f"/namespaces/{namespace or 'default'}"
        p += f"/{plural}"
        if name:
            p += f"/{name}"
        if sub:
            p += f"/{sub}"
        return p

    @staticmethod
    def _obj_path_args(obj: dict) -> dict:
        md = obj.get("metadata") or {}
        return dict(name=md.get("name"), namespace=md.get("namespace"), api_version=obj.get("apiVersion"))

    # ------------------------------------------------------------------ CRUD (ApiServer surface)
    def create(self, obj: dict) -> dict:
        if "kind" not in obj or not (obj.get("metadata") or {}).get("name"):
            raise BadRequest("object needs kind and metadata.name")
        a = self._obj_path_args(obj)
        if obj["kind"] in CLUSTER_SCOPED:
            obj = copy.deepcopy(obj)
            obj["metadata"].pop("namespace", None)
        return self.request("POST", self.path(obj["kind"], None, a["namespace"], a["api_version"]), obj)

    def get(self, kind: str, name: str, namespace: str | None = None) -> dict:
        o = self.request("GET", self.path(kind, name, namespace))
        o.setdefault("kind", kind)
        return o

    def try_get(self, kind: str, name: str, namespace: str | None = None) -> dict | None:
        try:
            return self.get(kind, name, namespace)
        except NotFound:
            return None

    def _list_raw(self, kind: str, namespace: str | None = None, labels: dict | None = None) -> dict:
        q = {}
        if labels:
            q["labelSelector"] = ",".join(f"{k}={v}" for k, v in sorted(labels.items()))
        return self.request("GET", self.path(kind, None, namespace, all_namespaces=namespace is None), query=q)

    def list(self, kind: str, namespace: str | None = None, labels: dict | None = None) -> list[dict]:
        items = self._list_raw(kind, namespace, labels).get("items", [])
        av = KINDS.get(kind, (None,))[0]
        for o in items:  # list items omit kind/apiVersion on real servers
            o.setdefault("kind", kind)
            if av:
                o.setdefault("apiVersion", av)
        return sorted(items, key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))

    def update(self, obj: dict, subresource: str | None = None) -> dict:
        a = self._obj_path_args(obj)
        return self.request("PUT", self.path(obj["kind"], a["name"], a["namespace"], a["api_version"], sub=subresource),
                            obj)

    def update_status(self, obj: dict) -> dict:
        return self.update(obj, subresource="status")

    def apply(self, obj: dict) -> dict:
        """Create, or update the live object's spec / labels / annotations / owners (render's
        ApplyObject semantics); retried on a resourceVersion conflict."""
        for _ in range(5):
            a = self._obj_path_args(obj)
            cur = self.try_get(obj["kind"], a["name"], a["namespace"])
            if cur is None:
                try:
                    return self.create(obj)
                except AlreadyExists:
                    continue
            merged = copy.deepcopy(cur)
            for f, v in obj.items():
                if f == "metadata":
                    for mf in ("labels", "annotations", "ownerReferences"):
                        if mf in v:
                            merged["metadata"][mf] = v[mf]
                elif f != "status":
                    merged[f] = v
            try:
                return self.update(merged)
            except Conflict:
                continue
        raise Conflict(f"apply {obj['kind']} {obj['metadata']['name']}: persistent conflict")

    def delete(self, kind: str, name: str, namespace: str | None = None) -> None:
        self.request("DELETE", self.path(kind, name, namespace), {"kind": "DeleteOptions", "apiVersion": "v1",
                                                                  "propagationPolicy": "Background"})

    # ------------------------------------------------------------------ admission (server-side here)
    def register_validating(self, kind: str, fn) -> None:
        self.admission.setdefault(kind, []).append(fn)
        log.info("admission for %s runs in the cluster's webhook, not in this client", kind)

    register_mutating = register_validating

    # ------------------------------------------------------------------ watch
    def watch(self, kind: str, fn: Callable[[str, dict], None], replay: bool = True,
              namespace: str | None = None) -> Callable[[], None]:
        w = _Watch(self, kind, fn, replay, namespace)
        with self._lock:
            self._watches.append(w)
        w.start()
        w.ready.wait(self.timeout)

        def cancel():
            w.stop()
            with self._lock:
                if w in self._watches:
                    self._watches.remove(w)

        return cancel

    def close(self) -> None:
        for w in list(self._watches):
            w.stop()
        for f in self.cfg._tmp:
            try:
                os.unlink(f)
            except OSError:
                pass


class _Watch:
    """One reflector: list (+ ADDED replay), then stream ?watch=1 from the list's
    resourceVersion; resume from the last seen version, re-list on 410 Gone."""

    def __init__(self, client: RestClient, kind: str, fn, replay: bool, namespace: str | None):
        self.c, self.kind, self.fn, self.replay, self.ns = client, kind, fn, replay, namespace
        self.rv: str | None = None
        self.known: dict[tuple[str, str], dict] = {}   # last state of every object the handler saw
        self._stop = threading.Event()
        self.ready = threading.Event()
        self._sock = None
        self._t = threading.Thread(target=self._run, daemon=True, name=f"watch-{kind}")

    def start(self) -> None:
        self._t.start()

    def stop(self) -> None:
        self._stop.set()
        sk = self._sock  # the stream's socket (the response owns it once headers are read)
        if sk is not None:
            try:
                sk.shutdown(2)
            except OSError:
                pass
        self._t.join(timeout=5)

    def _emit(self, etype: str, obj: dict) -> None:
        obj.setdefault("kind", self.kind)
        try:
            self.fn(etype, obj)
        except Exception:  # a broken handler must not kill the reflector
            log.exception("watch handler for %s failed", self.kind)

    @staticmethod
    def _key(obj: dict) -> tuple[str, str]:
        md = obj.get("metadata") or {}
        return md.get("namespace") or "", md.get("name") or ""

    def _track(self, etype: str, obj: dict) -> None:
        if etype == "DELETED":
            self.known.pop(self._key(obj), None)
        elif etype in ("ADDED", "MODIFIED"):
            self.known[self._key(obj)] = obj

    def _list(self, first: bool) -> None:
        """List, then reconcile the handler's view with it (a reflector's Replace): on a re-list
        after a 410 / expired watch, objects that vanished during the gap produce DELETED (with
        their last known state), objects already known MODIFIED, new ones ADDED."""
        lst = self.c._list_raw(self.kind, self.ns)
        self.rv = (lst.get("metadata") or {}).get("resourceVersion")
        items = lst.get("items", [])
        if first:
            for o in items:
                self._track("ADDED", o)
                if self.replay:
                    self._emit("ADDED", o)
            return
        now = {self._key(o): o for o in items}
        for k in [k for k in self.known if k not in now]:
            gone = self.known.pop(k)
            self._emit("DELETED", gone)
        for k, o in now.items():
            t = "MODIFIED" if k in self.known else "ADDED"
            self.known[k] = o
            self._emit(t, o)

    def _run(self) -> None:
        backoff = 0.05
        first = True
        while not self._stop.is_set():
            try:
                if self.rv is None:
                    self._list(first)
                    first = False
                    self.ready.set()
                self._stream()
                backoff = 0.05
            except Exception as e:  # noqa: BLE001 - keep watching through transport errors
                if self._stop.is_set():
                    break
                log.debug("watch %s: %s; retrying", self.kind, e)
                self.ready.set()
                time.sleep(backoff)
                backoff = min(backoff * 2, 5.0)

    def _stream(self) -> None:
        q = {"watch": "1", "resourceVersion": self.rv or "0", "allowWatchBookmarks": "true", "timeoutSeconds": "300"}
        path = self.c.path(self.kind, None, self.ns, all_namespaces=self.ns is None)
        conn = self.c._conn(timeout=330)
        try:
            conn.connect()
            self._sock = conn.sock
            if self._stop.is_set():
                return
            conn.request("GET", self.c.prefix + path + "?" + urllib.parse.urlencode(q), headers=self.c._headers())
            r = conn.getresponse()
            if r.status == 410:
                self.rv = None
                return
            if r.status >= 300:
                _raise_for(r.status, r.read())
            while not self._stop.is_set():
                line = r.readline()
                if not line:
                    return  # server closed the stream: resume from self.rv
                line = line.strip()
                if not line:
                    continue
                ev = json.loads(line)
                t, obj = ev.get("type"), ev.get("object") or {}
                if t == "ERROR":
                    if obj.get("code") == 410:
                        self.rv = None  # too old: re-list
                    return
                rv = (obj.get("metadata") or {}).get("resourceVersion")
                if rv:
                    self.rv = rv
                if t == "BOOKMARK" or self._stop.is_set():
                    continue
                self._track(t, obj)
                self._emit(t, obj)
        finally:
            self._sock = None
            conn.close()


def connect(kubeconfig: str | None = None) -> RestClient | None:
    """A RestClient for the cluster this process runs in / points at, or None without one."""
    cfg = ClusterConfig.discover(kubeconfig)
    return RestClient(cfg) if cfg else None
