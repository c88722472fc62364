"""In-process Kubernetes API emulation (object store + watches + admission + GC + scheduling).

The reference runs its reconcilers against a real (Kind) API server in tests
(internal/testutils/kindcluster.go:162-214) and against OpenShift/MicroShift in production.
There is no Kubernetes in this environment, so the control plane here talks to this emulation,
which implements the semantics the reference relies on:

* typed unstructured objects keyed by (kind, namespace, name); cluster- vs namespace-scoped kinds
* uid / resourceVersion / generation / creationTimestamp bookkeeping; optimistic concurrency
  (stale resourceVersion on update -> Conflict)
* watch streams (ADDED / MODIFIED / DELETED) — what controller-runtime informers consume
* validating / mutating admission hooks (the DpuOperatorConfig webhook, the NRI mutating webhook)
* ownerReference garbage collection (background cascade), which is how the reference tears down
  the daemon / VSP DaemonSets owned by the DpuOperatorConfig (render.go:75-79)
* a pod scheduler that honours nodeSelector and extended-resource requests against node
  allocatable — the "N+1 SFCs -> last one Pending" behaviour of e2e_test.go:525-592
* a DaemonSet controller that creates one pod per matching node.

`ApiServer` is thread-safe; watchers are called synchronously under no lock.
"""
from __future__ import annotations

import copy
import itertools
import threading
import time
import uuid
from collections import defaultdict
from typing import Callable

CLUSTER_SCOPED = {
    "Namespace", "Node", "DpuOperatorConfig", "ClusterRole", "ClusterRoleBinding",
    "CustomResourceDefinition", "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration",
    "ClusterVersion", "PersistentVolume",
}


class ApiError(Exception):
    code = 500
    reason = "InternalError"


class NotFound(ApiError):
    code, reason = 404, "NotFound"


class AlreadyExists(ApiError):
    code, reason = 409, "AlreadyExists"


class Conflict(ApiError):
    code, reason = 409, "Conflict"


class Forbidden(ApiError):
    code, reason = 403, "Forbidden"


class BadRequest(ApiError):
    code, reason = 400, "BadRequest"


def is_not_found(e: Exception) -> bool:
    return isinstance(e, NotFound)


def key_of(obj: dict) -> tuple[str, str, str]:
    md = obj.get("metadata") or {}
    kind = obj.get("kind", "")
    ns = "" if kind in CLUSTER_SCOPED else (md.get("namespace") or "default")
    return kind, ns, md.get("name", "")


def match_labels(labels: dict | None, selector: dict | None) -> bool:
    if not selector:
        return True
    labels = labels or {}
    return all(labels.get(k) == v for k, v in selector.items())


def parse_quantity(q) -> int:
    if isinstance(q, (int, float)):
        return int(q)
    s = str(q).strip()
    units = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40, "k": 10**3, "M": 10**6, "G": 10**9}
    for u, m in units.items():
        if s.endswith(u):
            return int(float(s[: -len(u)]) * m)
    if s.endswith("m"):
        return max(1, int(s[:-1]) // 1000)
    return int(float(s))


Watcher = Callable[[str, dict], None]
Admission = Callable[[str, dict, dict | None], object]


class ApiServer:
    def __init__(self, scheduler: bool = True, scheme=None):
        """`scheme` (api/scheme.py): when given, objects of unregistered kinds / apiVersions
        and schema violations are rejected with BadRequest, as a real API server does."""
        self.scheme = scheme
        self._lock = threading.RLock()
        self._objs: dict[tuple[str, str, str], dict] = {}
        self._rv = itertools.count(1)
        self._watchers: dict[str, list[Watcher]] = defaultdict(list)
        self._validating: dict[str, list[Admission]] = defaultdict(list)
        self._mutating: dict[str, list[Admission]] = defaultdict(list)
        self.scheduler_enabled = scheduler
        self.events: list[tuple[str, str, str, str]] = []   # (type, kind, ns/name, reason)

    # ------------------------------------------------------------------ admission / watch
    def register_validating(self, kind: str, fn: Admission) -> None:
        self._validating[kind].append(fn)

    def register_mutating(self, kind: str, fn: Admission) -> None:
        self._mutating[kind].append(fn)

    def watch(self, kind: str, fn: Watcher, replay: bool = True, namespace: str | None = None) -> Callable[[], None]:
        if namespace is not None and kind not in CLUSTER_SCOPED:
            inner = fn

            def fn(etype: str, obj: dict, _inner=inner) -> None:  # noqa: F811 - namespace-filtered watch
                if (obj.get("metadata") or {}).get("namespace", "") == namespace:
                    _inner(etype, obj)
        with self._lock:
            self._watchers[kind].append(fn)
            existing = [copy.deepcopy(o) for k, o in self._objs.items()
                        if k[0] == kind and (namespace is None or kind in CLUSTER_SCOPED or k[1] == namespace)] \
                if replay else []
        for o in existing:
            fn("ADDED", o)

        def cancel():
            with self._lock:
                if fn in self._watchers[kind]:
                    self._watchers[kind].remove(fn)

        return cancel

    def _notify(self, etype: str, obj: dict) -> None:
        for fn in list(self._watchers.get(obj["kind"], [])) + list(self._watchers.get("*", [])):
            try:
                fn(etype, copy.deepcopy(obj))
            except Exception:  # a broken watcher must not break the API server
                pass

    def _admit(self, op: str, obj: dict, old: dict | None) -> dict:
        for fn in self._mutating.get(obj["kind"], []):
            r = fn(op, obj, old)
            if isinstance(r, dict):
                obj = r
        for fn in self._validating.get(obj["kind"], []):
            try:
                fn(op, obj, old)
            except Exception as e:  # noqa: BLE001 - any validator error denies
                raise Forbidden(f'admission webhook denied the request: {e}') from e
        return obj

    def _check_scheme(self, obj: dict) -> None:
        if self.scheme is None:
            return
        try:
            self.scheme.check(obj)
        except ValueError as e:
            raise BadRequest(str(e)) from e

    # ------------------------------------------------------------------ CRUD
    def create(self, obj: dict) -> dict:
        obj = copy.deepcopy(obj)
        if "kind" not in obj or not (obj.get("metadata") or {}).get("name"):
            raise BadRequest("object needs kind and metadata.name")
        self._check_scheme(obj)
        md = obj.setdefault("metadata", {})
        if obj["kind"] not in CLUSTER_SCOPED:
            md.setdefault("namespace", "default")
        else:
            md.pop("namespace", None)
        obj = self._admit("CREATE", obj, None)
        k = key_of(obj)
        with self._lock:
            if k in self._objs:
                raise AlreadyExists(f"{k[0]} {k[1]}/{k[2]} already exists")
            md = obj["metadata"]
            md["uid"] = str(uuid.uuid4())
            md["resourceVersion"] = str(next(self._rv))
            md["generation"] = 1
            md["creationTimestamp"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
            obj.setdefault("status", obj.get("status") or {})
            self._objs[k] = obj
            out = copy.deepcopy(obj)
        self._notify("ADDED", out)
        self._after_change(out)
        return copy.deepcopy(out)

    def get(self, kind: str, name: str, namespace: str | None = None) -> dict:
        ns = "" if kind in CLUSTER_SCOPED else (namespace or "default")
        with self._lock:
            o = self._objs.get((kind, ns, name))
            if o is None:
                raise NotFound(f'{kind} "{name}" not found')
            return copy.deepcopy(o)

    def try_get(self, kind: str, name: str, namespace: str | None = None) -> dict | None:
        try:
            return self.get(kind, name, namespace)
        except NotFound:
            return None

    def list(self, kind: str, namespace: str | None = None, labels: dict | None = None) -> list[dict]:
        with self._lock:
            out = [copy.deepcopy(o) for k, o in self._objs.items()
                   if k[0] == kind and (namespace is None or k[1] == namespace)
                   and match_labels((o.get("metadata") or {}).get("labels"), labels)]
        return sorted(out, key=lambda o: (o["metadata"].get("namespace", ""), o["metadata"]["name"]))

    def update(self, obj: dict, subresource: str | None = None) -> dict:
        obj = copy.deepcopy(obj)
        self._check_scheme(obj)
        k = key_of(obj)
        with self._lock:
            cur = self._objs.get(k)
            if cur is None:
                raise NotFound(f'{k[0]} "{k[2]}" not found')
            rv = obj["metadata"].get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{k[0]} {k[2]}: the object has been modified")
            old = copy.deepcopy(cur)
        if subresource != "status":
            obj = self._admit("UPDATE", obj, old)
        with self._lock:
            cur = self._objs.get(k)
            if cur is None:
                raise NotFound(f'{k[0]} "{k[2]}" not found')
            new = copy.deepcopy(cur)
            if subresource == "status":
                new["status"] = obj.get("status") or {}
            else:
                for f in list(obj.keys()):
                    if f not in ("metadata", "status"):
                        new[f] = obj[f]
                for f in ("labels", "annotations", "ownerReferences", "finalizers"):
                    if f in obj["metadata"]:
                        new["metadata"][f] = obj["metadata"][f]
                if {k2: v for k2, v in new.items() if k2 not in ("metadata", "status")} != \
                        {k2: v for k2, v in cur.items() if k2 not in ("metadata", "status")}:
                    new["metadata"]["generation"] = cur["metadata"].get("generation", 1) + 1
                if "status" in obj and obj["status"]:
                    new["status"] = obj["status"]
            new["metadata"]["resourceVersion"] = str(next(self._rv))
            self._objs[k] = new
            out = copy.deepcopy(new)
        self._notify("MODIFIED", out)
        self._after_change(out)
        return copy.deepcopy(out)

    def update_status(self, obj: dict) -> dict:
        return self.update(obj, subresource="status")

    def apply(self, obj: dict) -> dict:
        """Create, or update the existing object's spec/labels/annotations/owners (ApplyObject)."""
        k = key_of(obj)
        with self._lock:
            cur = self._objs.get(k)
        if cur is None:
            return self.create(obj)
        merged = copy.deepcopy(cur)
        for f, v in obj.items():
            if f == "metadata":
                for mf in ("labels", "annotations", "ownerReferences"):
                    if mf in v:
                        merged["metadata"][mf] = v[mf]
            elif f != "status":
                merged[f] = v
        merged["metadata"].pop("resourceVersion", None)
        return self.update(merged)

    def delete(self, kind: str, name: str, namespace: str | None = None) -> None:
        ns = "" if kind in CLUSTER_SCOPED else (namespace or "default")
        with self._lock:
            o = self._objs.pop((kind, ns, name), None)
        if o is None:
            raise NotFound(f'{kind} "{name}" not found')
        o["metadata"]["deletionTimestamp"] = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        self._notify("DELETED", copy.deepcopy(o))
        self._gc(o["metadata"]["uid"])
        if kind == "Pod":
            self._schedule_pending()
        elif kind == "Node":
            self._schedule_pending()

    # ------------------------------------------------------------------ GC / controllers
    def _gc(self, owner_uid: str) -> None:
        with self._lock:
            deps = [o for o in self._objs.values()
                    if any(r.get("uid") == owner_uid for r in (o["metadata"].get("ownerReferences") or []))]
        for d in deps:
            try:
                self.delete(d["kind"], d["metadata"]["name"], d["metadata"].get("namespace"))
            except NotFound:
                pass

    def _after_change(self, obj: dict) -> None:
        if obj["kind"] == "DaemonSet":
            self._reconcile_daemonset(obj)
        elif obj["kind"] == "Node":
            for ds in self.list("DaemonSet"):
                self._reconcile_daemonset(ds)
            self._schedule_pending()
        elif obj["kind"] == "Pod" and self.scheduler_enabled and not obj.get("spec", {}).get("nodeName"):
            self._schedule_pending()

    def _reconcile_daemonset(self, ds: dict) -> None:
        tmpl = (ds.get("spec") or {}).get("template") or {}
        sel = (tmpl.get("spec") or {}).get("nodeSelector")
        name = ds["metadata"]["name"]
        ns = ds["metadata"].get("namespace", "default")
        want = {n["metadata"]["name"] for n in self.list("Node") if match_labels(n["metadata"].get("labels"), sel)}
        have = {p["spec"].get("nodeName"): p for p in self.list("Pod", ns)
                if any(r.get("uid") == ds["metadata"]["uid"] for r in p["metadata"].get("ownerReferences") or [])}
        for node in sorted(want - set(have)):
            pod = {
                "apiVersion": "v1", "kind": "Pod",
                "metadata": {"name": f"{name}-{node}", "namespace": ns,
                             "labels": dict((tmpl.get("metadata") or {}).get("labels") or {}),
                             "ownerReferences": [{"apiVersion": ds["apiVersion"], "kind": "DaemonSet", "name": name,
                                                  "uid": ds["metadata"]["uid"], "controller": True}]},
                "spec": dict(copy.deepcopy(tmpl.get("spec") or {}), nodeName=node),
                "status": {"phase": "Running"},
            }
            try:
                self.create(pod)
            except AlreadyExists:
                pass
        for node, pod in have.items():
            if node not in want:
                try:
                    self.delete("Pod", pod["metadata"]["name"], ns)
                except NotFound:
                    pass

    @staticmethod
    def _pod_requests(pod: dict) -> dict[str, int]:
        req: dict[str, int] = defaultdict(int)
        for c in (pod.get("spec") or {}).get("containers") or []:
            res = c.get("resources") or {}
            r = dict(res.get("limits") or {})
            r.update(res.get("requests") or {})
            for k, v in r.items():
                if "/" in k:  # extended resources only (cpu/memory are not modelled)
                    req[k] += parse_quantity(v)
        return req

    def _schedule_pending(self) -> None:
        if not self.scheduler_enabled:
            return
        for pod in self.list("Pod"):
            if pod["spec"].get("nodeName"):
                continue
            req = self._pod_requests(pod)
            placed = False
            for node in self.list("Node"):
                if (node.get("spec") or {}).get("unschedulable"):
                    continue  # cordoned (drain)
                if not match_labels(node["metadata"].get("labels"), pod["spec"].get("nodeSelector")):
                    continue
                alloc = {k: parse_quantity(v) for k, v in ((node.get("status") or {}).get("allocatable") or {}).items()}
                used: dict[str, int] = defaultdict(int)
                for p in self.list("Pod"):
                    if p["spec"].get("nodeName") == node["metadata"]["name"]:
                        for k, v in self._pod_requests(p).items():
                            used[k] += v
                if all(alloc.get(k, 0) - used[k] >= v for k, v in req.items()):
                    pod["spec"]["nodeName"] = node["metadata"]["name"]
                    pod["status"] = {"phase": "Running", "conditions": [{"type": "PodScheduled", "status": "True"}]}
                    pod["metadata"].pop("resourceVersion", None)
                    self._raw_replace(pod)
                    placed = True
                    break
            if not placed and (pod.get("status") or {}).get("phase") != "Pending":
                pod["status"] = {"phase": "Pending", "conditions": [
                    {"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                     "message": f"Insufficient resources {dict(req)}"}]}
                self._raw_replace(pod)
                self.events.append(("Warning", "Pod", f"{pod['metadata']['namespace']}/{pod['metadata']['name']}",
                                    "FailedScheduling"))

    def _raw_replace(self, obj: dict) -> None:
        k = key_of(obj)
        with self._lock:
            if k not in self._objs:
                return
            obj["metadata"]["resourceVersion"] = str(next(self._rv))
            self._objs[k] = copy.deepcopy(obj)
        self._notify("MODIFIED", copy.deepcopy(obj))


def owner_reference(owner: dict, controller: bool = True) -> dict:
    return {"apiVersion": owner["apiVersion"], "kind": owner["kind"], "name": owner["metadata"]["name"],
            "uid": owner["metadata"]["uid"], "controller": controller, "blockOwnerDeletion": True}


def set_controller_reference(owner: dict, obj: dict) -> dict:
    """controllerutil.SetControllerReference: one controller owner per object."""
    refs = [r for r in (obj.setdefault("metadata", {}).get("ownerReferences") or []) if not r.get("controller")]
    refs.append(owner_reference(owner))
    obj["metadata"]["ownerReferences"] = refs
    return obj


def make_node(name: str, labels: dict | None = None, allocatable: dict | None = None) -> dict:
    return {"apiVersion": "v1", "kind": "Node",
            "metadata": {"name": name, "labels": dict(labels or {})},
            "status": {"allocatable": dict(allocatable or {}), "capacity": dict(allocatable or {})}}
