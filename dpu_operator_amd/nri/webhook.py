"""Network Resources Injector: mutating admission that turns pod network attachments into
extended-resource requests.

Reference: cmd/nri/networkresourcesinjector.go:43-253 + the vendored
k8snetworkplumbingwg/network-resources-injector (webhook.go:252-761, controlswitches.go:28-191)
(SURVEY N1).  For a pod whose `k8s.v1.cni.cncf.io/networks` annotation names NADs (comma list
`[ns/]name[@if]` or a JSON list of selection elements), every NAD carrying a resource-name
annotation (`k8s.v1.cni.cncf.io/resourceName` by default) adds one unit of that resource to the
first container's requests and limits (or to the existing amount with honor-resources); a NAD
`k8s.v1.cni.cncf.io/nodeSelector` annotation adds a node selector; with the hugepage Downward API
switch the pod gets a `podnetinfo` volume.  Control switches come from flags and can be
overridden at run time by the `nri-control-switches` ConfigMap (`{"features": {...}}`).
The result is an RFC 6902 JSON patch in an AdmissionReview v1 response.
"""
from __future__ import annotations

import base64
import copy
import json
import logging
import re
import threading
import time

log = logging.getLogger("dpu.nri")

NETWORKS_ANNOTATION = "k8s.v1.cni.cncf.io/networks"
DEFAULT_RESOURCE_NAME_KEY = "k8s.v1.cni.cncf.io/resourceName"
NODE_SELECTOR_KEY = "k8s.v1.cni.cncf.io/nodeSelector"
CONTROL_SWITCHES_CM = "nri-control-switches"
FEATURES_KEY = "features"
HUGEPAGE_DOWNAPI = "enableHugePageDownApi"
HONOR_EXISTING = "enableHonorExistingResources"
_NAME_RE = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")


class ControlSwitches:
    def __init__(self, inject_hugepage_down_api: bool = False, honor_resources: bool = False,
                 resource_name_keys: str = DEFAULT_RESOURCE_NAME_KEY):
        self._initial = {HUGEPAGE_DOWNAPI: inject_hugepage_down_api, HONOR_EXISTING: honor_resources}
        self._active = dict(self._initial)
        self._keys_flag = resource_name_keys
        self.resource_name_keys = [k.strip() for k in resource_name_keys.split(",")]
        self._lock = threading.Lock()

    def hugepage_down_api(self) -> bool:
        return self._active[HUGEPAGE_DOWNAPI]

    def honor_existing(self) -> bool:
        return self._active[HONOR_EXISTING]

    def resource_names_enabled(self) -> bool:
        return len(self._keys_flag) > 0

    def state(self) -> str:
        return (f"HugePageInject: {str(self.hugepage_down_api()).lower()} / HonorExistingResources: "
                f"{str(self.honor_existing()).lower()} / EnableResourceNames: {str(self.resource_names_enabled()).lower()}")

    def process_configmap(self, cm: dict | None) -> None:
        """Apply `{"features": {name: bool}}` from the ConfigMap; features missing there (or a bad
        ConfigMap) fall back to their flag values."""
        with self._lock:
            self._active = dict(self._initial)
            if not cm:
                return
            raw = (cm.get("data") or {}).get(FEATURES_KEY)
            if raw is None:
                log.warning("control switches ConfigMap has no %r key", FEATURES_KEY)
                return
            try:
                feats = json.loads(raw)
            except ValueError as e:
                log.warning("control switches ConfigMap: bad JSON (%s), using initial state", e)
                return
            if not isinstance(feats, dict):
                return
            for k in self._active:
                if isinstance(feats.get(k), bool):
                    self._active[k] = feats[k]


class NadCache:
    """TTL cache of NAD annotations (the injector's netcache); `getter(ns, name)` -> NAD or None."""

    def __init__(self, getter, ttl: float = 60.0):
        self.getter = getter
        self.ttl = ttl
        self._c: dict[tuple[str, str], tuple[float, dict]] = {}

    def get(self, ns: str, name: str) -> dict | None:
        hit = self._c.get((ns, name))
        if hit and time.monotonic() - hit[0] < self.ttl:
            return hit[1]
        nad = self.getter(ns, name)
        if nad is None:
            return None
        ann = dict((nad.get("metadata") or {}).get("annotations") or {})
        self._c[(ns, name)] = (time.monotonic(), ann)
        return ann

    def invalidate(self, ns: str, name: str) -> None:
        self._c.pop((ns, name), None)


def parse_selection_element(sel: str, default_ns: str) -> dict:
    units = sel.split("/")
    if len(units) == 1:
        ns, name = default_ns, units[0]
    elif len(units) == 2:
        ns, name = units
    else:
        raise ValueError(f"invalid network selection element - more than one '/' rune in: '{sel}'")
    parts = name.split("@")
    if len(parts) > 2:
        raise ValueError(f"invalid network selection element - more than one '@' rune in: '{sel}'")
    name, iface = parts[0], parts[1] if len(parts) == 2 else ""
    for u in (ns, name, iface):
        if u and not _NAME_RE.match(u):
            raise ValueError(f"at least one of the network selection units is invalid: error found at '{u}'")
    return {"namespace": ns, "name": name, "interface": iface}


def parse_network_selections(networks: str, default_ns: str) -> list[dict] | None:
    if not networks:
        raise ValueError("empty string passed as network selection elements list")
    try:
        raw = json.loads(networks)
        if not isinstance(raw, list):
            raise ValueError
        sels = [{"namespace": e.get("namespace", ""), "name": e["name"], "interface": e.get("interface", "")}
                for e in raw]
    except (ValueError, KeyError, TypeError, AttributeError):
        sels = [parse_selection_element(s.strip(), default_ns) for s in networks.split(",")]
    for s in sels:
        if not s["namespace"]:
            if not default_ns:
                return None  # no usable namespace: the injector ignores the pod
            s["namespace"] = default_ns
    return sels


def _safe(key: str) -> str:
    return key.replace("~", "~0").replace("/", "~1")


def mutate_pod(pod: dict, nads: NadCache, switches: ControlSwitches, namespace: str = "") -> list[dict]:
    """-> JSON patch operations (empty: nothing to inject).  Raises ValueError to deny the pod."""
    meta = pod.get("metadata") or {}
    nets = (meta.get("annotations") or {}).get(NETWORKS_ANNOTATION)
    if not nets:
        return []
    ns = meta.get("namespace") or namespace
    sels = parse_network_selections(nets, ns)
    if not sels:
        return []
    reqs: dict[str, int] = {}
    node_sel: dict[str, str] = {}
    for s in sels:
        ann = nads.get(s["namespace"], s["name"])
        if ann is None:
            raise ValueError(f"could not find network attachment definition '{s['namespace']}/{s['name']}'")
        for key in switches.resource_name_keys:
            if key in ann:
                reqs[ann[key]] = reqs.get(ann[key], 0) + 1
        if NODE_SELECTOR_KEY in ann:
            kv = ann[NODE_SELECTOR_KEY].split("=")
            if len(kv) > 2:
                raise ValueError(f"node selector in net-attach-def {s['name']} has more than one label")
            node_sel[kv[0].strip()] = kv[1].strip() if len(kv) == 2 else ""
    patch: list[dict] = []
    containers = (pod.get("spec") or {}).get("containers") or []
    if reqs and containers:
        res0 = containers[0].get("resources") or {}
        requests, limits = dict(res0.get("requests") or {}), dict(res0.get("limits") or {})
        if not res0:
            patch.append({"op": "add", "path": "/spec/containers/0/resources", "value": {}})
        if not requests:
            patch.append({"op": "add", "path": "/spec/containers/0/resources/requests", "value": {}})
        if not limits:
            patch.append({"op": "add", "path": "/spec/containers/0/resources/limits", "value": {}})
        if switches.honor_existing():
            for name, n in sorted(reqs.items()):
                rq = n + int(requests.get(name, 0))
                lm = n + int(limits.get(name, 0))
                patch.append({"op": "add", "path": f"/spec/containers/0/resources/requests/{_safe(name)}", "value": str(rq)})
                patch.append({"op": "add", "path": f"/spec/containers/0/resources/limits/{_safe(name)}", "value": str(lm)})
        else:
            for name in list(reqs):
                for c in containers:
                    r = c.get("resources") or {}
                    if name in (r.get("limits") or {}) or name in (r.get("requests") or {}):
                        reqs.pop(name, None)
            for name, n in sorted(reqs.items()):
                patch.append({"op": "add", "path": f"/spec/containers/0/resources/requests/{_safe(name)}", "value": str(n)})
                patch.append({"op": "add", "path": f"/spec/containers/0/resources/limits/{_safe(name)}", "value": str(n)})
    if node_sel:
        desired = dict((pod.get("spec") or {}).get("nodeSelector") or {})
        desired.update(node_sel)
        patch.append({"op": "add", "path": "/spec/nodeSelector", "value": desired})
    if switches.hugepage_down_api() and containers:
        vols = (pod.get("spec") or {}).get("volumes")
        vol = {"name": "podnetinfo", "downwardAPI": {"items": [
            {"path": "labels", "fieldRef": {"fieldPath": "metadata.labels"}},
            {"path": "annotations", "fieldRef": {"fieldPath": "metadata.annotations"}}]}}
        patch.append({"op": "add", "path": "/spec/volumes/-" if vols else "/spec/volumes", "value": vol if vols else [vol]})
        for i, c in enumerate(containers):
            mounts = c.get("volumeMounts")
            m = {"name": "podnetinfo", "readOnly": True, "mountPath": "/etc/podnetinfo"}
            patch.append({"op": "add", "path": f"/spec/containers/{i}/volumeMounts/-" if mounts
                          else f"/spec/containers/{i}/volumeMounts", "value": m if mounts else [m]})
    return patch


def apply_patch(obj: dict, patch: list[dict]) -> dict:
    """Minimal RFC 6902 `add` application (what the API server does with the response)."""
    out = copy.deepcopy(obj)
    for op in patch:
        if op["op"] != "add":
            raise ValueError(f"unsupported patch op {op['op']}")
        parts = [p.replace("~1", "/").replace("~0", "~") for p in op["path"].split("/")[1:]]
        cur = out
        for p in parts[:-1]:
            cur = cur[int(p)] if isinstance(cur, list) else cur.setdefault(p, {})
        last = parts[-1]
        if isinstance(cur, list):
            if last == "-":
                cur.append(copy.deepcopy(op["value"]))
            else:
                cur.insert(int(last), copy.deepcopy(op["value"]))
        else:
            cur[last] = copy.deepcopy(op["value"])
    return out


def admission_response(review: dict, nads: NadCache, switches: ControlSwitches) -> dict:
    """AdmissionReview v1 request -> AdmissionReview v1 response."""
    req = review.get("request") or {}
    resp = {"uid": req.get("uid", ""), "allowed": True}
    try:
        if (req.get("kind") or {}).get("kind", "Pod") == "Pod":
            patch = mutate_pod(req.get("object") or {}, nads, switches, req.get("namespace", ""))
            if patch:
                resp["patchType"] = "JSONPatch"
                resp["patch"] = base64.b64encode(json.dumps(patch).encode()).decode()
    except ValueError as e:
        resp = {"uid": req.get("uid", ""), "allowed": False, "status": {"message": str(e), "code": 400}}
    return {"apiVersion": review.get("apiVersion", "admission.k8s.io/v1"), "kind": "AdmissionReview", "response": resp}


def api_admission_hook(api, switches: ControlSwitches | None = None):
    """Register the injector as a mutating admission hook of the in-process API server."""
    switches = switches or ControlSwitches()

    def getter(ns, name):
        return api.try_get("NetworkAttachmentDefinition", name, ns)

    nads = NadCache(getter, ttl=0.0)

    def hook(op: str, obj: dict, old: dict | None) -> dict:
        from ..k8s.apiserver import Forbidden

        if op != "CREATE":
            return obj
        try:
            patch = mutate_pod(obj, nads, switches)
        except ValueError as e:
            raise Forbidden(f"admission webhook network-resources-injector denied the request: {e}") from e
        return apply_patch(obj, patch) if patch else obj

    api.register_mutating("Pod", hook)
    return nads
