"""Node drain helper.

Reference: pkgs/drain/drain.go:15-43 wraps the sriov-network-operator drainer (SURVEY D1;
tested, not wired into a runtime path).  Same two calls here, implemented on the API:
* drain_node(node, force): cordon (spec.unschedulable = true), then evict the node's pods —
  DaemonSet-managed and mirror (static) pods stay; pods without a controller are evicted only
  with `force` (kubectl drain semantics); returns True when the node holds no evictable pods.
* complete_drain_node(node): uncordon; pods Pending on the node's resources can schedule again.
An optional `on_drain(node)` / `on_complete(node)` hook lets the GPU data plane quiesce (stop
admitting new flows, harvest counters) around the drain.
"""
from __future__ import annotations

import logging

from .k8s.apiserver import ApiServer, NotFound

log = logging.getLogger("dpu.drain")

MIRROR_POD_ANNOTATION = "kubernetes.io/config.mirror"


class Drainer:
    def __init__(self, api: ApiServer, on_drain=None, on_complete=None):
        self.api = api
        self.on_drain = on_drain
        self.on_complete = on_complete

    def _set_unschedulable(self, name: str, value: bool) -> None:
        node = self.api.get("Node", name)
        spec = node.setdefault("spec", {})
        if bool(spec.get("unschedulable")) != value:
            spec["unschedulable"] = value
            self.api.update(node)

    @staticmethod
    def _controller(pod: dict) -> dict | None:
        for r in pod["metadata"].get("ownerReferences") or []:
            if r.get("controller"):
                return r
        return None

    def evictable(self, pod: dict, force: bool) -> bool:
        if MIRROR_POD_ANNOTATION in (pod["metadata"].get("annotations") or {}):
            return False
        ctl = self._controller(pod)
        if ctl is not None and ctl.get("kind") == "DaemonSet":
            return False
        return ctl is not None or force

    def drain_node(self, node: dict | str, force: bool = False) -> bool:
        name = node if isinstance(node, str) else node["metadata"]["name"]
        self._set_unschedulable(name, True)
        if self.on_drain:
            self.on_drain(name)
        blocked = 0
        for p in self.api.list("Pod"):
            if (p.get("spec") or {}).get("nodeName") != name:
                continue
            if not self.evictable(p, force):
                ctl = self._controller(p)
                if ctl is None or ctl.get("kind") != "DaemonSet":
                    if MIRROR_POD_ANNOTATION not in (p["metadata"].get("annotations") or {}):
                        blocked += 1
                continue
            try:
                self.api.delete("Pod", p["metadata"]["name"], p["metadata"].get("namespace"))
                log.info("evicted %s/%s from %s", p["metadata"].get("namespace"), p["metadata"]["name"], name)
            except NotFound:
                pass
        return blocked == 0

    def complete_drain_node(self, node: dict | str) -> bool:
        name = node if isinstance(node, str) else node["metadata"]["name"]
        self._set_unschedulable(name, False)
        if self.on_complete:
            self.on_complete(name)
        return True
