"""Lease-based leader election (controller-runtime's --leader-elect, cmd/main.go:53-85).

A `coordination.k8s.io/v1` Lease named by the election id holds `holderIdentity`,
`leaseDurationSeconds`, `acquireTime`, `renewTime`, `leaseTransitions`.  A candidate acquires a
missing or expired lease and renews it every `renew` seconds; writes use the API server's
optimistic concurrency, so two candidates racing for one lease cannot both win (the loser sees
Conflict / AlreadyExists).  `on_started` / `on_stopped` fire on gaining / losing leadership.
"""
from __future__ import annotations

import threading
import time

from .apiserver import AlreadyExists, ApiServer, Conflict, NotFound


def _now() -> float:
    return time.time()


class LeaderElector:
    def __init__(self, api: ApiServer, lease_name: str, namespace: str, identity: str,
                 lease_duration: float = 15.0, renew: float = 2.0, on_started=None, on_stopped=None,
                 release_on_cancel: bool = True):
        self.api = api
        self.name, self.ns, self.identity = lease_name, namespace, identity
        self.duration, self.renew = lease_duration, renew
        self.on_started, self.on_stopped = on_started, on_stopped
        self.release_on_cancel = release_on_cancel
        self.leader = False
        self._stop = threading.Event()
        self._t: threading.Thread | None = None

    def _lease(self) -> dict:
        return {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                "metadata": {"name": self.name, "namespace": self.ns},
                "spec": {"holderIdentity": self.identity, "leaseDurationSeconds": self.duration,
                         "acquireTime": _now(), "renewTime": _now(), "leaseTransitions": 0}}

    def try_acquire_or_renew(self) -> bool:
        try:
            cur = self.api.get("Lease", self.name, self.ns)
        except NotFound:
            try:
                self.api.create(self._lease())
                return True
            except AlreadyExists:
                return False
        spec = cur.setdefault("spec", {})
        holder = spec.get("holderIdentity")
        expired = _now() > float(spec.get("renewTime", 0)) + float(spec.get("leaseDurationSeconds", self.duration))
        if holder != self.identity and holder and not expired:
            return False
        if holder != self.identity:
            spec["leaseTransitions"] = int(spec.get("leaseTransitions", 0)) + 1
            spec["acquireTime"] = _now()
            spec["holderIdentity"] = self.identity
        spec["renewTime"] = _now()
        spec["leaseDurationSeconds"] = self.duration
        try:
            self.api.update(cur)
            return True
        except (Conflict, NotFound):
            return False

    def _set(self, leader: bool) -> None:
        if leader and not self.leader:
            self.leader = True
            if self.on_started:
                self.on_started()
        elif not leader and self.leader:
            self.leader = False
            if self.on_stopped:
                self.on_stopped()

    def _run(self) -> None:
        while not self._stop.is_set():
            self._set(self.try_acquire_or_renew())
            self._stop.wait(self.renew)

    def start(self) -> "LeaderElector":
        self._t = threading.Thread(target=self._run, daemon=True, name=f"leader-{self.identity}")
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=5)
        if self.leader and self.release_on_cancel:
            try:
                cur = self.api.get("Lease", self.name, self.ns)
                if cur["spec"].get("holderIdentity") == self.identity:
                    cur["spec"]["holderIdentity"] = ""
                    self.api.update(cur)
            except (Conflict, NotFound):
                pass
        self._set(False)
