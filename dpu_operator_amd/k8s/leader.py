"""Lease-based leader election (controller-runtime's --leader-elect, cmd/main.go:53-85).

A `coordination.k8s.io/v1` Lease named by the election id holds `holderIdentity`,
`leaseDurationSeconds`, `acquireTime`, `renewTime`, `leaseTransitions`.  A candidate acquires a
missing or expired lease and renews it every `renew` seconds; writes use the API server's
optimistic concurrency, so two candidates racing for one lease cannot both win (the loser sees
Conflict / AlreadyExists).  `on_started` / `on_stopped` fire on gaining / losing leadership.

Failure handling follows controller-runtime's renew deadline: a leader that fails to renew
(Conflict, transport or API errors alike) keeps leadership only until `renew_deadline` seconds
after its last successful renew, which is shorter than the lease duration, so it steps down
before another candidate can take the expired lease.  No exception ever ends the election loop.
"""
from __future__ import annotations

import logging
import threading
import time

from .apiserver import AlreadyExists, ApiServer, Conflict, NotFound

log = logging.getLogger("dpu.leader")


def _now() -> float:
    return time.time()


class LeaderElector:
    def __init__(self, api: ApiServer, lease_name: str, namespace: str, identity: str,
                 lease_duration: float = 15.0, renew: float = 2.0, on_started=None, on_stopped=None,
                 release_on_cancel: bool = True, renew_deadline: float | None = None):
        self.api = api
        self.name, self.ns, self.identity = lease_name, namespace, identity
        self.duration, self.renew = lease_duration, renew
        self.on_started, self.on_stopped = on_started, on_stopped
        self.release_on_cancel = release_on_cancel
        # controller-runtime defaults: lease 15 s, renew deadline 10 s, retry period 2 s
        self.renew_deadline = renew_deadline if renew_deadline is not None else lease_duration * 2 / 3
        if not renew < self.renew_deadline < lease_duration:
            raise ValueError("need renew period < renew deadline < lease duration")
        self.leader = False
        self.errors = 0
        self._last_renew = 0.0
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

    def _tick(self) -> None:
        try:
            ok = self.try_acquire_or_renew()
        except Exception as e:  # noqa: BLE001 - API/transport failure counts as a failed renew
            self.errors += 1
            log.warning("leader election %s/%s: renew failed: %s", self.ns, self.name, e)
            ok = False
        now = time.monotonic()
        if ok:
            self._last_renew = now
            self._set(True)
        elif not self.leader or now - self._last_renew >= self.renew_deadline:
            self._set(False)

    def _run(self) -> None:
        while not self._stop.is_set():
            self._tick()
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
            except Exception:  # noqa: BLE001 - best effort: the lease expires on its own
                pass
        self._set(False)
