"""Minimal controller-runtime: watches -> work queue -> Reconcile(request) -> Result.

Semantics kept from controller-runtime (as used by the reference's reconcilers,
internal/controller/dpuoperatorconfig_controller.go:207-211, internal/daemon/sfc-reconciler/sfc.go:139-144):
requests are de-duplicated NamespacedNames; an error or ``Result(requeue=True)`` re-enqueues with
exponential backoff; ``requeue_after`` schedules a delayed retry; owned-object events map to the
controller owner's request.  The manager can run in a background thread (``start``) or be stepped
deterministically (``drain``) by tests.
"""
from __future__ import annotations

import heapq
import logging
import threading
import time
from dataclasses import dataclass
from typing import Callable, Protocol

from .apiserver import ApiServer
from ..utils.metrics import CONTROL

log = logging.getLogger("dpu.manager")


@dataclass(frozen=True)
class Request:
    namespace: str
    name: str


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0


class Reconciler(Protocol):
    def reconcile(self, req: Request) -> Result: ...


@dataclass
class _Ctl:
    name: str
    rec: Reconciler
    kind: str
    owns: tuple[str, ...]
    namespace: str | None
    predicate: Callable[[dict], bool] | None


class Manager:
    def __init__(self, api: ApiServer, namespace: str | None = None):
        self.api = api
        self.namespace = namespace
        self._ctls: list[_Ctl] = []
        self._queue: list[tuple[float, int, str, Request]] = []
        self._seq = 0
        self._pending: set[tuple[str, Request]] = set()
        self._failures: dict[tuple[str, Request], int] = {}
        self._cv = threading.Condition()
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self._cancels: list[Callable[[], None]] = []
        self.healthy = True
        self.reconcile_count = 0
        self.errors: list[tuple[str, Request, str]] = []

    def add(self, name: str, rec: Reconciler, kind: str, owns=(), namespace: str | None = None,
            predicate: Callable[[dict], bool] | None = None) -> None:
        self._ctls.append(_Ctl(name, rec, kind, tuple(owns), namespace if namespace is not None else self.namespace,
                               predicate))

    # ------------------------------------------------------------------ queue
    def enqueue(self, ctl: str, req: Request, delay: float = 0.0) -> None:
        with self._cv:
            key = (ctl, req)
            if delay <= 0 and key in self._pending:
                return
            self._pending.add(key)
            self._seq += 1
            heapq.heappush(self._queue, (time.monotonic() + delay, self._seq, ctl, req))
            self._cv.notify_all()

    def _on_event(self, ctl: _Ctl, owned: bool):
        def fn(etype: str, obj: dict) -> None:
            md = obj.get("metadata") or {}
            if ctl.namespace is not None and md.get("namespace", "") not in ("", ctl.namespace):
                return
            if owned:
                for r in md.get("ownerReferences") or []:
                    if r.get("controller") and r.get("kind") == ctl.kind:
                        self.enqueue(ctl.name, Request(md.get("namespace", "") if ctl.kind != "DpuOperatorConfig" else "",
                                                       r["name"]))
                return
            if ctl.predicate and not ctl.predicate(obj):
                return
            self.enqueue(ctl.name, Request(md.get("namespace", ""), md["name"]))

        return fn

    def _subscribe(self) -> None:
        for ctl in self._ctls:
            self._cancels.append(self.api.watch(ctl.kind, self._on_event(ctl, False), namespace=ctl.namespace))
            for k in ctl.owns:
                self._cancels.append(self.api.watch(k, self._on_event(ctl, True), replay=False, namespace=ctl.namespace))

    def _process_one(self, block: bool, timeout: float) -> bool:
        with self._cv:
            deadline = time.monotonic() + timeout
            while True:
                now = time.monotonic()
                if self._queue and self._queue[0][0] <= now:
                    _, _, cname, req = heapq.heappop(self._queue)
                    self._pending.discard((cname, req))
                    break
                if not block or self._stop.is_set() or now >= deadline:
                    return False
                wait = min(deadline - now, (self._queue[0][0] - now) if self._queue else deadline - now)
                self._cv.wait(max(wait, 0.001))
        ctl = next(c for c in self._ctls if c.name == cname)
        key = (cname, req)
        try:
            res = ctl.rec.reconcile(req) or Result()
            self.reconcile_count += 1
            CONTROL.reconciles.labels(cname, "requeue" if (res.requeue or res.requeue_after) else "success").inc()
            if res.requeue_after > 0:
                self._failures.pop(key, None)
                self.enqueue(cname, req, res.requeue_after)
            elif res.requeue:
                n = self._failures.get(key, 0) + 1
                self._failures[key] = n
                self.enqueue(cname, req, min(0.005 * (2 ** n), 1.0))
            else:
                self._failures.pop(key, None)
        except Exception as e:  # noqa: BLE001
            n = self._failures.get(key, 0) + 1
            self._failures[key] = n
            self.errors.append((cname, req, repr(e)))
            CONTROL.reconciles.labels(cname, "error").inc()
            log.warning("reconcile %s %s failed (%d): %s", cname, req, n, e)
            self.enqueue(cname, req, min(0.005 * (2 ** n), 1.0))
        return True

    # ------------------------------------------------------------------ run
    def start(self) -> "Manager":
        self._subscribe()
        self._thread = threading.Thread(target=self._run, name="dpu-manager", daemon=True)
        self._thread.start()
        return self

    def _run(self) -> None:
        while not self._stop.is_set():
            self._process_one(True, 0.1)

    def stop(self) -> None:
        self._stop.set()
        with self._cv:
            self._cv.notify_all()
        for c in self._cancels:
            c()
        self._cancels.clear()
        if self._thread:
            self._thread.join(timeout=5)

    def setup(self) -> "Manager":
        """Subscribe without a thread (use drain())."""
        self._subscribe()
        return self

    def drain(self, timeout: float = 2.0, settle: float = 0.0) -> int:
        """Process queued requests until idle (delayed requeues due within `settle` included)."""
        n = 0
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if self._process_one(False, 0):
                n += 1
                continue
            with self._cv:
                nxt = self._queue[0][0] if self._queue else None
            if nxt is not None and nxt - time.monotonic() <= settle:
                time.sleep(max(0.0, nxt - time.monotonic()))
                continue
            break
        return n
