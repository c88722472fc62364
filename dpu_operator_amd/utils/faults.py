"""Fault injection.

The reference has none.  Named injection points are checked by the components
(`faults.check("vsp.CreateBridgePort")`); a point can be armed to raise an error (optionally a
gRPC-style UNAVAILABLE the retry policies react to), to sleep, or to corrupt/drop — for `count`
hits or forever, optionally only every `every`-th hit.  Arm from code (`FAULTS.arm(...)`) or the
environment: DPU_FAULTS="vsp.Init:unavailable:3,cni.ADD:delay=0.5:1".
Points wired in: vsp.<Rpc> (VSP wire adapters), cni.<ADD|DEL> (CNI server), deviceplugin.GetDevices,
dataplane.commit, daemon.detect.
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass


class FaultError(RuntimeError):
    def __init__(self, point: str, kind: str):
        super().__init__(f"injected fault at {point} ({kind})")
        self.point, self.kind = point, kind


@dataclass
class _Arm:
    kind: str            # error | unavailable | delay | drop
    count: int = -1      # remaining activations (-1 = unlimited)
    delay: float = 0.0
    every: int = 1
    hits: int = 0
    fired: int = 0


class FaultInjector:
    def __init__(self):
        self._arms: dict[str, _Arm] = {}
        self._lock = threading.Lock()
        self.log: list[tuple[str, str]] = []

    def arm(self, point: str, kind: str = "error", count: int = 1, delay: float = 0.0, every: int = 1) -> None:
        if kind not in ("error", "unavailable", "delay", "drop"):
            raise ValueError(f"unknown fault kind {kind}")
        with self._lock:
            self._arms[point] = _Arm(kind, count, delay, max(1, every))

    def disarm(self, point: str | None = None) -> None:
        with self._lock:
            if point is None:
                self._arms.clear()
            else:
                self._arms.pop(point, None)

    def load_env(self, spec: str | None = None) -> None:
        spec = os.environ.get("DPU_FAULTS", "") if spec is None else spec
        for item in filter(None, (s.strip() for s in spec.split(","))):
            parts = item.split(":")
            point, kind = parts[0], parts[1] if len(parts) > 1 else "error"
            delay = 0.0
            if kind.startswith("delay="):
                kind, delay = "delay", float(kind.split("=", 1)[1])
            count = int(parts[2]) if len(parts) > 2 else 1
            self.arm(point, kind, count, delay)

    def check(self, point: str) -> bool:
        """Returns True when the caller should DROP the operation; raises for error kinds."""
        with self._lock:
            a = self._arms.get(point)
            if a is None or a.count == 0:
                return False
            a.hits += 1
            if a.hits % a.every:
                return False
            if a.count > 0:
                a.count -= 1
            a.fired += 1
            self.log.append((point, a.kind))
            kind, delay = a.kind, a.delay
        if kind == "delay":
            time.sleep(delay)
            return False
        if kind == "drop":
            return True
        raise FaultError(point, kind)

    def fired(self, point: str) -> int:
        with self._lock:
            a = self._arms.get(point)
            return a.fired if a else 0


FAULTS = FaultInjector()
FAULTS.load_env()
