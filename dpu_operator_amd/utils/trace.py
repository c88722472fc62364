"""Lightweight tracing: spans in a bounded ring, exported as Chrome trace JSON (Perfetto).

The reference has no tracing; GPU kernels are profiled with rocprofv3.  Host-side
control and data-plane paths open spans (`with TRACER.span("cni.ADD", pod=...)`): CNI requests,
VSP RPCs, data-plane batch launches and table commits.  Disabled unless DPU_TRACE=1 or
`TRACER.enable()`; when disabled a span costs one attribute check.
"""
from __future__ import annotations

import json
import os
import threading
import time
from collections import deque
from contextlib import contextmanager


class Tracer:
    def __init__(self, capacity: int = 65536):
        self.enabled = os.environ.get("DPU_TRACE", "") == "1"
        self._events: deque = deque(maxlen=capacity)
        self._lock = threading.Lock()
        self._pid = os.getpid()

    def enable(self, on: bool = True) -> None:
        self.enabled = on

    @contextmanager
    def span(self, name: str, **attrs):
        if not self.enabled:
            yield
            return
        t0 = time.perf_counter_ns()
        err = None
        try:
            yield
        except BaseException as e:
            err = repr(e)
            raise
        finally:
            dur = time.perf_counter_ns() - t0
            args = dict(attrs)
            if err:
                args["error"] = err
            ev = {"name": name, "ph": "X", "ts": t0 / 1000.0, "dur": dur / 1000.0, "pid": self._pid,
                  "tid": threading.get_ident(), "args": args}
            with self._lock:
                self._events.append(ev)

    def events(self, name: str | None = None) -> list[dict]:
        with self._lock:
            return [e for e in self._events if name is None or e["name"] == name]

    def clear(self) -> None:
        with self._lock:
            self._events.clear()

    def export(self, path: str) -> int:
        with self._lock:
            evs = list(self._events)
        with open(path, "w") as f:
            json.dump({"traceEvents": evs, "displayTimeUnit": "ms"}, f)
        return len(evs)


TRACER = Tracer()
