"""Latency histograms of the packet path, exported through the data-plane metrics collector.

Log-2 buckets from 250 ns to ~4 s (the GPU's realtime counter ticks at 100 MHz, so 10 ns is the
finest device sample; host stages are µs and up).  Observations are folded in bulk with
`np.searchsorted`, so a whole batch of device latency samples costs one numpy call.  Thread-safe:
the live path observes from its loop thread while the metrics server scrapes from another.

Stages recorded by the live packet path (dataplane/netio.py), one observation per batch:
  rx        reads of the ready vport fds (from poll's wake-up) until the batch is formed
  pipeline  header slots -> data plane (upload, fused kernel, download) -> egress meta on the host
  side      side pass readout (flood / mirror replicas, learn events, tunnel headers)
  tx        frame assembly + writes to the egress fds
  batch     the whole cycle
and per packet (GPU only, 1 in 16 packets sampled by the fused kernel):
  device    batch release (`t0` stamp) -> the packet's egress decision written, on the GPU clock
"""
from __future__ import annotations

import threading

import numpy as np

BOUNDS = tuple(250e-9 * 2.0 ** k for k in range(25))  # 250 ns .. ~4.2 s


class LatencyHist:
    def __init__(self, bounds=BOUNDS):
        self.bounds = np.asarray(bounds, np.float64)
        self.counts = np.zeros(len(bounds) + 1, np.int64)   # last = +Inf
        self.sum = 0.0
        self._mu = threading.Lock()

    def observe(self, seconds: float) -> None:
        i = int(np.searchsorted(self.bounds, seconds, side="left"))
        with self._mu:
            self.counts[i] += 1
            self.sum += float(seconds)

    def observe_many(self, seconds) -> None:
        v = np.asarray(seconds, np.float64).ravel()
        if not v.size:
            return
        idx = np.searchsorted(self.bounds, v, side="left")
        c = np.bincount(idx, minlength=len(self.counts))
        with self._mu:
            self.counts += c
            self.sum += float(v.sum())

    @property
    def count(self) -> int:
        return int(self.counts.sum())

    def quantile(self, q: float) -> float:
        """Upper bound of the bucket holding quantile q (0 when empty)."""
        with self._mu:
            c = self.counts.copy()
        tot = c.sum()
        if not tot:
            return 0.0
        i = int(np.searchsorted(np.cumsum(c), q * tot, side="left"))
        return float(self.bounds[i]) if i < len(self.bounds) else float("inf")

    def buckets(self) -> tuple[list[tuple[str, float]], float]:
        """Prometheus form: cumulative (le, count) pairs ending in +Inf, and the sum."""
        with self._mu:
            cum = np.cumsum(self.counts)
            s = self.sum
        out = [(repr(float(b)), float(cum[i])) for i, b in enumerate(self.bounds)]
        out.append(("+Inf", float(cum[-1])))
        return out, s


class LatencyStats:
    """Named histograms (stage -> LatencyHist)."""

    def __init__(self):
        self._h: dict[str, LatencyHist] = {}
        self._mu = threading.Lock()

    def hist(self, stage: str) -> LatencyHist:
        with self._mu:
            h = self._h.get(stage)
            if h is None:
                h = self._h[stage] = LatencyHist()
            return h

    def observe(self, stage: str, seconds: float) -> None:
        self.hist(stage).observe(seconds)

    def observe_many(self, stage: str, seconds) -> None:
        self.hist(stage).observe_many(seconds)

    def items(self):
        with self._mu:
            return sorted(self._h.items())
