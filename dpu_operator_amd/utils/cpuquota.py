"""The CPU share this process may use: cgroup CFS bandwidth quota and its throttling counters.

The live pod -> pod path is host-CPU work (pod generators, rx / tx engine threads that poll), so
its rate depends on how much CPU time the box grants, not on how many CPUs `nproc` shows.  A CFS
quota (`cpu.max` on cgroup v2, `cpu.cfs_quota_us` / `cpu.cfs_period_us` on v1) caps the CPU time
per period of all the process's threads together; once spent, every thread is frozen until the
period ends, which shows up as throughput collapse and millisecond tails when more threads poll
than the quota covers.  `snapshot()` reads the quota and the throttling counters, `delta()` gives
what a measured interval cost (CPU seconds used, periods throttled, time frozen).

Pure /proc and /sys reads; every field is None where the hierarchy does not expose it.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

_ROOT = "/sys/fs/cgroup"


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _kv(text: Optional[str]) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for line in (text or "").splitlines():
        parts = line.split()
        if len(parts) == 2 and parts[1].lstrip("-").isdigit():
            out[parts[0]] = int(parts[1])
    return out


def _cgroup_paths(proc_cgroup: Optional[str]) -> Dict[str, str]:
    """controller -> relative cgroup path ('' key: the v2 unified path)."""
    out: Dict[str, str] = {}
    for line in (proc_cgroup or "").splitlines():
        parts = line.split(":", 2)
        if len(parts) != 3:
            continue
        for c in (parts[1].split(",") if parts[1] else [""]):
            out[c] = parts[2]
    return out


def _first_dir(cands) -> Optional[str]:
    for d in cands:
        if d and os.path.isdir(d):
            return d
    return None


def _dirs(root: str, proc_cgroup: Optional[str]):
    """(v2 dir, v1 cpu dir, v1 cpuacct dir): the process's own cgroup where it is visible (a cgroup
    namespace shows it at the root of the mount), else the mount root."""
    paths = _cgroup_paths(proc_cgroup)
    v2 = None
    if os.path.exists(os.path.join(root, "cgroup.controllers")):
        rel = paths.get("", "/").lstrip("/")
        v2 = _first_dir([os.path.join(root, rel) if rel else None, root])
    cpu_rel = next((p for c, p in paths.items() if "cpu" in c.split(",") or c == "cpu,cpuacct"), "/").lstrip("/")
    v1cpu = _first_dir([os.path.join(root, d, cpu_rel) for d in ("cpu", "cpu,cpuacct") if cpu_rel] +
                       [os.path.join(root, d) for d in ("cpu", "cpu,cpuacct")])
    acct_rel = paths.get("cpuacct", cpu_rel).lstrip("/")
    v1acct = _first_dir([os.path.join(root, d, acct_rel) for d in ("cpuacct", "cpu,cpuacct") if acct_rel] +
                        [os.path.join(root, d) for d in ("cpuacct", "cpu,cpuacct")])
    return v2, v1cpu, v1acct


def snapshot(root: str = _ROOT, proc_cgroup_path: str = "/proc/self/cgroup") -> dict:
    """Quota (CPUs, None = unlimited), period, usage and throttling counters, plus the affinity."""
    v2, v1cpu, v1acct = _dirs(root, _read(proc_cgroup_path))
    snap = {"cgroup": None, "quota_cpus": None, "period_us": None, "usage_s": None, "nr_periods": None,
            "nr_throttled": None, "throttled_s": None}
    try:
        snap["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        snap["affinity_cpus"] = os.cpu_count()
    if v2 and _read(os.path.join(v2, "cpu.max")) is not None:
        snap["cgroup"] = "v2"
        q = (_read(os.path.join(v2, "cpu.max")) or "max 100000").split()
        period = int(q[1]) if len(q) > 1 and q[1].isdigit() else 100000
        snap["period_us"] = period
        snap["quota_cpus"] = None if q[0] == "max" else round(int(q[0]) / period, 3)
        st = _kv(_read(os.path.join(v2, "cpu.stat")))
        snap["usage_s"] = st["usage_usec"] / 1e6 if "usage_usec" in st else None
        snap["nr_periods"] = st.get("nr_periods")
        snap["nr_throttled"] = st.get("nr_throttled")
        snap["throttled_s"] = st["throttled_usec"] / 1e6 if "throttled_usec" in st else None
        eff = _read(os.path.join(v2, "cpuset.cpus.effective"))
        if eff:
            snap["cpuset"] = eff
        return snap
    if v1cpu:
        snap["cgroup"] = "v1"
        quota = _read(os.path.join(v1cpu, "cpu.cfs_quota_us"))
        period = _read(os.path.join(v1cpu, "cpu.cfs_period_us"))
        if period and period.isdigit():
            snap["period_us"] = int(period)
        if quota and quota.lstrip("-").isdigit() and int(quota) > 0 and snap["period_us"]:
            snap["quota_cpus"] = round(int(quota) / snap["period_us"], 3)
        st = _kv(_read(os.path.join(v1cpu, "cpu.stat")))
        snap["nr_periods"] = st.get("nr_periods")
        snap["nr_throttled"] = st.get("nr_throttled")
        snap["throttled_s"] = st["throttled_time"] / 1e9 if "throttled_time" in st else None
        if v1acct:
            u = _read(os.path.join(v1acct, "cpuacct.usage"))
            if u and u.isdigit():
                snap["usage_s"] = int(u) / 1e9
    return snap


def delta(before: dict, after: dict, wall_s: float) -> dict:
    """What an interval of `wall_s` seconds cost: CPUs used on average, throttled periods / time."""
    def d(k):
        a, b = after.get(k), before.get(k)
        return None if a is None or b is None else a - b

    used = d("usage_s")
    out = {"wall_s": round(wall_s, 4),
           "cpus_used": None if used is None or wall_s <= 0 else round(used / wall_s, 2),
           "periods": d("nr_periods"), "throttled_periods": d("nr_throttled"),
           "throttled_s": None if d("throttled_s") is None else round(d("throttled_s"), 4)}
    return out


def process_cpu_s() -> float:
    """CPU seconds this process has used (all threads): the fallback when no cgroup counter exists."""
    t = os.times()
    return t.user + t.system


class Meter:
    """Context manager: `with Meter() as m: ...` then `m.result` (delta() plus the process's own
    CPU seconds, which count even where the cgroup hides its counters)."""

    def __enter__(self):
        import time

        self._t = time.perf_counter()
        self._s = snapshot()
        self._p = process_cpu_s()
        return self

    def __exit__(self, *exc):
        import time

        wall = time.perf_counter() - self._t
        self.result = delta(self._s, snapshot(), wall)
        self.result["process_cpus_used"] = round((process_cpu_s() - self._p) / max(wall, 1e-9), 2)
        return False


def cpu_share(counts=(4, 8, 16, 24, 32), seconds: float = 0.25) -> dict:
    """The CPUs this process is really granted, measured: N native threads busy-loop together
    (nfdp.cpu_share_probe, no fork) for each N; `cpus` is the most any N got.  Where a CFS quota
    hides behind a cgroup the process cannot read, this is the only way to see it (the GPU box:
    256 CPUs listed, 16 granted)."""
    from dpu_operator_amd.native import nfdp

    nf = nfdp()
    curve = []
    for n in counts:
        cpu, wall = nf.cpu_share_probe(int(n), float(seconds))
        curve.append({"threads": int(n), "cpus_granted": round(cpu / max(wall, 1e-9), 2)})
    return {"cpus": max(c["cpus_granted"] for c in curve), "curve": curve, "probe_s": seconds}
