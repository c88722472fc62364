"""Live-path diagnostics: saturated pod -> pod Mpps per engine configuration, repeated trials, with the
process's CPU quota and what each trial cost in CPU time and CFS throttling (utils/cpuquota.py).

Answers "why does the same configuration give 50 Mpps in one place and 104 in another" and "why
do 8 queues collapse": every trial reports cpus_used and throttled periods next to its Mpps.

    python tools/live_diag.py [--trials 3] [--duration 1.0] [--configs 4x2g4,8x2g4,...] [--out f.jsonl]

A config `QxWgG[z][e]` is Q rx queues, W tx workers per queue (0 = run-to-completion: the rx thread
delivers), G generator threads; `e` adds GPU-direct egress, `z` zero-copy rx.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dpu_operator_amd.utils import cpuquota  # noqa: E402


def parse_cfg(s: str) -> dict:
    m = re.fullmatch(r"(\d+)x(\d+)g(\d+)([ze]*)", s)
    if not m:
        raise SystemExit(f"bad config {s!r} (want QxWgG[z][e])")
    return {"queues": int(m.group(1)), "tx_workers": int(m.group(2)), "threads": int(m.group(3)),
            "zero_copy": "z" in m.group(4), "gpu_egress": "e" in m.group(4)}


def _spin(seconds: float) -> None:
    import time as _t

    end = _t.perf_counter() + seconds
    x = 0
    while _t.perf_counter() < end:
        x += 1


def cpu_probe(counts=(1, 2, 4, 8, 12, 16, 24, 32), seconds: float = 1.0) -> list:
    """How much CPU time the box grants: N processes busy-loop for `seconds` together; the CPUs
    they got on average (children's CPU seconds / wall).  Flat beyond some N = the real share."""
    import multiprocessing as mp
    import resource

    out = []
    ctx = mp.get_context("fork")
    for n in counts:
        r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        t0 = time.perf_counter()
        ps = [ctx.Process(target=_spin, args=(seconds,)) for _ in range(n)]
        for p in ps:
            p.start()
        for p in ps:
            p.join()
        wall = time.perf_counter() - t0
        r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        used = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
        out.append({"procs": n, "cpus_granted": round(used / wall, 2), "wall_s": round(wall, 3)})
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--duration", type=float, default=1.0)
    ap.add_argument("--flows", type=int, default=1 << 20)
    ap.add_argument("--configs", default="4x2g4,4x2g4,1x2g4,2x2g4,8x2g4,4x1g4,8x1g4")
    ap.add_argument("--full-first", action="store_true", help="run the bench's full live block first (as bench.py)")
    ap.add_argument("--out", default="")
    ap.add_argument("--cpu-probe", action="store_true", help="first measure the CPU time the box grants N spinners")
    a = ap.parse_args()
    import importlib.util

    spec = importlib.util.spec_from_file_location("live_bench", os.path.join(os.path.dirname(__file__), "live_bench.py"))
    lb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lb)
    fout = open(a.out, "a") if a.out else None

    def emit(rec):
        line = json.dumps(rec)
        print(line, flush=True)
        if fout:
            fout.write(line + "\n")
            fout.flush()

    emit({"quota": cpuquota.snapshot(), "pid": os.getpid(), "nproc": os.cpu_count()})
    if a.cpu_probe:
        emit({"cpu_probe": cpu_probe()})
    if a.full_first:
        with cpuquota.Meter() as m:
            r = lb.run(device=a.device, flows=a.flows, duration=0.5)
        emit({"phase": "full_first", "mpps": r.get("mpps"), "half_p99_us": r.get("half_p99_us"),
              "idle_p50_us": r.get("idle_p50_us"), "load90_p99_us": r.get("load90_p99_us"), "cpu": m.result,
              "engine": r.get("engine"), "error": r.get("error")})
    for cs in a.configs.split(","):
        c = parse_cfg(cs)
        for t in range(a.trials):
            t0 = time.perf_counter()
            with cpuquota.Meter() as m:
                r = lb.run(device=a.device, flows=a.flows, duration=a.duration, saturated_only=True, **c)
            emit({"config": cs, "trial": t, **c, "mpps": r.get("mpps"), "offered_mpps": r.get("offered_mpps"),
                  "p50_us": r.get("p50_us"), "p99_us": r.get("p99_us"), "engine": r.get("engine"),
                  "cpu": m.result, "wall_s": round(time.perf_counter() - t0, 2), "error": r.get("error")})


if __name__ == "__main__":
    main()
