"""Saturated live pod -> pod Mpps over engine geometries (queues x tx workers x generator threads,
header copies vs zero copy) in one process: where the box's CPU share goes.  One JSON line per
configuration.  Usage: python tools/live_sweep.py [--duration 0.3]"""
import argparse
import importlib.util
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (queues, tx workers, generator threads, zero copy, GPU-direct egress)
GRID = [(4, 2, 4, False, False), (5, 1, 8, False, True), (4, 1, 6, False, True), (4, 1, 4, False, True),
        (6, 1, 6, False, True)] * 3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--duration", type=float, default=0.3)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    spec = importlib.util.spec_from_file_location("live_bench", os.path.join(os.path.dirname(__file__), "live_bench.py"))
    lb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lb)
    for q, w, g, zc, gde in GRID:
        r = lb.run(device=a.device, duration=a.duration, queues=q, tx_workers=w, threads=g, zero_copy=zc,
                   saturated_only=True, gpu_egress=gde)
        print(json.dumps({"queues": q, "tx_workers": w, "gen_threads": g, "zero_copy": zc, "gpu_egress": gde,
                          "mpps": r.get("mpps"), "p50_us": r.get("p50_us"), "engine": r.get("engine"),
                          "gde": r.get("gde"), "error": r.get("error")}), flush=True)


if __name__ == "__main__":
    main()
