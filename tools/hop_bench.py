"""The SFC hop pipeline across GPUs, measured alone (bench.py runs it as a child process).

The headline chain (acl -> nat -> l2fwd over 1M flows) split after nat: acl + nat on the first
plane, l2fwd + egress on the second.  `--devices cuda:0,cuda:1` puts the planes on two GPUs (the
hand-off's peer stores cross xGMI); `cuda:0,cuda:0` rehearses on one.  Prints one JSON line:
pipeline Mpps / ms per batch at --batch, and the per-hop latency split of a 64K batch (first GPU's
kernel, hand-off, resuming GPU's kernel; GPU event clock).  A child process, so a fault on the
peer path cannot take the bench's headline with it.

Usage: python tools/hop_bench.py [--devices cuda:0,cuda:0] [--batch 4194304] [--flows 1048576] [--steps 20]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default="cuda:0,cuda:0")
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--flows", type=int, default=1 << 20)
    ap.add_argument("--acl", type=int, default=256)
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--hash", default="lds")
    ap.add_argument("--split", default="acl,nat,l2fwd@1")
    a = ap.parse_args()
    import torch

    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.multi import MultiDataPlane
    from dpu_operator_amd.ops import packets as P
    from dpu_operator_amd.parallel.hops import HopPipeline

    devs = a.devices.split(",")
    multi = MultiDataPlane(devs, placement="port", hash_mode=a.hash,
                           flow_buckets=1 << max(10, int(math.ceil(math.log2(a.flows / 2)))))
    sc = S.build_sfc(multi, n_pods=a.pods, n_flows=a.flows, n_acl=a.acl, hops=tuple(a.split.split(",")))
    multi.commit()
    d0 = devs[0]
    bs = []
    for r in range(2):
        pk, im = S.traffic(sc, a.batch, seed=9500 + r)
        bs.append((torch.from_numpy(pk).to(d0), torch.from_numpy(im.view(np.int32)).to(d0)))
    hp = HopPipeline(multi.planes, a.batch)
    for k in range(3):
        hp.step(*bs[k % 2])
    hp.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        hp.step(*bs[k % 2])
    hp.synchronize()
    el = time.perf_counter() - t0
    out, meta = hp.results(a.batch)
    rs = P.meta_fields(meta)[2]
    res = {"split": a.split, "planes": devs, "peer": devs[0] != devs[1], "batch": a.batch, "steps": a.steps,
           "mpps": round(a.batch * a.steps / el / 1e6, 1), "ms_per_batch": round(el / a.steps * 1e3, 4),
           "forwarded_fraction": round(float(np.mean(rs == 0)), 4),
           "handoff_bytes_per_frame": 64 + 32 + 4}
    # per-hop latency: one 64K batch at a time, GPU event clock at each stage boundary
    nsm = min(1 << 16, a.batch)
    del hp
    hs = HopPipeline(multi.planes, nsm)
    small = (bs[0][0][:nsm].contiguous(), bs[0][1][:nsm].contiguous())
    f_us, h_us, r_us = [], [], []
    for k in range(60):
        tm = {}
        hs.step(*small, timing=tm)
        hs.synchronize()
        if k >= 10:
            f_us.append(tm["t0"].elapsed_time(tm["fused"]) * 1e3)
            h_us.append(tm["fused"].elapsed_time(tm["handoff"]) * 1e3)
            r_us.append(tm["handoff"].elapsed_time(tm["resume"]) * 1e3)
    res["per_hop_us"] = {"batch": nsm, "first_gpu_kernel": round(float(np.median(f_us)), 2),
                         "handoff": round(float(np.median(h_us)), 2),
                         "resume_gpu_kernel": round(float(np.median(r_us)), 2),
                         "total": round(float(np.median(np.add(np.add(f_us, h_us), r_us))), 2)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
