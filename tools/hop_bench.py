"""The SFC hop pipeline alone (bench.py measure_hops without the rest): two data planes on one GPU,
the headline chain split after nat, N timed batches.  For rocprofv3 --kernel-trace --stats runs.

Usage: python tools/hop_bench.py [--batch 4194304] [--flows 1048576] [--steps 20]
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
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--flows", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--split", default="acl,nat,l2fwd@1")
    a = ap.parse_args()
    import torch

    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.multi import MultiDataPlane
    from dpu_operator_amd.parallel.hops import HopPipeline

    dev = "cuda:0"
    multi = MultiDataPlane([dev, dev], placement="port",
                           flow_buckets=1 << max(10, int(math.ceil(math.log2(a.flows / 2)))))
    sc = S.build_sfc(multi, n_pods=8, n_flows=a.flows, n_acl=256, hops=tuple(a.split.split(",")))
    multi.commit()
    bs = []
    for r in range(2):
        pk, im = S.traffic(sc, a.batch, seed=9500 + r)
        bs.append((torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev)))
    hp = HopPipeline(multi.planes, a.batch)
    for k in range(3):
        hp.step(*bs[k % 2])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        hp.step(*bs[k % 2])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"batch": a.batch, "steps": a.steps, "ms_per_batch": round(el / a.steps * 1e3, 4),
                      "mpps": round(a.batch * a.steps / el / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
