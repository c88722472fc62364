"""Flow-table scale sweep on one MI355X: the headline SFC (ACL 256 -> SNAT -> L2, 64-B frames,
4M-packet batches) with 1M, 16M, 64M (and 256M) flows (tables of 64 MB, 1 GB, 4 GB and 16 GB at
50 % load), so the random bucket fetch moves from Infinity-Cache-resident to HBM-bound.  One JSON
line per size.

python tools/flow_scale.py [--flows 1M,16M,64M,256M] [--steps 20]
"""
import argparse
import gc
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.ops import packets as P  # noqa: E402


def size(s: str) -> int:
    s = s.strip().upper()
    mul = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}.get(s[-1], 1)
    return int(s[:-1] if s[-1] in "KMG" else s) * mul


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", default="1M,16M,64M")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1 << 22)
    a = ap.parse_args()
    # a 256M-flow build runs ~7 min on the host, mostly in native / numpy calls that hold the GIL
    # (a Python heartbeat thread stalls with them): run it beside a shell heartbeat that appends
    # to a file under gpurun_out/ (profiles/r2_s42_flow_scale_256m.log)
    for f in [size(x) for x in a.flows.split(",")]:
        t0 = time.time()
        print(f"# building {f} flows", flush=True)
        dp = DataPlane(device="cuda", flow_buckets=max(f // 2, 1 << 10), hash_mode="lds", acl_mode="mfma")
        sc = S.build_sfc(dp, n_pods=8, n_flows=f, n_acl=256, seed=0)
        dp.commit(full=True)
        setup = time.time() - t0
        print(f"# built in {setup:.1f} s", flush=True)
        batches = []
        for r in range(2):
            pk, im = S.traffic(sc, a.batch, seed=11 + r)
            batches.append((torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()))
        out, meta, lat = dp.alloc_batch(a.batch)
        for k in range(3):
            dp.run(*batches[k % 2], out, meta, lat)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(a.steps):
            dp.run(*batches[k % 2], out, meta, lat)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        fwd = float(np.mean(P.meta_fields(meta.cpu().numpy().view(np.uint32))[2] == 0))
        table_mb = dp.flows.nbuckets * 128 / 2 ** 20
        print(json.dumps({"flows": f, "table_mb": round(table_mb), "mpps": round(a.batch * a.steps / el / 1e6, 1),
                          "ms_per_batch": round(el / a.steps * 1e3, 4), "forwarded_fraction": round(fwd, 4),
                          "setup_s": round(setup, 1)}), flush=True)
        del dp, sc, batches, out, meta, lat
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
