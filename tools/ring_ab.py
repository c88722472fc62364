"""Interleaved A/B of the persistent ring's throughput mode (bench `ring.loaded_mpps`): trials of
each configuration alternate, so box drift hits them all alike (3,519 Mpps in
the r4 driver run, 2,528 in r5's, 2,486-3,544 across r5 sessions).

Configurations: workgroups per CU (resident grid size) x chunks in flight x batch per publish; the
host thread publishes and reaps in C++ (RingEngine.probe).  Also the 64K-batch fused-kernel p50
(bench `p50_latency_us_64k_batch`) in the same process, 5 trials.

python tools/ring_ab.py [--trials 5]
"""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.dataplane.ring import RingPath  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=5)
    ap.add_argument("--batches", type=int, default=10000)
    a = ap.parse_args()
    dp = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
    dp.commit(full=True)
    pk, im = S.traffic(sc, 1 << 18, seed=1)
    tpk, tim = torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()
    # (wgs per CU, in flight, batch, capacity)
    cfgs = {"w2_if32_b4096": (2, 32, 4096, 1 << 17), "w1_if32_b4096": (1, 32, 4096, 1 << 17),
            "w4_if32_b4096": (4, 32, 4096, 1 << 17), "w2_if64_b4096": (2, 64, 4096, 1 << 18),
            "w2_if16_b8192": (2, 16, 8192, 1 << 17)}
    res = {k: [] for k in cfgs}
    lat64 = []
    errs = {}
    out, meta, lat = dp.alloc_batch(1 << 16)
    for t in range(a.trials):
        print(f"trial {t}", file=sys.stderr, flush=True)
        for name, (w, inflight, batch, cap) in cfgs.items():
            rq = RingPath(dp, capacity=cap, wgs_per_cu=w, deadline_s=120.0, coop=False)
            rq.stage(tpk[:cap], tim[:cap])
            try:
                rq.start()
            except RuntimeError as ex:   # (a configuration the CU cannot hold: recorded, not fatal)
                errs[name] = str(ex)
                rq.close()
                continue
            rq.probe(batches=500, batch=batch, inflight=inflight)
            _, el = rq.probe(batches=a.batches, batch=batch, inflight=inflight)
            rq.stop()
            rq.close()
            res[name].append(a.batches * batch / el / 1e6)
        for _ in range(20):
            dp.run(tpk[: 1 << 16], tim[: 1 << 16], out, meta, lat)
        torch.cuda.synchronize()
        lat64.append(float(np.median(lat.cpu().numpy().view(np.uint32).astype(np.float64) * 0.01)))
        time.sleep(0.05)
    print(json.dumps({"ring_loaded_mpps": {k: {"median": round(float(np.median(v)), 1), "trials": [round(x, 1) for x in v]}
                                           for k, v in res.items() if v},
                      "errors": errs,
                      "p50_latency_us_64k_batch": {"median": round(float(np.median(lat64)), 2),
                                                   "trials": [round(x, 2) for x in lat64]}}), flush=True)


if __name__ == "__main__":
    main()
