"""What limits the headline kernel: same-process, interleaved timings of the fused kernel with one
cost centre changed at a time, plus the bytes the step moves.

Variants (all 4M 64-B packets of the headline SFC, 256 ACL rules, LDS Toeplitz, MFMA ACL):
  * base          1M flows (the headline: 64-MB bucket table + 8-MB flow counters);
  * flows_64k     64K flows: buckets and counters fit one XCD's L2 (the bucket fetch and the counter
                  RMW stop going to the Infinity Cache / HBM);
  * flows_16m     16M flows: 1-GB table, every fetch from HBM;
  * ctr_zero      flow-counter atomics add 0 (kernel flag 4: the atomic is still issued: the
                  difference to base is the counter lines' dirty write-back only);
  * no_lat        no latency samples, no port counters (flags 1 | 2);
  * wild / wild_no_early   the ClassBench-style 1025-rule ACL: the early-fetch 2-wave instance (its
                  default) and the 4-wave instance with per-tile prefilters (flag 256).
A build without the per-flow atomic at all is tools/ab_variants.py with -DNFDP_ABL_NO_FLOWCTR.

Byte model per packet (what has to cross HBM / MALL at minimum): frame in 64 B, frame out 64 B,
meta in + out 8 B, one 128-B bucket line, one 8-B counter RMW (a 64-B line read and written back
when it misses the caches).  Printed next to the measured rate so the fraction of roofline shows.

python tools/limiter.py [--rounds 5] [--iters 20]
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

HBM_TBS = 8.0   # MI355X HBM3E peak (TB/s)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    planes = {}
    for name, flows in (("base", 1 << 20), ("flows_64k", 1 << 16), ("flows_16m", 1 << 24)):
        g = DataPlane(device="cuda", flow_buckets=max(1 << 10, flows // 2), hash_mode="lds", acl_mode="mfma")
        sc = S.build_sfc(g, n_pods=8, n_flows=flows, n_acl=256, seed=0)
        g.commit(full=True)
        bs = []
        for r in range(2):
            pk, im = S.traffic(sc, a.batch, seed=1 + r)
            bs.append((torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()))
        planes[name] = (g, bs)
        print(f"plane {name} ready", file=sys.stderr, flush=True)
    # the ClassBench-style rule set (bench value_acl_wild) on the headline's flows: the early-fetch
    # 2-wave instance (default from 33 rule tiles) against the 4-wave instance with per-tile prefilters
    g = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(g, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
    S.install_acl_wild(g, 1024)
    g.commit(full=True)
    pk, im = S.traffic(sc, a.batch, seed=9001)
    planes["wild"] = (g, [(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())] * 2)
    g = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(g, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
    S.add_acl_rules(g, 1024)
    g.commit(full=True)
    pk, im = S.traffic(sc, a.batch, seed=9001)
    planes["acl1024"] = (g, [(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())] * 2)
    variants = {"base": ("base", 0), "flows_64k": ("flows_64k", 0), "flows_16m": ("flows_16m", 0),
                "ctr_zero": ("base", 4), "no_lat": ("base", 3), "wild": ("wild", 0), "wild_no_early": ("wild", 256),
                "acl1024": ("acl1024", 0), "acl1024_no_early": ("acl1024", 256)}
    res = {k: [] for k in variants}
    bufs = {k: planes[k][0].alloc_batch(a.batch) for k in planes}
    for rd in range(a.rounds):
        print(f"round {rd}", file=sys.stderr, flush=True)
        for v, (pl, flags) in variants.items():
            g, bs = planes[pl]
            out, meta, lat = bufs[pl]
            for k in range(3):
                g.run(*bs[k % 2], out, meta, lat, flags=flags)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.iters):
                g.run(*bs[k % 2], out, meta, lat, flags=flags)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / a.iters)
    out = {}
    min_bytes = 64 + 64 + 8 + 128 + 2 * 64
    for v, ts in res.items():
        t = float(np.median(ts))
        gpps = a.batch / t / 1e9
        out[v] = {"ms": round(t * 1e3, 4), "gpps": round(gpps, 3), "ms_min": round(min(ts) * 1e3, 4),
                  "ms_max": round(max(ts) * 1e3, 4)}
    b = out["base"]["gpps"]
    out["model"] = {"bytes_per_packet_min": min_bytes, "hbm_tbs": HBM_TBS,
                    "base_tbs_at_min_bytes": round(b * min_bytes / 1e3, 3),
                    "base_fraction_of_hbm_roofline": round(b * min_bytes / 1e3 / HBM_TBS, 3),
                    "roofline_gpps_at_min_bytes": round(HBM_TBS * 1e3 / min_bytes, 2)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
