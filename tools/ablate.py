"""Interleaved A/B ablation of the fused kernel's cost centres (one process, rule 24).

python tools/ablate.py [--batch N] [--rounds R]
"""
import argparse
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda"
    variants = {}
    base = None
    for name, hm, am, nacl in (("lds+mfmaACL256", "lds", "mfma", 256), ("mfma+mfmaACL256", "mfma", "mfma", 256),
                               ("lds+aclOff", "lds", "off", 256), ("mfma+mfmaACL1024", "mfma", "mfma", 1024),
                               ("lds+mfmaACL1024", "lds", "mfma", 1024), ("mfma+mfmaACL512", "mfma", "mfma", 512),
                               ("lds+scalarACL256", "lds", "scalar", 256), ("lds+mfmaWild", "lds", "mfma", "wild")):
        g = DataPlane(device=dev, flow_buckets=1 << 19, hash_mode=hm, acl_mode=am)
        sc = S.build_sfc(g, n_pods=8, n_flows=1 << 20, n_acl=nacl if nacl != "wild" else 256, seed=0)
        if nacl == "wild":   # ClassBench-style rule set (bench.py value_acl_wild)
            S.install_acl_wild(g)
        g.commit(full=True)
        variants[name] = (g, 0, True)
        if base is None:
            base = (g, sc)
    g0, sc = base
    for k in ("mfma+mfmaACL1024", "lds+mfmaACL1024", "mfma+mfmaACL512", "lds+mfmaACL256"):
        variants[k + "/noEarly"] = (variants[k][0], 256, True)   # kernels.hip kFlagNoEarly
    for k in ("mfma+mfmaACL512", "lds+mfmaACL256"):
        variants[k + "/early"] = (variants[k][0], 512, True)     # kernels.hip kFlagForceEarly
    variants["noPortCtr"] = (g0, 1, True)
    variants["noCounters+noLat"] = (g0, 3, False)

    pk, im = S.traffic(sc, a.batch, seed=5)
    tp = torch.from_numpy(pk).to(dev)
    ti = torch.from_numpy(im.view(np.int32)).to(dev)
    out, meta, lat = g0.alloc_batch(a.batch)
    res = {k: [] for k in variants}
    for r in range(a.rounds):
        for name, (g, flags, cf) in variants.items():
            g.count_flows = cf
            g.run(tp, ti, out, meta, lat, flags=flags)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                g.run(tp, ti, out, meta, lat, flags=flags)
            e1.record()
            torch.cuda.synchronize()
            res[name].append(e0.elapsed_time(e1) / a.iters)
            g.count_flows = True
    for name, v in res.items():
        v = np.array(v)
        print(f"{name:22s} median {np.median(v):.4f} ms  min {v.min():.4f}  -> {a.batch / np.median(v) / 1e3:8.1f} Mpps",
              flush=True)


if __name__ == "__main__":
    main()
