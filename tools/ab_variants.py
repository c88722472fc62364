"""Interleaved A/B of build variants of the headline kernel, one process per measurement.

Two builds of `_nfdp` cannot share a process (one module name), so each measurement is a child
process that loads one variant (NFDP_EXT_DIR, native/build.py NFDP_BUILD_OUT) and times the
headline step (1M flows, ACL 256 -> SNAT -> L2, 4M-packet batches) with HIP events; variants
alternate round by round so box drift hits them equally.

python tools/ab_variants.py base= variants/noreload [--rounds 4] [--iters 50] [--acl 256|wild|ipv6]
  (an empty directory means the in-tree build; name=dir:kernel launches a stamp kernel before every
  batch, the pre-r6 release stamp, instead of the fused kernel's own)
python tools/ab_variants.py --inline [--acl ...]   one in-process measurement of the in-tree build
  (for rocprofv3: no child process)
"""
import argparse
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys, numpy as np, torch
sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane.engine import DataPlane
iters, batch, acl = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
stamp_kernel = len(sys.argv) > 4 and sys.argv[4] == "kernel"
g = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
sc = S.build_sfc(g, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
if acl == "wild":
    S.install_acl_wild(g)
info6 = S.install_ipv6(g, sc, 1 << 16, 64) if acl == "ipv6" else None
g.commit(full=True)
bs = []
for r in range(4):
    if info6 is None:
        pk, im = S.traffic(sc, batch, seed=1 + r)
    else:   # bench.py's dual stack: half IPv6, shuffled
        pk4, im4 = S.traffic(sc, batch - batch // 2, seed=9200 + r)
        pk6, im6 = S.traffic_ipv6(sc, info6, batch // 2, seed=9300 + r)
        perm = np.random.default_rng(r).permutation(batch)
        pk = np.ascontiguousarray(np.concatenate([pk4, pk6])[perm])
        im = np.ascontiguousarray(np.concatenate([im4, im6])[perm])
    bs.append((torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()))
out, meta, lat = g.alloc_batch(batch)
def step(k):
    if stamp_kernel:   # the pre-r6 release stamp: a stamp kernel in front of every batch
        g.nf.launch_stamp(g._ptr("t0"), torch.cuda.current_stream().cuda_stream)
        g.run(*bs[k % 4], out, meta, lat, stamp=False)
    else:
        g.run(*bs[k % 4], out, meta, lat)
for k in range(10):
    step(k)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for k in range(iters):
    step(k)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / iters
print(json.dumps({"ms": ms, "mpps": batch / ms / 1e3}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*", help="name=dir (dir empty: in-tree build)")
    ap.add_argument("--inline", action="store_true", help="measure the in-tree build in this process")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1 << 22)
    ap.add_argument("--acl", default="256", choices=["256", "wild", "ipv6"])
    a = ap.parse_args()
    if a.inline:
        sys.argv = ["-", str(a.iters), str(a.batch), a.acl]
        exec(compile(CHILD, "ab_variants_child", "exec"), {"__name__": "__child__"})
        return
    vs = [v.split("=", 1) if "=" in v else (os.path.basename(v), v) for v in a.variants]
    res = {n: [] for n, _ in vs}
    for r in range(a.rounds):
        for n, d in vs:
            d, _, mode = d.partition(":")   # dir[:kernel] - "kernel": a stamp kernel before each batch
            env = dict(os.environ)
            env.pop("NFDP_EXT_DIR", None)
            if d:
                env["NFDP_EXT_DIR"] = os.path.abspath(d)
            p = subprocess.run([sys.executable, "-c", CHILD, str(a.iters), str(a.batch), a.acl, mode or "self"], env=env,
                               capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if not line:
                print(json.dumps({"variant": n, "error": p.stderr[-1500:]}), flush=True)
                sys.exit(1)
            res[n].append(json.loads(line[-1])["mpps"])
            print(json.dumps({"round": r, "variant": n, "mpps": round(res[n][-1], 1)}), flush=True)
    print(json.dumps({"summary": {n: {"median_mpps": round(sorted(v)[len(v) // 2], 1), "all": [round(x, 1) for x in v]}
                                  for n, v in res.items()}, "acl": a.acl, "batch": a.batch}), flush=True)


if __name__ == "__main__":
    main()
