"""Debug: where do GPU and oracle egress slots differ on the >2^24-slot batch?"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402

g = DataPlane(device="cuda", flow_buckets=1 << 12)
c = DataPlane(device="cpu", flow_buckets=1 << 12)
for dp in (g, c):
    sc = S.build_sfc(dp, n_pods=8, n_flows=4096, n_acl=64, seed=0)
    dp.commit(full=True)
pk1, im1 = S.traffic(sc, 1 << 20, seed=3)
for n in ((1 << 20), (1 << 24) + (1 << 16)):
    reps = n // len(pk1) + 1
    pk = np.tile(pk1, (reps, 1))[:n]
    im = np.tile(im1, reps)[:n]
    for trial in range(2):
        r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
        torch.cuda.synchronize()
        rc = c.run(pk, im)
        go = r.out.cpu().numpy()
        d = np.nonzero((go != rc.out).any(axis=1))[0]
        print(f"n={n} trial={trial}: {len(d)} rows differ", flush=True)
        if len(d):
            print("  first rows", d[:10].tolist(), "launch of each:", (d[:10] >> 24).tolist())
            cols = np.nonzero((go[d] != rc.out[d]).any(axis=0))[0]
            print("  differing byte columns", cols.tolist())
            i = int(d[0])
            print("  gpu", go[i].tolist())
            print("  cpu", rc.out[i].tolist())
            print("  in ", pk[i].tolist(), "im", hex(int(im[i])))
