"""Debug: mismatch pattern of the fused kernel vs the oracle on the small bit-exact test traffic.

python tools/dbg/spill_diff.py [hash_mode] [acl_mode]
Prints which slots (lane = slot % 64, slot % 4), which byte columns and which values differ.
"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_dataplane_gpu import _build, _traffic  # noqa: E402

hm = sys.argv[1] if len(sys.argv) > 1 else "lds"
am = sys.argv[2] if len(sys.argv) > 2 else "mfma"
cpu, sc = _build("cpu")
pk, im = _traffic(sc)
rc = cpu.run(pk, im)
g, _ = _build("cuda", hm, am)
for trial in range(3):
    r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    go = r.out.cpu().numpy()
    gm = r.meta.cpu().numpy().view(np.uint32)
    d = np.nonzero((go != rc.out).any(axis=1))[0]
    print(f"trial {trial}: {len(d)} of {len(go)} slots differ; meta differ {(gm != rc.meta).sum()}", flush=True)
    if not len(d):
        continue
    lanes = d % 64
    print("  lane histogram (mod 4):", np.bincount(lanes % 4, minlength=4).tolist())
    print("  lanes:", np.unique(lanes).tolist()[:64])
    print("  slots:", d[:16].tolist())
    cols = np.nonzero((go[d] != rc.out[d]).any(axis=0))[0]
    print("  byte columns:", cols.tolist())
    for i in d[:4].tolist():
        w = go[i].view(np.uint32)
        c = rc.out[i].view(np.uint32)
        dw = np.nonzero(w != c)[0]
        print(f"  slot {i}: dwords {dw.tolist()} gpu {[hex(x) for x in w[dw]]} cpu {[hex(x) for x in c[dw]]}"
              f" meta {hex(int(rc.meta[i]))}")
