"""Debug: which rows / byte positions of the P4-feature trace differ between the GPU kernel
(whatever NFDP_EXT_DIR selects) and the oracle."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_dataplane_gpu as T  # noqa: E402

cpu, sc, vfs = T._p4_plane("cpu")
gpu, _, _ = T._p4_plane("cuda")
pk, im = T._p4_traffic(sc, vfs)
rc = cpu.run(pk, im)
rg = gpu.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
torch.cuda.synchronize()
og = rg.out.cpu().numpy()
bad = np.nonzero((og != rc.out).any(axis=1))[0]
print("rows differ:", len(bad), "of", len(og))
if len(bad):
    cols = np.nonzero((og[bad] != rc.out[bad]).any(axis=0))[0]
    print("byte columns:", cols.tolist())
    print("rows mod 64:", np.bincount(bad % 64, minlength=64).tolist())
    print("rows // 1024 (block):", np.bincount(bad // 1024).tolist())
    for r in bad[:4]:
        print(r, "in ", pk[r].tobytes().hex())
        print(r, "cpu", rc.out[r].tobytes().hex())
        print(r, "gpu", og[r].tobytes().hex())
print("side cpu", cpu.side_result()["n_rep"], "gpu", gpu.side_result()["n_rep"])
