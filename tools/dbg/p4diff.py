import sys, numpy as np, torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_dataplane_gpu import _p4_plane, _p4_traffic
from dpu_operator_amd.ops import packets as P
cpu, sc, vfs = _p4_plane("cpu")
gpu, _, _ = _p4_plane("cuda")
pk, im = _p4_traffic(sc, vfs)
rc = cpu.run(pk, im)
rg = gpu.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
torch.cuda.synchronize()
og = rg.out.cpu().numpy()
bad = np.where((og != rc.out).any(1))[0]
print("nbad", len(bad), "of", len(pk))
for i in bad[:6]:
    print(i, P.meta_fields(rc.meta[i:i+1]), "in", pk[i][:20].tobytes().hex())
    print(" cpu", rc.out[i].tobytes().hex())
    print(" gpu", og[i].tobytes().hex())
print("side cpu", cpu.side_result()["n_rep"], "gpu", gpu.side_result()["n_rep"])
