"""Kernel-level cost of bench.py's value_vxlan step (run under rocprofv3 --kernel-trace --stats):
the headline data plane + a VTEP port, 2M VXLAN frames (4M slots) per step, fresh copies."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
sys.path.insert(0, __import__("os").environ.get("GRAFT_REPO_ROOT", "."))
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402

dev = torch.device("cuda", 0)
dp = DataPlane(device="cuda:0", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
egress = len(sys.argv) > 1 and sys.argv[1] == "egress"
if egress:   # the headline's traffic leaving encapsulated (every packet on the side list)
    S.install_vxlan_egress(dp, sc)
    dp.commit(full=True)
    pk, im = S.traffic(sc, 1 << 22, seed=1)
else:
    ports = S.install_vxlan(dp, sc)
    dp.commit(full=True)
    pk, im, _ = S.traffic_vxlan(sc, ports, 1 << 21, seed=1)
src = (torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev))
work = [(src[0].clone(), src[1].clone()) for _ in range(12)]
out, meta, lat = dp.alloc_batch(1 << 22)
for k in range(2):
    dp.run(*work[k], out, meta, lat)
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(2, 12):
    dp.run(*work[k], out, meta, lat)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / 10
nf = (1 << 22) if egress else (1 << 21)
print({"mode": "egress" if egress else "terminate", "ms_per_step": round(el * 1e3, 4), "frames": nf,
       "mpps": round(nf / el / 1e6, 1), "side": {k: v for k, v in dp.side_result().items() if k.startswith("n_")}}, flush=True)
