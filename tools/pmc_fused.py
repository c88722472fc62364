"""Minimal driver for PMC passes: the bench's 1-GPU config (1M flows, 256 ACL rules, 4M-packet
batches), 3 fused-kernel launches, nothing else on the GPU worth counting."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402

import os

ACL = int(os.environ.get("PMC_ACL", "256"))        # rule count
FLAGS = int(os.environ.get("PMC_FLAGS", "0"))      # launch flags (kernels.hip: 256 = no early fetch)
dp = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=min(ACL, 256), seed=0)
if ACL > 256:
    S.add_acl_rules(dp, ACL)
if os.environ.get("PMC_WILD"):   # the bench's ClassBench-style set instead (acl_wild variant)
    S.install_acl_wild(dp, 1024)
dp.commit(full=True)
pk, im = S.traffic(sc, 1 << 22, seed=1)
pk, im = torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()
out, meta, lat = dp.alloc_batch(1 << 22)
for _ in range(3):
    dp.run(pk, im, out, meta, lat, flags=FLAGS)
torch.cuda.synchronize()
print("done")
