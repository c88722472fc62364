"""IPv6 flows on a batch larger than one grid-stride pass (v6_kernel / V6 fused instances):
GPU vs oracle, which packet indices differ."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.ops import packets as P  # noqa: E402


def build(dev, n_acl):
    dp = DataPlane(device=dev, flow_buckets=1 << 16, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 16, n_acl=n_acl, seed=0)
    info6 = S.install_ipv6(dp, sc, 1 << 14, 64)
    dp.commit(full=True)
    return dp, sc, info6


for n_acl in (256, 1024):
    g, sc, info6 = build("cuda:0", n_acl)
    c, _, _ = build("cpu", n_acl)
    n = 1 << 20
    pk6, im6 = S.traffic_ipv6(sc, info6, n, seed=5)
    rc = c.run(pk6, im6)
    for name, flags in (("default", 0), ("no_early", 1 << 8)):
        r = g.run(torch.from_numpy(pk6).cuda(), torch.from_numpy(im6.view(np.int32)).cuda(), flags=flags)
        torch.cuda.synchronize()
        m = r.meta.cpu().numpy().view(np.uint32)
        bad = np.where(m != rc.meta)[0]
        print(n_acl, name, "tiles", g._acl_tiles, "mismatch", len(bad), "first", bad[:8].tolist(),
              "min", int(bad.min()) if len(bad) else -1, dict(zip(*[x.tolist() for x in np.unique(P.meta_fields(m)[2], return_counts=True)])),
              flush=True)
