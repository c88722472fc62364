"""GPU vs oracle on the bench's IPv6 variant tables (1M IPv4 flows, 1024 IPv4 rules -> the EARLY
instances, 64K IPv6 flows, 64 IPv6 rules): disposition histograms per instance choice."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.ops import packets as P  # noqa: E402


def build(dev):
    dp = DataPlane(device=dev, flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
    dp.commit(full=True)
    S.add_acl_rules(dp, 1024)
    dp.commit()
    info6 = S.install_ipv6(dp, sc, 1 << 16, 64)
    dp.commit()
    return dp, sc, info6


g, sc, info6 = build("cuda:0")
c, _, _ = build("cpu")
pk6, im6 = S.traffic_ipv6(sc, info6, 1 << 16, seed=9300)
rc = c.run(pk6, im6)
for name, flags in (("default", 0), ("no_early", 1 << 8)):
    r = g.run(torch.from_numpy(pk6).cuda(), torch.from_numpy(im6.view(np.int32)).cuda(), flags=flags)
    torch.cuda.synchronize()
    m = r.meta.cpu().numpy().view(np.uint32)
    rs = P.meta_fields(m)[2]
    print(name, "tiles", g._acl_tiles, dict(zip(*[x.tolist() for x in np.unique(rs, return_counts=True)])),
          "equal_meta", bool(np.array_equal(m, rc.meta)), "equal_out", bool(np.array_equal(r.out.cpu().numpy(), rc.out)),
          flush=True)
print("oracle", dict(zip(*[x.tolist() for x in np.unique(P.meta_fields(rc.meta)[2], return_counts=True)])))
