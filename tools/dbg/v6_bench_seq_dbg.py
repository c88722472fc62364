"""bench.py's variant sequence on a smaller batch, then the IPv6 traffic's dispositions."""
import sys
import types

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.ops import packets as P  # noqa: E402

dev = torch.device("cuda", 0)
dp = DataPlane(device="cuda:0", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
dp.commit(full=True)
a = types.SimpleNamespace(batch=1 << 20, variant_steps=3)
res = bench.measure_variants(a, dp, sc, dev, torch, S, P)
print({k: v for k, v in res.items() if k != "imix"}, flush=True)
info6 = {"src": None}
rng = np.random.default_rng(0)
# the v6 flows install_ipv6 made (same seed): regenerate the traffic from its return value
from dpu_operator_amd.dataplane import tables as T  # noqa: E402
print("flow6_on", dp._flow6_on, "full", dp._flow6_full, "n6", len(dp.flows6), "rules6", len(dp.acl.rules6),
      "tables", {k: v for k, v in dp.tables_ptrs().items() if k in ("flow6_on", "n_acl6", "acl6_tiles", "n_acl")}, flush=True)
