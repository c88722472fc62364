"""Ring latency attribution: the bench's coop-ring probe (64-packet chunks, one in flight) on the
headline tables, 3 trials of 4000 chunks, p50 / p99 of the host-clock round trip."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, ".")
import dpu_operator_amd  # noqa: F401,E402
import torch  # noqa: E402

from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.dataplane.ring import RingPath  # noqa: E402

dp = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
dp.commit(full=True)
pk, im = S.traffic(sc, 1 << 16, seed=1)
pk_t = torch.from_numpy(pk).cuda()
im_t = torch.from_numpy(im.view(np.int32)).cuda()
out = {"variant": os.environ.get("NFDP_EXT_DIR", "base").rsplit("/", 1)[-1], "p50": [], "p99": []}
for trial in range(3):
    rp = RingPath(dp, capacity=1 << 16, deadline_s=60.0, coop=True)
    rp.stage(pk_t, im_t)
    rp.start()
    lat, _ = rp.probe(batches=4000, batch=64, inflight=1)
    rp.stop()
    rp.close()
    lat = np.asarray(lat)[400:]
    out["p50"].append(round(float(np.percentile(lat, 50)), 2))
    out["p99"].append(round(float(np.percentile(lat, 99)), 2))
print(json.dumps(out), flush=True)
