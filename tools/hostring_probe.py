"""Persistent ring with zero-copy HOST slots vs device slots: latency (64-packet chunks, one in
flight) and loaded throughput (4096-packet chunks, 32 in flight), 1M-flow SFC, 1 GPU.
python tools/hostring_probe.py"""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.dataplane.ring import RingPath  # noqa: E402

dp = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
dp.commit(full=True)
pk, im = S.traffic(sc, 1 << 17, seed=1)
pk, im = torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()
for host in (False, True):
    out = {"host_slots": host}
    r = RingPath(dp, capacity=1 << 16, deadline_s=60.0, coop=True, host_slots=host)
    r.stage(pk[: 1 << 16], im[: 1 << 16])
    r.start()
    lat, _ = r.probe(batches=2000, batch=64, inflight=1)
    r.stop()
    r.close()
    out["p50_us"] = round(float(np.median(lat[200:])), 2)
    out["p99_us"] = round(float(np.percentile(lat[200:], 99)), 2)
    q = RingPath(dp, capacity=1 << 17, wgs_per_cu=2, deadline_s=60.0, coop=False, host_slots=host)
    q.stage(pk, im)
    q.start()
    lat2, el2 = q.probe(batches=1000, batch=4096, inflight=32)
    q.stop()
    q.close()
    out["loaded_mpps"] = round(1000 * 4096 / el2 / 1e6, 1)
    out["loaded_p50_us"] = round(float(np.median(lat2[100:])), 2)
    print(json.dumps(out), flush=True)
