"""Single-GPU cost probe of the replicated multi-GPU step (fused REMOTE kernel + egress kernel).

Builds one rank of a W-GPU layout (full 1M-flow tables, 8 pods per GPU, traffic from this GPU's
pods to random pods) and times, with HIP events, the per-chunk kernels that run on each GPU:
fused REMOTE (classify + lookup + chain + write local / per-peer segments) and egress (count +
stamp what peers sent; here the rank's own send buffer stands in for the received one).  The
xGMI all-to-all itself needs real peers and is measured by bench.py at N > 1.
"""
from __future__ import annotations

import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.parallel.replicated import ReplicatedDataPlane  # noqa: E402


def probe(world: int, batch: int, flows: int, iters: int = 20) -> dict:
    dev = torch.device("cuda", 0)
    dp = DataPlane(device="cuda:0", flow_buckets=1 << int(np.ceil(np.log2(flows / 2))), hash_mode="lds",
                   acl_mode="mfma")
    n_pods = 8 * world
    pod_gpu = np.arange(n_pods) // 8
    sc = S.build_sfc(dp, n_pods=n_pods, n_flows=flows, n_acl=256, pod_gpu=pod_gpu)
    dp.commit(full=True)
    pk, im = S.traffic(sc, batch, seed=7, src_pods=np.where(pod_gpu == 0)[0])
    pk, im = torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev)
    eng = ReplicatedDataPlane(dp, 0, world, batch, chunks=1)
    s = eng.slots[0]
    for _ in range(3):
        eng._fused(s, 0, batch, pk, im)
        s.recv.copy_(s.send)
        eng._egress(s)
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    tf = te = 0.0
    for _ in range(iters):
        e0.record()
        eng._fused(s, 0, batch, pk, im)
        e1.record()
        s.recv.copy_(s.send)
        e2.record()
        eng._egress(s)
        e2.synchronize()
        tf += e0.elapsed_time(e1)
    # egress alone
    t0 = time.perf_counter()
    for _ in range(iters):
        eng._egress(s)
    torch.cuda.synchronize()
    te = (time.perf_counter() - t0) * 1e3 / iters
    fused_ms = tf / iters
    meta = eng.out_meta_t.cpu().numpy().view(np.uint32)[:batch]
    remote = float(np.mean(((meta >> 24) & 0x7F) == 10))
    return {"world": world, "batch": batch, "fused_remote_ms": round(fused_ms, 4), "egress_ms": round(te, 4),
            "gpps_fused": round(batch / fused_ms / 1e6, 3), "remote_fraction": round(remote, 4),
            "xgmi_bytes_per_step": int(remote * batch * 68)}


def main() -> None:
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    for w in (2, 4, 8):
        print(json.dumps(probe(w, batch, 1 << 20)), flush=True)


if __name__ == "__main__":
    main()
