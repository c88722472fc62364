"""Single-GPU cost probe of one rank's RSS (flow-affine) multi-GPU step vs the 1-GPU fused kernel.

Builds rank 0 of a W-GPU layout exactly as bench.py --mode rss does (1M flows per shard, the
rank's shard only, host-RSS-steered traffic with --remote-frac 1 % misdirected) and times with
HIP events, on the same batch: the plain fused kernel (what N = 1 runs) and the per-step kernels
of the RSS engine (steering pass over the batch + the fused kernel on the gathered packets,
with the rank's own send segments standing in for what peers sent).  The xGMI all-to-all itself
needs real peers; bench.py measures it at N > 1.
"""
from __future__ import annotations

import json
import math
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.parallel.rss import RssShardedDataPlane, flow_owner, rss_traffic  # noqa: E402
from dpu_operator_amd.ops import packets as P  # noqa: E402
from dpu_operator_amd.parallel.sharded import shard_filter  # noqa: E402


def _time(fn, iters: int) -> float:
    """ms per call, device-wide (the RSS engine's rx pass runs on its own stream)."""
    import time

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / iters


def probe(world: int, batch: int, flows: int, frac: float, iters: int = 30) -> dict:
    dev = torch.device("cuda", 0)
    buckets = 1 << max(10, int(math.ceil(math.log2(flows / 2))))
    dp = DataPlane(device="cuda:0", flow_buckets=buckets, hash_mode="lds", acl_mode="mfma")
    n_pods = 8 * world
    pod_gpu = np.arange(n_pods) // 8
    sc = S.build_sfc(dp, n_pods=n_pods, n_flows=flows * world, n_acl=256, seed=0, pod_gpu=pod_gpu,
                     flow_filter=shard_filter(0, world))
    dp.commit(full=True)
    owner = flow_owner(sc.keys, world, dp.flows.rss_key)
    pk, im = rss_traffic(sc, batch, 0, world, owner, frac, seed=1)
    pk, im = torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev)
    out, meta, lat = dp.alloc_batch(batch)
    fused_ms = _time(lambda: dp.run(pk, im, out, meta, lat), iters)
    res = {"world": world, "batch": batch, "fused_ms": round(fused_ms, 4)}
    eng = RssShardedDataPlane(dp, 0, world, batch, remote_frac=frac)
    s = eng.slots[0]
    steer_ms = _time(lambda: eng._local(s, pk, im, batch), iters)
    if eng.use_list:   # the LIST fused kernel alone (steer_kernel skipped), then restore
        real = eng.nf

        class _NoSteer:
            def __getattr__(self, k):
                return (lambda *a, **kw: None) if k == "launch_steer" else getattr(real, k)

        eng.nf = _NoSteer()
        res["list_kernel_ms"] = round(_time(lambda: eng._local(s, pk, im, batch), iters), 4)
        eng.nf = real
        eng._local(s, pk, im, batch)
        torch.cuda.synchronize()
    cnt = s.pcnt.cpu().numpy().copy()
    s.recv.copy_(s.send)            # rank 0 "receives" what it sent its peers (timing only)
    s.recv.view(world, eng.pseg)[:, :4].view(torch.int32)[:, 0].copy_(s.pcnt)
    eng.hcnt[1].copy_(s.pcnt.cpu())
    rx_ms = _time(lambda: eng._receive(s), iters)
    _, _, rs = P.meta_fields(eng.out_meta_t.cpu().numpy().view(np.uint32)[:batch])
    # the engine's step sequence (exchange stood in by the prepared receive segments): local pass
    # of step k on the compute stream, rx pass of step k - 1 on the rx stream
    s2 = eng.slots[1]
    s2.recv.copy_(s.recv)
    kk = [0]

    def pipe():
        k = kk[0]
        eng._local(eng.slots[k & 1], pk, im, batch)
        eng._receive(eng.slots[(k + 1) & 1])
        kk[0] += 1

    step_ms = _time(pipe, iters)
    res.update(rss_local_ms=round(steer_ms, 4), rss_rx_ms=round(rx_ms, 4), list_mode=eng.use_list,
               steered_fraction=round(float(np.mean(rs == 10)), 4), segment_counts=cnt.tolist(),
               per_gpu_vs_1gpu_serial=round(fused_ms / (steer_ms + rx_ms), 3),
               rss_step_ms=round(step_ms, 4), per_gpu_vs_1gpu=round(fused_ms / step_ms, 3))
    return res


def main() -> None:
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 22
    for w in (2, 8):
        print(json.dumps(probe(w, batch, 1 << 20, 0.01)), flush=True)


if __name__ == "__main__":
    main()
