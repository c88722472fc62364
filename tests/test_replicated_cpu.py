"""Multi-process (gloo, CPU) test of the replicated-table multi-GPU data plane: every rank holds
the full tables, runs the fused pipeline on its own ingress (CPU twin of the REMOTE kernel) and
ships frames for peer-owned pods in one all_to_all_single per chunk.  Every frame must come out
exactly as a single-process oracle produces it, on the rank owning the egress pod, and the tx
counters of each rank must account for every frame delivered to its pods."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, chunks):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.ops import packets as P
    from dpu_operator_amd.parallel.replicated import ReplicatedDataPlane

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n_pods = 4 * world
        pod_gpu = np.arange(n_pods) // 4
        dp = DataPlane("cpu", flow_buckets=1 << 14)
        sc = S.build_sfc(dp, n_pods=n_pods, n_flows=20000, n_acl=32, pod_gpu=pod_gpu)
        dp.commit(full=True)
        pk, im = S.traffic(sc, 3000, seed=10 + rank, src_pods=np.where(pod_gpu == rank)[0])
        eng = ReplicatedDataPlane(dp, rank, world, 3000, chunks=chunks, record_rx=True)
        eng.step(torch.from_numpy(pk), torch.from_numpy(im.view(np.int32)))
        meta = eng.out_meta()
        outs = eng.outputs()
        rs = P.meta_fields(meta)[2]
        ref = DataPlane("cpu", flow_buckets=1 << 14)
        S.build_sfc(ref, n_pods=n_pods, n_flows=20000, n_acl=32, pod_gpu=pod_gpu)
        ref.commit(full=True)
        rr = ref.run(pk, im)
        rrs = P.meta_fields(rr.meta)[2]
        ok = bool(((rs == 10) | (rs == rrs)).all())
        loc = rs == 0
        ok &= bool(np.array_equal(outs[loc], rr.out[loc]))
        rx, rx_meta = eng.received()
        objs = [None] * world
        dist.all_gather_object(objs, rx.tobytes())
        allrx = b"".join(objs)
        got = {allrx[i * 64:(i + 1) * 64] for i in range(len(allrx) // 64)}
        rem = np.where(rs == 10)[0]
        ok &= len(rem) > 0 and all(rr.out[i].tobytes() in got for i in rem)
        # every received frame's egress port belongs to this rank
        ok &= bool(all(dp.ports.a[int(m) & 0xFFFF]["gpu"] == rank for m in rx_meta))
        # tx accounting: local egress + frames received from peers
        tx = dp.port_counters()[:, 2].sum()
        ok &= int(tx) == int(loc.sum()) + len(rx_meta)
        q.put((rank, ok, int((rs == 10).sum()), int(loc.sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 4)])
def test_replicated_gloo(world, chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res
    assert all(p.exitcode == 0 for p in procs)
