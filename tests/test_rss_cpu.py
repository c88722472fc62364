"""Multi-process (gloo, CPU) test of the flow-affine (RSS) sharded data plane.

Every rank holds ONLY the flows whose Toeplitz hash it owns; its ingress is host-RSS-steered
traffic plus a fraction of misdirected packets.  Misdirected packets must leave the ingress rank
unprocessed (reason `remote`) and come out of their OWNER exactly as a single-table oracle
produces them; every other packet must match the oracle on its ingress rank.  Also checks the
pipelined step (exchange of step k processed during step k+1) over several steps."""
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


def _worker(rank, world, port, q, steps, frac, flush_each=True):
    import sys

    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.ops import packets as P
    from dpu_operator_amd.parallel.rss import RssShardedDataPlane, flow_owner, rss_traffic
    from dpu_operator_amd.parallel.sharded import shard_filter

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dp = DataPlane("cpu", flow_buckets=1 << 13)
        sc = S.build_sfc(dp, n_pods=8, n_flows=20000, n_acl=32, flow_filter=shard_filter(rank, world))
        dp.commit(full=True)
        ref = DataPlane("cpu", flow_buckets=1 << 14)
        S.build_sfc(ref, n_pods=8, n_flows=20000, n_acl=32)
        ref.commit(full=True)
        owner = flow_owner(sc.keys, world, dp.flows.rss_key)
        assert len(dp.flows) == int((owner == rank).sum())
        eng = RssShardedDataPlane(dp, rank, world, 2000, remote_frac=frac)
        ok, n_remote, n_rx = True, 0, 0
        for k in range(steps):
            pk, im = rss_traffic(sc, 2000, rank, world, owner, frac, seed=100 * k + rank)
            eng.step(torch.from_numpy(pk), torch.from_numpy(im.view(np.int32)))
            meta = eng.out_meta()
            rs = P.meta_fields(meta)[2]
            rr = ref.run(pk, im)
            loc = rs != 10
            n_remote += int((~loc).sum())
            ok &= bool(np.array_equal(meta[loc], rr.meta[loc]))
            ok &= bool(np.array_equal(eng.outputs()[loc], rr.out[loc]))
            if not flush_each:
                continue      # pipelined: exchanges complete `lag` steps later (checked by the totals below)
            # what this rank sent must come out of the owners as the oracle says
            sent = {pk[i].tobytes(): (rr.out[i].tobytes(), int(rr.meta[i])) for i in np.where(~loc)[0]}
            objs = [None] * world
            dist.all_gather_object(objs, sent)
            expect = {}
            for o in objs:
                expect.update(o)
            eng.flush()
            rin, rout, rmeta = eng.received()
            n_rx += len(rin)
            for a, b, m in zip(rin, rout, rmeta):
                e = expect.get(a.tobytes())
                ok &= e is not None and e == (b.tobytes(), int(m))
        ok &= "overflow" not in dp.drop_counters()          # nothing dropped for lack of room
        if not flush_each:
            eng.flush()
            n_rx = eng.stats["received"]
            ok &= eng.stats["sent"] == n_remote
        q.put((rank, ok, n_remote, n_rx))
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, False, repr(ex), 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,frac", [(2, 0.2), (3, 0.1), (4, 0.05), (8, 0.05),
                                        # loss-free at any misdirected fraction (count-first exchange):
                                        # half the traffic, and a producer that does not steer at all
                                        (2, 0.5), (3, 2 / 3), (4, 0.75)])
def test_rss_gloo(world, frac):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, 3, frac)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res
    assert sum(r[2] for r in res) == sum(r[3] for r in res) > 0  # every misdirected packet processed once


def test_rss_gloo_pipelined_lagged_exchange():
    """Six steps with no flush in between: each step's exchange completes `lag` (2) steps later
    (the host never waits for fresh counts); every misdirected packet still reaches its owner."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, 6, 0.1, False)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res
    assert sum(r[2] for r in res) == sum(r[3] for r in res) > 0


def test_bench_exchange_block_matches_the_protocol():
    """bench.py's `exchange` block (what the driver's multi-GPU runs print) carries the protocol
    facts tests/test_multigpu.py asserts: two collective launches per step, every key present."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    info = bench.rss_exchange_info(0.002, 4096.0, 700, 0.01, 2)
    assert set(info) == set(bench.RSS_EXCHANGE_KEYS)
    assert info["a2a_per_step"] == bench.RSS_A2A_PER_STEP == 2
    assert info["xgmi_bytes_out_per_gpu_per_step"] == 4096 * 68 and info["host_lag_steps"] == 2


def test_bench_unsteered_block_keys():
    """bench.py's exchange-bound variant at N > 1 (`unsteered`: (N-1)/N of every batch crosses
    xGMI): the block's keys and arithmetic.  The loss-free exchange at those fractions is
    test_rss_gloo's (3, 2/3) and (4, 3/4) cases; the GPU run asserts the same keys
    (tests/test_multigpu.py::test_bench_rss_two_gpus)."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    u = bench.rss_unsteered_info(0.010, 10, 4, 1 << 20, 786432.0, 1.0)
    assert set(u) == set(bench.RSS_UNSTEERED_KEYS)
    assert u["remote_frac"] == 0.75 and u["ms_per_step"] == 1.0
    assert u["mpps"] == round(4 * (1 << 20) / 1e-3 / 1e6, 2) and u["mpps_per_gpu"] * 4 == pytest.approx(u["mpps"], rel=1e-3)
    assert u["xgmi_bytes_out_per_gpu_per_step"] == 786432 * 68
