"""The RSS engine's three streams (compute: local pass, comm: exchange, rx: gather + fused over
what peers sent) on one GPU, with the exchange stood in by a device copy on the comm stream: the
pipelined step sequence must give exactly what a serial run (synchronize after every stage)
gives, so the slot events order the reuse of the exchange slots and receive buffers correctly.
(The real exchange needs >= 2 GPUs: tests/test_multigpu.py.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine():
    import torch

    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.parallel.rss import RssShardedDataPlane, flow_owner, rss_traffic
    from dpu_operator_amd.parallel.sharded import shard_filter

    world, batch = 2, 1 << 16
    dp = DataPlane(device="cuda:0", flow_buckets=1 << 14, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=16, n_flows=1 << 15, n_acl=64, seed=0, pod_gpu=np.arange(16) // 8,
                     flow_filter=shard_filter(0, world))
    dp.commit(full=True)
    owner = flow_owner(sc.keys, world, dp.flows.rss_key)
    batches = []
    for k in range(4):
        pk, im = rss_traffic(sc, batch, 0, world, owner, 0.05, seed=10 + k)
        batches.append((torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()))
    eng = RssShardedDataPlane(dp, 0, world, batch, remote_frac=0.05)
    return eng, batches


def _fake_exchange(eng, serial):
    """Loopback exchange on the engine's streams ("peers sent" what this rank sent them): counts
    enqueued at the step, transfer completed `lag` steps later, as the real protocol does."""
    import torch

    def counts(s):
        cs = eng.comm
        with torch.cuda.stream(cs):
            cs.wait_event(s.ev)
            if s.used:
                cs.wait_event(s.rev)
            s.rcnt.copy_(s.pcnt)
            s.recv.copy_(s.send)
            s.recv.view(eng.world, eng.pseg)[:, :4].view(torch.int32)[:, 0].copy_(s.rcnt)
            eng.hcnt[s.idx][1].copy_(s.rcnt, non_blocking=True)
            s.hev.record(cs)

    def transfer(s):
        s.hev.synchronize()
        eng.stats["received"] += int(eng.hcnt[s.idx][1].sum())
        s.cev.record(eng.comm)
        if serial:
            torch.cuda.synchronize()
        return s
    return counts, transfer


def _run(serial):
    import torch

    eng, batches = _engine()
    eng._counts, eng._transfer = _fake_exchange(eng, serial)
    for k in range(8):
        eng.step(*batches[k % 4])
        if serial:
            torch.cuda.synchronize()
    eng.flush()
    eng.sync()
    pk, o, m = eng.received()
    # the steer list's order within a workgroup follows wave scheduling, so the received batch is
    # compared as a set of (input slot, egress slot, egress meta) rows
    rows = np.concatenate([pk.reshape(len(pk), -1), o.reshape(len(o), -1), m.view(np.uint8).reshape(len(m), 4)], axis=1)
    rows = rows[np.lexsort(rows.T[::-1])] if len(rows) else rows
    dp = eng.dp
    return (rows, eng.out_meta().copy(), eng.outputs().copy(), eng.harvest_flow_counters().copy(),
            dp.port_counters().copy(), dp.drop_counters(), eng.stats["received"])


def test_rss_pipelined_streams_match_serial():
    a = _run(serial=False)
    b = _run(serial=True)
    for x, y in zip(a[:5], b[:5]):
        assert np.array_equal(x, y)
    assert a[5] == b[5] and a[6] == b[6] and a[6] > 0 and len(a[0]) > 0
    assert int(a[3][:, 0].sum()) > 0
