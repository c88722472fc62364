"""SFC hop pipeline across GPUs on the GPU: split chains (kHopXfer) bit-exact with one plane.

Rehearsal on one MI355X: two (or three) data planes on cuda:0, each with its own tables, counters
and stream.  The hand-off is the real code path - the entry plane's XFER fused instance, then
hop_pack_kernel storing slot + HopState + index into the resuming plane's inbox, then
resume_kernel there - with the planes on different GPUs the same stores cross xGMI (peer access).
Checked against the same chain on one plane (GPU) and against the oracle (CPU).
"""
import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.multi import MultiDataPlane

pytestmark = pytest.mark.gpu
REMOTE = 10


def _program(dp, hops, n_flows=1 << 14, seed=0):
    sc = S.build_sfc(dp, n_pods=8, n_flows=n_flows, n_acl=200, hops=hops, seed=seed, install_flows=False)
    act = sc.actions.copy()
    v = np.zeros(len(act), np.uint32)
    v[::3] = 100 + (np.arange(len(act))[::3] % 50)
    v[1::6] = 0xFFFF
    act[:, 2] = (act[:, 2] & 0xFFFF) | (v << 16)
    dp.flows.insert_many(sc.keys, act)
    deny = S.install_deny_flows(dp, sc, k=512, seed=5)
    dp.commit()
    return sc, deny


def _compare(m1, o1, m2, o2):
    m1, m2 = np.asarray(m1, np.uint32), np.asarray(m2, np.uint32)
    assert not (((m2 >> 26) & 0xF) == REMOTE).any(), "a hand-off was left unresolved"
    np.testing.assert_array_equal(m1, m2)
    fwd = ((m1 >> 26) & 0xF) == 0
    assert fwd.mean() > 0.5
    o1, o2 = np.asarray(o1), np.asarray(o2)
    bad = np.nonzero(fwd & (o1 != o2).any(1))[0]
    for i in bad[:6]:   # (what differs, if anything: frame, meta, byte columns, values)
        cols = np.nonzero(o1[i] != o2[i])[0]
        print("frame", i, hex(int(m1[i])), "cols", cols.tolist(), o1[i][cols].tolist(), o2[i][cols].tolist())
    assert len(bad) == 0, f"{len(bad)} forwarded frames differ"


@pytest.mark.parametrize("hash_mode", ["mfma", "lds"])
@pytest.mark.parametrize("split,whole", [
    (("acl", "nat", "ttl@1", "l2fwd@1"), ("acl", "nat", "ttl", "l2fwd")),
    (("acl", "vlan", "nat@1", "ttl@1", "l2fwd@0"), ("acl", "vlan", "nat", "ttl", "l2fwd")),
])
def test_hop_pipeline_two_planes_on_one_gpu(hash_mode, split, whole):
    import torch

    from dpu_operator_amd.parallel.hops import HopPipeline

    one = DataPlane(device="cuda:0", hash_mode=hash_mode)
    sc, deny = _program(one, whole)
    multi = MultiDataPlane(["cuda:0", "cuda:0"], placement="port", hash_mode=hash_mode)
    _program(multi, split)
    orc = DataPlane(device="cpu")
    _program(orc, whole)
    n = 1 << 16
    pk, im = S.traffic_mixed(sc, deny, n, seed=7, miss=0.05, deny_frac=0.05)
    tpk, tim = torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()
    r1 = one.run(tpk, tim)
    torch.cuda.synchronize()
    m1, o1 = r1.meta.cpu().numpy().view(np.uint32), r1.out.cpu().numpy()
    ro = orc.run(pk, im)
    _compare(ro.meta, ro.out, m1, o1)   # (the whole chain: GPU == oracle)

    hp = HopPipeline(multi.planes, n)
    hp.step(tpk, tim)
    o2, m2 = hp.results(n)
    _compare(m1, o1, m2, o2)
    # counters: rx on the entry plane, tx where the chain ended - summed, the one plane's
    np.testing.assert_array_equal(one.port_counters(), multi.port_counters())
    d1, d2 = one.drop_counters(), multi.drop_counters()
    assert d2.pop("remote", 0) >= int((((m1 >> 26) & 0xF) == 0).sum())
    assert d1 == d2
    # a second batch through the same inboxes (the publish step reset the fill counters)
    hp.step(tpk, tim)
    o3, m3 = hp.results(n)
    _compare(m1, o1, m3, o3)


def test_route_before_the_split_on_gpu():
    """acl, nat, route on plane 0 -> ttl on plane 1 (the XFER instance, pack, resume_kernel): the
    routed egress port crosses in the resume word; bit-exact with the whole chain and the oracle."""
    import torch

    from dpu_operator_amd.parallel.hops import HopPipeline

    whole, split = ("acl", "nat", "route", "ttl"), ("acl", "nat", "route", "ttl@1")
    one = DataPlane(device="cuda:0")
    sc, deny = _program(one, whole)
    multi = MultiDataPlane(["cuda:0", "cuda:0"], placement="port")
    _program(multi, split)
    orc = DataPlane(device="cpu")
    _program(orc, whole)
    for dp, hops in ((one, whole), (multi, split), (orc, whole)):
        S.install_l3_routes(dp, sc, n_background=2000)
        dp.chains.set(sc.chain_id, list(hops))
        dp.commit()
    n = 1 << 16
    pk, im = S.traffic_mixed(sc, deny, n, seed=11, miss=0.05, deny_frac=0.05)
    tpk, tim = torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()
    r1 = one.run(tpk, tim)
    torch.cuda.synchronize()
    m1, o1 = r1.meta.cpu().numpy().view(np.uint32), r1.out.cpu().numpy()
    ro = orc.run(pk, im)
    _compare(ro.meta, ro.out, m1, o1)
    hp = HopPipeline(multi.planes, n)
    hp.step(tpk, tim)
    o2, m2 = hp.results(n)
    _compare(m1, o1, m2, o2)
    np.testing.assert_array_equal(one.port_counters(), multi.port_counters())


def test_multidataplane_run_resolves_handoffs_on_gpu():
    """The host-array API (MultiDataPlane.run): flow placement, frames enter on their owner plane
    and hand off device to device."""
    one = DataPlane(device="cuda:0")
    sc, deny = _program(one, ("acl", "nat", "ttl", "l2fwd"))
    multi = MultiDataPlane(["cuda:0", "cuda:0"], placement="flow")
    _program(multi, ("acl", "nat", "ttl@1", "l2fwd@1"))
    pk, im = S.traffic_mixed(sc, deny, 1 << 14, seed=9, miss=0.05, deny_frac=0.05)
    import torch

    r1 = one.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    r2 = multi.run(pk, im)
    assert r2.extra["handoff_rounds"] == 1
    _compare(r1.meta.cpu().numpy().view(np.uint32), r1.out.cpu().numpy(), r2.meta, r2.out)
    np.testing.assert_array_equal(one.port_counters(), multi.port_counters())


def test_hop_pipeline_back_to_back_steps_on_distinct_streams():
    """Consecutive steps reuse the inboxes: with each plane on its own stream (as on two GPUs), the
    next step's pack must wait for the previous step's resume over the same inbox.
    Four steps of alternating batches are queued without any host wait; the last step's frames and
    the summed counters must equal the one-plane chain run four times."""
    import torch

    from dpu_operator_amd.parallel.hops import HopPipeline

    one = DataPlane(device="cuda:0")
    sc, deny = _program(one, ("acl", "nat", "ttl", "l2fwd"))
    multi = MultiDataPlane(["cuda:0", "cuda:0"], placement="port")
    _program(multi, ("acl", "nat", "ttl@1", "l2fwd@1"))
    n = 1 << 16
    batches = []
    for s in range(2):
        pk, im = S.traffic_mixed(sc, deny, n, seed=20 + s, miss=0.05, deny_frac=0.05)
        batches.append((torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()))
    for k in range(4):
        r1 = one.run(*batches[k % 2])
    torch.cuda.synchronize()
    m1, o1 = r1.meta.cpu().numpy().view(np.uint32), r1.out.cpu().numpy()
    streams = [torch.cuda.Stream(device="cuda:0"), torch.cuda.Stream(device="cuda:0")]
    hp = HopPipeline(multi.planes, n, streams=streams)
    for k in range(4):
        hp.step(*batches[k % 2])
    o2, m2 = hp.results(n)
    _compare(m1, o1, m2, o2)
    np.testing.assert_array_equal(one.port_counters(), multi.port_counters())
    d1, d2 = one.drop_counters(), multi.drop_counters()
    d2.pop("remote", 0)
    assert d1 == d2
