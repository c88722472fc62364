"""SFC hop pipeline across GPUs: chains whose hops are placed on different GPU planes (kHopXfer).

A split chain (``"ttl@1"``: the rest of the chain runs on plane 1) must give exactly what the same
chain gives on one plane: every out slot and meta word, the port counters summed over the planes,
the drop counters (less the REMOTE hand-off count) and the flow counters.  CPU: the oracle planes
(csrc/nfdp/host.cpp oracle_run / oracle_resume).  The GPU twin (XFER fused instances, peer-store
hand-off, resume_kernel) is tests/test_hop_pipeline_gpu.py.

Reference: the Marvell VSP realises an SFC as hops across NF ports
(/root/reference/internal/daemon/vendor-specific-plugins/marvell/main.go:490-563); here each hop
may sit on its own GPU and the frame's header slot + state cross xGMI between them.
"""
import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.multi import MultiDataPlane

REMOTE = 10


def _program(dp, hops, n_flows=4096, vlan_every=3, seed=0):
    sc = S.build_sfc(dp, n_pods=8, n_flows=n_flows, n_acl=64, hops=hops, seed=seed, install_flows=False)
    act = sc.actions.copy()
    # some flows push a vlan, some pop, the rest leave it (exercises the vlan hop and its replay)
    v = np.zeros(len(act), np.uint32)
    v[::vlan_every] = 100 + (np.arange(len(act))[::vlan_every] % 50)
    v[1::vlan_every * 2] = 0xFFFF
    act[:, 2] = (act[:, 2] & 0xFFFF) | (v << 16)
    dp.flows.insert_many(sc.keys, act)
    return sc


def _traffic(dp, sc, n=6000, seed=3):
    deny = S.install_deny_flows(dp, sc, k=256, seed=seed)
    return S.traffic_mixed(sc, deny, n, seed=seed, miss=0.05, deny_frac=0.05)


def _pair(split_hops, whole_hops, placement="flow", planes=2, **kw):
    one = DataPlane(device="cpu")
    multi = MultiDataPlane(["cpu"] * planes, placement=placement)
    s1 = _program(one, whole_hops, **kw)
    s2 = _program(multi, split_hops, **kw)
    one.commit()
    multi.commit()
    return one, multi, s1, s2


def _check(one, multi, sc, n=6000, seed=3):
    pk, im = _traffic(one, sc, n, seed)
    _traffic(multi, sc, n, seed)   # (same deny flows, same seed: identical tables)
    multi.commit()
    one.commit()
    r1 = one.run(pk, im)
    r2 = multi.run(pk, im)
    m1, m2 = np.asarray(r1.meta, np.uint32), np.asarray(r2.meta, np.uint32)
    assert r2.extra["handoff_rounds"] >= 1
    assert not ((m2 >> 26) & 0xF == REMOTE).any(), "a hand-off was left unresolved"
    np.testing.assert_array_equal(m1, m2)
    fwd = ((m1 >> 26) & 0xF) == 0
    assert fwd.sum() > n // 2
    np.testing.assert_array_equal(np.asarray(r1.out)[fwd], np.asarray(r2.out)[fwd])
    np.testing.assert_array_equal(one.port_counters(), multi.port_counters())
    d1, d2 = one.drop_counters(), multi.drop_counters()
    d2.pop("remote", None)
    assert d1 == d2
    for f in range(0, len(sc.keys), 97):
        assert one.flow_counters(sc.keys[f]) == multi.flow_counters(sc.keys[f])
    return m2


def test_expand_hops():
    assert T.expand_hops(["acl", "nat", "ttl@1", "l2fwd@1"]) == [1, 2, 0x11, 4, 3]
    assert T.expand_hops(["acl", "@1", "nat", "@2", "ttl"]) == [1, 0x11, 2, 0x12, 4]
    # a route hop before a hand-off: its egress port travels with the frame (hop_resume_word)
    assert T.expand_hops(["route", "ttl@1"]) == [T.HOP_ROUTE, 0x11, 4]
    with pytest.raises(ValueError):
        T.expand_hops(["ttl@16"])
    c = T.ChainTable()
    c.add(["acl", "nat"])
    assert not c.split()
    c.add(["acl", "nat@2", "ttl@3"])
    assert c.split() and c.xfer_planes() == {2, 3}
    with pytest.raises(ValueError):   # 4 hops + 4 hand-offs
        c.add(["acl@1", "nat@2", "ttl@3", "l2fwd@4"])


@pytest.mark.parametrize("placement", ["flow", "port"])
def test_split_chain_matches_one_plane(placement):
    one, multi, sc, _ = _pair(("acl", "nat", "ttl@1", "l2fwd@1"), ("acl", "nat", "ttl", "l2fwd"), placement)
    m = _check(one, multi, sc)
    # every frame of the chain that passed the ACL was handed over once (counted where it left)
    fwd = ((m >> 26) & 0xF) == 0
    assert multi.drop_counters()["remote"] >= fwd.sum()


def test_three_segment_chain_with_vlan_replay():
    """acl, vlan on plane 0 -> nat, ttl on plane 1 -> l2fwd back on plane 0: the vlan push / pop
    decided on plane 0 is applied at the very end (its replay), the frame crosses twice."""
    one, multi, sc, _ = _pair(("acl", "vlan", "nat@1", "ttl@1", "l2fwd@0"), ("acl", "vlan", "nat", "ttl", "l2fwd"))
    _check(one, multi, sc)


def test_acl_and_vlan_after_the_split():
    """The ACL verdict (classified on the first plane over the ingress key) travels in the record."""
    one, multi, sc, _ = _pair(("nat", "ttl@1", "acl@1", "vlan@1", "l2fwd@1"), ("nat", "ttl", "acl", "vlan", "l2fwd"))
    _check(one, multi, sc)


def test_hairpin_before_the_split():
    one, multi, sc, _ = _pair(("hairpin", "ttl@1"), ("hairpin", "ttl"))
    _check(one, multi, sc)


def test_route_before_the_split():
    """acl, nat, route on plane 0 -> ttl, then back for nothing: the routed egress port (ECMP over
    the rewritten header) crosses with the frame instead of being recomputed on plane 1."""
    one, multi, sc, _ = _pair(("acl", "nat", "route", "ttl@1"), ("acl", "nat", "route", "ttl"))
    for dp in (one, multi):
        S.install_l3_routes(dp, sc, n_background=2000)
    one.chains.set(sc.chain_id, ["acl", "nat", "route", "ttl"])
    multi.chains.set(sc.chain_id, ["acl", "nat", "route", "ttl@1"])
    m = _check(one, multi, sc)
    fwd = ((m >> 26) & 0xF) == 0
    assert multi.drop_counters()["remote"] >= fwd.sum()


def test_four_planes_relay():
    one, multi, sc, _ = _pair(("acl", "nat@1", "ttl@2", "l2fwd@3"), ("acl", "nat", "ttl", "l2fwd"), planes=4)
    _check(one, multi, sc)


def test_hop_on_a_missing_gpu_is_dropped():
    one, multi, sc, _ = _pair(("acl", "nat@5", "l2fwd@5"), ("acl", "nat", "l2fwd"))
    pk, im = S.traffic(sc, 500, seed=9)
    r = multi.run(pk, im)
    m = np.asarray(r.meta, np.uint32)
    assert (((m >> 26) & 0xF) == 1).all()   # bad_port: plane 5 does not exist


def test_resume_record_layout():
    """The oracle's HopState record: in_port | len << 16, hash, acl rule, resume hop, action."""
    dp = DataPlane(device="cpu")
    sc = S.build_sfc(dp, n_pods=4, n_flows=64, n_acl=8, hops=("acl", "nat@1", "l2fwd@1"))
    dp.commit()
    pk, im = S.traffic(sc, 32, seed=1)
    r = dp.run(pk, im)
    m = np.asarray(r.meta, np.uint32)
    assert (((m >> 26) & 0xF) == REMOTE).all() and ((m & 0xFFF) == 1).all()
    hs = r.extra["hop_state"]
    assert ((hs[:, 0] & 0xFFFF) == (im & 0xFFFF)).all()
    assert ((hs[:, 0] >> 16) == ((m >> 12) & 0x3FFF)).all()   # the frame length, untagged
    np.testing.assert_array_equal(hs[:, 1], r.extra["hash"])
    np.testing.assert_array_equal(hs[:, 2].view(np.int32), r.extra["acl"])
    assert (hs[:, 3] & 0xFF == 2).all()   # acl, xfer -> resumes at hop 2 (nat)
    # the egress port decided before the hand-off (bit 15: present): here the flow's own port
    assert (hs[:, 3] & 0x8000 != 0).all()
    assert ((hs[:, 3] >> 16) == (hs[:, 4] >> 16)).all()
    assert (hs[:, 4] & 0xFFFF == sc.chain_id).all()


def test_vsp_places_gpu_nf_hops_on_gpus(tmp_path):
    """gpu-nf://ttl@1 through the VSP: a split chain on a 2-GPU node, refused on a GPU it lacks."""
    from dpu_operator_amd.utils.paths import PathManager
    from dpu_operator_amd.cni.netlink import FakeNetlink
    from dpu_operator_amd.vsp.gpu import GpuVsp

    vsp = GpuVsp(PathManager(str(tmp_path)), device="cpu", nl=FakeNetlink(), flow_buckets=1 << 8, gpus=2)
    cid = vsp.on_gpu_chain("sfc-a", ["acl", "nat", "ttl@1", "l2fwd@1"])
    assert vsp.dp.chains.split() and vsp.dp.chains.xfer_planes() == {1}
    assert list(vsp.dp.chains.a[cid]["hop"][:5]) == [1, 2, 0x11, 4, 3]
    with pytest.raises(ValueError):
        vsp.on_gpu_chain("sfc-b", ["acl", "ttl@2"])
