"""The SFC fed through a VXLAN overlay (bench value_vxlan): frames arrive encapsulated on an
underlay VTEP port as wide header pairs, are terminated in one pass and run the chain (ACL ->
SNAT -> L2 steer) as received on the tunnel port.  Every head egresses to its flow's destination
pod, every continuation reports kCont; the GPU run (more slots than one grid-stride pass) matches
the oracle bit for bit."""
import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P


def _build(dev, flows=1 << 12):
    dp = DataPlane(device=dev, flow_buckets=max(1 << 10, flows // 2))
    sc = S.build_sfc(dp, n_pods=8, n_flows=flows, n_acl=64, seed=0)
    ports = S.install_vxlan(dp, sc)
    dp.commit(full=True)
    return dp, sc, ports


def test_vxlan_overlay_sfc_oracle():
    dp, sc, ports = _build("cpu")
    slots, im, f = S.traffic_vxlan(sc, ports, 512, seed=3)
    r = dp.run(slots, im)
    port, ln, rs = P.meta_fields(r.meta)
    assert (rs[0::2] == 0).all() and (rs[1::2] == 15).all()
    assert np.array_equal(port[0::2], sc.pod_port[sc.flow_dst_pod[f]])
    # the inner frame (60 B) leaves tagged with the destination pod's vlan and SNATed
    assert (ln[0::2] == 64).all()
    pc = dp.port_counters()
    assert int(pc[ports["vtep"], 0]) == 512 and int(pc[ports["tunnel"], 0]) == 512


@pytest.mark.gpu
def test_vxlan_overlay_sfc_gpu_bit_exact():
    import torch

    (g, sc, ports), (c, _, _) = _build("cuda", 1 << 16), _build("cpu", 1 << 16)
    slots, im, _ = S.traffic_vxlan(sc, ports, 1 << 19, seed=4)
    rc = c.run(slots, im)
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert np.array_equal(g.port_counters(), c.port_counters())


def _build_egress(dev, flows=1 << 12):
    dp = DataPlane(device=dev, flow_buckets=max(1 << 10, flows // 2))
    sc = S.build_sfc(dp, n_pods=8, n_flows=flows, n_acl=64, seed=0)
    S.install_vxlan_egress(dp, sc)
    dp.commit(full=True)
    return dp, sc


def test_vxlan_egress_every_packet_gets_an_outer_header_oracle():
    dp, sc = _build_egress("cpu")
    pk, im = S.traffic(sc, 512, seed=3)
    r = dp.run(pk, im)
    port, ln, rs = P.meta_fields(r.meta)
    assert (rs == 0).all() and P.meta_xhdr(r.meta).all()
    x = dp.side_result()["xhdr"]
    assert (x[:512, 12:14] == [0x08, 0x00]).all() and (x[:512, 46:49] == [0x00, 0x13, 0x88]).all()   # VNI 5000


@pytest.mark.gpu
def test_vxlan_egress_gpu_bit_exact():
    """Every packet of a 1M batch on the side list (outer-header records): the wave-aggregated
    side-list claim, the side pass, the records."""
    import torch

    (g, sc), (c, _) = _build_egress("cuda", 1 << 16), _build_egress("cpu", 1 << 16)
    pk, im = S.traffic(sc, 1 << 20, seed=4)
    rc = c.run(pk, im)
    xc = c.side_result()["xhdr"][: 1 << 20].copy()
    r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    sg = g.side_result()
    assert sg["side_dropped"] == 0 and sg["n_side"] == 1 << 20
    assert np.array_equal(sg["xhdr"][: 1 << 20], xc)
