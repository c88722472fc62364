"""All of a node's GPUs behind the VSP (vsp/gpu.py gpus=N, dataplane/multi.py, the native I/O
engine steering by RSS owner).  On CPU the planes are oracle planes, so the whole multi-GPU control
and data path runs here: SetNumVfs -> CreateBridgePort -> CreateNetworkFunction -> traffic through
shared-memory vports; results are compared with a single-plane data plane fed the same frames.
The GPU variant needs >= 2 MI355X and skips below."""
import shutil
import tempfile
import time
from pathlib import Path

import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.multi import MultiDataPlane
from dpu_operator_amd.dataplane.native_io import MemifVport, NativeLivePath, memif_dir
from dpu_operator_amd.native import nfdp
from dpu_operator_amd.ops import packets as P
from dpu_operator_amd.vsp.gpu import WIRE_PORT, GpuVsp


@pytest.fixture
def shm():
    d = Path(tempfile.mkdtemp(prefix="dpu-vspmg-", dir=memif_dir()))
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _until(fn, t=5.0):
    end = time.monotonic() + t
    while time.monotonic() < end:
        if fn():
            return True
        time.sleep(0.003)
    return bool(fn())


def _gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:  # noqa: BLE001
        return 0


@pytest.mark.parametrize("n", [2, 3])
def test_sharded_flows_match_one_plane(n):
    """Flows land on their owner only; a batch split by owner gives the single-plane result bit
    for bit, counters summed (ports) or read from the owner (flows)."""
    m = MultiDataPlane(["cpu"] * n, flow_buckets=1 << 12)
    sc = S.build_sfc(m, n_pods=6, n_flows=6000, n_acl=64, seed=0)
    m.commit(full=True)
    ref = DataPlane("cpu", flow_buckets=1 << 13)
    S.build_sfc(ref, n_pods=6, n_flows=6000, n_acl=64, seed=0)
    ref.commit(full=True)
    own = m.flows.owner(sc.keys)
    assert [len(p.flows) for p in m.planes] == [int((own == g).sum()) for g in range(n)]
    pk, im = S.traffic(sc, 4000, seed=2)
    r, rr = m.run(pk, im), ref.run(pk, im)
    assert np.array_equal(r.out, rr.out) and np.array_equal(r.meta, rr.meta)
    assert len(np.unique(r.extra["owner"])) == n
    assert np.array_equal(m.port_counters(), ref.port_counters())
    f = int(np.argmax(np.bincount(np.asarray(S.traffic(sc, 4000, seed=2, return_flows=True)[2]))))
    assert m.flow_counters(sc.keys[f]) == ref.flow_counters(sc.keys[f]) != (0, 0)


def test_engine_owner_matches_the_flow_shards(shm):
    """The native engine's ingress owner (iox.cpp frame_owner) is the owner the flow shards use."""
    nf = nfdp()
    m = MultiDataPlane(["cpu"] * 4, flow_buckets=1 << 12)
    sc = S.build_sfc(m, n_pods=4, n_flows=2000, n_acl=8, seed=1)
    m.commit(full=True)
    pk, im, f = S.traffic(sc, 500, seed=3, return_flows=True)
    assert np.array_equal(m.owners(pk, im), m.flows.owner(sc.keys[f]))
    eng = nf.IoEngine(64, 8, 1)
    for _ in range(4):
        eng.add_backend(nf.OracleBackend(256))
    eng.set_steering(np.ascontiguousarray(m.ports.a), bytes(m.flows.rss_key))
    assert [eng.owner_of_frame(bytes(pk[i]), int(im[i] & 0xFFFF)) for i in range(50)] == list(m.owners(pk, im)[:50])


def _vsp_multi(shm, n, device="cpu"):
    vsp = GpuVsp(device=device, gpus=n, live=True, vport_kind="memif", memif_dir=str(shm), flow_buckets=1 << 12,
                 tx_workers=2)
    vsp.init(True, "gpu")
    vsp.set_num_vfs(6)
    return vsp


def _pod_frame(src_mac, dst_mac, sport, n=1):
    fr, ln = P.craft(n, dmac=dst_mac, smac=src_mac, src_ip=0x0A000001, dst_ip=0x0A000002, sport=sport, dport=80)
    return [bytes(fr[i, : ln[i]]) for i in range(n)]


@pytest.mark.parametrize("n", [2, 3])
def test_vsp_multi_gpu_bridge_ports_and_network_function(shm, n):
    """VSP API on an N-plane data plane: two bridge ports talk L2 through the planes (frames of
    different flows spread over them), then a network function is inserted and pod traffic goes
    VF -> NF-in, NF-out -> wire as the reference's OvS rules would steer it."""
    nf = nfdp()
    vsp = _vsp_multi(shm, n)
    try:
        assert len(vsp.dp.planes) == n and vsp.live_engine == "native"
        macs = ["02:00:00:00:aa:01", "02:00:00:00:aa:02"]
        vsp.create_bridge_port("host0-0", bytes.fromhex(macs[0].replace(":", "")), 0, ["2"])
        vsp.create_bridge_port("host0-1", bytes.fromhex(macs[1].replace(":", "")), 0, ["3"])
        ep = {i: nf.MemifEndpoint(vsp.vport_path(i)) for i in range(6)}
        frames = [f for s in range(64) for f in _pod_frame(macs[0], macs[1], 1000 + s)]
        assert ep[0].send(frames) == len(frames)
        got = []
        assert _until(lambda: got.extend(ep[1].recv()) or len(got) >= len(frames)), vsp.livepath.stats
        assert sorted(got) == sorted(frames)                  # plain L2: delivered unchanged
        planes_used = sum(1 for p in vsp.dp.planes if p.port_counters()[0, 0] > 0)
        assert planes_used == n                               # the flows spread over every plane
        assert int(vsp.dp.port_counters()[0, 0]) == len(frames)
        # a network function on vports 4 / 5: VF traffic now enters the NF first
        vsp.create_network_function(vsp.vports[4]["mac"], vsp.vports[5]["mac"])
        fr2 = [f for s in range(32) for f in _pod_frame(macs[0], macs[1], 2000 + s)]
        ep[0].send(fr2)
        got_nf = []
        assert _until(lambda: got_nf.extend(ep[4].recv()) or len(got_nf) >= len(fr2)), vsp.livepath.stats
        assert sorted(got_nf) == sorted(fr2)
        assert all(d == "Healthy" for d in vsp.get_devices().values())
    finally:
        vsp.stop()


def test_vsp_port_placement_runs_each_hop_on_its_gpu(shm):
    """--placement port on 3 planes (GpuVsp placement="port"): vport i is served by plane i % 3,
    so with a network function inserted the VF's frames are classified on the VF's plane and the
    NF's output on the NF-out port's plane — the chain's hops pipeline across the GPUs."""
    nf = nfdp()
    vsp = GpuVsp(device="cpu", gpus=3, live=True, vport_kind="memif", memif_dir=str(shm), flow_buckets=1 << 12,
                 tx_workers=2, placement="port")
    vsp.init(True, "gpu")
    vsp.set_num_vfs(6)
    try:
        assert vsp.dp.placement == "port"
        # lane groups: every plane brings its own rx queue (io_queues = 1 each), and a vport is
        # read by a queue of its plane's group
        lp = vsp.livepath
        assert lp.queues == 3 and lp.stats["queues"] == 3
        assert [lp.group_of(lp.port_queue(i)) for i in range(6)] == [i % 3 for i in range(6)]
        macs = ["02:00:00:00:dd:01", "02:00:00:00:dd:02"]
        vsp.create_bridge_port("host0-0", bytes.fromhex(macs[0].replace(":", "")), 0, ["2"])
        vsp.create_bridge_port("host0-1", bytes.fromhex(macs[1].replace(":", "")), 0, ["3"])
        ep = {i: nf.MemifEndpoint(vsp.vport_path(i)) for i in range(6)}
        frames = [f for s in range(64) for f in _pod_frame(macs[0], macs[1], 1000 + s)]
        assert ep[0].send(frames) == len(frames)
        got = []
        assert _until(lambda: got.extend(ep[1].recv()) or len(got) >= len(frames)), vsp.livepath.stats
        assert sorted(got) == sorted(frames)
        rx0 = [int(p.port_counters()[0, 0]) for p in vsp.dp.planes]
        assert rx0 == [len(frames), 0, 0]                     # every flow of vport 0 on plane 0
        vsp.create_network_function(vsp.vports[4]["mac"], vsp.vports[5]["mac"])
        fr2 = [f for s in range(32) for f in _pod_frame(macs[0], macs[1], 2000 + s)]
        ep[0].send(fr2)
        got_nf = []
        assert _until(lambda: got_nf.extend(ep[4].recv()) or len(got_nf) >= len(fr2)), vsp.livepath.stats
        assert sorted(got_nf) == sorted(fr2)
        ep[5].send(got_nf)                                    # the NF passes them on: the next hop
        assert _until(lambda: int(vsp.dp.planes[2].port_counters()[5, 0]) == len(fr2))
        assert [int(p.port_counters()[5, 0]) for p in vsp.dp.planes[:2]] == [0, 0]
    finally:
        vsp.stop()


def test_vsp_unhealthy_while_the_engine_restarts(shm):
    """A failed native engine makes every vport Unhealthy (device plugin), the supervisor
    rebuilds it, and the vports come back Healthy and forwarding."""
    nf = nfdp()
    vsp = _vsp_multi(shm, 2)
    try:
        macs = ["02:00:00:00:bb:01", "02:00:00:00:bb:02"]
        vsp.create_bridge_port("host0-0", bytes.fromhex(macs[0].replace(":", "")), 0, ["2"])
        vsp.create_bridge_port("host0-1", bytes.fromhex(macs[1].replace(":", "")), 0, ["3"])
        lp = vsp.livepath
        seen = []
        lp.healthy = False                      # what the supervisor sets on an engine error
        seen.append(set(vsp.get_devices().values()))
        lp.healthy = True
        lp.fault("injected")
        assert _until(lambda: lp.restarts >= 1)
        assert seen[0] == {"Unhealthy"} and set(vsp.get_devices().values()) == {"Healthy"}
        ep0, ep1 = nf.MemifEndpoint(vsp.vport_path(0)), nf.MemifEndpoint(vsp.vport_path(1))
        fr = _pod_frame(macs[0], macs[1], 7, 8)
        ep0.send(fr)
        got = []
        assert _until(lambda: got.extend(ep1.recv()) or len(got) >= 8)
    finally:
        vsp.stop()


@pytest.mark.gpu
@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 MI355X")
def test_vsp_two_gpus_native_path(shm):
    nf = nfdp()
    vsp = _vsp_multi(shm, 2, device="cuda")
    try:
        macs = ["02:00:00:00:cc:01", "02:00:00:00:cc:02"]
        vsp.create_bridge_port("host0-0", bytes.fromhex(macs[0].replace(":", "")), 0, ["2"])
        vsp.create_bridge_port("host0-1", bytes.fromhex(macs[1].replace(":", "")), 0, ["3"])
        ep0, ep1 = nf.MemifEndpoint(vsp.vport_path(0)), nf.MemifEndpoint(vsp.vport_path(1))
        frames = [f for s in range(256) for f in _pod_frame(macs[0], macs[1], 3000 + s)]
        ep0.send(frames)
        got = []
        assert _until(lambda: got.extend(ep1.recv()) or len(got) >= len(frames), 10)
        assert sorted(got) == sorted(frames)
        assert all(int(p.port_counters()[0, 0]) > 0 for p in vsp.dp.planes)
    finally:
        vsp.stop()


@pytest.mark.parametrize("n", [2, 3])
def test_ipv6_flows_sharded_match_one_plane(n):
    """IPv6 flows on a multi-GPU plane: each lands on the owner of its folded 5-tuple, frames are
    steered by the same hash (owners() / the native engine with v6 steering), and the dual-stack
    result equals one plane holding every flow."""
    from dpu_operator_amd.dataplane import tables as T

    def v6flows(dp):
        for i in range(64):
            dp.add_flow6(f"fd00::{i + 1:x}", f"fd00::{(i * 7) % 50 + 100:x}", 1000 + i, 80, 17, 1,
                         T.flow_action(chain_id=1, out_port=i % 6, flow_id=i)[0])

    m = MultiDataPlane(["cpu"] * n, flow_buckets=1 << 12)
    sc = S.build_sfc(m, n_pods=6, n_flows=4000, n_acl=32, seed=0)
    v6flows(m)
    m.acl.add(permit=False, dst="fd00::80/124", family=6)
    m.commit(full=True)
    ref = DataPlane("cpu", flow_buckets=1 << 13)
    S.build_sfc(ref, n_pods=6, n_flows=4000, n_acl=32, seed=0)
    v6flows(ref)
    ref.acl.add(permit=False, dst="fd00::80/124", family=6)
    ref.commit(full=True)
    assert sum(len(p.flows6) for p in m.planes) == 64 and sum(1 for p in m.planes if p.flows6) > 1
    frames = []
    for i in range(64):
        fr, ln = P.craft6_full(1, dmac=S.GW_MAC, smac=S.pod_mac(i % 6), src6=f"fd00::{i + 1:x}",
                               dst6=f"fd00::{(i * 7) % 50 + 100:x}", sport=1000 + i, dport=80, frame_len=62)
        t = np.zeros(66, np.uint8)
        t[:12], t[12:14], t[14:16], t[16:] = fr[0, :12], (0x81, 0), (0, (i % 6) + 2), fr[0, 12:]
        frames.append(t)
    s6 = P.header_slots(np.stack(frames), np.full(64, 66, np.uint32))
    i6 = P.inmeta(sc.pod_port[np.arange(64) % 6], np.full(64, 66, np.uint32))
    pk4, im4 = S.traffic(sc, 512, seed=3)
    pk, im = np.concatenate([pk4, s6]), np.concatenate([im4, i6])
    r, rr = m.run(pk, im), ref.run(pk, im)
    assert np.array_equal(r.meta, rr.meta) and np.array_equal(r.out, rr.out)
    _, _, rs = P.meta_fields(r.meta[512:])
    assert (rs == 0).sum() > 40 and (rs == 4).sum() >= 1      # IPv6 flows hit; the /124 deny applies
