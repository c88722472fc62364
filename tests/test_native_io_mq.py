"""Multi-queue native I/O engine (csrc/nfdp/iox.{h,cpp}): several rx threads each owning a group of
ports and a ring queue on every backend, the per-burst CPU side pass (tunnel outer headers, flood
replicas, learning) with no ring drain, copy-on-write configuration (tunnel redirects replaced as a
whole), byte-table Toeplitz steering, and a memif peer that corrupts the shared region header.

Everything runs on the C++ oracle backends here; the GPU twins (ring kernel queues) are marked gpu.
Expected frames come from the batch path of an identical data plane (`DataPlane.run` + its side
results), assembled by ops/packets.assemble."""
import os
import shutil
import struct
import tempfile
import time
from pathlib import Path

import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.multi import MultiDataPlane
from dpu_operator_amd.dataplane.native_io import MemifVport, NativeLivePath, memif_dir
from dpu_operator_amd.native import nfdp
from dpu_operator_amd.ops import packets as P


@pytest.fixture
def shm():
    d = Path(tempfile.mkdtemp(prefix="dpu-iomq-", dir=memif_dir()))
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _until(fn, t=8.0):
    end = time.monotonic() + t
    while time.monotonic() < end:
        v = fn()
        if v:
            return v
        time.sleep(0.002)
    return fn()


def _sfc(device="cpu", n_pods=6, n_flows=4096, egress=False):
    dp = DataPlane(device=device, flow_buckets=1 << 12)
    sc = S.build_sfc(dp, n_pods=n_pods, n_flows=n_flows, n_acl=64, seed=0)
    extra = S.install_vxlan_egress(dp, sc) if egress else None
    dp.commit(full=True)
    return dp, sc, extra


def _expected(ref, slots, im):
    """Batch-path egress frames by destination port (outer headers from its side pass)."""
    r = ref.run(slots, im)
    side = ref.side_result() if ref.side_active() else None
    port, _, reason = P.meta_fields(r.meta)
    lens = im >> 16
    exp: dict[int, list[bytes]] = {}
    for i in np.nonzero(reason == 0)[0]:
        x = side["xhdr"][i] if (side is not None and side["xhdr"] is not None and P.meta_xhdr(r.meta[i:i + 1])[0]) else None
        exp.setdefault(int(port[i]), []).append(P.assemble(r.out[i], int(r.meta[i]), slots[i], int(lens[i]), x))
    return exp, int((reason != 0).sum())


def _send_all(nf, paths, slots, im, src_ports):
    eps = {p: nf.MemifEndpoint(paths[p]) for p in paths}
    src = im & 0xFFFF
    for p in src_ports:
        fr = [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == p)[0]]
        sent = 0
        t_end = time.monotonic() + 10
        while sent < len(fr) and time.monotonic() < t_end:
            sent += eps[p].send(fr[sent:])
    return eps


def _collect(eps, want):
    got: dict[int, list[bytes]] = {p: [] for p in eps}

    def done():
        for p, e in eps.items():
            got[p] += e.recv()
        return sum(map(len, got.values())) >= want

    return got, done


@pytest.mark.parametrize("queues,workers", [(3, 1), (2, 2), (2, 0)])
def test_multiqueue_bit_exact(shm, queues, workers):
    """Ports spread over `queues` rx threads (least loaded first), each with its own ring queue:
    every frame comes out as the batch path makes it, counters equal."""
    nf = nfdp()
    dp, sc, _ = _sfc()
    ref, _, _ = _sfc()
    slots, im = S.traffic(sc, 3000, seed=3)
    exp, drops = _expected(ref, slots, im)
    paths = {int(p): str(shm / f"q{int(p)}") for p in sc.pod_port}
    live = NativeLivePath(dp, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=128,
                          ring_capacity=1024, queues=queues, tx_workers=workers).start()
    try:
        qs = [live.port_queue(p) for p in paths]
        assert sorted(set(qs)) == list(range(queues))            # every queue owns ports
        assert max(qs.count(q) for q in range(queues)) - min(qs.count(q) for q in range(queues)) <= 1
        eps = _send_all(nf, paths, slots, im, list(paths))
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
        st = live.stats
        assert st["rx"] == len(slots) and st["tx"] == len(slots) - drops and live.error is None
        assert st["queues"] == queues
        assert np.array_equal(dp.port_counters(), ref.port_counters())
        dp.harvest(); ref.harvest()
        assert np.array_equal(dp.flow_totals, ref.flow_totals)
        # per-port rx counters (one burst tally per rx call) match what each pod sent
        src = im & 0xFFFF
        for p in paths:
            assert live.port(p).counters()["rx"] == int((src == p).sum())
    finally:
        live.stop()


def test_toeplitz_tables_match_the_bitwise_hash():
    """The engine steers with byte-table Toeplitz (iox ToeplitzTab); owners equal the bit-serial
    frame_owner on IPv4 and (folded) IPv6 frames, for 3 backends."""
    nf = nfdp()
    m = MultiDataPlane(["cpu"] * 3, flow_buckets=1 << 12)
    sc = S.build_sfc(m, n_pods=4, n_flows=2000, n_acl=8, seed=1)
    m.commit(full=True)
    pk, im = S.traffic(sc, 400, seed=9)
    f6, l6 = P.craft6_full(64, dmac=S.GW_MAC, smac="02:00:00:00:66:01", src6="2001:db8::1", dst6="2001:db8::2",
                           sport=np.arange(64) + 100, dport=53)
    slots6 = P.header_slots(f6, l6)
    im6 = P.inmeta(np.full(64, int(sc.pod_port[0])), l6)
    for v6 in (False, True):
        eng = nf.IoEngine(64, 8, 1)
        for _ in range(3):
            eng.add_backend(nf.OracleBackend(256))
        eng.set_steering(np.ascontiguousarray(m.ports.a), bytes(m.flows.rss_key), v6)
        for s, i in ((pk, im), (slots6, im6)):
            ref = nf.owner_of_frames(np.ascontiguousarray(s), np.ascontiguousarray(i, np.uint32),
                                     np.ascontiguousarray(m.ports.a), bytes(m.flows.rss_key), 3, v6)
            got = [eng.owner_of_frame(bytes(s[k][: int(i[k] >> 16)]), int(i[k] & 0xFFFF)) for k in range(len(s))]
            assert got == list(ref)
    own = m.owners(pk, im)
    assert len(np.unique(own)) == 3


def test_vxlan_egress_side_pass_per_burst_and_redirect_cleared(shm):
    """Every pod VF a VXLAN tunnel port: the tx leader builds each packet's outer header on the CPU
    (pipeline.h side_stage with table Toeplitz) and the frame leaves on the underlay port, byte for
    byte as the batch path's side kernel makes it, without any ring drain.  Then the ports stop
    being tunnels: the redirect map is replaced as a whole and frames go straight to the pods."""
    nf = nfdp()
    dp, sc, eg = _sfc(egress=True)
    ref, _, _ = _sfc(egress=True)
    slots, im = S.traffic(sc, 1500, seed=5)
    exp, drops = _expected(ref, slots, im)
    und = eg["underlay"]
    # the meta names the tunnel port (the destination pod's VF); the frame leaves on its underlay
    assert und not in exp
    exp = {und: [f for v in exp.values() for f in v]}
    paths = {int(p): str(shm / f"x{int(p)}") for p in list(sc.pod_port) + [und]}
    live = NativeLivePath(dp, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=256,
                          ring_capacity=2048, queues=2).start()
    try:
        eps = _send_all(nf, paths, slots, im, [int(p) for p in sc.pod_port])
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done), (live.stats, live.error)
        assert sorted(got[und]) == sorted(exp[und])
        assert live.stats["side_passes"] >= 1 and live.error is None
        # tunnels off (the slots stay set in the tunnel table): plain delivery to the pods
        for p in sc.pod_port:
            dp.ports.a[int(p)]["flags"] &= ~np.uint32(T.PORT_TUNNEL)
        dp.ports.version += 1
        dp.commit()
        for p in sc.pod_port:
            ref.ports.a[int(p)]["flags"] &= ~np.uint32(T.PORT_TUNNEL)
        ref.ports.version += 1
        ref.commit()
        slots2, im2 = S.traffic(sc, 800, seed=6)
        exp2, _ = _expected(ref, slots2, im2)
        assert und not in exp2
        for e in eps.values():
            e.recv()
        eps2 = _send_all(nf, paths, slots2, im2, [int(p) for p in sc.pod_port])
        got2, done2 = _collect(eps2, sum(map(len, exp2.values())))
        assert _until(done2), (live.stats, live.error)
        for port, frames in exp2.items():
            assert sorted(got2[port]) == sorted(frames), port
        assert got2[und] == []
    finally:
        live.stop()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("egress", [False, True])
def test_zero_copy_rx_bit_exact(shm, device, egress):
    """Zero-copy rx (iox Engine::set_zero_copy): the pipeline reads every memif frame where the pod
    wrote it — on the GPU through the pinned, mapped region (ring.hip ring_frames_gather), on the
    CPU oracle through the same per-slot addresses — and the frames, the side pass's outer headers
    and the counters come out as the batch path makes them."""
    nf = nfdp()
    dp, sc, eg = _sfc(device=device, egress=egress)
    ref, _, _ = _sfc(egress=egress)
    slots, im = S.traffic(sc, 3000, seed=11)
    exp, drops = _expected(ref, slots, im)
    ports = [int(p) for p in sc.pod_port]
    if egress:
        exp = {eg["underlay"]: [f for v in exp.values() for f in v]}
        ports_all = ports + [eg["underlay"]]
    else:
        ports_all = ports
    paths = {p: str(shm / f"z{p}") for p in ports_all}
    live = NativeLivePath(dp, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=128,
                          ring_capacity=1024, queues=2, zero_copy=True).start()
    try:
        eps = _send_all(nf, paths, slots, im, ports)
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done, 20.0), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
        st = live.stats
        assert st["rx"] == len(slots) and live.error is None
        assert st["zero_copy_frames"] == len(slots)          # not one frame copied into a slot
        assert np.array_equal(dp.port_counters(), ref.port_counters())
    finally:
        live.stop()


@pytest.mark.parametrize("devices", [["cpu", "cpu"], pytest.param(["cuda:0", "cuda:0"], marks=pytest.mark.gpu)])
def test_multi_plane_native_matches_one_plane(shm, devices):
    """Two planes behind one engine with two queues (RSS owner steering in each rx thread): the
    frames and summed counters equal a single plane's.  On a GPU box both planes are ring kernels
    of the same MI355X (two lanes per queue on one device: the multi-GPU code path on one card)."""
    nf = nfdp()
    m = MultiDataPlane(devices, flow_buckets=1 << 12)
    sc = S.build_sfc(m, n_pods=6, n_flows=4096, n_acl=64, seed=0)
    m.commit(full=True)
    ref, _, _ = _sfc()
    slots, im = S.traffic(sc, 3000, seed=7)
    exp, drops = _expected(ref, slots, im)
    paths = {int(p): str(shm / f"m{int(p)}") for p in sc.pod_port}
    live = NativeLivePath(m, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=128,
                          ring_capacity=1024, queues=2).start()
    try:
        assert len(live.dps) == 2
        eps = _send_all(nf, paths, slots, im, list(paths))
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
        assert all(int(p.port_counters()[:, 0].sum()) > 0 for p in m.planes)   # both planes worked
        # (ring kernels flush their LDS counter tallies when their waves next go idle)
        ok = _until(lambda: np.array_equal(m.port_counters(), ref.port_counters()), 2.0)
        if not ok:
            got_c, want_c = m.port_counters(), ref.port_counters()
            bad = np.nonzero((got_c != want_c).any(1))[0]
            per = [p.port_counters()[bad] for p in m.planes]
            st = dict(live.stats)
            live.stop()
            after = m.port_counters()
            raise AssertionError(f"ports {bad.tolist()}: got {got_c[bad].tolist()} want {want_c[bad].tolist()} "
                                 f"per plane {[x.tolist() for x in per]} after stop {after[bad].tolist()} "
                                 f"equal after stop {np.array_equal(after, want_c)} stats {st}")
        # a commit of the multi-plane data plane pauses the engine once and keeps forwarding
        m.ports.set_mtu(int(sc.pod_port[0]), 1400)
        ref.ports.set_mtu(int(sc.pod_port[0]), 1400)
        m.commit()
        ref.commit()
        slots2, im2 = S.traffic(sc, 500, seed=8)
        exp2, _ = _expected(ref, slots2, im2)
        eps2 = _send_all(nf, paths, slots2, im2, list(paths))
        got2, done2 = _collect(eps2, sum(map(len, exp2.values())))
        assert _until(done2), (live.stats, live.error)
        for port, frames in exp2.items():
            assert sorted(got2[port]) == sorted(frames), port
    finally:
        live.stop()


@pytest.mark.parametrize("devices", [["cpu", "cpu", "cpu"], pytest.param(["cuda:0", "cuda:0"], marks=pytest.mark.gpu)])
def test_port_placement_hop_pipeline(shm, devices):
    """MultiDataPlane(placement="port"), the SFC hop pipeline across GPUs: every frame runs on the
    GPU its ingress port (one NF hop) is placed on — batch and live (the engine steers by the
    port table, iox Steer::port_owner) — with flows replicated: frames equal one plane's, each
    plane's rx counters hold only its own ports, and the flow counters summed over the planes
    equal one plane's.  A port moved to another GPU (place_port + commit) is served there."""
    nf = nfdp()
    m = MultiDataPlane(devices, placement="port", flow_buckets=1 << 12)
    sc = S.build_sfc(m, n_pods=6, n_flows=4096, n_acl=64, seed=0)
    m.commit(full=True)
    ref, _, _ = _sfc()
    n = len(devices)
    pods = [int(p) for p in sc.pod_port]
    assert len(m.flows) == len(ref.flows) and all(len(p.flows) == len(ref.flows) for p in m.planes)
    # batch: split by ingress port
    slots, im = S.traffic(sc, 3000, seed=9)
    r = m.run(slots, im)
    r0 = ref.run(slots, im)
    assert np.array_equal(r.meta, r0.meta) and np.array_equal(r.out, r0.out)
    assert np.array_equal(r.extra["owner"], (im & 0xFFFF).astype(np.int64) % n)
    m.reset_counters(); ref.reset_counters()
    m.harvest(); ref.harvest()
    # live: the engine steers by ingress port
    exp, drops = _expected(ref, slots, im)
    paths = {p: str(shm / f"h{p}") for p in pods}
    live = NativeLivePath(m, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=128,
                          ring_capacity=1024, queues=2).start()
    try:
        eps = _send_all(nf, paths, slots, im, pods)
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
        src = (im & 0xFFFF).astype(np.int64)

        def per_plane_rx_ok():
            for g, p in enumerate(m.planes):
                rx = p.port_counters()[:, 0]
                for q in pods:
                    want = int((src == q).sum()) if q % n == g else 0
                    if int(rx[q]) != want:
                        return False
            return True

        assert _until(per_plane_rx_ok, 2.0), [p.port_counters()[pods, 0].tolist() for p in m.planes]
        assert _until(lambda: np.array_equal(m.port_counters(), ref.port_counters()), 2.0)
        m.harvest(); ref.harvest()
        assert np.array_equal(m.flow_totals, ref.flow_totals)
        k = sc.keys[0]
        assert m.flow_counters(k) == ref.flow_counters(k)
        # move the first pod's port to another GPU: its next frames are processed there
        q0 = pods[0]
        g_new = (q0 + 1) % n
        before = [int(p.port_counters()[q0, 0]) for p in m.planes]
        m.place_port(q0, g_new)
        m.commit()
        sel = np.nonzero(src == q0)[0][:200]
        for e in eps.values():
            e.recv()
        eps[q0].send([bytes(slots[k, : int(im[k] >> 16)]) for k in sel])
        assert _until(lambda: int(m.planes[g_new].port_counters()[q0, 0]) - before[g_new] == len(sel), 4.0), \
            ([int(p.port_counters()[q0, 0]) for p in m.planes], before)
        assert int(m.planes[q0 % n].port_counters()[q0, 0]) == before[q0 % n]
    finally:
        live.stop()


def test_learning_reaches_every_plane(shm):
    """MAC learning from the per-burst side pass goes through the learner thread into EVERY plane's
    MAC table (one learning bridge per node), not only the plane that saw the frame."""
    nf = nfdp()
    m = MultiDataPlane(["cpu", "cpu"], flow_buckets=1 << 10, mac_slots=1 << 10)
    for p in range(4):
        m.ports.set(p, flags=T.PORT_VALID | T.PORT_LEARN, bridge_id=7)
    m.flood.set_members(7, [0, 1, 2, 3])
    m.commit(full=True)
    paths = {p: str(shm / f"l{p}") for p in range(4)}
    live = NativeLivePath(m, {p: MemifVport(paths[p]) for p in paths}, queues=2).start()
    try:
        eps = {p: nf.MemifEndpoint(paths[p]) for p in paths}
        macs = [f"02:00:00:00:1c:{k:02x}" for k in range(16)]
        frames = []
        for k, mac in enumerate(macs):
            fr, ln = P.craft(1, dmac="ff:ff:ff:ff:ff:ff", smac=mac, src_ip=0x0A000001 + k, dst_ip=0x0A0000FE,
                             sport=1000 + k, dport=80)
            frames.append(bytes(fr[0, : ln[0]]))
        assert eps[2].send(frames) == len(frames)
        got = {p: [] for p in (0, 1, 3)}
        assert _until(lambda: [got[p].extend(eps[p].recv()) for p in got] and all(len(got[p]) >= 16 for p in got))
        live.flush_learning()
        for plane in m.planes:
            tab = plane._dev["macs"].view(T.MAC_DTYPE)
            learned = {(int(e["mac_lo"]), int(e["mac_hi"])) for e in tab if int(e["valid"]) == 3}
            for mac in macs:
                lo, hi = T.mac_raw(mac)
                assert (int(lo), int(hi)) in learned, mac
        assert live.stats["learn_events"] >= 16 and live.stats["learn_applied"] >= 16
    finally:
        live.stop()


def test_memif_peer_corrupting_the_header_cannot_reach_outside_the_region(shm):
    """The engine snapshots the region geometry when it creates it: a pod that rewrites ring_size /
    buf_size / its head index in the shared header while traffic flows garbles at most its own
    frames; the engine keeps running and the other pods keep talking."""
    nf = nfdp()
    dp, sc, _ = _sfc(n_pods=4)
    paths = {int(p): str(shm / f"c{int(p)}") for p in sc.pod_port}
    live = NativeLivePath(dp, {p: MemifVport(paths[p], ring_size=256) for p in paths}, ring_capacity=1024).start()
    try:
        bad = int(sc.pod_port[0])
        with open(paths[bad], "r+b") as f:
            f.seek(12)
            f.write(struct.pack("<II", 1 << 30, 1 << 16))   # ring_size, buf_size
            f.seek(64)
            f.write(struct.pack("<I", 0x7FFFFFF0))          # ring 0 head: a bogus producer index
        time.sleep(0.2)
        assert live.error is None and live.healthy
        good = [int(p) for p in sc.pod_port[1:]]
        slots, im = S.traffic(sc, 600, seed=11, src_pods=np.arange(1, len(sc.pod_port)))
        eps = {p: nf.MemifEndpoint(paths[p]) for p in good}
        src = im & 0xFFFF
        for p in good:
            fr = [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == p)[0]]
            assert eps[p].send(fr) == len(fr)
        n = [0]
        assert _until(lambda: n.__setitem__(0, n[0] + sum(len(e.recv()) for e in eps.values())) or n[0] > 0)
        assert live.error is None
    finally:
        live.stop()


def test_memif_tx_rings_per_queue(shm):
    """A memif vport has one data-plane -> pod ring per engine queue: each queue's tx thread writes
    its own ring (no shared lock or cache line between queues), the pod drains all of them, and
    frames of one ring stay in order."""
    nf = nfdp()
    path = str(shm / "p0")
    port = nf.MemifPort(path, 64, 2048, 3)
    assert port.tx_rings == 3
    ep = nf.MemifEndpoint(path)
    eng = nf.IoEngine(64, 8, 1, 3, 0)
    be = nf.WireBackend(256, 3, [(int.from_bytes(bytes([2, 0, 0, 0, 0, 1]), "little"), 0)])
    eng.add_backend(be)
    srcs = [nf.MemifPort(str(shm / f"s{q}"), 64, 2048, 3) for q in range(3)]
    eng.add_port(0, port, 0)
    for q, s in enumerate(srcs):
        eng.add_port(1 + q, s, q)          # source pod q is read by queue q
    eng.start()
    try:
        frame = lambda q, i: bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 9, 0x88, 0xB5, q, i]) + bytes(44)  # noqa: E731
        for q in range(3):
            e = nf.MemifEndpoint(str(shm / f"s{q}"))
            assert e.send([frame(q, i) for i in range(20)]) == 20
        got = []
        _until(lambda: got.extend(ep.recv()) or len(got) >= 60)
        assert len(got) == 60
        st = eng.stats()
        assert st["rx"] == 60 and st["tx"] == 60
        # each source queue's frames arrive in order (they share one tx ring)
        for q in range(3):
            seq = [f[15] for f in got if f[14] == q]
            assert seq == list(range(20))
    finally:
        eng.stop()


def test_coalescing_never_delays_an_idle_lane(shm):
    """Publication coalescing (Engine::set_coalesce) gathers frames only while bursts of the lane
    are in flight: with a one-second window, single frames on an idle engine still come out at
    once, every one of them."""
    nf = nfdp()
    eng = nf.IoEngine(64, 8, 1, 1, 0)
    eng.set_coalesce(64, 1e6)
    eng.add_backend(nf.WireBackend(256, 1, [(int.from_bytes(bytes([2, 0, 0, 0, 0, 1]), "little"), 0)]))
    dst = nf.MemifPort(str(shm / "d"), 64, 2048, 1)
    src = nf.MemifPort(str(shm / "s"), 64, 2048, 1)
    eng.add_port(0, dst)
    eng.add_port(1, src)
    eng.start()
    try:
        a, b = nf.MemifEndpoint(str(shm / "s")), nf.MemifEndpoint(str(shm / "d"))
        for i in range(20):
            t0 = time.perf_counter()
            assert a.send([bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 9, 0x88, 0xB5, i]) + bytes(45)]) == 1
            got = _until(lambda: b.recv(), t=0.5)
            assert got and got[0][14] == i
            assert time.perf_counter() - t0 < 0.25      # far below the 1 s window
    finally:
        eng.stop()


def test_memif_region_recreated_at_the_same_path(shm):
    """A port re-created at the path of one still alive (a removed port the engine keeps while its
    frames drain) gets a fresh file: the old mapping is never truncated under it, and the old
    port going away later does not unlink its successor's file."""
    import gc
    import os

    nf = nfdp()
    path = str(shm / "again")
    old = nf.MemifPort(path, 256, 2048)
    ep_old = nf.MemifEndpoint(path)
    new = nf.MemifPort(path, 256, 2048)
    assert ep_old.send([bytes(64)]) == 1          # the old region is intact (not truncated)
    del old, ep_old
    gc.collect()
    assert os.path.exists(path)                     # still the new port's file
    ep = nf.MemifEndpoint(path)
    assert ep.send([bytes(64)]) == 1
    del ep, new
    gc.collect()
    assert not os.path.exists(path)


@pytest.mark.parametrize("devices", [["cpu", "cpu"], pytest.param(["cuda:0", "cuda:0"], marks=pytest.mark.gpu)])
def test_live_soak_under_churn(shm, devices):
    """~10 s of pod traffic through two planes (on a GPU box: two ring kernels on one MI355X; port
    placement, zero-copy rx)
    while the control plane churns: ACL rules added and removed (live table-set flips), ports moved
    between the planes, link flaps through the device control mailbox, a spare vport removed and
    re-added.  Traffic never stops, the engine never fails, the removed vports' pinned regions stay
    bounded (maintenance restarts of the rings release them), and once the churn is undone a final
    batch is bit-exact with a CPU plane holding the same tables."""
    import ipaddress
    import threading

    from dpu_operator_amd.dataplane import tables as T2

    nf = nfdp()
    m = MultiDataPlane(devices, placement="port", flow_buckets=1 << 14)
    sc = S.build_sfc(m, n_pods=6, n_flows=8192, n_acl=64, seed=0)
    m.commit(full=True)
    ref, _, _ = _sfc(n_flows=8192)
    pods = [int(p) for p in sc.pod_port]
    spare = max(pods) + 4
    paths = {p: str(shm / f"s{p}") for p in pods + [spare]}
    live = NativeLivePath(m, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=128,
                          ring_capacity=2048, queues=2, zero_copy=True).start()
    eps = {p: nf.MemifEndpoint(paths[p]) for p in pods}
    slots, im = S.traffic(sc, 6000, seed=12)
    src = im & 0xFFFF
    by_pod = {p: [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == p)[0]] for p in pods}
    stop = threading.Event()
    windows: list[int] = []
    lock = threading.Lock()

    def sender():
        got = 0
        t_win = time.monotonic()
        while not stop.is_set():
            for p in pods:
                eps[p].send(by_pod[p][:64])
            for p in pods:
                got += len(eps[p].recv())
            if time.monotonic() - t_win >= 1.0:
                with lock:
                    windows.append(got)
                got, t_win = 0, time.monotonic()
            time.sleep(0.0005)

    th = threading.Thread(target=sender, daemon=True)
    th.start()
    rng = np.random.default_rng(5)
    ops = {"acl": 0, "move": 0, "flap": 0, "spare": 0}
    try:
        import os

        t_end = time.monotonic() + float(os.environ.get("DPU_SOAK_SECONDS", "10"))   # (longer soaks: the env)
        while time.monotonic() < t_end:
            k = int(rng.integers(0, 4))
            if k == 0:      # a deny rule in, then out (two live table-set flips)
                pod = int(rng.integers(0, 6))
                m.acl.add(permit=False, dst=f"{ipaddress.IPv4Address(S.POD_NET + pod)}/32")
                m.acl.rules.insert(0, m.acl.rules.pop())
                m.acl.version += 1
                m.commit()
                m.acl.rules.pop(0)
                m.acl.version += 1
                m.commit()
                ops["acl"] += 1
            elif k == 1:    # a pod's port moves to the other plane
                p = pods[int(rng.integers(0, len(pods)))]
                m.place_port(p, 1 - int(m.port_owner[p]))
                m.commit()
                ops["move"] += 1
            elif k == 2:    # link flap through the control mailbox (no commit)
                p = pods[int(rng.integers(0, len(pods)))]
                for on in (False, True):
                    if on:
                        m.ports.a[p]["flags"] |= np.uint32(T2.PORT_VALID)
                    else:
                        m.ports.a[p]["flags"] &= ~np.uint32(T2.PORT_VALID)
                    # through the running rings' control mailbox; a commit when none runs (CPU
                    # planes, or rings in a maintenance restart - what GpuVsp.set_port_state does)
                    if not (m.gpu and m.ctrl_ports([p])):
                        m.ports.version += 1
                        m.commit()
                ops["flap"] += 1
            else:           # the spare vport goes away and comes back
                live.remove_port(spare)
                time.sleep(0.005)
                live.add_port(spare, MemifVport(paths[spare], ring_size=4096))
                ops["spare"] += 1
            time.sleep(0.02)
        stop.set()
        th.join(timeout=10)
        assert live.error is None and live.restarts == 0, (live.error, live.restarts)
        assert min(ops.values()) >= 3, ops
        if m.gpu:
            # removed zero-copy regions stay pinned while rings run: bounded by maintenance restarts
            assert nf.deferred_host_unmaps() <= live.max_deferred_unmaps + 1, nf.deferred_host_unmaps()
            if ops["spare"] > live.max_deferred_unmaps + 1:
                assert live.unmap_restarts >= 1
        with lock:
            assert len(windows) >= 8 and min(windows) > 0, windows     # traffic never stopped
        # undo: every pod on its default plane, tables as the reference's; then a final exact batch
        for p in pods:
            m.place_port(p, p % 2)
        m.commit()
        time.sleep(0.2)
        for p in pods:
            eps[p].recv()
        slots2, im2 = S.traffic(sc, 2000, seed=13)
        exp, _ = _expected(ref, slots2, im2)
        eps2 = _send_all(nf, {p: paths[p] for p in pods}, slots2, im2, pods)
        got, done = _collect(eps2, sum(map(len, exp.values())))
        assert _until(done, 15.0), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
    finally:
        stop.set()
        live.stop()


def test_bursts_in_flight_keep_their_publish_time_configuration(shm):
    """A burst is side-passed and delivered with the configuration current when it was published
    (iox Burst::cfg), not with whatever a commit swapped in while it was in flight: VXLAN-egress
    bursts held in flight (the oracle's completion gate) while the tunnel redirects are cleared still
    leave encapsulated on the underlay, byte for byte; bursts published afterwards follow the new map."""
    nf = nfdp()
    dp, sc, eg = _sfc(egress=True)
    ref, _, _ = _sfc(egress=True)
    slots, im = S.traffic(sc, 600, seed=7)
    exp, _ = _expected(ref, slots, im)
    und = eg["underlay"]
    exp = {und: [f for v in exp.values() for f in v]}
    paths = {int(p): str(shm / f"g{int(p)}") for p in list(sc.pod_port) + [und]}
    live = NativeLivePath(dp, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=256,
                          ring_capacity=2048, queues=1).start()
    try:
        be = live._backends[0]
        be.set_completion_gate(True)
        eps = _send_all(nf, paths, slots, im, [int(p) for p in sc.pod_port])
        assert _until(lambda: live.stats["rx"] >= len(slots)), live.stats
        assert _until(lambda: live.stats["bursts"] >= 1)
        time.sleep(0.05)
        assert live.stats["tx"] == 0                     # nothing completed: every burst in flight
        live._eng.set_redirects([])                      # a commit's configuration swap, mid-flight
        be.set_completion_gate(False)
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done), (live.stats, live.error)
        assert sorted(got[und]) == sorted(exp[und])
        assert all(got[int(p)] == [] for p in sc.pod_port)
        # published after the swap: no redirect, so the frames are delivered to the tunnel port
        # itself (the pod), still with their outer header
        eps[und].recv()
        slots2, im2 = S.traffic(sc, 64, seed=8)
        _send_all(nf, paths, slots2, im2, [int(p) for p in sc.pod_port])
        got2, done2 = _collect(eps, 1)
        assert _until(done2), (live.stats, live.error)
        assert got2[und] == []
        assert live.error is None
    finally:
        live.stop()


def test_removed_port_released_once_its_bursts_are_delivered(shm):
    """A removed port is held only while a burst may still point into its rx memory (iox
    Engine::reap_retired): with its frames delivered it is released within moments, not after a
    fixed grace time, and a port removed while frames of it are in flight is kept until they are."""
    nf = nfdp()
    dp, sc, _ = _sfc()
    slots, im = S.traffic(sc, 400, seed=11)
    paths = {int(p): str(shm / f"r{int(p)}") for p in sc.pod_port}
    live = NativeLivePath(dp, {p: MemifVport(paths[p], ring_size=1024) for p in paths}, burst=128,
                          ring_capacity=1024, queues=2).start()
    try:
        eng = live._eng
        src = int(sc.pod_port[0])
        be = live._backends[0]
        be.set_completion_gate(True)                       # frames of `src` stay in flight
        eps = _send_all(nf, paths, slots, im, [src])
        n_src = int(((im & 0xFFFF) == src).sum())
        assert _until(lambda: live.stats["rx"] >= n_src), live.stats
        live.remove_port(src)
        time.sleep(0.05)
        assert eng.retired_ports() == 1                     # its bursts are not delivered yet
        be.set_completion_gate(False)
        assert _until(lambda: eng.retired_ports() == 0, 2.0), eng.retired_ports()
        assert live.error is None
        eps.clear()
    finally:
        live.stop()


def test_cpulist_and_lane_group_pinning(shm):
    """sysfs cpulists parse; each lane group's threads run on the CPUs given for it (set_queue_cpus
    before start; refused after) and the engine forwards bit-exact as before."""
    from dpu_operator_amd.dataplane.native_io import parse_cpulist

    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []
    nf = nfdp()
    eng = nf.IoEngine(128, 16, 1, 2, 0)
    with pytest.raises(ValueError):
        eng.set_queue_cpus(5, [0])
    dp, sc, _ = _sfc()
    ref, _, _ = _sfc()
    slots, im = S.traffic(sc, 500, seed=12)
    exp, _ = _expected(ref, slots, im)
    paths = {int(p): str(shm / f"c{int(p)}") for p in sc.pod_port}
    cpus = sorted(os.sched_getaffinity(0))
    live = NativeLivePath([dp], {p: MemifVport(paths[p], ring_size=2048) for p in paths}, burst=128,
                          ring_capacity=1024, queues=2, lane_groups=True, pin_cpus={0: cpus[:2]}).start()
    try:
        with pytest.raises(RuntimeError):
            live._eng.set_queue_cpus(0, cpus[:1])           # running: too late
        eps = _send_all(nf, paths, slots, im, list(paths))
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
    finally:
        live.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("placement,split,whole", [
    ("port", ("acl", "nat", "l2fwd@1"), ("acl", "nat", "l2fwd")),
    ("flow", ("acl", "nat@1", "ttl@0", "l2fwd@1"), ("acl", "nat", "ttl", "l2fwd")),
])
def test_split_chain_live_crosses_planes(shm, placement, split, whole):
    """SFC hops across GPUs in the LIVE path (ring.h XferEntry): two ring planes behind one engine,
    a chain whose hops sit on both.  Each frame's first hops run on the plane it entered, the rest
    on the other plane's resident grid (its inbox), which stores the final header into the entry
    ring's out slot; the engine delivers the burst once every frame is back.  Frames equal the
    whole chain on one plane; summed port counters too (tx counted where the chain ended); the
    drops equal one plane's besides the hand-offs.  The second case crosses twice (0 -> 1 -> 0 -> 1
    for frames entering on plane 0)."""
    nf = nfdp()
    m = MultiDataPlane(["cuda:0", "cuda:0"], placement=placement, flow_buckets=1 << 12)
    sc = S.build_sfc(m, n_pods=6, n_flows=4096, n_acl=64, seed=0, hops=split)
    m.commit(full=True)
    ref = DataPlane(device="cpu", flow_buckets=1 << 12)
    S.build_sfc(ref, n_pods=6, n_flows=4096, n_acl=64, seed=0, hops=whole)
    ref.commit(full=True)
    slots, im = S.traffic(sc, 3000, seed=11)
    exp, drops = _expected(ref, slots, im)
    paths = {int(p): str(shm / f"x{int(p)}") for p in sc.pod_port}
    live = NativeLivePath(m, {p: MemifVport(paths[p], ring_size=4096) for p in paths}, burst=128,
                          ring_capacity=1024, queues=2).start()
    try:
        assert live.xfer and live.xfer_active() == [True, True]
        eps = _send_all(nf, paths, slots, im, list(paths))
        got, done = _collect(eps, sum(map(len, exp.values())))
        assert _until(done), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
        assert live.error is None
        assert _until(lambda: np.array_equal(m.port_counters(), ref.port_counters()), 2.0), \
            (m.port_counters()[sc.pod_port].tolist(), ref.port_counters()[sc.pod_port].tolist())
        d1, d2 = ref.drop_counters(), m.drop_counters()
        assert d2.pop("remote", 0) >= int(sum(map(len, exp.values())))   # every forwarded frame crossed
        assert d1 == d2, (d1, d2)
    finally:
        live.stop()
    st = [r.eng.xfer_stats() for r in live._rings] if live._rings else None
    assert st is None or all(len(x) == 8 and x[4] > 0 for x in st if x[0])
