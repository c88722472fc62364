"""Native I/O engine (csrc/nfdp/iox.{h,cpp}, dataplane/native_io.py): shared-memory vports ->
C++ rx thread -> data plane (C++ oracle backend here; the persistent ring kernel on a GPU) -> C++
tx thread -> vports.  Every test checks the frames that come out against the oracle run of the
same frames assembled by ops/packets.assemble (the Python LivePath's rule), so the native path is
bit-exact with the batch path."""
import os
import time

import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.native_io import MemifVport, NativeLivePath, memif_dir
from dpu_operator_amd.native import nfdp
from dpu_operator_amd.ops import packets as P


def _until(fn, t=5.0):
    end = time.monotonic() + t
    while time.monotonic() < end:
        v = fn()
        if v:
            return v
        time.sleep(0.002)
    return fn()


def _sfc(device, n_pods=4, n_flows=4096):
    dp = DataPlane(device=device, flow_buckets=1 << 12)
    sc = S.build_sfc(dp, n_pods=n_pods, n_flows=n_flows, n_acl=64, seed=0)
    dp.commit(full=True)
    return dp, sc


@pytest.fixture
def tmp_path():
    """Regions on tmpfs (/dev/shm): a disk-backed MAP_SHARED file pays writeback faults."""
    import shutil
    import tempfile
    from pathlib import Path

    d = Path(tempfile.mkdtemp(prefix="dpu-iox-", dir=memif_dir()))
    yield d
    shutil.rmtree(d, ignore_errors=True)


def _vports(tmp_path, n, tag="v"):
    return {i: MemifVport(str(tmp_path / f"{tag}{i}"), ring_size=4096) for i in range(n)}


def _expected(dp_ref, slots, im):
    """Oracle run of the same frames: egress frames grouped by destination port."""
    r = dp_ref.run(slots, im)
    port, olen, reason = P.meta_fields(r.meta)
    exp: dict[int, list[bytes]] = {}
    lens = im >> 16
    for i in np.nonzero(reason == 0)[0]:
        f = P.assemble(r.out[i], int(r.meta[i]), slots[i], int(lens[i]))
        exp.setdefault(int(port[i]), []).append(f)
    return exp, int((reason != 0).sum())


@pytest.mark.parametrize("workers", [0, 1, 3])
def test_memif_sfc_bit_exact_with_the_batch_path(tmp_path, workers):
    nf = nfdp()
    dp, sc = _sfc("cpu")
    ref, _ = _sfc("cpu")
    slots, im = S.traffic(sc, 2000, seed=3)
    exp, drops = _expected(ref, slots, im)
    live = NativeLivePath(dp, _vports(tmp_path, sc.n_pods), burst=128, ring_capacity=1024, tx_workers=workers).start()
    try:
        eps = {i: nf.MemifEndpoint(str(tmp_path / f"v{i}")) for i in range(sc.n_pods)}
        src = im & 0xFFFF
        for i in range(sc.n_pods):
            fr = [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == i)[0]]
            sent = 0
            while sent < len(fr):
                sent += eps[i].send(fr[sent:])
        got: dict[int, list[bytes]] = {i: [] for i in range(sc.n_pods)}

        def drained():
            for i in range(sc.n_pods):
                got[i] += eps[i].recv()
            return sum(map(len, got.values())) >= sum(map(len, exp.values()))

        assert _until(drained), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
        st = live.stats
        assert st["rx"] == len(slots) and st["tx"] == len(slots) - drops and live.error is None
        assert np.array_equal(dp.port_counters(), ref.port_counters())
        dp.harvest(); ref.harvest()
        assert np.array_equal(dp.flow_totals, ref.flow_totals)
    finally:
        live.stop()


def test_trafgen_through_the_native_path(tmp_path):
    """The C++ pod-side generator / sink (trafgen.h) drives all vports; every frame sent in the
    measured window arrives, and one-way latencies come back."""
    nf = nfdp()
    dp, sc = _sfc("cpu")
    live = NativeLivePath(dp, _vports(tmp_path, sc.n_pods, "t"), burst=256, ring_capacity=2048).start()
    try:
        pods = []
        for i in range(sc.n_pods):
            slots, im = S.traffic(sc, 256, seed=10 + i, src_pods=np.array([i]))
            pods.append((str(tmp_path / f"t{i}"), slots, (im >> 16).astype(np.uint32)))
        r = nf.trafgen_run(pods, duration_s=0.3, warmup_s=0.05, threads=2, inflight=256)
        assert r["sent"] > 1000 and r["bad"] == 0
        assert len(r["lat_us"]) and np.median(r["lat_us"]) > 0
        # frames still in flight at the end of the window arrive afterwards: nothing is lost
        eps = [nf.MemifEndpoint(p[0]) for p in pods]
        late = [0]

        def drained():
            late[0] += sum(len(e.recv()) for e in eps)
            return r["received"] + late[0] >= r["sent"]

        _until(drained, 5.0)
        assert r["received"] + late[0] + live.stats["tx_full"] >= r["sent"], (r["received"], late[0], live.stats)
        assert live.error is None
    finally:
        live.stop()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_flood_learn_and_arp_punt_native(tmp_path, device):
    """OvS NORMAL through the native path: broadcast ARP flooded to every other member (primary +
    replicas from the side pass), its copy punted to the slow path, the source MAC learned."""
    nf = nfdp()
    dp = DataPlane(device=device, flow_buckets=1 << 10, mac_slots=1 << 10)
    for p in range(4):
        dp.ports.set(p, flags=T.PORT_VALID | T.PORT_LEARN | T.PORT_ARP_TRAP, bridge_id=5)
    dp.flood.set_members(5, [0, 1, 2, 3])
    dp.commit(full=True)
    punts = []
    live = NativeLivePath(dp, _vports(tmp_path, 4, "f"), on_punt=lambda f, p, r: punts.append((p, r))).start()
    try:
        eps = {i: nf.MemifEndpoint(str(tmp_path / f"f{i}")) for i in range(4)}
        arp, al = P.craft_arp(1, smac="02:00:00:00:0a:01", sender_ip=0x0A000001, target_ip=0x0A000002)
        assert eps[0].send([bytes(arp[0, : al[0]])]) == 1
        got = {}
        assert _until(lambda: all(got.setdefault(i, []) or got[i].extend(eps[i].recv()) or got[i] for i in (1, 2, 3)))
        assert all(g == [bytes(arp[0, : al[0]])] for g in (got[1], got[2], got[3]))
        assert _until(lambda: punts) and punts[0] == (0, 12)
        dp.pull_learned()
        assert (5, "02:00:00:00:0a:01", 0) in dp.macs.learned()
        assert live.stats["replicas"] == 2 and live.stats["side_passes"] >= 1
    finally:
        live.stop()


def test_commit_under_traffic_and_failure_restart(tmp_path):
    """Table commits while the engine runs (paused around each one), then an injected engine
    failure: unhealthy, restarted by the supervisor, forwarding again."""
    nf = nfdp()
    dp, sc = _sfc("cpu")
    live = NativeLivePath(dp, _vports(tmp_path, sc.n_pods, "c"), ring_capacity=1024).start()
    try:
        eps = {i: nf.MemifEndpoint(str(tmp_path / f"c{i}")) for i in range(sc.n_pods)}
        slots, im = S.traffic(sc, 64, seed=4, src_pods=np.array([0]))
        frames = [bytes(slots[k, : int(im[k] >> 16)]) for k in range(len(slots))]

        def rx_all():
            return sum(len(eps[i].recv()) for i in range(sc.n_pods))

        for rnd in range(5):
            eps[0].send(frames)
            dp.ports.set_mtu(3, 1400 + rnd)       # a port-table change: a full commit mid-traffic
            dp.commit()
        seen = [0]
        assert _until(lambda: seen.__setitem__(0, seen[0] + rx_all()) or seen[0] >= 5 * 64), (seen, live.stats)
        live.fault("injected I/O failure")
        assert _until(lambda: live.restarts >= 1), live.error
        assert live.healthy and "injected" in (live.error or "")
        eps[0].send(frames)
        seen = [0]
        assert _until(lambda: seen.__setitem__(0, seen[0] + rx_all()) or seen[0] >= 64), (seen, live.stats)
    finally:
        live.stop()


@pytest.mark.gpu
@pytest.mark.parametrize("queues,gpu_egress", [(1, False), (2, False), (1, True), (2, True)])
def test_native_path_gpu_ring_bit_exact(tmp_path, queues, gpu_egress):
    """The GPU backend: header slots into the persistent ring kernel's pinned host slots (one
    ring queue per engine queue); frames bit-exact and counters exact.  gpu_egress: the grid
    writes the frames into the pods' rings itself (ring.h GdeRing), the same frames arrive."""
    nf = nfdp()
    dp, sc = _sfc("cuda")
    ref, _ = _sfc("cpu")
    slots, im = S.traffic(sc, 3000, seed=5)
    exp, drops = _expected(ref, slots, im)
    live = NativeLivePath(dp, _vports(tmp_path, sc.n_pods, "g"), burst=256, ring_capacity=4096,
                          queues=queues, gpu_egress=gpu_egress).start()
    try:
        eps = {i: nf.MemifEndpoint(str(tmp_path / f"g{i}")) for i in range(sc.n_pods)}
        src = im & 0xFFFF
        for i in range(sc.n_pods):
            fr = [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == i)[0]]
            sent = 0
            while sent < len(fr):
                sent += eps[i].send(fr[sent:])
        got: dict[int, list[bytes]] = {i: [] for i in range(sc.n_pods)}

        def drained():
            for i in range(sc.n_pods):
                got[i] += eps[i].recv()
            return sum(map(len, got.values())) >= sum(map(len, exp.values()))

        assert _until(drained, 10), (live.stats, live.error)
        for port, frames in exp.items():
            assert sorted(got[port]) == sorted(frames), port
        st = live.stats
        if gpu_egress:   # every forwarded 64-B frame went out from the GPU, none through the tx threads
            assert st["gpu_tx"] == sum(map(len, exp.values())) and st["tx"] == 0, st
        else:
            assert st["gpu_tx"] == 0
        # counters: the ring kernel's LDS tallies reach the device counters when its waves idle
        if not _until(lambda: np.array_equal(dp.port_counters(), ref.port_counters()), 2.0):
            g, w = dp.port_counters(), ref.port_counters()
            bad = np.nonzero((g != w).any(1))[0]
            raise AssertionError(f"ports {bad.tolist()}: got {g[bad].tolist()} want {w[bad].tolist()} {live.stats}")
    finally:
        live.stop()


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_native_sanitizer_stress(kind, tmp_path):
    """Race / memory-error detection on the native I/O engine (csrc/nfdp/iox_stress.cpp, host-only
    TSan or ASan+UBSan build): two queues x two oracle backends x two tx workers under memif
    traffic, while commits pause / hold the engine and swap its configuration, a port is removed
    and re-added, statistics are read, and an injected failure rebuilds the engine; one backend
    reads its frames by address in the pods' regions (zero-copy rx)."""
    import subprocess

    from dpu_operator_amd.native.build import build_sanitized

    try:
        exe = build_sanitized(kind, target="iox")
    except RuntimeError as e:  # toolchain without the sanitizer runtime
        pytest.skip(str(e)[:200])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path), "1.5"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert r.stdout.strip().endswith("ok")


@pytest.mark.gpu
def test_live_commits_at_1khz_under_traffic(tmp_path):
    """CreateBridgePort-style port edits, ACL edits and agent link flaps committed at ~1 kHz while
    pods send through the GPU live path: every commit is a live table-set flip under the running
    ring (no pause, no drain), nothing is lost, and the one-way p99 with the churn stays within
    10 us of the p99 without it (the table sets are in HBM: a flip's restage never crosses PCIe;
    +1.1 to +2.6 us measured, profiles/r5_s3_live_commit_hwq_ab.txt).  One re-measurement of both
    runs is allowed: a single host-scheduling stall of the 1-s run is not the commit's cost."""
    import threading

    nf = nfdp()
    dp, sc = _sfc("cuda")
    dp.ports.set(100, flags=T.PORT_VALID, bridge_id=0)     # a spare port for the link flaps
    dp.commit()
    live = NativeLivePath(dp, _vports(tmp_path, sc.n_pods, "k"), burst=256, ring_capacity=8192, queues=2).start()
    try:
        pods = []
        for i in range(sc.n_pods):
            slots, im = S.traffic(sc, 512, seed=30 + i, src_pods=np.array([i]))
            pods.append((str(tmp_path / f"k{i}"), slots, (im >> 16).astype(np.uint32)))
        kw = dict(duration_s=1.0, warmup_s=0.1, threads=2, burst=4, rate_pps=4e5)
        stop, err, n = threading.Event(), [], [0]
        flips0 = dp.flip_stats.get("table_flips", 0)

        def control():
            k = 0
            try:
                while not stop.is_set():
                    port = int(sc.pod_port[k % sc.n_pods])
                    dp.ports.update(port, mtu=1400 + (k % 50))
                    if k % 3 == 0:
                        dp.ports.set_link(100, k % 2 == 0)
                    if k % 7 == 0:
                        dp.acl.add(permit=False, dst=f"192.0.{k % 250}.0/24", dport=9)
                    dp.commit()
                    n[0] += 1
                    k += 1
                    time.sleep(0.001)
            except Exception as e:  # noqa: BLE001
                err.append(e)

        def measure():
            base = nf.trafgen_run(pods, **kw)
            stop.clear()
            n[0] = 0
            f0 = dp.flip_stats.get("table_flips", 0)
            th = threading.Thread(target=control)
            th.start()
            churn = nf.trafgen_run(pods, **kw)
            stop.set()
            th.join()
            assert not err, err
            flips = dp.flip_stats.get("table_flips", 0) - f0
            b99, c99 = np.percentile(base["lat_us"], 99), np.percentile(churn["lat_us"], 99)
            print(f"live commits {n[0]} in 1 s ({flips} table flips); one-way p50/p99 us: without "
                  f"{np.percentile(base['lat_us'], 50):.1f}/{b99:.1f}, with {np.percentile(churn['lat_us'], 50):.1f}/{c99:.1f}")
            assert n[0] >= 300 and flips >= n[0] - 1          # every commit a live flip: nothing paused
            assert live.error is None and churn["bad"] == 0
            assert churn["received"] >= 0.99 * churn["sent"]
            return b99, c99

        b99, c99 = measure()
        if not c99 < b99 + 10.0:
            b99, c99 = measure()
        assert c99 < b99 + 10.0
        assert dp.flip_stats.get("table_flips", 0) > flips0
    finally:
        live.stop()


@pytest.mark.gpu
def test_ctrl_mailbox_link_state_without_commit(tmp_path):
    """ctrl-net link state through the rings' control mailbox (ring.h RingCtrlRing): the resident
    grid writes the port entry itself and every workgroup restages its LDS port copy.  No commit,
    no epoch change; frames to the downed port are dropped exactly as the oracle drops them, and
    flow again once the link comes back - bit-exact with the batch path both ways."""
    nf = nfdp()
    dp, sc = _sfc("cuda")
    ref, _ = _sfc("cpu")
    live = NativeLivePath(dp, _vports(tmp_path, sc.n_pods, "x"), burst=256, ring_capacity=4096, queues=2).start()
    try:
        eps = {i: nf.MemifEndpoint(str(tmp_path / f"x{i}")) for i in range(sc.n_pods)}
        victim = int(sc.pod_port[2])

        def run(seed):
            slots, im = S.traffic(sc, 2000, seed=seed)
            exp, drops = _expected(ref, slots, im)
            src = im & 0xFFFF
            for i in range(sc.n_pods):
                fr = [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == i)[0]]
                sent = 0
                while sent < len(fr):
                    sent += eps[i].send(fr[sent:])
            got = {i: [] for i in range(sc.n_pods)}
            want = sum(map(len, exp.values()))

            def drained():
                for i in range(sc.n_pods):
                    got[i] += eps[i].recv()
                return sum(map(len, got.values())) >= want

            assert _until(drained, 10), (live.stats, live.error)
            time.sleep(0.05)
            for i in range(sc.n_pods):
                got[i] += eps[i].recv()
            for port in range(sc.n_pods):
                assert sorted(got[port]) == sorted(exp.get(port, [])), port
            return drops

        run(41)
        ring = live._rings[0]
        epoch0, flips0 = ring.eng.epoch, dp.flip_stats.get("table_flips", 0)
        for up in (False, True):
            dp.ports.set_link(victim, up)
            ref.ports.set_link(victim, up)
            ref.commit()
            t0 = time.perf_counter()
            assert dp.ctrl_ports([victim])
            dt = time.perf_counter() - t0
            drops = run(42 if not up else 43)
            print(f"link {'up' if up else 'down'} via the control mailbox in {dt * 1e6:.0f} us "
                  f"({dp.flip_stats['ctrl_last_s'] * 1e6:.1f} us of it from post to applied on the GPU); "
                  f"{drops} frames dropped by the oracle")
            if not up:
                assert drops > 0
        assert ring.eng.epoch == epoch0 and dp.flip_stats.get("table_flips", 0) == flips0   # no commit
        assert ring.eng.ctrl_done == ring.eng.ctrl_posted >= 2
        # the engine refuses writes outside the registered table buffers
        with pytest.raises(Exception):
            ring.eng.post_write(8, b"\0" * 4)
    finally:
        live.stop()
