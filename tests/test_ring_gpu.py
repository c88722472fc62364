"""Persistent ring kernel (csrc/nfdp/ring.hip): bit-exact with the oracle, drain-on-stop, table
commits while running (flow updates by epoch flip, other tables by a table-set flip: the
kernel is never stopped), flow churn at >= 100K flows/s under a forwarding ring, device-side deadline,
closed-loop latency probe."""
import threading
import time

import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.ring import RingPath

CAP = 8192


def _build(device, n_flows=4000, seed=0, hash_mode="lds", n_acl=64):
    dp = DataPlane(device=device, flow_buckets=1 << 11, hash_mode=hash_mode, acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=16, n_flows=n_flows, n_acl=n_acl, seed=seed)
    dp.commit(full=True)
    return dp, sc


def _traffic(sc, n=CAP, seed=3):
    pk, im = S.traffic(sc, n, seed=seed)
    im[5] = (im[5] & 0xFFFF) | (10 << 16)   # malformed
    pk[7, 15] ^= 1                           # wrong vlan
    pk[9, 11] ^= 1                           # spoofed
    return pk, im


def test_ring_needs_gpu():
    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    with pytest.raises(RuntimeError):
        RingPath(dp, capacity=1024)


@pytest.mark.gpu
@pytest.mark.parametrize("coop,host_slots,hash_mode,n_acl", [
    (True, False, "lds", 64), (False, False, "lds", 64), (True, True, "lds", 64),
    # MFMA-hash kernels test two rule tiles per pass-1 branch; with coop each of the 4 waves scans
    # tiles wave, wave+4, ... so 200 rules (13 tiles, not a multiple of 8) exercise the nu == nt
    # clamp across waves
    (True, False, "mfma", 200), (False, False, "mfma", 200)])
def test_ring_bit_exact_and_counters(coop, host_slots, hash_mode, n_acl):
    g, sc = _build("cuda", hash_mode=hash_mode, n_acl=n_acl)
    c, _ = _build("cpu", hash_mode=hash_mode, n_acl=n_acl)
    pk, im = _traffic(sc)
    ring = RingPath(g, capacity=CAP, deadline_s=30.0, coop=coop, host_slots=host_slots)
    try:
        ring.stage(pk, im)
        ring.start()
        for _ in range(4):
            end = ring.publish(CAP // 4)
        ring.wait(end, 10.0)
        ring.stop()
        out, meta = ring.results()
    finally:
        ring.close()
    rc = c.run(pk, im)
    assert np.array_equal(meta, rc.meta)
    assert np.array_equal(out, rc.out)
    assert np.array_equal(g.port_counters(), c.port_counters())
    assert g.drop_counters() == c.drop_counters()
    g.harvest()
    c.harvest()
    assert np.array_equal(g.flow_totals, c.flow_totals)
    svc = ring.service_ticks()
    assert (svc > 0).all()


@pytest.mark.gpu
def test_ring_laps_and_commit_while_running():
    """Several laps of the ring, then a flow update while the kernel is resident: commit()
    writes the idle flow-table copy and flips the epoch (the kernel keeps running), and the next
    lap sees the new table.  Then a port change: a table-set flip, also without a relaunch."""
    g, sc = _build("cuda")
    c, _ = _build("cpu")
    pk, im = _traffic(sc)
    ring = RingPath(g, capacity=CAP, deadline_s=30.0)
    try:
        ring.stage(pk, im)
        ring.start()
        for _ in range(3):                       # three full laps, one lap in flight at a time
            end = ring.publish(CAP)
            ring.wait(end, 10.0)
        assert ring.completed() == 3 * CAP
        # steer every flow of the first pod's traffic to a drop chain: erase flows
        victims = [tuple(int(x) for x in k) for k in sc.keys[:500]]
        for dp in (g, c):
            for k in victims:
                dp.flows.erase(k)
        sent = g.commit()                        # flows only: epoch flip under the running kernel
        assert sent.get("flip") == 1 and g.flip_stats["flips"] == 1 and ring.eng.epoch & 1 == 1
        assert ring.running
        end = ring.publish(CAP)
        ring.wait(end, 10.0)
        assert ring.eng.grace_over()
        ring.stop()
        out, meta = ring.results()
        c.commit()
        rc = c.run(pk, im)
        assert np.array_equal(meta, rc.meta)
        assert np.array_equal(out, rc.out)
        # a port change is staged in LDS by the kernel: the coop ring flips to a new table set,
        # its workgroups restage LDS at the next chunk (no drain, no relaunch)
        ring.start()
        launches = ring.launches
        for dp in (g, c):
            dp.ports.update(int(sc.pod_port[1]), mtu=20)   # everything to pod 1 is now too big
        sent = g.commit()
        assert sent.get("table_flip") and ring.running and ring.launches == launches
        end = ring.publish(CAP)
        ring.wait(end, 10.0)
        ring.stop()
        out, meta = ring.results()
    finally:
        ring.close()
    c.commit()
    rc = c.run(pk, im)
    assert np.array_equal(meta, rc.meta)
    assert np.array_equal(out, rc.out)


@pytest.mark.gpu
def test_ring_deadline_and_idle_stop():
    g, sc = _build("cuda")
    pk, im = _traffic(sc, 1024)
    ring = RingPath(g, capacity=1024, deadline_s=0.5)
    try:
        ring.stage(pk, im)
        ring.start()
        time.sleep(1.0)                          # nothing published: the grid exits on its own
        t0 = time.time()
        ring.stop(timeout_s=10.0)
        assert time.time() - t0 < 5.0
        ring.start()                             # and can be relaunched
        end = ring.publish(1024)
        ring.wait(end, 10.0)
        ring.stop()
    finally:
        ring.close()


@pytest.mark.gpu
def test_ring_probe_latency():
    g, sc = _build("cuda")
    pk, im = _traffic(sc)
    ring = RingPath(g, capacity=CAP, deadline_s=60.0)
    try:
        ring.stage(pk, im)
        ring.start()
        lat, el = ring.probe(batches=400, batch=64, inflight=1)
        lat2, el2 = ring.probe(batches=200, batch=1024, inflight=4)
        ring.stop()
    finally:
        ring.close()
    assert len(lat) == 400 and len(lat2) == 200
    p50 = float(np.median(lat[40:]))
    print(f"ring p50 {p50:.2f} us  p99 {np.percentile(lat[40:], 99):.2f} us; "
          f"loaded p50 {np.median(lat2):.2f} us, {200 * 1024 / el2 / 1e6:.1f} Mpps")
    assert 0 < p50 < 2000


@pytest.mark.gpu
def test_ring_host_slots_latency():
    """Zero-copy host rings: the resident kernel reads/writes the frames in pinned host memory."""
    g, sc = _build("cuda")
    pk, im = _traffic(sc)
    ring = RingPath(g, capacity=CAP, deadline_s=60.0, host_slots=True)
    try:
        ring.stage(pk, im)
        ring.start()
        lat, _ = ring.probe(batches=400, batch=64, inflight=1)
        lat2, el2 = ring.probe(batches=200, batch=1024, inflight=4)
        ring.stop()
    finally:
        ring.close()
    p50 = float(np.median(lat[40:]))
    print(f"host-slot ring p50 {p50:.2f} us  p99 {np.percentile(lat[40:], 99):.2f} us; "
          f"loaded p50 {np.median(lat2):.2f} us, {200 * 1024 / el2 / 1e6:.1f} Mpps")
    assert 0 < p50 < 2000


def _nat(f, v):
    """(nat_ip, nat_port) of flow f at version v: each field names the flow and the version."""
    f = np.asarray(f, np.uint32)
    v = np.asarray(v, np.uint32)
    return (f << np.uint32(12)) | (v & np.uint32(0xFFF)), (f * np.uint32(7) + v) & np.uint32(0xFFFF)


@pytest.mark.gpu
def test_ring_live_flow_churn_no_torn_lookups():
    """>= 100K flow inserts / erases / action changes per second while the ring forwards: no
    lookup ever returns another flow's action or a half-updated one, flows that are never erased
    never miss, every published chunk completes, and the kernel is never stopped."""
    from dpu_operator_amd.dataplane import tables as T

    NT, CAPL = 16384, 1 << 16
    dp = DataPlane(device="cuda", flow_buckets=1 << 15, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=2 * NT, n_acl=32, seed=0, install_flows=False)
    keys = sc.keys
    ver = np.zeros(len(keys), np.int64)
    acts = sc.actions.copy()
    ip, port = _nat(np.arange(len(keys)), 0)
    acts[:, 1], acts[:, 2] = ip, port
    dp.flows.insert_many(keys, acts)
    dp.commit(full=True)
    pk, im, fl = S.traffic(sc, CAPL, seed=3, flows=np.arange(NT), return_flows=True)
    churn = np.arange(NT // 2, NT)              # trace flows that get erased and re-inserted
    rng = np.random.default_rng(9)
    fresh_base = 0x0B000000
    stop = threading.Event()
    stats = {"ops": 0, "commits": 0, "err": None}
    committed = {"ver": ver.copy()}   # versions every commit so far has made visible

    def updater():
        erased = np.zeros(0, np.int64)
        fresh_live = np.zeros((0, 4), np.uint32)
        k = 0
        try:
            while not stop.is_set():
                # 1) in-place action changes of 1000 trace flows (never-erased ones included)
                upd = rng.choice(NT // 2, 1000, replace=False)
                ver[upd] += 1
                a = acts[upd].copy()
                a[:, 1], a[:, 2] = _nat(upd, ver[upd])
                dp.flows.insert_many(keys[upd], a)
                # 2) re-insert the flows erased last round (new version), erase 500 others
                if len(erased):
                    ver[erased] += 1
                    a = acts[erased].copy()
                    a[:, 1], a[:, 2] = _nat(erased, ver[erased])
                    dp.flows.insert_many(keys[erased], a)
                cand = np.setdiff1d(churn, erased)
                erased = rng.choice(cand, 500, replace=False)
                dp.flows.erase_many(keys[erased])
                # 3) 1000 fresh flows in, the previous 1000 out (bucket churn, cuckoo moves)
                fk = T.flow_key(fresh_base + k * 1000 + np.arange(1000), 0x0A800001, 5000, 6000, 17, sc.bridge)
                dp.flows.insert_many(fk, np.tile(acts[:1], (1000, 1)))
                if len(fresh_live):
                    dp.flows.erase_many(fresh_live)
                fresh_live = fk
                k += 1
                snap = ver.copy()
                dp.commit()
                committed["ver"] = snap
                stats["ops"] += 1000 + 2 * 500 + 2 * 1000
                stats["commits"] += 1
        except BaseException as e:  # noqa: BLE001
            stats["err"] = e

    ring = RingPath(dp, capacity=CAPL, deadline_s=60.0, coop=False)
    laps = torn = stable_miss = churn_miss = hits = 0
    try:
        ring.stage(pk, im)
        ring.start()
        base = np.concatenate([ring.probe(batches=CAPL // 1024, batch=1024, inflight=2)[0] for _ in range(20)])
        th = threading.Thread(target=updater, daemon=True)
        t0 = time.perf_counter()
        th.start()
        p99 = []
        while time.perf_counter() - t0 < 3.0 and stats["err"] is None:
            v_lo = committed["ver"].copy()           # committed before the lap's first publish
            lat, _ = ring.probe(batches=CAPL // 1024, batch=1024, inflight=2)   # one lap, host-paced
            v_hi = ver.copy()
            p99.append(np.percentile(lat, 99))
            out, meta = ring.peek()
            port, _, reason = __import__("dpu_operator_amd.ops.packets", fromlist=["x"]).meta_fields(meta)
            ok = reason == 0
            nat_ip = out[:, 30:34].copy().view("<u4").ravel()
            nat_port = out[:, 38:40].copy().view("<u2").ravel().astype(np.uint32)
            f_ip = nat_ip >> 12
            v_ip = nat_ip & 0xFFF
            # the action of the flow itself, whole, and no older than what was committed before
            # the lap began (a stale cached bucket line would show an older version)
            good = (ok & (f_ip == fl) & (nat_port == ((fl.astype(np.uint32) * 7 + v_ip) & 0xFFFF))
                    & (v_ip >= (v_lo[fl] & 0xFFF)) & (v_ip <= (v_hi[fl] & 0xFFF)))
            torn += int((ok & ~good).sum())
            hits += int(good.sum())
            is_churn = fl >= NT // 2
            stable_miss += int((~ok & ~is_churn).sum())
            churn_miss += int((~ok & is_churn).sum())
            laps += 1
        stop.set()
        th.join(10)
        elapsed = time.perf_counter() - t0
        assert stats["err"] is None, stats["err"]
        assert ring.running
        assert ring.completed() == ring.eng.published      # no dropped chunk
        # for comparison: a change of an LDS-staged table still drains and relaunches the kernel
        t1 = time.perf_counter()
        dp.ports.update(int(sc.pod_port[0]), mtu=9000)
        dp.commit()
        relaunch_ms = (time.perf_counter() - t1) * 1e3
        assert ring.running
        ring.stop()
    finally:
        stop.set()
        ring.close()
    rate = stats["ops"] / elapsed
    print(f"live churn: {rate / 1e3:.0f}K flow ops/s, {stats['commits']} flips, {laps} laps, {hits} hits, "
          f"{churn_miss} churn misses; batch latency p99 {np.median(p99):.1f} us under churn vs "
          f"{np.percentile(base, 99):.1f} us without; relaunch commit {relaunch_ms:.2f} ms; flip stats {dp.flip_stats}")
    assert torn == 0 and stable_miss == 0
    assert laps >= 10 and hits > 0.9 * laps * CAPL * 0.5
    assert rate >= 100e3, rate
    assert dp.flip_stats["flips"] == stats["commits"]


@pytest.mark.gpu
def test_ring_table_updates_live_without_drain():
    """Port / ACL / link-state changes at ~1 kHz while a coop ring forwards: every commit flips
    the ring's table set (its workgroups restage LDS), the grid is never stopped or relaunched,
    every published chunk completes, and the final lap is bit-exact with the oracle holding the
    final tables."""
    g, sc = _build("cuda", n_acl=64)
    c, _ = _build("cpu", n_acl=64)
    pk, im = _traffic(sc)
    ring = RingPath(g, capacity=CAP, deadline_s=60.0, coop=True)
    stop = threading.Event()
    done = {"commits": 0, "laps": 0}
    err = []
    try:
        ring.stage(pk, im)
        ring.start()
        launches = ring.launches

        def control():
            k = 0
            try:
                while not stop.is_set():
                    port = int(sc.pod_port[k % 4 + 4])
                    g.ports.update(port, mtu=1400 + (k % 50))        # CreateBridgePort-style edits
                    if k % 3 == 0:
                        g.ports.set_link(port, k % 2 == 0)          # agent link flaps
                    if k % 7 == 0:
                        g.acl.add(permit=False, dst=f"192.0.{k % 250}.0/24", dport=9)   # ACL edits
                    g.commit()
                    done["commits"] += 1
                    k += 1
                    time.sleep(0.001)
            except Exception as e:  # noqa: BLE001
                err.append(e)

        th = threading.Thread(target=control)
        th.start()
        t_end = time.time() + 3.0
        while time.time() < t_end:
            end = ring.publish(CAP)
            ring.wait(end, 10.0)
            done["laps"] += 1
        stop.set()
        th.join()
        assert not err, err
        assert ring.running and ring.eng.alive() and ring.launches == launches
        assert done["commits"] >= 500 and g.flip_stats["table_flips"] >= done["commits"] - 1
        assert ring.completed() == ring.eng.published
        per_commit_ms = 1e3 * g.flip_stats["table_update_s"] / g.flip_stats["table_flips"]
        print(f"live table commits: {done['commits']} in 3 s, {per_commit_ms:.3f} ms each, ring stall 0, "
              f"{done['laps']} laps")
        # the stall a commit costs the packets: closed-loop chunk latency with and without a
        # table flip every millisecond (a workgroup restages its LDS copy at the first chunk of
        # a new set; nothing is drained)
        base, _ = ring.probe(batches=3000, batch=64, inflight=1)
        stop.clear()
        th = threading.Thread(target=control)
        th.start()
        flips0 = g.flip_stats["table_flips"]
        churn, el = ring.probe(batches=20000, batch=64, inflight=1)
        stop.set()
        th.join()
        assert not err, err
        nflip = g.flip_stats["table_flips"] - flips0
        stall = float(np.max(churn) - np.percentile(base, 50))
        print(f"probe p50/p99/max us: idle {np.percentile(base, 50):.2f}/{np.percentile(base, 99):.2f}/"
              f"{np.max(base):.2f}, with {nflip} table flips {np.percentile(churn, 50):.2f}/"
              f"{np.percentile(churn, 99):.2f}/{np.max(churn):.2f}; worst commit stall {stall:.2f} us")
        assert nflip >= 100 and ring.launches == launches
        assert np.percentile(churn, 99) < np.percentile(base, 99) + 50.0
        # the final tables: mirror them into the oracle and compare one more lap
        c.ports.a[:] = g.ports.a
        c.ports.version += 1
        c.acl.rules = list(g.acl.rules)
        c.acl.version += 1
        c.commit()
        g.commit()
        end = ring.publish(CAP)
        ring.wait(end, 10.0)
        ring.stop()
        out, meta = ring.results()
    finally:
        stop.set()
        ring.close()
    rc = c.run(pk, im)
    assert np.array_equal(meta, rc.meta)
    assert np.array_equal(out, rc.out)
