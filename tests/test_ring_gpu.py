"""Persistent ring kernel (csrc/nfdp/ring.hip): bit-exact with the oracle, drain-on-stop, table
commits while running, device-side deadline, closed-loop latency probe."""
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
    """Several laps of the ring, then a table update while the kernel is resident: commit()
    drains + relaunches, and the next lap sees the new table."""
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
        g.commit()                               # ring is stopped, tables pushed, ring relaunched
        assert ring.running
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
