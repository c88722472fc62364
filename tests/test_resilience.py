"""Checkpoint/resume, fault injection and tracing (SURVEY §5 aux subsystems)."""
from __future__ import annotations

import json
import os
import shutil
import tempfile

import grpc
import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane import snapshot
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P
from dpu_operator_amd.proto import vendor
from dpu_operator_amd.proto.grpcutil import Stub, retry_service_config, unix_target
from dpu_operator_amd.utils.faults import FAULTS, FaultError, FaultInjector
from dpu_operator_amd.utils.journal import Journal
from dpu_operator_amd.utils.paths import PathManager
from dpu_operator_amd.utils.trace import Tracer
from dpu_operator_amd.cni.netlink import FakeNetlink


@pytest.fixture
def tmp():
    d = tempfile.mkdtemp(prefix="dpur", dir="/tmp")
    yield d
    shutil.rmtree(d, ignore_errors=True)


def test_journal_snapshot_and_torn_tail(tmp):
    j = Journal(tmp, "t", compact_every=3)
    for i in range(2):
        j.append({"i": i})
    assert not j.needs_compaction()
    j.append({"i": 2})
    assert j.needs_compaction()
    j.compact({"upto": 2})
    j.append({"i": 3})
    with open(j.log_path, "a") as f:
        f.write('{"i": 4, "trunc')  # crash mid-append
    snap, recs = Journal(tmp, "t").load()
    assert snap == {"upto": 2, "_journal_seq": 3} and recs == [{"i": 3, "seq": 4}]


def test_dataplane_snapshot_roundtrip(tmp):
    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    sc = S.build_sfc(dp, n_pods=8, n_flows=1500, n_acl=64, seed=3)
    dp.commit(full=True)
    pk, im = S.traffic(sc, 2048, seed=5)
    r1 = dp.run(pk, im)
    path = os.path.join(tmp, "dp.npz")
    info = snapshot.save(dp, path)
    assert info["flows"] == 1500
    dp2 = DataPlane(device="cpu", flow_buckets=1 << 10)
    snapshot.load(dp2, path)
    r2 = dp2.run(pk, im)
    assert np.array_equal(r1.meta, r2.meta) and np.array_equal(r1.out, r2.out)
    dp.run(pk, im)
    dp.harvest()
    dp2.harvest()
    # counters follow the flow key across the restore (bucket positions may differ)
    got = [(dp.flow_counters(k), dp2.flow_counters(k)) for k in sc.keys[:400]]
    assert all(a == b for a, b in got)
    assert sum(a != (0, 0) for a, _ in got) > 100


def _populate(vsp):
    vsp._call("Init", vsp.init, True, "dpu0")
    vsp._call("SetNumVfs", vsp.set_num_vfs, 8)
    vsp._call("CreateBridgePort", vsp.create_bridge_port, "host0-0", bytes.fromhex("001122334455"), 1, ["2"])
    vsp._call("CreateNetworkFunction", vsp.create_network_function, vsp.vports[6]["mac"], vsp.vports[7]["mac"])


def _probe(vsp):
    frames, _ = P.craft(1, dmac="02:00:00:00:ff:01", smac="00:11:22:33:44:55", src_ip=0x0A000002,
                        dst_ip=0x08080808, sport=1234, dport=53)
    reply, _ = P.craft(1, dmac="00:11:22:33:44:55", smac="02:00:00:00:ff:01", src_ip=0x08080808,
                       dst_ip=0x0A000002, sport=53, dport=1234)
    return [vsp.process(frames, [0])[1][0], vsp.process(reply, [6])[1][0], vsp.process(reply, [4000])[1][0]]


def test_gpu_vsp_resumes_from_journal(tmp):
    from dpu_operator_amd.vsp.gpu import GpuVsp

    pm = PathManager(tmp)
    nl = FakeNetlink()
    a = GpuVsp(pm, device="cpu", nl=nl, flow_buckets=1 << 8, state_dir=os.path.join(tmp, "state"))
    _populate(a)
    a.on_gpu_chain("sfc-a", ["nat", "ttl"])
    before = _probe(a)
    macs = {i: v["mac"] for i, v in a.vports.items()}
    # "crash": a new process on the same state dir (fresh netlink: the taps are recreated too)
    b = GpuVsp(pm, device="cpu", nl=FakeNetlink(), flow_buckets=1 << 8, state_dir=os.path.join(tmp, "state"))
    assert b.restored == 5
    assert {i: v["mac"] for i, v in b.vports.items()} == macs
    assert b.bridge_ports == {"host0-0": 0} and len(b.nfs) == 1 and b.gpu_chains == a.gpu_chains
    assert _probe(b) == before
    assert int(P.meta_fields(np.array([before[0]]))[0][0]) == 6  # VF -> NF ingress


def test_gpu_vsp_checkpoint_then_tail(tmp):
    from dpu_operator_amd.vsp.gpu import GpuVsp

    pm = PathManager(tmp)
    sd = os.path.join(tmp, "state")
    a = GpuVsp(pm, device="cpu", nl=FakeNetlink(), flow_buckets=1 << 8, state_dir=sd)
    _populate(a)
    keys = np.array([[0x0A000002, 0x08080808, (1234 << 16) | 53, 17]], np.uint32)
    acts = np.zeros((1, 4), np.uint32)
    acts[0, 0] = 5 << 16
    a.install_flows(keys, acts)
    a.checkpoint()
    a._call("DeleteBridgePort", a.delete_bridge_port, "host0-0")  # journal tail after the snapshot
    b = GpuVsp(pm, device="cpu", nl=FakeNetlink(), flow_buckets=1 << 8, state_dir=sd)
    assert b.restored == 1 and b.bridge_ports == {} and len(b.nfs) == 1
    assert b.dp.flows.find(keys[0]) >= 0
    assert b.vports[0]["role"] == "free"


def test_gpu_vsp_flows_survive_without_checkpoint(tmp):
    """Flows installed after the last checkpoint are journaled: a crash before the
    next checkpoint must not lose them; bulk installs checkpoint instead."""
    from dpu_operator_amd.vsp import gpu as G

    pm = PathManager(tmp)
    sd = os.path.join(tmp, "state")
    a = G.GpuVsp(pm, device="cpu", nl=FakeNetlink(), flow_buckets=1 << 12, state_dir=sd)
    _populate(a)
    keys = np.array([[0x0A000002, 0x08080808, (1234 << 16) | 53, 17],
                     [0x0A000003, 0x08080404, (999 << 16) | 80, 6]], np.uint32)
    acts = np.zeros((2, 4), np.uint32)
    acts[:, 0] = 5 << 16
    a.install_flows(keys, acts)              # no checkpoint afterwards
    b = G.GpuVsp(pm, device="cpu", nl=FakeNetlink(), flow_buckets=1 << 12, state_dir=sd)
    assert all(b.dp.flows.find(k) >= 0 for k in keys)
    big = np.zeros((G.JOURNAL_FLOWS_MAX + 1, 4), np.uint32)
    big[:, 0] = 0x0B000000 + np.arange(len(big))
    big[:, 3] = 17
    b.install_flows(big, np.zeros_like(big))
    assert os.path.getsize(b.journal.log_path) == 0     # bulk load -> checkpoint, no giant record
    c = G.GpuVsp(pm, device="cpu", nl=FakeNetlink(), flow_buckets=1 << 12, state_dir=sd)
    assert len(c.dp.flows) == len(big) + 2


def test_journal_compaction_crash_does_not_replay_twice(tmp):
    """Crash between snapshot replace and log truncate: records covered by the snapshot carry
    seq <= _journal_seq and are skipped on load."""
    j = Journal(tmp, "t")
    for i in range(3):
        j.append({"i": i})
    log = open(j.log_path).read()
    j.compact({"upto": 3})
    with open(j.log_path, "w") as f:   # the truncate "never happened"
        f.write(log)
    j2 = Journal(tmp, "t")
    snap, recs = j2.load()
    assert snap["upto"] == 3 and recs == []
    j2.append({"i": 3})
    assert [r["i"] for r in j2.load()[1]] == [3] and j2.seq == 4


def test_fault_injector_semantics():
    f = FaultInjector()
    f.arm("x", "error", count=2, every=2)
    assert f.check("x") is False
    with pytest.raises(FaultError):
        f.check("x")
    f.check("x")
    with pytest.raises(FaultError):
        f.check("x")
    assert f.check("x") is False and f.fired("x") == 2
    f.load_env("y:drop:1,z:delay=0.01:1")
    assert f.check("y") is True and f.check("y") is False
    assert f.check("z") is False and f.fired("z") == 1


def test_vsp_unavailable_is_retried_by_client(tmp):
    """An injected UNAVAILABLE on the VSP is absorbed by the daemon's gRPC retry policy."""
    from dpu_operator_amd.vsp.base import MockVsp

    pm = PathManager(tmp)
    vsp = MockVsp(pm).start()
    FAULTS.arm("vsp.Init", "unavailable", count=2)
    try:
        ch = grpc.insecure_channel(unix_target(pm.vendor_plugin_socket()),
                                   options=[("grpc.service_config", retry_service_config(initial="0.05s")),
                                            ("grpc.enable_retries", 1)])
        stub = Stub(ch, vendor, "LifeCycleService")
        r = stub.Init(vendor.InitRequest(dpu_mode=True, dpu_identifier="x"), timeout=20)
        assert r.port == 50051 and FAULTS.fired("vsp.Init") == 2
        FAULTS.arm("vsp.Init", "error", count=1)
        with pytest.raises(grpc.RpcError) as ei:
            stub.Init(vendor.InitRequest(dpu_mode=True, dpu_identifier="x"), timeout=20)
        assert ei.value.code() == grpc.StatusCode.INTERNAL
        ch.close()
    finally:
        FAULTS.disarm()
        vsp.stop()


def test_tracer_exports_chrome_trace(tmp):
    t = Tracer()
    t.enable()
    with t.span("a", k=1):
        pass
    with pytest.raises(ValueError):
        with t.span("b"):
            raise ValueError("boom")
    path = os.path.join(tmp, "trace.json")
    assert t.export(path) == 2
    evs = json.load(open(path))["traceEvents"]
    assert [e["name"] for e in evs] == ["a", "b"] and "boom" in evs[1]["args"]["error"]
    assert all(e["ph"] == "X" and e["dur"] >= 0 for e in evs)


def test_dataplane_spans_recorded():
    from dpu_operator_amd.utils.trace import TRACER

    TRACER.clear()
    TRACER.enable()
    try:
        dp = DataPlane(device="cpu", flow_buckets=1 << 8)
        sc = S.build_sfc(dp, n_pods=4, n_flows=100, n_acl=8)
        dp.commit(full=True)
        pk, im = S.traffic(sc, 64)
        dp.run(pk, im)
        assert TRACER.events("dataplane.run") and TRACER.events("dataplane.commit")
    finally:
        TRACER.enable(False)
        TRACER.clear()


class _SockPort:
    """A TAP stand-in: one end of an AF_UNIX datagram socketpair (frame boundaries kept)."""

    def __init__(self, sock):
        import socket as _s

        self.s = sock
        self.s.setblocking(False)
        self.fd = sock.fileno()
        self._err = (BlockingIOError, _s.timeout)

    def read(self):
        try:
            return self.s.recv(1 << 16)
        except self._err:
            return None

    def write(self, frame):
        self.s.send(frame)
        return True


def test_livepath_cycle_failure_marks_unhealthy_and_recovers():
    """A failing LivePath cycle (fault point livepath.poll) marks the path unhealthy and the loop
    restarts itself; once cycles succeed again it is healthy and forwards."""
    import socket
    import time

    from dpu_operator_amd.dataplane import tables as T
    from dpu_operator_amd.dataplane.netio import LivePath

    dp = DataPlane(device="cpu", flow_buckets=1 << 10, mac_slots=1 << 10)
    for p in range(2):
        dp.ports.set(p, flags=T.PORT_VALID, bridge_id=3, default_out=1 - p)
    dp.commit(full=True)
    pairs = [socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM) for _ in range(2)]
    live = LivePath(dp, {0: _SockPort(pairs[0][0]), 1: _SockPort(pairs[1][0])})
    FAULTS.arm("livepath.poll", "error", count=3)
    try:
        live.start()
        end = time.monotonic() + 5
        while live.restarts < 3 and time.monotonic() < end:
            time.sleep(0.01)
        assert live.restarts >= 3 and isinstance(live.error, FaultError)
        while not live.healthy and time.monotonic() < end:
            time.sleep(0.01)
        assert live.healthy
        fr, ln = P.craft(1, dmac="02:00:00:00:00:02", smac="02:00:00:00:00:01", src_ip=1, dst_ip=2, sport=3, dport=4)
        pairs[0][1].send(bytes(fr[0, : ln[0]]))
        pairs[1][1].settimeout(5)
        assert pairs[1][1].recv(1 << 16) == bytes(fr[0, : ln[0]])
    finally:
        FAULTS.disarm("livepath.poll")
        live.stop()
        for a, b in pairs:
            a.close()
            b.close()
