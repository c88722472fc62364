"""Native control agent: mailbox ring, ctrl-net commands, heartbeat failure detection, reset,
plugin relay, standalone binary.

Mirrors what the reference's octep_cp_agent does (SURVEY NAT1-NAT10, K15) — the reference ships
no tests for it; expectations here come from its protocol definition (octep_ctrl_net.h command
set + version gating, octep_ctrl_mbox.c ring semantics).  The SoC config parser is checked
against the reference's own cn106xx.cfg text (read as text only).
"""
from __future__ import annotations

import os
import select
import signal
import socket
import struct
import subprocess
import tempfile
import time
from pathlib import Path

import pytest

from dpu_operator_amd import cpagent
from dpu_operator_amd.cpagent import GET, H2F, SET, Reply

A = cpagent.native()
REF_CFG = Path("/root/reference/internal/daemon/vendor-specific-plugins/marvell/vendor/pcie_ep_octeon_target/"
               "target/apps/octep_cp_agent/cn106xx.cfg")


@pytest.fixture
def tmp():
    d = tempfile.mkdtemp(prefix="cpa", dir="/tmp")
    yield Path(d)
    for p in Path(d).iterdir():
        p.unlink()
    os.rmdir(d)


def test_ring_fifo_wraparound_and_full(tmp):
    mb = A.Mailbox.create(str(tmp / "mb"), 288 + 2 * 256)
    assert mb.queue_bytes == 256
    sent = []
    got = []
    rng = __import__("random").Random(1)
    for i in range(400):  # many laps around a 256-B ring with odd sizes
        n = rng.randrange(0, 60)
        payload = bytes(rng.randrange(256) for _ in range(n))
        if mb.h2f_push(0, 1, -1 if i % 2 else 3, 1, i & 0xFFFF, payload):
            sent.append((i & 0xFFFF, payload, i % 2 == 0))
        while rng.random() < 0.5:
            m = mb.h2f_pop()
            if m is None:
                break
            got.append(m)
    while (m := mb.h2f_pop()) is not None:
        got.append(m)
    assert len(got) == len(sent) and len(sent) > 300
    for (mid, payload, is_vf), (pem, pf, vf_flag, vf_idx, flags, gid, data) in zip(sent, got):
        assert (gid, data, vf_flag, pf) == (mid, payload, is_vf, 1)
        assert vf_idx == (3 if is_vf else 0)
    # full: a 256-B ring holds at most 248 bytes of records
    assert mb.h2f_push(0, 0, -1, 1, 1, b"x" * 200)
    assert not mb.h2f_push(0, 0, -1, 1, 2, b"y" * 40)
    assert mb.h2f_pop()[6] == b"x" * 200
    with pytest.raises(ValueError):
        A.Mailbox.create(str(tmp / "small"), 300)


def _poke(path, off, fmt, *vals):
    with open(path, "r+b") as f:
        f.seek(off)
        f.write(struct.pack(fmt, *vals))


def test_ring_rejects_peer_corrupted_cursors_and_geometry(tmp):
    """The region is peer-writable: cursors >= sz or unaligned, mismatched or oversized queue
    sizes must be rejected instead of steering memcpy outside the mapping."""
    path = str(tmp / "mb")
    mb = A.Mailbox.create(path, 288 + 2 * 256)
    assert mb.h2f_push(0, 1, -1, 1, 7, b"abc")
    _poke(path, 256, "<I", 4096)            # H2F prod far beyond sz
    with pytest.raises(RuntimeError, match="cursor"):
        mb.h2f_pop()
    assert mb.h2f_pop() is None             # the corrupt ring was reset, not read
    _poke(path, 256 + 4, "<I", 13)          # H2F cons not 8-aligned
    with pytest.raises(RuntimeError, match="cursor"):
        mb.h2f_push(0, 1, -1, 1, 8, b"x")
    # the shared sz field is ignored after binding (cached) ...
    _poke(path, 256 + 8, "<I", 1 << 30)
    assert mb.h2f_push(0, 1, -1, 1, 9, b"ok") and mb.h2f_pop()[6] == b"ok"
    # ... and a region whose queues no longer fit is refused at open
    with pytest.raises(RuntimeError, match="geometry"):
        A.Mailbox.open(path)
    _poke(path, 256 + 8, "<I", 256)
    _poke(path, 272 + 8, "<I", 128)         # H2F and F2H sizes disagree
    with pytest.raises(RuntimeError, match="geometry"):
        A.Mailbox.open(path)
    _poke(path, 272 + 8, "<I", 256)
    assert A.Mailbox.open(path).queue_bytes == 256


def test_parse_reference_soc_config():
    if not REF_CFG.exists():
        pytest.skip("reference config not mounted")
    summary = A.config_summary(REF_CFG.read_text())
    pem_idx, pfs = summary[0]
    assert pem_idx == 0 and len(pfs) == 1
    pf = pfs[0]
    assert pf["hb_interval"] == 1000 and pf["hb_miss_count"] == 20 and pf["speed"] == 10000
    assert pf["mac"][:5] == bytes([0, 0, 0, 1, 1])
    assert len(pf["vfs"]) >= 4 and pf["vfs"][1][1] == bytes([0, 0, 0, 2, 1, 1])
    tree = A.parse_config('a = 0x10L; b = [1, 2,]; c = ( { x = "p" "q"; } ); /* c */ d : true; # e\n')
    assert tree == {"a": 16, "b": [1, 2], "c": [{"x": "pq"}], "d": True}
    with pytest.raises(RuntimeError, match="line 2"):
        A.parse_config("a = 1;\nb = ;")


@pytest.fixture
def running(tmp):
    ag = A.Agent(str(tmp / "mbox"), cpagent.default_config(n_vfs=4, hb_interval_ms=20, hb_miss_count=3))
    ag.start()
    host = A.HostCtrl(str(tmp / "mbox"))
    assert host.wait_ready(2000)
    yield ag, host
    ag.stop()


def test_ctrl_net_commands(running):
    ag, host = running
    r = host.request(0, 0, 1, H2F.MTU, GET)
    assert r["reply"] == Reply.OK and r["val"] == 1500
    assert host.request(0, 0, 1, H2F.MTU, SET, 9000)["val"] == 9000
    assert host.request(0, 0, 1, H2F.MTU, SET, 20)["reply"] == Reply.INVALID_PARAM
    assert ag.iface(0, 0, 1)["mtu"] == 9000
    mac = bytes([2, 1, 2, 3, 4, 5])
    assert host.request(0, 0, 2, H2F.MAC, SET, mac=mac)["mac"] == mac
    assert host.request(0, 0, 2, H2F.MAC, SET, mac=bytes([1, 0, 0, 0, 0, 1]))["reply"] == Reply.INVALID_PARAM
    assert host.request(0, 0, -1, H2F.LINK_STATUS, SET, 0)["val"] == 0
    assert host.request(0, 0, -1, H2F.RX_STATE, GET)["val"] == 1
    li = host.request(0, 0, 0, H2F.LINK_INFO, GET)["link_info"]
    assert li["speed"] == 200000 and li["supported_modes"] == 3
    assert host.request(0, 0, 0, H2F.LINK_INFO, SET, link={"advertised_modes": 4})["reply"] == Reply.INVALID_PARAM
    assert host.request(0, 0, 0, H2F.LINK_INFO, SET, link={"advertised_modes": 2, "speed": 100000})["link_info"][
        "advertised_modes"] == 2
    info = host.request(0, 0, -1, H2F.GET_INFO)["info"]
    assert info["hb_interval_ms"] == 20 and info["hb_miss_count"] == 3
    ag.update_stats(0, 0, 3, 10, 640, 7, 448, 1, 0)
    st = host.request(0, 0, 3, H2F.GET_IF_STATS)
    assert (st["rx"]["pkts"], st["rx"]["octets"], st["tx"]["pkts"], st["rx"]["dropped"]) == (10, 640, 7, 1)
    assert host.request(0, 0, 3, H2F.OFFLOADS, SET, offloads=(3, 5))["tx_offloads"] == 5
    assert host.request(0, 0, 9, H2F.MTU)["reply"] == Reply.INVALID_PARAM          # unknown VF
    assert host.request(0, 0, 0, 0)["reply"] == Reply.INVALID_PARAM                 # invalid command
    assert host.request(0, 0, 3, H2F.DEV_REMOVE)["reply"] == Reply.OK
    assert host.request(0, 0, 3, H2F.MTU)["reply"] == Reply.INVALID_PARAM          # removed
    c = ag.counters()
    assert c["requests"] >= 14 and c["bad_msgs"] == 0


def test_version_gating(tmp):
    ag = A.Agent(str(tmp / "mbox"), cpagent.default_config(n_vfs=1))
    ag.start()
    try:
        host = A.HostCtrl(str(tmp / "mbox"), A.version(1, 0, 0))
        assert host.wait_ready(2000)
        assert host.request(0, 0, 0, H2F.OFFLOADS)["reply"] == Reply.UNSUPPORTED  # added in 1.0.1
        assert host.request(0, 0, 0, H2F.MTU)["reply"] == Reply.OK
    finally:
        ag.stop()


def test_link_notify_reset_and_heartbeat_failure_detection(running):
    ag, host = running
    ag.set_link(0, 0, 2, False)
    deadline = time.time() + 2
    notes = []
    while time.time() < deadline and not notes:
        notes = host.notifications()
        time.sleep(0.005)
    assert notes == [(1, 0)]  # F2H LINK_STATUS, down
    host.request(0, 0, 1, H2F.MTU, SET, 4000)
    assert host.reset(2000)  # PERST: state reloaded from the configuration
    assert host.request(0, 0, 1, H2F.MTU)["val"] == 1500
    assert ag.counters()["resets"] == 1
    time.sleep(0.1)
    assert host.fw_alive()
    ag.stop()  # fw dies: heartbeat stops
    time.sleep(0.2)
    assert not host.fw_alive()  # 3 missed 20-ms intervals
    with pytest.raises(RuntimeError, match="timed out"):
        host.request(0, 0, 1, H2F.MTU, timeout_ms=50)


def _frame(typ, payload=b"", seq=0):
    return struct.pack("<IHHII", 0x50555044, typ, 0, len(payload), seq) + payload


def _read_frame(s, timeout=2.0):
    buf = b""
    end = time.time() + timeout
    while time.time() < end:
        if len(buf) >= 16:
            magic, typ, _, n, seq = struct.unpack("<IHHII", buf[:16])
            if len(buf) >= 16 + n:
                return typ, buf[16:16 + n]
        r, _, _ = select.select([s], [], [], 0.05)
        if r:
            chunk = s.recv(4096)
            if not chunk:
                break
            buf += chunk
    raise TimeoutError("no frame")


def test_plugin_relay(tmp):
    ag = A.Agent(str(tmp / "mbox"), cpagent.default_config(n_vfs=1))
    ag.start(plugin_port=0)
    try:
        host = A.HostCtrl(str(tmp / "mbox"))
        assert host.wait_ready(2000)
        port = ag.plugin_port
        assert port > 0
        c1 = socket.create_connection(("127.0.0.1", port))
        c1.sendall(_frame(1))
        typ, body = _read_frame(c1)
        assert typ == 2 and struct.unpack("<I", body)[0] == A.CP_VERSION_MAX
        # host custom message -> plugin
        assert host.send_custom(0, 0, b"hello plugin")
        typ, body = _read_frame(c1)
        assert typ == 4 and body[16:] == b"hello plugin"
        # plugin message -> host (custom flag)
        hdr = struct.pack("<HHIIHH", 0, 0, 0, 0, 0, 0)
        c1.sendall(_frame(3, hdr + b"from plugin"))
        deadline = time.time() + 2
        got = []
        while time.time() < deadline and not got:
            got = host.custom()
            time.sleep(0.005)
        assert got and got[0][6] == b"from plugin" and got[0][4] == cpagent.FLAG_CUSTOM
        # at most two plugin clients
        c2 = socket.create_connection(("127.0.0.1", port))
        c3 = socket.create_connection(("127.0.0.1", port))
        c3.settimeout(2)
        time.sleep(0.1)
        assert c3.recv(16) == b""  # closed by the server
        # reset is broadcast as an event
        assert host.reset(2000)
        typ, body = _read_frame(c1)
        assert typ == 5 and struct.unpack("<I", body[:4])[0] == 1
        for c in (c1, c2, c3):
            c.close()
    finally:
        ag.stop()


def test_standalone_binary(tmp):
    from dpu_operator_amd.native import build

    exe = build.build_exe("dpu-cp-agent")
    cfg = tmp / "a.cfg"
    cfg.write_text(cpagent.default_config(n_vfs=2, hb_interval_ms=50))
    mbox = tmp / "mbox"
    p = subprocess.Popen([str(exe), str(cfg), "--mbox", str(mbox), "--plugin-port", "-1"], stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE, text=True)
    try:
        line = p.stdout.readline()
        assert "ready" in line and "3 functions" in line
        host = A.HostCtrl(str(mbox))
        assert host.wait_ready(2000)
        assert host.request(0, 0, 1, H2F.MTU, SET, 2000)["val"] == 2000
    finally:
        p.send_signal(signal.SIGTERM)
        out, err = p.communicate(timeout=10)
    assert p.returncode == 0 and "stopped" in out


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_agent_sanitizer_stress(kind):
    """Race / memory-error detection on the native agent: ring torture + agent under concurrent
    requests, link flaps, stats updates, notification drains and PERST resets (host-only
    sanitizer build of csrc/agent/stress_main.cpp)."""
    import subprocess

    from dpu_operator_amd.native.build import build_sanitized

    try:
        exe = build_sanitized(kind)
    except RuntimeError as e:  # toolchain without the sanitizer runtime
        pytest.skip(str(e)[:200])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(exe), "1.5"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")


def test_doorbell_request_latency(running):
    """Requests wake the agent through the H2F futex doorbell and responses wake the host through
    the F2H one: the round trip is not bounded below by a polling period."""
    _, host = running
    for _ in range(20):
        host.request(0, 0, 1, H2F.MTU)
    ts = []
    for _ in range(200):
        t = time.perf_counter()
        host.request(0, 0, 1, H2F.MTU)
        ts.append(time.perf_counter() - t)
    ts.sort()
    p50_us = ts[len(ts) // 2] * 1e6
    print(f"mailbox round trip p50 {p50_us:.1f} us")
    assert p50_us < 150, f"p50 mailbox round trip {p50_us:.0f} us"
