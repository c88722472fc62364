"""The live packet loop (dataplane/netio.py LivePath) over socket-pair "netdevs": no privileges
needed, so it runs everywhere (the TAP + network-namespace version is tests/test_livepath.py).

A socket pair stands in for each vport: the test writes frames into one end (what the pod sends)
and reads what the data plane delivered from the same end (what the pod receives).  The bridge is
OvS-NORMAL style (learning, ARP copies to the slow path, flooding, a mirror port), the traffic mixes
broadcast ARP, unknown unicast, learned unicast and jumbo frames.

* CPU: the batch engine over the C++ oracle; delivered frames are checked against the bridge's
  expected behaviour.
* GPU: the persistent ring kernel with its slots in pinned host memory (engine="ring") must
  deliver exactly what the oracle's batch loop delivers (per port, as multisets: replicas come off
  the side list in atomic order).
"""
from __future__ import annotations

import socket

import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.netio import LivePath
from dpu_operator_amd.ops import packets as P

MACS = ["02:00:00:00:0a:01", "02:00:00:00:0b:01", "02:00:00:00:0c:01", "02:00:00:00:0d:01"]
BR = 5


class SockPort:
    """A vport made of a datagram socket pair: `a` is the data plane's end, `b` the pod's."""

    def __init__(self):
        self.a, self.b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
        for s in (self.a, self.b):
            s.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 1 << 21)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 21)
        self.a.setblocking(False)
        self.b.setblocking(False)
        self.fd = self.a.fileno()

    # data-plane side (LivePath)
    def read(self):
        try:
            return self.a.recv(1 << 16)
        except BlockingIOError:
            return None

    def write(self, frame: bytes) -> bool:
        self.a.send(frame)
        return True

    # pod side (the test)
    def inject(self, frame: bytes) -> None:
        self.b.send(frame)

    def drain(self) -> list[bytes]:
        out = []
        while True:
            try:
                out.append(self.b.recv(1 << 16))
            except BlockingIOError:
                return out

    def close(self) -> None:
        self.a.close()
        self.b.close()


def _bridge(device):
    dp = DataPlane(device=device, flow_buckets=1 << 10, mac_slots=1 << 10)
    for p in range(4):
        dp.ports.set(p, flags=T.PORT_VALID | T.PORT_LEARN | T.PORT_ARP_TRAP, bridge_id=BR)
    dp.flood.set_members(BR, [0, 1, 2, 3])
    dp.ports.set_mirror(2, 3)
    dp.commit(full=True)
    return dp


def _frame(dst, src, size, seq):
    fr, ln = P.craft_full(1, dmac=dst, smac=src, src_ip=0x0A000001 + seq, dst_ip=0x0A000002, sport=1000 + seq,
                          dport=2000, frame_len=size, payload_seed=seq)
    return bytes(fr[0, : int(ln[0])])


def _trace():
    """(in_port, frame) bursts: ARP broadcast, replies, unknown unicast, learned unicast, jumbo."""
    arp, al = P.craft_arp(1, smac=MACS[0], sender_ip=0x0A000001, target_ip=0x0A000002)
    b1 = [(0, bytes(arp[0, : int(al[0])]))]
    b2 = [(1, _frame(MACS[0], MACS[1], 64, 1)), (2, _frame("02:00:00:00:0f:0f", MACS[2], 200, 2))]
    b3 = [(0, _frame(MACS[1], MACS[0], 1500, 3)), (0, _frame(MACS[2], MACS[0], 9000, 4)),
          (3, _frame(MACS[0], MACS[3], 576, 5)), (2, _frame(MACS[0], MACS[2], 64, 6))]
    return [b1, b2, b3]


def _run(dp, engine):
    ports = {i: SockPort() for i in range(4)}
    punts = []
    live = LivePath(dp, ports, engine=engine, ring_capacity=1024,
                    on_punt=lambda f, p, r: punts.append((p, r, f)))
    got = []
    try:
        for burst in _trace():
            for p, f in burst:
                ports[p].inject(f)
            n = 0
            for _ in range(20):
                n += live.poll_once(0.05)
                if n >= len(burst):
                    break
            assert n == len(burst)
            got.append({p: sorted(ports[p].drain()) for p in ports})
        return got, punts, live.stats, dp
    finally:
        live.stop()
        for p in ports.values():
            p.close()


def test_batch_engine_over_socket_ports_oracle():
    got, punts, stats, dp = _run(_bridge("cpu"), "batch")
    b1, b2, b3 = got
    # ARP broadcast from port 0: flooded to 1, 2, 3 and copied to the slow path
    assert [len(b1[p]) for p in range(4)] == [0, 1, 1, 1]
    assert [r for _, r, _ in punts] == [12]
    # the reply to the learned MAC goes to port 0 only; unknown unicast from port 2 floods to
    # 0, 1, 3, and port 3 (port 2's mirror) also gets the mirror copy
    assert [len(b2[p]) for p in range(4)] == [2, 1, 0, 2]
    # learned unicast incl. a 9000-B jumbo frame
    assert any(len(f) == 9000 for f in b3[2]) and any(len(f) == 1500 for f in b3[1])
    assert stats["rx"] == 7 and stats["replicas"] == 6
    assert [len(f) for f in b3[3]] == [64]          # port 2's mirror copy of its frame to port 0
    dp.pull_learned()
    assert {(b, m) for b, m, _ in dp.macs.learned()} >= {(BR, MACS[0]), (BR, MACS[1]), (BR, MACS[2])}


@pytest.mark.gpu
def test_ring_engine_matches_batch_oracle():
    want, wpunts, _, _ = _run(_bridge("cpu"), "batch")
    got, gpunts, stats, dp = _run(_bridge("cuda"), "ring")
    assert got == want
    assert sorted((p, r, f) for p, r, f in gpunts) == sorted((p, r, f) for p, r, f in wpunts)
    assert stats["rx"] == 7 and stats.get("ring_relaunch") == 0
    dp.pull_learned()
    assert {(b, m) for b, m, _ in dp.macs.learned()} >= {(BR, MACS[0]), (BR, MACS[1]), (BR, MACS[2])}


def test_ipsec_boundary_on_the_uplink():
    """Port 3 is the uplink with the ESP engine at its boundary: pod traffic to the protected
    destination leaves it as ESP (tunnel mode), other traffic in clear (SPD bypass); ESP from the
    peer is authenticated, decrypted and bridged to the pod; a tampered packet is dropped."""
    from dpu_operator_amd.dataplane import ipsec as I

    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    for p in (0, 3):
        dp.ports.set(p, flags=T.PORT_VALID, bridge_id=BR)
    dp.macs.insert(BR, MACS[3], 3)
    dp.macs.insert(BR, MACS[0], 0)
    dp.commit(full=True)
    eng = dp.ipsec
    eng.add_sa(0, key=bytes(range(16)), salt=b"\x01\x02\x03\x04", spi=0x11, mode=I.TUNNEL, src="192.0.2.1",
               dst="192.0.2.2", smac=MACS[0], dmac=MACS[3])
    eng.add_sa(1, key=bytes(range(16, 32)), salt=b"\x05\x06\x07\x08", spi=0x22, mode=I.TUNNEL,
               src="192.0.2.2", dst="192.0.2.1")
    eng.set_spd("10.0.0.2", 17, I.PROTECT, 0)
    eng.set_rx_sa("192.0.2.2", "192.0.2.1", 0x22, 1)
    # the peer's engine: the mirror image (its SA 0 = our SA 1)
    peer = I.IpsecEngine()
    peer.add_sa(0, key=bytes(range(16, 32)), salt=b"\x05\x06\x07\x08", spi=0x22, mode=I.TUNNEL, src="192.0.2.2",
                dst="192.0.2.1", smac=MACS[3], dmac=MACS[0])
    peer.set_spd("10.0.0.1", 17, I.PROTECT, 0)
    peer.add_sa(1, key=bytes(range(16)), salt=b"\x01\x02\x03\x04", spi=0x11, mode=I.TUNNEL)
    peer.set_rx_sa("192.0.2.1", "192.0.2.2", 0x11, 1)
    ports = {0: SockPort(), 3: SockPort()}
    live = LivePath(dp, ports)
    live.ipsec_ports = {3}
    try:
        prot = _frame(MACS[3], MACS[0], 300, 1)                      # to 10.0.0.2: protected
        clear = bytes(bytearray(prot[:30]) + bytes([10, 0, 0, 9]) + prot[34:])   # to 10.0.0.9: bypass
        ports[0].inject(prot)
        ports[0].inject(clear)
        for _ in range(10):
            if live.poll_once(0.05):
                break
        out = ports[3].drain()
        assert len(out) == 2 and live.stats["esp_out"] == 2
        esp = next(f for f in out if f[23] == 50)
        assert clear in out and int.from_bytes(esp[34:38], "big") == 0x11
        dec, st = peer.decrypt([esp])
        assert st[0] == I.DONE and dec[0][14:] == prot[14:]
        # the peer answers through its SA; a tampered copy is dropped
        fr, ln = P.craft_full(1, dmac=MACS[0], smac=MACS[3], src_ip=0x0A000002, dst_ip=0x0A000001, sport=7, dport=9,
                              frame_len=500)
        reply = bytes(fr[0, : int(ln[0])])
        enc, _ = peer.encrypt([reply, reply])
        bad = bytearray(enc[1])
        bad[100] ^= 1
        ports[3].inject(enc[0])
        ports[3].inject(bytes(bad))
        for _ in range(10):
            if live.poll_once(0.05):
                break
        got = ports[0].drain()
        assert len(got) == 1 and got[0][14:] == reply[14:] and live.stats["esp_in"] == 1 and live.stats["esp_drop"] == 1
    finally:
        live.stop()
        for p in ports.values():
            p.close()


def test_ipv6_underlay_tunnel_through_the_live_path():
    """Pod -> IPv6-underlay VXLAN tunnel port -> underlay netdev carries the 70-B outer header; the
    reply arriving on the underlay is recognised by the kernel (recirc6), resolved on the whole
    frame (the VNI lies past the header slot) and re-enters on the tunnel port, bridged to the pod."""
    import ipaddress

    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    dp.ports.set(1, flags=T.PORT_VALID, bridge_id=BR)
    dp.ports.set(21, flags=T.PORT_VALID | T.PORT_TUNNEL | T.PORT_TUNNEL6, bridge_id=BR)
    dp.ports.a[21]["lag"] = 0
    dp.ports.set(30, flags=T.PORT_VALID | T.PORT_VTEP)
    dp.tunnels6.set(0, src="2001:db8:f::1", dst="2001:db8:f::2", vni=7000, out_port=30, smac=MACS[2], dmac=MACS[3])
    dp.vtep6.set("2001:db8:f::1")
    dp.terms6.insert("2001:db8:f::2", 7000, 21)
    dp.macs.insert(BR, MACS[1], 21)
    dp.macs.insert(BR, MACS[0], 1)
    dp.commit(full=True)
    ports = {1: SockPort(), 30: SockPort()}
    live = LivePath(dp, ports)
    try:
        f = _frame(MACS[1], MACS[0], 300, 1)
        ports[1].inject(f)
        for _ in range(10):
            if live.poll_once(0.05):
                break
        out = ports[30].drain()
        assert len(out) == 1 and out[0][12:14] == b"\x86\xdd" and out[0][70:] == f
        # the remote VTEP's reply: outer addresses swapped, inner MACs swapped
        b = bytearray(out[0])
        b[22:38], b[38:54] = out[0][38:54], out[0][22:38]
        inner = bytearray(b[70:])
        inner[0:6], inner[6:12] = inner[6:12], inner[0:6]
        b[70:] = inner
        ports[30].inject(bytes(b))
        got = []
        for _ in range(10):
            live.poll_once(0.05)
            got += ports[1].drain()
            if got:
                break
        assert got == [bytes(inner)] and live.stats["recirc"] == 1
        assert ipaddress.IPv6Address(bytes(b[22:38])) == ipaddress.IPv6Address("2001:db8:f::2")
    finally:
        live.stop()
        for p in ports.values():
            p.close()
