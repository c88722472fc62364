"""Network-namespace helpers for live-path tests: endpoints (netns + a data-plane TAP moved into
it, addressed and up), an ICMP echo client that runs inside a namespace, and a bump-in-the-wire
network function (a namespace whose two interfaces forward every frame to each other, like the
reference e2e's NF pod between its ingress and egress DPU netdevs)."""
from __future__ import annotations

import os
import select
import socket
import struct
import threading
import time

from ..cni.netlink import RtNetlink, create_netns, delete_netns, in_netns


def netns_path(name: str) -> str:
    """Where a named test namespace is bound: `DPU_NETNS_DIR` (a private directory when the tests
    run in a user namespace of their own) or /var/run/netns, where `ip netns` keeps them."""
    return os.path.join(os.environ.get("DPU_NETNS_DIR", "/var/run/netns"), name)


def privileged() -> bool:
    """True when this process can create network namespaces and TAP devices."""
    if not os.path.exists("/dev/net/tun"):
        return False
    path = netns_path(f"dpu-probe-{os.getpid()}")
    try:
        create_netns(path)
    except OSError:
        return False
    delete_netns(path)
    return True


def _csum(b: bytes) -> int:
    if len(b) % 2:
        b += b"\0"
    s = sum(struct.unpack(f"!{len(b) // 2}H", b))
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def ping(ns: str, dst: str, timeout: float = 3.0, ident: int = 0x4D49, seq: int = 1, payload: bytes = b"mi355x",
         dev: str | None = None) -> float | None:
    """One ICMP echo from inside netns `ns` (out of interface `dev` if given); the RTT in seconds
    or None."""

    def run():
        s = socket.socket(socket.AF_INET, socket.SOCK_RAW, socket.IPPROTO_ICMP)
        if dev:
            s.setsockopt(socket.SOL_SOCKET, socket.SO_BINDTODEVICE, dev.encode())
        s.settimeout(0.2)
        try:
            hdr = struct.pack("!BBHHH", 8, 0, 0, ident, seq)
            pkt = struct.pack("!BBHHH", 8, 0, _csum(hdr + payload), ident, seq) + payload
            end = time.monotonic() + timeout
            t0 = time.monotonic()
            s.sendto(pkt, (dst, 0))
            last = t0
            while time.monotonic() < end:
                if time.monotonic() - last > 0.5:  # retry: the first try may wait for ARP
                    t0 = last = time.monotonic()
                    s.sendto(pkt, (dst, 0))
                try:
                    data, addr = s.recvfrom(65535)
                except socket.timeout:
                    continue
                ihl = (data[0] & 0xF) * 4
                t, _c, _ck, i, q = struct.unpack_from("!BBHHH", data, ihl)
                if t == 0 and i == ident and q == seq and addr[0] == dst:
                    return time.monotonic() - t0
            return None
        finally:
            s.close()

    return in_netns(ns, run)


def udp_exchange(src_ns: str, dst_ns: str, dst_ip: str, payload: bytes, port: int = 47000, timeout: float = 3.0,
                 tries: int = 5) -> bytes | None:
    """One UDP datagram from a socket in `src_ns` to `dst_ip`:`port`, received by a socket in
    `dst_ns` through the kernels' own UDP stacks (so checksums are verified on receipt); what
    arrived, or None."""
    rx = in_netns(dst_ns, lambda: socket.socket(socket.AF_INET, socket.SOCK_DGRAM))
    tx = in_netns(src_ns, lambda: socket.socket(socket.AF_INET, socket.SOCK_DGRAM))
    try:
        rx.bind(("0.0.0.0", port))
        rx.settimeout(timeout / tries)
        for _ in range(tries):      # (the first may wait for ARP)
            tx.sendto(payload, (dst_ip, port))
            try:
                data, _addr = rx.recvfrom(65535)
                return data
            except socket.timeout:
                continue
        return None
    finally:
        rx.close()
        tx.close()


class Endpoint:
    """A namespace with one interface: `ifname` moved in, `cidr` assigned, interface + lo up."""

    def __init__(self, ns_name: str, ifname: str, cidr: str, nl: RtNetlink | None = None):
        self.nl = nl or RtNetlink()
        self.ns = create_netns(netns_path(ns_name))
        self.ifname = ifname
        self.nl.link_set_ns(ifname, self.ns)
        self.nl.link_set_up("lo", self.ns)
        self.nl.addr_add(ifname, cidr, self.ns)
        self.nl.link_set_up(ifname, self.ns)
        self.mac = self.nl.link_by_name(ifname, self.ns).mac

    def close(self) -> None:
        delete_netns(self.ns)


class WireNF:
    """An NF pod: namespace `ns_name` holding `if_in` and `if_out` (moved in and brought up, no
    addresses) and a thread that copies every frame received on one to the other (AF_PACKET
    sockets opened inside the namespace)."""

    ETH_P_ALL = 0x0003

    def __init__(self, ns_name: str, if_in: str, if_out: str, nl: RtNetlink | None = None,
                 existing_ns: str | None = None):
        """existing_ns: the interfaces are already in that namespace (an NF pod's, moved in by the
        CNI); it is not deleted on close."""
        self.nl = nl or RtNetlink()
        self.own_ns = existing_ns is None
        self.ns = existing_ns or create_netns(netns_path(ns_name))
        self.ifs = (if_in, if_out)
        self.macs = []
        for i in self.ifs:
            if existing_ns is None:
                self.nl.link_set_ns(i, self.ns)
            self.nl.link_set_up(i, self.ns)
            self.macs.append(self.nl.link_by_name(i, self.ns).mac)
        self.forwarded = 0
        self._stop = threading.Event()
        self._ready = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name=f"nf-{ns_name}")
        self._t.start()
        self._ready.wait(5)

    def _run(self) -> None:
        from ..cni.netlink import setns_current_thread

        setns_current_thread(self.ns)
        socks = []
        for i in self.ifs:
            s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(self.ETH_P_ALL))
            s.bind((i, 0))
            s.setblocking(False)
            socks.append(s)
        self._ready.set()
        try:
            while not self._stop.is_set():
                r, _, _ = select.select(socks, [], [], 0.05)
                for s in r:
                    peer = socks[1 - socks.index(s)]
                    while True:
                        try:
                            data, addr = s.recvfrom(65535)
                        except BlockingIOError:
                            break
                        except OSError:                      # interface went down / away: NF is done
                            return
                        if addr[2] == socket.PACKET_OUTGOING:   # our own transmissions
                            continue
                        try:
                            peer.send(data)
                        except OSError:
                            return
                        self.forwarded += 1
        finally:
            for s in socks:
                s.close()

    def close(self) -> None:
        self._stop.set()
        self._t.join(5)
        if self.own_ns:
            delete_netns(self.ns)


class RawPod:
    """A pod namespace holding one interface (moved in, up, no addresses, IPv6 off so the kernel
    sends nothing of its own) and an AF_PACKET socket bound to it, opened inside the namespace:
    `send` puts whole Ethernet frames on the wire exactly as given, `recv` returns what arrived
    (the pod's own transmissions filtered out)."""

    ETH_P_ALL = 0x0003

    def __init__(self, ns_name: str, ifname: str, nl: RtNetlink | None = None, existing_ns: str | None = None):
        self.nl = nl or RtNetlink()
        self.ns = existing_ns or create_netns(netns_path(ns_name))
        self.own_ns = existing_ns is None
        self.ifname = ifname
        if existing_ns is None:
            self.nl.link_set_ns(ifname, self.ns)

        def setup():
            for p in (f"/proc/sys/net/ipv6/conf/{ifname}/disable_ipv6", "/proc/sys/net/ipv6/conf/all/disable_ipv6"):
                try:
                    with open(p, "w") as f:
                        f.write("1")
                except OSError:
                    pass
            s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(self.ETH_P_ALL))
            s.bind((ifname, 0))
            s.setblocking(False)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 22)
            s.setsockopt(self.SOL_PACKET, self.PACKET_AUXDATA, 1)   # 802.1Q tags the kernel strips
            return s

        self.nl.link_set_up(ifname, self.ns)
        self.sock = in_netns(self.ns, setup)

    def send(self, frames: list[bytes]) -> int:
        n = 0
        for f in frames:
            for _ in range(200):
                try:
                    self.sock.send(f)
                    n += 1
                    break
                except BlockingIOError:
                    time.sleep(0.0005)
        return n

    SOL_PACKET, PACKET_AUXDATA = 263, 8
    TP_STATUS_VLAN_VALID, TP_STATUS_VLAN_TPID_VALID = 1 << 4, 1 << 6

    def recv(self) -> list[bytes]:
        """Frames as they were on the wire: a VLAN tag the kernel moved to the aux data (VLAN
        offload) goes back in front of the ethertype."""
        out = []
        while True:
            try:
                data, anc, _flags, addr = self.sock.recvmsg(65535, socket.CMSG_SPACE(20))
            except BlockingIOError:
                return out
            if addr[2] == socket.PACKET_OUTGOING:
                continue
            for lvl, typ, cd in anc:
                if lvl == self.SOL_PACKET and typ == self.PACKET_AUXDATA and len(cd) >= 20:
                    st, _l, _sl, _mac, _net, tci, tpid = struct.unpack_from("=IIIHHHH", cd)
                    if st & self.TP_STATUS_VLAN_VALID and (tci or st & self.TP_STATUS_VLAN_TPID_VALID):
                        tpid = tpid if st & self.TP_STATUS_VLAN_TPID_VALID and tpid else 0x8100
                        data = data[:12] + struct.pack("!HH", tpid, tci) + data[12:]
            out.append(data)

    def close(self) -> None:
        self.sock.close()
        if self.own_ns:
            delete_netns(self.ns)
