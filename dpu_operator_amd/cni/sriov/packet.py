"""Gratuitous ARP and unsolicited IPv6 Neighbor Advertisement frames.

Reference: dpu-cni/pkgs/sriovutils/packet.go:32-198 — after an interface gets its IPs, announce
them so switches/neighbours learn the (possibly new) MAC.  Builders return raw frames; `announce`
sends them on an AF_PACKET socket when the process has the privilege (best effort, like the
reference, which only logs failures).
"""
from __future__ import annotations

import ipaddress
import socket
import struct


def _mac(m: str) -> bytes:
    return bytes(int(x, 16) for x in m.split(":"))


def garp_frame(src_mac: str, ip: str) -> bytes:
    """Ethernet + 28-B ARP request with sender == target IP, broadcast."""
    ipb = ipaddress.IPv4Address(ip).packed
    eth = b"\xff" * 6 + _mac(src_mac) + b"\x08\x06"
    arp = struct.pack("!HHBBH", 1, 0x0800, 6, 4, 1) + _mac(src_mac) + ipb + b"\x00" * 6 + ipb
    return eth + arp


def _icmp6_csum(src: bytes, dst: bytes, payload: bytes) -> int:
    pseudo = src + dst + struct.pack("!I", len(payload)) + b"\x00\x00\x00\x3a"
    data = pseudo + payload
    if len(data) % 2:
        data += b"\0"
    s = sum(struct.unpack(f"!{len(data) // 2}H", data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def unsolicited_na_frame(src_mac: str, ip: str) -> bytes:
    """Ethernet + IPv6 (hop limit 255, to ff02::1) + 32-B ICMPv6 NA with target link-layer option."""
    src = ipaddress.IPv6Address(ip).packed
    dst = ipaddress.IPv6Address("ff02::1").packed
    # type 136, code 0, csum, flags (override=0x20000000), target, option(type 2, len 1, mac)
    body = struct.pack("!BBHI", 136, 0, 0, 0x20000000) + src + struct.pack("!BB", 2, 1) + _mac(src_mac)
    csum = _icmp6_csum(src, dst, body)
    body = body[:2] + struct.pack("!H", csum) + body[4:]
    ip6 = struct.pack("!IHBB", 6 << 28, len(body), 58, 255) + src + dst
    eth = b"\x33\x33\x00\x00\x00\x01" + _mac(src_mac) + b"\x86\xdd"
    return eth + ip6 + body


def announce(ifname: str, mac: str, ips: list[str], netns: str = "") -> int:
    """Send a GARP (IPv4) / unsolicited NA (IPv6) per address out of `ifname` - inside `netns`
    (the pod's namespace, where the VF lives after SetupVF; packet.go:166-198 runs in the
    container's netns too).  Returns the number of frames sent."""
    if netns:
        from ..netlink import in_netns

        try:
            return in_netns(netns, lambda: announce(ifname, mac, ips))
        except OSError:
            return 0
    sent = 0
    try:
        s = socket.socket(socket.AF_PACKET, socket.SOCK_RAW)
        s.bind((ifname, 0))
    except OSError:
        return 0
    try:
        for ip in ips:
            addr = ip.split("/")[0]
            frame = garp_frame(mac, addr) if ":" not in addr else unsolicited_na_frame(mac, addr)
            try:
                s.send(frame)
                sent += 1
            except OSError:
                pass
    finally:
        s.close()
    return sent
