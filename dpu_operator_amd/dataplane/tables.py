"""Host-side models of the data-plane tables (numpy, byte-identical to csrc/nfdp/nfdp.h).

Tables (what they replace in the reference):

* ``PortTable``  — vports (VF / NF / wire / representor).  Replaces SR-IOV VF config
  (vlan / spoofchk / trust, ``dpu-cni/pkgs/sriov/sriov.go:200-282``) and the P4
  ``tx_source_port`` / ``source_port_to_pr_map`` tables (``p4rtclient.go:674-718``).
* ``ChainTable`` — service-function chains of built-in GPU NFs (``api/v1/servicefunctionchain_types.go``).
* ``MacTable``   — (bridge, dst MAC) -> port, the ``l2_fwd_*`` tables (``p4info.txt:600-692``) and
  OvS dl_dst steering (``ovsdp.go:125-131``).
* ``AclTable``   — priority/ternary rules over the 128-bit FlowKey (TCAM; MFMA-evaluated).
* ``FlowTable``  — 1M+ exact-match 5-tuple flows (native cuckoo, ``_nfdp.FlowTable``).
"""
from __future__ import annotations

import ipaddress
from dataclasses import dataclass

import numpy as np

from ..native import nfdp as _nfdp_mod
from ..ops.packets import ip_raw, mac_raw, port_raw

MAX_PORTS = 4096        # port table rows (buffer sizes)
MAX_PORT_ID = 4094      # usable port ids: 4094 / 4095 encode none / punt in the 12-bit egress meta port
PORT_NONE = 0xFFFF
PORT_PUNT = 0xFFFE
FLOOD_WAYS = 16         # nfdp.h kFloodWays

# port flags (nfdp.h PortFlags)
PORT_VALID = 1 << 0
PORT_SPOOFCHK = 1 << 1
PORT_VLAN_ISOLATE = 1 << 2
PORT_TAG_EGRESS = 1 << 3
PORT_VLAN_BRIDGE = 1 << 4
PORT_TRUST = 1 << 5
PORT_HAS_DEFAULT = 1 << 6
PORT_INGRESS_TAG = 1 << 7   # frames from the port leave tagged with ext[11:0] (P4 add_vlan_and_send_to_port)
PORT_MIRROR = 1 << 8        # forwarded frames are also copied to ext[31:16] (P4 mirror_and_send)
PORT_LAG = 1 << 9           # egress picks member lag_members[lag][hash & 7] (P4 tx_lag_table)
PORT_VSI_LOOKUP = 1 << 10   # L2 lookup on (bridge, 00:VSI:00:00:00:00), VSI = dst MAC byte 1 (P4 vsi_to_vsi_loopback)
PORT_LEARN = 1 << 11        # (bridge, src MAC) -> port learned from this port's frames (OvS NORMAL)
PORT_ARP_TRAP = 1 << 12     # ARP frames from this port are also copied to the slow path (always_trap_arp_table)
PORT_ROUTED = 1 << 13       # router interface: IPv4 to the port's own MAC is routed (LPM) on a flow miss
PORT_TUNNEL = 1 << 14       # tunnel port: egress = VXLAN / GENEVE encap with tunnels[lag]
PORT_VTEP = 1 << 15         # underlay port: VXLAN / GENEVE to ext (local VTEP IPv4, raw) is terminated
PORT_RX_OFF = 1 << 16       # ctrl-net RX_STATE down: frames to the port are dropped (bad_port)
PORT_LINK_DOWN = 1 << 17    # ctrl-net LINK_STATUS down / DEV_REMOVE: the port neither receives nor sends
PORT_TUNNEL6 = 1 << 18      # with PORT_TUNNEL: IPv6 underlay, the tunnel is tunnels6[lag]
LAG_WAYS = 8

# hop opcodes (nfdp.h Hop)
HOP_NONE, HOP_ACL, HOP_NAT, HOP_L2FWD, HOP_TTL, HOP_HAIRPIN, HOP_VLAN, HOP_DROP, HOP_PUNT, HOP_ROUTE = range(10)
HOP_NAMES = {
    "acl": HOP_ACL, "nat": HOP_NAT, "l2fwd": HOP_L2FWD, "ttl": HOP_TTL, "hairpin": HOP_HAIRPIN,
    "vlan": HOP_VLAN, "drop": HOP_DROP, "punt": HOP_PUNT, "route": HOP_ROUTE,
}

# reasons (nfdp.h Reason)
REASONS = {
    0: "ok", 1: "bad_port", 2: "vlan_drop", 3: "spoof", 4: "acl_deny", 5: "no_route",
    6: "too_big", 7: "chain_drop", 8: "ttl_expired", 9: "malformed", 10: "remote", 11: "overflow",
    12: "arp_trap", 13: "recirc", 14: "recirc6", 15: "cont",
}

PORT_DTYPE = np.dtype(
    [
        ("flags", "<u4"), ("vlan", "<u2"), ("bridge_id", "<u2"),
        ("mac_lo", "<u4"), ("mac_hi", "<u2"), ("gpu", "<u2"),
        ("peer_mac_lo", "<u4"), ("peer_mac_hi", "<u2"), ("default_out", "<u2"),
        ("ext", "<u4"), ("lag", "<u2"), ("mtu", "<u2"),
    ]
)
CHAIN_DTYPE = np.dtype([("nhops", "u1"), ("hop", "u1", (7,)), ("acl_id", "<u2"), ("flags", "<u2"), ("pad", "<u4")])
MAC_DTYPE = np.dtype(
    [("mac_lo", "<u4"), ("mac_hi", "<u2"), ("bridge_id", "<u2"), ("out_port", "<u2"), ("valid", "<u2"), ("stamp", "<u4")]
)
MAC_EMPTY, MAC_STATIC, MAC_TOMB, MAC_LEARNED = 0, 1, 2, 3   # nfdp.h MacValid
NH_DTYPE = np.dtype([("dmac_lo", "<u4"), ("dmac_hi", "<u2"), ("port", "<u2"), ("smac_lo", "<u4"), ("smac_hi", "<u2"),
                     ("valid", "<u2")])
TUNNEL_DTYPE = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("sport", "<u2"), ("dport", "<u2"), ("vni", "<u4"),
                         ("smac_lo", "<u4"), ("smac_hi", "<u2"), ("out_port", "<u2"), ("dmac_lo", "<u4"),
                         ("dmac_hi", "<u2"), ("type", "<u2")])
TERM_DTYPE = np.dtype([("src_ip", "<u4"), ("vni", "<u4"), ("port", "<u2"), ("valid", "<u2"), ("pad", "<u4")])
TERM6_DTYPE = np.dtype([("src", "<u4", (4,)), ("vni", "<u4"), ("port", "<u2"), ("valid", "<u2"), ("pad", "<u4", (2,))])
PORT_CONT = 0xFFFD      # in-meta port of a wide header pair's continuation slot (nfdp.h kPortCont)
VMMAC_DTYPE = np.dtype([("ip", "<u4"), ("kind", "<u4"), ("mac_lo", "<u4"), ("mac_hi", "<u4")])   # nfdp.h VmMacEntry
VMMAC_SRC, VMMAC_DST = 1, 2
TUNNEL6_DTYPE = np.dtype([("src", "<u4", (4,)), ("dst", "<u4", (4,)), ("sport", "<u2"), ("dport", "<u2"), ("vni", "<u4"),
                          ("smac_lo", "<u4"), ("smac_hi", "<u2"), ("out_port", "<u2"), ("dmac_lo", "<u4"),
                          ("dmac_hi", "<u2"), ("type", "<u2"), ("tc_flow", "<u4"), ("hop_limit", "<u4")])
assert NH_DTYPE.itemsize == 16 and TUNNEL_DTYPE.itemsize == 32 and TERM_DTYPE.itemsize == 16
assert TUNNEL6_DTYPE.itemsize == 64
TUN_VXLAN, TUN_GENEVE = 1, 2
VXLAN_PORT, GENEVE_PORT = 4789, 6081
LPM_EXT, ROUTE_NH, ROUTE_ECMP = 1 << 31, 1 << 28, 2 << 28
ECMP_WAYS = 8
assert PORT_DTYPE.itemsize == 32 and CHAIN_DTYPE.itemsize == 16 and MAC_DTYPE.itemsize == 16

# Microsoft RSS verification key (40 B) — standard Toeplitz key.
RSS_KEY = bytes(
    [
        0x6D, 0x5A, 0x56, 0xDA, 0x25, 0x5B, 0x0E, 0xC2, 0x41, 0x67, 0x25, 0x3D, 0x43, 0xA3, 0x8F, 0xB0,
        0xD0, 0xCA, 0x2B, 0xCB, 0xAE, 0x7B, 0x30, 0xB4, 0x77, 0xCB, 0x2D, 0xA3, 0x80, 0x30, 0xF2, 0x0C,
        0x6A, 0x42, 0xB7, 0x3B, 0xBE, 0xAC, 0x01, 0xFA,
    ]
)


def fmix32(h):
    h = np.asarray(h, dtype=np.uint32).copy()
    with np.errstate(over="ignore"):
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return h


def ip_to_int(ip) -> int:
    if isinstance(ip, (int, np.integer)):
        return int(ip)
    return int(ipaddress.IPv4Address(ip))


def flow_key(src_ip, dst_ip, sport=0, dport=0, proto=17, zone=0) -> np.ndarray:
    """Vectorized FlowKey construction (host-order ints in) -> uint32[n,4] raw words."""
    src = ip_raw(np.asarray(src_ip, np.uint32))
    dst = ip_raw(np.asarray(dst_ip, np.uint32))
    ports = port_raw(sport) | (port_raw(dport) << np.uint32(16))
    meta = (np.asarray(proto, np.uint32) & 0xFF) | ((np.asarray(zone, np.uint32) & 0xFFFF) << np.uint32(16))
    n = max(np.size(src), np.size(dst), np.size(ports), np.size(meta))
    k = np.zeros((n, 4), np.uint32)
    k[:, 0], k[:, 1], k[:, 2], k[:, 3] = src, dst, ports, meta
    return k


KEY_V6 = 0x200   # FlowKey.meta bit of an IPv6 key (nfdp.h kKeyV6)
# ACL key port-class bits (nfdp.h acl_key_meta): meta of the ACL key only, never of a flow key
ACL_SPORT_HI, ACL_DPORT_HI = 0x400, 0x800


def acl_key(keys: np.ndarray) -> np.ndarray:
    """Flow keys uint32[n, 4] -> the ACL keys the TCAM matches (port-class bits added to meta)."""
    k = np.array(keys, np.uint32, copy=True).reshape(-1, 4)
    ports = k[:, 2]
    k[:, 3] |= np.where(ports & np.uint32(0xFC), np.uint32(ACL_SPORT_HI), np.uint32(0))
    k[:, 3] |= np.where(ports & np.uint32(0xFC0000), np.uint32(ACL_DPORT_HI), np.uint32(0))
    return k
SLOT_USED = 0x100


def fold6(words) -> int:
    """nfdp.h fold6: the four raw words of an IPv6 address -> one FlowKey word."""
    w = [np.uint32(x) for x in words]
    with np.errstate(over="ignore"):
        h = fmix32(w[3] ^ np.uint32(0x6B43A9B5))
        h = fmix32(w[2] ^ h)
        h = fmix32(w[1] ^ h)
        h = fmix32(w[0] ^ h)
    return int(h)


def flow_key6(src, dst, sport=0, dport=0, proto=17, zone=0) -> tuple[np.ndarray, np.ndarray]:
    """IPv6 5-tuple -> (the folded FlowKey uint32[4] the data plane probes, the 8 raw address
    words of its side entry).  Ports count for TCP / UDP only (nfdp.h v6_ports)."""
    s6, d6 = ip6_raw(src), ip6_raw(dst)
    ports = 0
    if proto in (6, 17):
        ports = int(port_raw(np.uint32(sport))) | (int(port_raw(np.uint32(dport))) << 16)
    meta = (proto & 0xFF) | KEY_V6 | ((zone & 0xFFFF) << 16)
    key = np.array([fold6(s6), fold6(d6), ports, meta], np.uint32)
    return key, np.concatenate([s6, d6]).astype(np.uint32)


def flow_action(chain_id=0, out_port=0, nat_ip=0, nat_port=0, vlan=0, flow_id=0) -> np.ndarray:
    """Vectorized FlowAction -> uint32[n,4] (nat ip/port host order in)."""
    w0 = (np.asarray(chain_id, np.uint32) & 0xFFFF) | ((np.asarray(out_port, np.uint32) & 0xFFFF) << np.uint32(16))
    w1 = ip_raw(np.asarray(nat_ip, np.uint32))
    w2 = port_raw(nat_port) | ((np.asarray(vlan, np.uint32) & 0xFFFF) << np.uint32(16))
    w3 = np.asarray(flow_id, np.uint32)
    n = max(np.size(w0), np.size(w1), np.size(w2), np.size(w3))
    a = np.zeros((n, 4), np.uint32)
    a[:, 0], a[:, 1], a[:, 2], a[:, 3] = w0, w1, w2, w3
    return a


class PortTable:
    def __init__(self):
        self.a = np.zeros(MAX_PORTS, PORT_DTYPE)
        self.version = 0

    def set(self, idx: int, *, flags=PORT_VALID, vlan=0, bridge_id=0, mac="00:00:00:00:00:00",
            peer_mac="00:00:00:00:00:00", gpu=0, default_out: int | None = None, mtu: int = 0) -> None:
        if not 0 <= idx < MAX_PORT_ID:
            raise ValueError(f"port index {idx} out of range")
        if not 0 <= mtu <= 0xFFFF:
            raise ValueError("mtu must be in [0, 65535] (0 = no per-port limit)")
        lo, hi = mac_raw(mac)
        plo, phi = mac_raw(peer_mac)
        if default_out is not None:
            flags |= PORT_HAS_DEFAULT
        self.a[idx] = (flags | PORT_VALID, vlan, bridge_id, lo, hi, gpu, plo, phi,
                       0 if default_out is None else default_out, 0, 0, mtu)
        self.version += 1

    def update(self, idx: int, **fields) -> None:
        """Change individual fields of an existing port (e.g. default_out when an NF appears)."""
        for k, v in fields.items():
            if k == "default_out":
                if v is None:
                    self.a[idx]["flags"] &= ~np.uint32(PORT_HAS_DEFAULT)
                else:
                    self.a[idx]["flags"] |= np.uint32(PORT_HAS_DEFAULT)
                    self.a[idx]["default_out"] = v
            elif k in ("mac", "peer_mac"):
                lo, hi = mac_raw(v)
                pre = "" if k == "mac" else "peer_"
                self.a[idx][pre + "mac_lo"], self.a[idx][pre + "mac_hi"] = lo, hi
            else:
                self.a[idx][k] = v
        self.version += 1

    def clear(self, idx: int) -> None:
        self.a[idx] = np.zeros((), PORT_DTYPE)
        self.version += 1

    def valid(self, idx: int) -> bool:
        return bool(self.a[idx]["flags"] & PORT_VALID)

    def set_flag(self, idx: int, bit: int, on: bool = True) -> None:
        self._flag(idx, bit, on)
        self.version += 1

    def set_link(self, idx: int, up: bool) -> None:
        """Link state (ctrl-net LINK_STATUS, DEV_REMOVE): a down port neither receives nor sends.
        Kept apart from PORT_VALID, so link flaps never undo the port's configuration."""
        self._flag(idx, PORT_LINK_DOWN, not up)
        self.version += 1

    def set_rx(self, idx: int, on: bool) -> None:
        """RX state (ctrl-net RX_STATE): with RX off nothing is delivered to the port."""
        self._flag(idx, PORT_RX_OFF, not on)
        self.version += 1

    def set_mtu(self, idx: int, mtu: int) -> None:
        """Egress MTU in L3 bytes (ctrl-net SET_MTU); frames above it are dropped as too_big."""
        if not 0 <= mtu <= 0xFFFF:
            raise ValueError("mtu must be in [0, 65535]")
        self.a[idx]["mtu"] = mtu
        self.version += 1

    def _flag(self, idx: int, bit: int, on: bool) -> None:
        if on:
            self.a[idx]["flags"] |= np.uint32(bit)
        else:
            self.a[idx]["flags"] &= ~np.uint32(bit)

    def set_ingress_tag(self, idx: int, vid: int | None) -> None:
        """P4 add_vlan_and_send_to_port: frames from `idx` leave tagged with `vid` (None: off)."""
        if vid is not None and not 1 <= vid <= 4094:
            raise ValueError("vid must be 1..4094")
        ext = int(self.a[idx]["ext"]) & ~0xFFF
        self.a[idx]["ext"] = ext | (vid or 0)
        self._flag(idx, PORT_INGRESS_TAG, vid is not None)
        self.version += 1

    def set_mirror(self, idx: int, mirror_port: int | None) -> None:
        """P4 mirror_and_send: frames forwarded from `idx` are also copied to `mirror_port`."""
        ext = int(self.a[idx]["ext"]) & 0xFFFF
        self.a[idx]["ext"] = ext | ((mirror_port or 0) << 16)
        self._flag(idx, PORT_MIRROR, mirror_port is not None)
        self.version += 1

    def set_lag(self, idx: int, group: int | None) -> None:
        """Egress to `idx` (a LAG port) picks a member of `group` by hash[2:0]."""
        self.a[idx]["lag"] = group or 0
        self._flag(idx, PORT_LAG, group is not None)
        self.version += 1

    def mirror_port(self, idx: int) -> int | None:
        return int(self.a[idx]["ext"]) >> 16 if self.a[idx]["flags"] & PORT_MIRROR else None


class RouteTable:
    """IPv4 routes (P4 ipv4_table, LPM) -> nexthop id or ECMP group, compiled to the DIR-24-8 arrays
    the kernels read (nfdp.h lpm_lookup): tbl24 (2^24 x u32, 64 MB of HBM) + 256-entry tbl8
    groups for prefixes longer than /24."""

    def __init__(self):
        self.routes: dict[tuple[int, int], int] = {}
        self.version = 0

    @staticmethod
    def _net(cidr) -> tuple[int, int]:
        n = ipaddress.IPv4Network(cidr, strict=False)
        return int(n.network_address), n.prefixlen

    def add(self, cidr, nexthop: int | None = None, ecmp_group: int | None = None) -> None:
        if (nexthop is None) == (ecmp_group is None):
            raise ValueError("a route points at exactly one of nexthop / ecmp_group")
        res = (ROUTE_NH | nexthop) if nexthop is not None else (ROUTE_ECMP | ecmp_group)
        if (nexthop or ecmp_group or 0) > 0xFFFF:
            raise ValueError("nexthop / group id must fit 16 bits")
        self.routes[self._net(cidr)] = res
        self.version += 1

    def remove(self, cidr) -> bool:
        ok = self.routes.pop(self._net(cidr), None) is not None
        self.version += ok
        return ok

    def __len__(self) -> int:
        return len(self.routes)

    def lookup(self, ip) -> int:
        """Reference LPM (longest prefix wins), for tests: the route result or 0."""
        x = int(ipaddress.IPv4Address(ip)) if not isinstance(ip, (int, np.integer)) else int(ip)
        best, res = -1, 0
        for (net, plen), r in self.routes.items():
            m = 0 if plen == 0 else (0xFFFFFFFF << (32 - plen)) & 0xFFFFFFFF
            if (x & m) == net and plen > best:
                best, res = plen, r
        return res

    def build(self) -> tuple[np.ndarray, np.ndarray]:
        t24 = np.zeros(1 << 24, np.uint32)
        t8: list[np.ndarray] = []
        for (net, plen), res in sorted(self.routes.items(), key=lambda kv: kv[0][1]):
            if plen <= 24:  # ascending prefix length: longer prefixes overwrite shorter ones
                lo = net >> 8
                t24[lo:lo + (1 << (24 - plen))] = res
            else:
                i = net >> 8
                if not t24[i] & LPM_EXT:
                    t8.append(np.full(256, t24[i], np.uint32))
                    t24[i] = LPM_EXT | (len(t8) - 1)
                g = int(t24[i] & ~np.uint32(LPM_EXT))
                lo = net & 0xFF
                t8[g][lo:lo + (1 << (32 - plen))] = res
        tbl8 = np.concatenate(t8) if t8 else np.zeros(256, np.uint32)
        return t24, tbl8


class Route6Table:
    """IPv6 routes (P4 ipv6_table, LPM) -> nexthop id or ECMP group.  Compiled (native
    `build_lpm6`) to one open-addressing table over (masked prefix, length) plus the distinct
    lengths present, longest first; the kernels probe the lengths in that order (nfdp.h
    lpm6_lookup): a handful of probes for a real FIB's few lengths, no 2^24-entry array."""

    def __init__(self):
        self.routes: dict[tuple[int, int], int] = {}
        self.version = 0

    @staticmethod
    def _net(cidr) -> tuple[int, int]:
        n = ipaddress.IPv6Network(cidr, strict=False)
        return int(n.network_address), n.prefixlen

    def add(self, cidr, nexthop: int | None = None, ecmp_group: int | None = None) -> None:
        if (nexthop is None) == (ecmp_group is None):
            raise ValueError("a route points at exactly one of nexthop / ecmp_group")
        if (nexthop or ecmp_group or 0) > 0xFFFF:
            raise ValueError("nexthop / group id must fit 16 bits")
        self.routes[self._net(cidr)] = (ROUTE_NH | nexthop) if nexthop is not None else (ROUTE_ECMP | ecmp_group)
        self.version += 1

    def remove(self, cidr) -> bool:
        ok = self.routes.pop(self._net(cidr), None) is not None
        self.version += ok
        return ok

    def __len__(self) -> int:
        return len(self.routes)

    def lookup(self, ip) -> int:
        """Reference LPM for tests: the route result or 0."""
        x = int(ipaddress.IPv6Address(ip)) if not isinstance(ip, (int, np.integer)) else int(ip)
        best, res = -1, 0
        for (net, plen), r in self.routes.items():
            m = 0 if plen == 0 else ((1 << 128) - 1) ^ ((1 << (128 - plen)) - 1)
            if (x & m) == net and plen > best:
                best, res = plen, r
        return res

    def build(self):
        """-> (table [slots, 8] u32, lengths u8, n_lengths)."""
        from ..native import nfdp

        rows = np.zeros((len(self.routes), 6), np.uint32)
        for i, ((net, plen), res) in enumerate(self.routes.items()):
            rows[i, :4] = [(net >> (96 - 32 * w)) & 0xFFFFFFFF for w in range(4)]
            rows[i, 4], rows[i, 5] = plen, res
        return nfdp().build_lpm6(rows)


class NextHopTable:
    """nexthop_table + rif_mod_table: id -> (egress port, neighbour MAC, router-interface MAC)."""

    def __init__(self, capacity: int = 4096):
        self.a = np.zeros(capacity, NH_DTYPE)
        self.n = 0
        self.version = 0

    def set(self, nh: int, port: int, dmac, smac) -> None:
        if not 0 <= nh < len(self.a):
            raise ValueError("nexthop id out of range")
        dlo, dhi = mac_raw(dmac)
        slo, shi = mac_raw(smac)
        self.a[nh] = (dlo, dhi, port, slo, shi, 1)
        self.n = max(self.n, nh + 1)
        self.version += 1

    def clear(self, nh: int) -> None:
        self.a[nh] = np.zeros((), NH_DTYPE)
        self.version += 1


class EcmpTable:
    """ECMP groups (ecmp_hash_table): ECMP_WAYS nexthop ids per group, member = hash[2:0]."""

    def __init__(self, groups: int = 1024):
        self.a = np.zeros(groups * ECMP_WAYS, np.uint16)
        self.n = 0
        self.version = 0

    def set_group(self, g: int, nexthops: list[int]) -> None:
        if not nexthops:
            raise ValueError("an ECMP group needs members")
        self.a[g * ECMP_WAYS:(g + 1) * ECMP_WAYS] = [nexthops[i % len(nexthops)] for i in range(ECMP_WAYS)]
        self.n = max(self.n, g + 1)
        self.version += 1

    def set_slot(self, g: int, h: int, nh: int) -> None:
        self.a[g * ECMP_WAYS + (h & (ECMP_WAYS - 1))] = nh
        self.n = max(self.n, g + 1)
        self.version += 1


class TunnelTable:
    """VXLAN / GENEVE tunnels (vxlan_encap_mod_table / geneve_encap_mod_table + l2_to_tunnel_v4):
    the outer headers of a tunnel port.  Addresses host-order ints / dotted strings in."""

    def __init__(self, capacity: int = 1024):
        self.a = np.zeros(capacity, TUNNEL_DTYPE)
        self.n = 0
        self.version = 0

    def set(self, idx: int, *, src, dst, vni: int, out_port: int, smac, dmac, kind: int = TUN_VXLAN,
            dport: int | None = None, sport: int = 0) -> None:
        dport = dport or (VXLAN_PORT if kind == TUN_VXLAN else GENEVE_PORT)
        slo, shi = mac_raw(smac)
        dlo, dhi = mac_raw(dmac)
        self.a[idx] = (int(ip_raw(np.uint32(ip_to_int(src)))), int(ip_raw(np.uint32(ip_to_int(dst)))),
                       int(port_raw(np.uint32(sport))) if sport else 0, int(port_raw(np.uint32(dport))),
                       vni & 0xFFFFFF, slo, shi, out_port, dlo, dhi, kind)
        self.n = max(self.n, idx + 1)
        self.version += 1

    def bytes_of(self, idx: int) -> bytes:
        return self.a[idx].tobytes()


def ip6_raw(addr) -> np.ndarray:
    """IPv6 address (text / int) -> the 16 network-order bytes as 4 little-endian u32 words."""
    a = ipaddress.IPv6Address(int(addr) if isinstance(addr, (int, np.integer)) else addr)
    return np.frombuffer(a.packed, "<u4").copy()


class Tunnel6Table:
    """IPv6-underlay VXLAN / GENEVE tunnels (vxlan_encap_v6_mod_table / geneve_encap_v6_mod_table +
    l2_to_tunnel_v6): the outer headers of a PORT_TUNNEL | PORT_TUNNEL6 port."""

    def __init__(self, capacity: int = 256):
        self.a = np.zeros(capacity, TUNNEL6_DTYPE)
        self.n = 0
        self.version = 0

    def set(self, idx: int, *, src, dst, vni: int, out_port: int, smac, dmac, kind: int = TUN_VXLAN,
            dport: int | None = None, sport: int = 0, traffic_class: int = 0, flow_label: int = 0,
            hop_limit: int = 64) -> None:
        dport = dport or (VXLAN_PORT if kind == TUN_VXLAN else GENEVE_PORT)
        slo, shi = mac_raw(smac)
        dlo, dhi = mac_raw(dmac)
        e = self.a[idx]
        e["src"], e["dst"] = ip6_raw(src), ip6_raw(dst)
        e["sport"] = int(port_raw(np.uint32(sport))) if sport else 0
        e["dport"] = int(port_raw(np.uint32(dport)))
        e["vni"] = vni & 0xFFFFFF
        e["smac_lo"], e["smac_hi"], e["out_port"], e["dmac_lo"], e["dmac_hi"] = slo, shi, out_port, dlo, dhi
        e["type"] = kind
        e["tc_flow"] = ((traffic_class & 0xFF) << 20) | (flow_label & 0xFFFFF)
        e["hop_limit"] = hop_limit & 0xFF
        self.a[idx] = e
        self.n = max(self.n, idx + 1)
        self.version += 1

    def bytes_of(self, idx: int) -> bytes:
        return self.a[idx].tobytes()


class Vtep6:
    """The local IPv6 VTEP address: VTEP (underlay) ports hand IPv6 VXLAN / GENEVE addressed to it to
    the termination path (kernel reason recirc6, Term6Table finishes it)."""

    def __init__(self):
        self.a = np.zeros(4, np.uint32)
        self.active = False
        self.version = 0

    def set(self, addr) -> None:
        self.a[:] = ip6_raw(addr)
        self.active = True
        self.version += 1

    def clear(self) -> None:
        self.a[:] = 0
        self.active = False
        self.version += 1


class Term6Table:
    """ipv6_tunnel_term_table + rx_ipv6_tunnel_source_port: (outer IPv6 source, VNI) -> the tunnel
    port the inner frame enters on.  The VNI lies past a 64-B header slot (frame bytes 66..68):
    a frame that arrives as a wide header pair (128 B, nfdp.h kPortCont) is terminated by the
    kernels from the device copy `a` (open addressing over term6_hash, 32-B entries) in the same
    pass; a plain 64-B slot is only recognised (reason recirc6) and finished on the whole frame by
    the I/O layer with `lookup` (`DataPlane.resolve_recirc6`)."""

    SLOTS = 256

    def __init__(self):
        self.entries: dict[tuple[int, int], int] = {}
        self.version = 0
        self.a = np.zeros(self.SLOTS, TERM6_DTYPE)
        self.mask = self.SLOTS - 1

    def _rebuild(self) -> None:
        a = np.zeros(self.SLOTS, TERM6_DTYPE)
        for (src, vni), port in self.entries.items():
            w = np.frombuffer(ipaddress.IPv6Address(src).packed, "<u4").astype(np.uint32)
            with np.errstate(over="ignore"):
                h = fmix32(w[3] ^ (np.uint32(vni) * np.uint32(0x9E3779B1)))
                h = fmix32(w[2] ^ h)
                h = fmix32(w[1] ^ h)
                h = int(fmix32(w[0] ^ h))
            for q in range(8):
                i = (h + q) & self.mask
                if not a[i]["valid"]:
                    a[i] = (w, vni, port, 1, (0, 0))
                    break
            else:
                raise RuntimeError("term6 table probe limit reached")
        self.a = a

    def insert(self, src, vni: int, port: int) -> None:
        self.entries[(int(ipaddress.IPv6Address(int(src) if isinstance(src, (int, np.integer)) else src)),
                      vni & 0xFFFFFF)] = int(port)
        self._rebuild()
        self.version += 1

    def clear(self) -> None:
        self.entries.clear()
        self._rebuild()
        self.version += 1

    def lookup(self, frame: bytes) -> tuple[int, int] | None:
        """(tunnel port, inner offset) of an IPv6 VXLAN / GENEVE frame (an outer 802.1Q tag
        allowed), or None: VXLAN needs its I flag, GENEVE version 0, no options, not OAM, an
        Ethernet payload (the checks the kernel leaves to the whole frame: pipeline.h
        tunnel_hdr_ok)."""
        off = 4 if frame[12:14] == b"\x81\x00" else 0
        if len(frame) < 84 + off or frame[12 + off:14 + off] != b"\x86\xdd" or frame[20 + off] != 17:
            return None
        t = 62 + off
        dport = int.from_bytes(frame[56 + off:58 + off], "big")
        if dport == 4789:
            if not frame[t] & 0x08:
                return None
        elif dport == 6081:
            if frame[t] != 0 or frame[t + 1] & 0x80 or frame[t + 2:t + 4] != b"\x65\x58":
                return None
        else:
            return None
        src = int.from_bytes(frame[22 + off:38 + off], "big")
        vni = int.from_bytes(frame[t + 4:t + 7], "big")
        p = self.entries.get((src, vni))
        return None if p is None else (p, t + 8)

    def __len__(self) -> int:
        return len(self.entries)


class TermTable:
    """Tunnel termination (ipv4_tunnel_term_table + rx_ipv4_tunnel_source_port):
    (outer source IPv4, VNI) -> the tunnel port the inner frame re-enters on."""

    def __init__(self, slots: int = 1024):
        if slots & (slots - 1):
            raise ValueError("term table size must be a power of two")
        self.a = np.zeros(slots, TERM_DTYPE)
        self.mask = slots - 1
        self.n = 0
        self.version = 0

    def insert(self, src, vni: int, port: int) -> None:
        raw = int(ip_raw(np.uint32(ip_to_int(src))))
        with np.errstate(over="ignore"):
            h = int(fmix32(np.uint32(raw) ^ (np.uint32(vni) * np.uint32(0x9E3779B1))))
        for q in range(8):
            i = (h + q) & self.mask
            was = bool(self.a[i]["valid"])
            if not was or (self.a[i]["src_ip"] == raw and self.a[i]["vni"] == vni):
                self.a[i] = (raw, vni, port, 1, 0)
                self.n += 0 if was else 1
                self.version += 1
                return
        raise RuntimeError("term table probe limit reached")


class VmMacTable:
    """VM IPv4 -> MAC maps (P4 vm_src_ip4_mac_map_table / vm_dst_ip4_mac_map_table): a routed
    packet from a mapped source IP leaves with that MAC as its source MAC, one to a mapped
    destination IP with that MAC as its destination MAC (nfdp.h vmmac_lookup, applied in
    pipeline.h route_ipv4 after the nexthop's MACs).  Open addressing over (ip, kind)."""

    PROBE = 8

    def __init__(self, slots: int = 4096):
        if slots & (slots - 1):
            raise ValueError("vmmac table size must be a power of two")
        self.a = np.zeros(slots, VMMAC_DTYPE)
        self.mask = slots - 1
        self.n = 0
        self.version = 0

    @staticmethod
    def _hash(raw: int, kind: int) -> int:
        with np.errstate(over="ignore"):
            return int(fmix32(np.uint32(raw) ^ (np.uint32(kind) * np.uint32(0x85EBCA77))))

    def set(self, ip, kind: int, mac) -> None:
        if kind not in (VMMAC_SRC, VMMAC_DST):
            raise ValueError("kind must be VMMAC_SRC or VMMAC_DST")
        raw = int(ip_raw(np.uint32(ip_to_int(ip))))
        lo, hi = mac_raw(mac)
        h = self._hash(raw, kind)
        for q in range(self.PROBE):
            i = (h + q) & self.mask
            was = int(self.a[i]["kind"])
            if not was or (self.a[i]["ip"] == raw and was == kind):
                self.a[i] = (raw, kind, lo, hi)
                self.n += 0 if was else 1
                self.version += 1
                return
        raise RuntimeError("vmmac table probe limit reached")

    def clear(self) -> None:
        if self.n:
            self.a[:] = np.zeros((), VMMAC_DTYPE)
            self.n = 0
            self.version += 1

    def lookup(self, ip, kind: int):
        """(mac_lo, mac_hi) or None (host-side twin of vmmac_lookup)."""
        raw = int(ip_raw(np.uint32(ip_to_int(ip))))
        h = self._hash(raw, kind)
        for q in range(self.PROBE):
            e = self.a[(h + q) & self.mask]
            if not e["kind"]:
                return None
            if e["ip"] == raw and e["kind"] == kind:
                return int(e["mac_lo"]), int(e["mac_hi"])
        return None


FLOOD_LINK = 0x8000      # nfdp.h kFloodLink: an entry >= this (!= PORT_NONE) links to overflow row entry - FLOOD_LINK
FLOOD_MAX_ROWS = 0x7000  # nfdp.h kFloodMaxRows


class FloodTable:
    """Per-bridge flood groups (OvS NORMAL broadcast / unknown-unicast flooding), any size.

    Row b (< ``bridges``) is bridge b's head row of ``FLOOD_WAYS`` entries.  A group of up to 16
    members fills its head row; a bigger one keeps 15 members per row and links the 16th entry
    to an overflow row (rows >= ``bridges``, allocated on demand and recycled), so the kernel's
    first-member search stays inside the head row and the side pass follows the chain."""

    def __init__(self, bridges: int = 4096):
        self.bridges = bridges
        self.a = np.full((bridges, FLOOD_WAYS), PORT_NONE, np.uint16)
        self.n = 0
        self.version = 0
        self._rows: dict[int, list[int]] = {}   # bridge -> its overflow rows
        self._free: list[int] = []

    def _alloc_row(self) -> int:
        if self._free:
            r = self._free.pop()
        else:
            r = len(self.a)
            if r >= FLOOD_MAX_ROWS:
                raise ValueError("flood table: out of overflow rows")
            grow = max(64, len(self.a) // 4)
            self.a = np.vstack([self.a, np.full((grow, FLOOD_WAYS), PORT_NONE, np.uint16)])
            self._free.extend(range(len(self.a) - 1, r, -1))
        self.a[r] = PORT_NONE
        return r

    def set_members(self, bridge: int, ports: list[int]) -> None:
        if not 0 <= bridge < self.bridges:
            raise ValueError("bridge id out of range")
        ports = [int(p) for p in ports]
        if any(not 0 <= p < MAX_PORTS for p in ports):
            raise ValueError("flood member out of range")
        for r in self._rows.pop(bridge, []):
            self.a[r] = PORT_NONE
            self._free.append(r)
        self.a[bridge] = PORT_NONE
        rows, row, rest = [], bridge, ports
        while len(rest) > FLOOD_WAYS:
            nxt = self._alloc_row()
            rows.append(nxt)
            self.a[row, : FLOOD_WAYS - 1] = rest[: FLOOD_WAYS - 1]
            self.a[row, FLOOD_WAYS - 1] = FLOOD_LINK + nxt
            rest, row = rest[FLOOD_WAYS - 1:], nxt
        self.a[row, : len(rest)] = rest
        if rows:
            self._rows[bridge] = rows
        self.n = max(self.n, bridge + 1) if ports else self.n
        self.version += 1

    def add_member(self, bridge: int, port: int) -> None:
        cur = self.members(bridge)
        if port not in cur:
            self.set_members(bridge, cur + [port])

    def remove_member(self, bridge: int, port: int) -> None:
        self.set_members(bridge, [p for p in self.members(bridge) if p != port])

    def members(self, bridge: int) -> list[int]:
        out, row = [], bridge
        for _ in range(FLOOD_MAX_ROWS):
            for p in self.a[row]:
                p = int(p)
                if p == PORT_NONE:
                    return out
                if p >= FLOOD_LINK:
                    row = p - FLOOD_LINK
                    break
                out.append(p)
            else:
                return out
        return out


class LagTable:
    """LAG groups: `LAG_WAYS` member slots per group indexed by hash[2:0] (P4 tx_lag_table)."""

    def __init__(self, groups: int = 64):
        self.a = np.full(groups * LAG_WAYS, PORT_NONE, np.uint16)
        self.n = 0
        self.version = 0

    def set_group(self, group: int, members: list[int]) -> None:
        """Spread `members` over the 8 hash buckets (round robin, like equal-weight LAG)."""
        if not 0 <= group < len(self.a) // LAG_WAYS:
            raise ValueError("LAG group out of range")
        if not members:
            row = [PORT_NONE] * LAG_WAYS
        else:
            row = [members[i % len(members)] for i in range(LAG_WAYS)]
        self.a[group * LAG_WAYS:(group + 1) * LAG_WAYS] = row
        self.n = max(self.n, group + 1)
        self.version += 1

    def set_slot(self, group: int, hash_bits: int, port: int) -> None:
        self.a[group * LAG_WAYS + (hash_bits & 7)] = port
        self.n = max(self.n, group + 1)
        self.version += 1


HOP_XFER = 0x10          # | plane: the rest of the chain runs on that GPU (nfdp.h kHopXfer)
MAX_XFER_PLANE = 15


def expand_hops(hops) -> list[int]:
    """Chain hops -> opcodes.  A hop may name the GPU it runs on, ``"ttl@1"``; the chain then hands
    the frame over (a kHopXfer op) wherever the GPU changes, and a hop without ``@`` runs where the
    previous one did (the first on the GPU the frame entered).  ``"@1"`` alone is an explicit
    hand-off.  A route hop may come before a hand-off: the egress port it decided travels with the
    frame (pipeline.h hop_resume_word), since it depends on the header the route rewrote."""
    codes: list[int] = []
    cur = None
    for h in hops:
        if isinstance(h, str):
            name, _, at = h.partition("@")
            if at:
                g = int(at)
                if not 0 <= g <= MAX_XFER_PLANE:
                    raise ValueError(f"hop {h!r}: GPU plane in [0, {MAX_XFER_PLANE}]")
                if g != cur:
                    codes.append(HOP_XFER | g)
                    cur = g
            if name:
                if name not in HOP_NAMES:
                    raise ValueError(f"unknown hop {name!r}")
                codes.append(HOP_NAMES[name])
        else:
            codes.append(int(h))
    return codes


class ChainTable:
    def __init__(self, capacity: int = 4096):
        self.a = np.zeros(capacity, CHAIN_DTYPE)
        self.n = 1  # chain 0 = empty chain (plain forward to flow.out_port)
        self.version = 0

    def xfer_planes(self) -> set[int]:
        """GPU planes that split chains hand frames to (empty: no chain crosses GPUs)."""
        a = self.a[: self.n]
        out: set[int] = set()
        for row in a[a["nhops"] > 0]:
            out.update(int(c) & MAX_XFER_PLANE for c in row["hop"][: int(row["nhops"])] if c >= HOP_XFER)
        return out

    def split(self) -> bool:
        a = self.a[: self.n]
        hop = a["hop"]
        live = np.arange(hop.shape[1])[None, :] < a["nhops"][:, None]
        return bool(((hop >= HOP_XFER) & live).any())

    def add(self, hops, acl_id: int = 0) -> int:
        if self.n >= len(self.a):
            raise RuntimeError("chain table full")
        cid = self.n
        self.set(cid, hops, acl_id)
        self.n += 1
        return cid

    def set(self, cid: int, hops, acl_id: int = 0) -> None:
        codes = expand_hops(hops)
        if len(codes) > 7:
            raise ValueError("at most 7 hops per chain (hand-offs to another GPU included)")
        hop = np.zeros(7, np.uint8)
        hop[: len(codes)] = codes
        self.a[cid]["nhops"] = len(codes)
        self.a[cid]["hop"] = hop
        self.a[cid]["acl_id"] = acl_id
        self.n = max(self.n, cid + 1)
        self.version += 1


class MacTable:
    """(bridge, dst MAC) -> port; open addressing, hash identical to nfdp.h mac_lookup."""

    def __init__(self, slots: int = 1 << 16):
        if slots & (slots - 1):
            raise ValueError("MAC table size must be a power of two")
        self.a = np.zeros(slots, MAC_DTYPE)
        self.mask = slots - 1
        self.version = 0

    def _h(self, bridge, lo, hi) -> int:
        with np.errstate(over="ignore"):
            x = np.uint32(lo) ^ (np.uint32(hi) << np.uint32(16)) ^ (np.uint32(bridge) * np.uint32(0x9E3779B1))
        return int(fmix32(x)) & self.mask

    # Deleted slots become tombstones (valid=2, bridge 0xFFFF which no port uses): the kernel's
    # probe keeps walking over them (it stops only at valid == 0) and never matches them.
    # Learned entries (valid=3) are inserted by the data plane itself (mac_learn_kernel) and
    # folded back into this model with merge_learned() before the host uploads the table.
    TOMBSTONE_BRIDGE = 0xFFFF

    def _find(self, bridge: int, lo: int, hi: int) -> tuple[int, int]:
        """-> (slot of the key or -1, first reusable slot or -1)."""
        h = self._h(bridge, lo, hi)
        free = -1
        for p in range(16):
            i = (h + p) & self.mask
            e = self.a[i]
            if not e["valid"]:
                return -1, free if free >= 0 else i
            if e["valid"] == MAC_TOMB:
                free = i if free < 0 else free
            elif e["mac_lo"] == lo and e["mac_hi"] == hi and e["bridge_id"] == bridge:
                return i, free
        return -1, free

    def insert(self, bridge: int, mac, out_port: int) -> None:
        if not 0 <= bridge < self.TOMBSTONE_BRIDGE:
            raise ValueError("bridge id must be in [0, 0xFFFF)")
        lo, hi = mac_raw(mac)
        at, free = self._find(bridge, lo, hi)
        slot = at if at >= 0 else free
        if slot < 0:
            raise RuntimeError("MAC table probe limit reached")
        self.a[slot] = (lo, hi, bridge, out_port, MAC_STATIC, 0)
        self.version += 1

    def insert_learned(self, bridge: int, lo: int, hi: int, out_port: int, stamp: int) -> bool:
        """Merge one entry the data plane learned (static entries win).  False: no slot."""
        at, free = self._find(bridge, lo, hi)
        if at >= 0:
            if self.a[at]["valid"] == MAC_STATIC:
                return True
            slot = at
        else:
            slot = free
        if slot < 0:
            return False
        self.a[slot] = (lo, hi, bridge, out_port, MAC_LEARNED, stamp)
        self.version += 1
        return True

    def merge_learned(self, dev: np.ndarray) -> int:
        """Fold the device table's learned entries (valid == 3) into this host model."""
        n = 0
        for e in dev[dev["valid"] == MAC_LEARNED]:
            n += self.insert_learned(int(e["bridge_id"]), int(e["mac_lo"]), int(e["mac_hi"]), int(e["out_port"]),
                                     int(e["stamp"]))
        return n

    def age(self, now: int, max_age: int) -> int:
        """Remove learned entries last seen more than `max_age` stamps ago (host aging)."""
        old = np.where((self.a["valid"] == MAC_LEARNED) & ((now - self.a["stamp"].astype(np.int64)) > max_age))[0]
        for i in old:
            self.a[i] = (0xFFFFFFFF, 0xFFFF, self.TOMBSTONE_BRIDGE, 0xFFFF, MAC_TOMB, 0)
        if len(old):
            self.version += 1
        return len(old)

    def learned(self) -> list[tuple[int, str, int]]:
        """(bridge, mac, port) of every learned entry."""
        from ..ops.packets import mac_str

        out = []
        for e in self.a[self.a["valid"] == MAC_LEARNED]:
            lo, hi = int(e["mac_lo"]), int(e["mac_hi"])
            raw = bytes([lo & 0xFF, lo >> 8 & 0xFF, lo >> 16 & 0xFF, lo >> 24 & 0xFF, hi & 0xFF, hi >> 8 & 0xFF])
            out.append((int(e["bridge_id"]), mac_str(raw), int(e["out_port"])))
        return out

    def lookup(self, bridge: int, mac) -> int:
        lo, hi = mac_raw(mac)
        at, _ = self._find(bridge, lo, hi)
        return int(self.a[at]["out_port"]) if at >= 0 else -1

    def remove(self, bridge: int, mac) -> bool:
        lo, hi = mac_raw(mac)
        at, _ = self._find(bridge, lo, hi)
        if at < 0:
            return False
        self.a[at] = (0xFFFFFFFF, 0xFFFF, self.TOMBSTONE_BRIDGE, 0xFFFF, MAC_TOMB, 0)
        self.version += 1
        return True

    def clear(self) -> None:
        self.a[:] = np.zeros((), MAC_DTYPE)
        self.version += 1


@dataclass
class AclRule:
    value: np.ndarray  # uint32[4] over the FlowKey words
    mask: np.ndarray
    permit: bool


def _prefix_mask(bits: int) -> int:
    return 0 if bits == 0 else ((0xFFFFFFFF << (32 - bits)) & 0xFFFFFFFF)


def range_to_prefixes(lo: int, hi: int, width: int = 16) -> list[tuple[int, int]]:
    """[lo, hi] -> list of (value, mask) ternary prefixes (TCAM range expansion)."""
    out = []
    full = (1 << width) - 1
    while lo <= hi:
        size = lo & -lo if lo else 1 << width
        while size > hi - lo + 1:
            size >>= 1
        out.append((lo, full & ~(size - 1)))
        lo += size
    return out


class AclTable:
    """Priority-ordered ternary rules (index = priority, first match wins), <= 4096 rules
    (12-bit rule index in the MFMA accumulator; the P4 tables hold 1024)."""

    MAX_RULES = 4096

    def __init__(self, default_permit: bool = True):
        self.rules: list[AclRule] = []
        self.rules6: list[AclRule] = []   # IPv6 rules (their own priority order)
        self.default_permit = default_permit
        self.version = 0

    def add_raw(self, value, mask, permit: bool) -> int:
        """An IPv4 rule over the FlowKey words.  The rule also requires kKeyV6 clear, so it never
        matches an IPv6 packet's key."""
        if len(self.rules) >= self.MAX_RULES:
            raise RuntimeError(f"ACL full ({self.MAX_RULES} rules)")
        m = np.asarray(mask, np.uint32).copy()
        m[3] |= np.uint32(KEY_V6)
        v = np.asarray(value, np.uint32) & m
        self.rules.append(AclRule(v, m, bool(permit)))
        self.version += 1
        return len(self.rules) - 1

    def add_raw6(self, value, mask, permit: bool) -> int:
        """An IPv6 rule over the 12 key6 words (nfdp.h key6_word: src6, dst6, ports, next header
        | zone << 16, 0, 0).  Returns its index among the IPv6 rules."""
        if len(self.rules6) >= self.MAX_RULES:
            raise RuntimeError(f"IPv6 ACL full ({self.MAX_RULES} rules)")
        m = np.asarray(mask, np.uint32)
        v = np.asarray(value, np.uint32) & m
        if v.shape != (12,):
            raise ValueError("IPv6 rule value / mask are 12 words")
        self.rules6.append(AclRule(v, m.copy(), bool(permit)))
        self.version += 1
        return len(self.rules6) - 1

    @staticmethod
    def _family(cidr):
        return None if cidr is None else ipaddress.ip_network(cidr, strict=False).version

    def add(self, *, permit: bool, src=None, dst=None, sport=None, dport=None, proto=None, zone=None,
            family=None) -> list[int]:
        """Add a rule from fields; CIDRs for src/dst, int or (lo, hi) ranges for ports.
        Port ranges expand to several ternary entries (returned indices).  IPv6 CIDRs make an
        IPv6 rule (indices among the IPv6 rules).  A rule with no address is an IPv4 rule, or
        with `family` 6 an IPv6 one, or with family "any" one of each (the IPv4 indices are
        returned).  (IPv6 rules switch the data plane to its IPv6-capable kernel instances.)"""
        fams = {f for f in (self._family(src), self._family(dst)) if f}
        if len(fams) > 1:
            raise ValueError("src and dst CIDRs must be the same address family")
        fam = fams.pop() if fams else {None: 4, 4: 4, 6: 6, "any": None}[family]

        def prefixes(p):
            if p is None:
                return [(0, 0)]
            if isinstance(p, tuple):
                return range_to_prefixes(p[0], p[1])
            return [(int(p), 0xFFFF)]

        if fam in (None, 6):
            v6 = np.zeros(12, np.uint32)
            m6 = np.zeros(12, np.uint32)
            for base, cidr in ((0, src), (4, dst)):
                if cidr is None:
                    continue
                net = ipaddress.IPv6Network(cidr, strict=False)
                v6[base:base + 4] = ip6_raw(int(net.network_address))
                m6[base:base + 4] = ip6_raw(int(net.netmask))
            if proto is not None:
                v6[9] |= np.uint32(proto & 0xFF)
                m6[9] |= np.uint32(0xFF)
            if zone is not None:
                v6[9] |= np.uint32((zone & 0xFFFF) << 16)
                m6[9] |= np.uint32(0xFFFF0000)
            idx6 = []
            for sv, sm in prefixes(sport):
                for dv, dm in prefixes(dport):
                    v, m = v6.copy(), m6.copy()
                    v[8] = port_raw(np.uint32(sv)) | (port_raw(np.uint32(dv)) << np.uint32(16))
                    m[8] = port_raw(np.uint32(sm)) | (port_raw(np.uint32(dm)) << np.uint32(16))
                    idx6.append(self.add_raw6(v, m, permit))
            if fam == 6:
                return idx6
        base_v = np.zeros(4, np.uint32)
        base_m = np.zeros(4, np.uint32)
        for word, cidr in ((0, src), (1, dst)):
            if cidr is None:
                continue
            net = ipaddress.IPv4Network(cidr, strict=False)
            base_v[word] = ip_raw(np.uint32(int(net.network_address)))
            base_m[word] = ip_raw(np.uint32(_prefix_mask(net.prefixlen)))
        if proto is not None:
            base_v[3] |= np.uint32(proto & 0xFF)
            base_m[3] |= np.uint32(0xFF)
        if zone is not None:
            base_v[3] |= np.uint32((zone & 0xFFFF) << 16)
            base_m[3] |= np.uint32(0xFFFF0000)

        def ports4(p, hi_bit):
            # [1024, 65535]: one entry on the ACL key's port-class bit (nfdp.h acl_key_meta)
            if isinstance(p, tuple) and (int(p[0]), int(p[1])) == (1024, 0xFFFF):
                return [(0, 0, hi_bit)]
            return [(v, m, 0) for v, m in prefixes(p)]

        idx = []
        for sv, sm, sf in ports4(sport, ACL_SPORT_HI):
            for dv, dm, df in ports4(dport, ACL_DPORT_HI):
                v, m = base_v.copy(), base_m.copy()
                v[2] = port_raw(np.uint32(sv)) | (port_raw(np.uint32(dv)) << np.uint32(16))
                m[2] = port_raw(np.uint32(sm)) | (port_raw(np.uint32(dm)) << np.uint32(16))
                v[3] |= np.uint32(sf | df)
                m[3] |= np.uint32(sf | df)
                idx.append(self.add_raw(v, m, permit))
        return idx

    def arrays6(self):
        """IPv6 rules: value / mask [n, 12], verdicts, n."""
        n = len(self.rules6)
        val = np.zeros((max(n, 1), 12), np.uint32)
        msk = np.zeros((max(n, 1), 12), np.uint32)
        per = np.zeros(max(n, 1), np.uint8)
        for i, r in enumerate(self.rules6):
            val[i], msk[i], per[i] = r.value, r.mask, 1 if r.permit else 0
        return val, msk, per, n

    def arrays(self):
        n = len(self.rules)
        val = np.zeros((max(n, 1), 4), np.uint32)
        msk = np.zeros((max(n, 1), 4), np.uint32)
        per = np.zeros(max(n, 1), np.uint8)
        for i, r in enumerate(self.rules):
            val[i], msk[i], per[i] = r.value, r.mask, 1 if r.permit else 0
        return val, msk, per, n


class FlowTable:
    """Thin wrapper over the native authoritative cuckoo table."""

    def __init__(self, nbuckets: int, rss_key: bytes = RSS_KEY):
        self.t = _nfdp_mod().FlowTable(nbuckets, rss_key)
        self.rss_key = rss_key

    def __len__(self) -> int:
        return len(self.t)

    @property
    def nbuckets(self) -> int:
        return self.t.nbuckets

    def insert(self, key, action) -> int:
        return self.t.insert(tuple(int(x) for x in key), tuple(int(x) for x in action))

    def insert_many(self, keys: np.ndarray, actions: np.ndarray) -> np.ndarray:
        return self.t.insert_many(np.ascontiguousarray(keys, np.uint32), np.ascontiguousarray(actions, np.uint32))

    def erase(self, key) -> bool:
        return self.t.erase(tuple(int(x) for x in key))

    def erase_many(self, keys: np.ndarray) -> int:
        return int(self.t.erase_many(np.ascontiguousarray(keys, np.uint32)))

    def find(self, key) -> int:
        return self.t.find(tuple(int(x) for x in key))
