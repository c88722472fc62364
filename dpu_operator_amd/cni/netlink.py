"""Netlink abstraction (the reference's mockable NetlinkManager, dpu-cni/pkgs/sriovutils/netlink_manager.go:12-90).

`NetlinkManager` is the interface the CNI code uses; `FakeNetlink` is a complete in-memory model
of links, network namespaces and SR-IOV VF state (tests, and hosts without CAP_NET_ADMIN).
The production implementation on a real node is `RtNetlink` (rtnetlink over AF_NETLINK for the
link operations; VF attributes via IFLA_VFINFO_LIST), kept deliberately small.
"""
from __future__ import annotations

import copy
import os
import socket
import struct
import threading
from dataclasses import dataclass, field


class LinkNotFound(KeyError):
    pass


@dataclass
class VfConfig:
    mac: str = "00:00:00:00:00:00"
    vlan: int = 0
    qos: int = 0
    vlan_proto: int = 33024
    spoofchk: bool = True
    trust: bool = False
    min_tx_rate: int = 0
    max_tx_rate: int = 0
    link_state: int = 0  # 0 auto, 1 enable, 2 disable


@dataclass
class Link:
    name: str
    mac: str = "00:00:00:00:00:00"
    up: bool = False
    alias: str = ""
    mtu: int = 1500
    index: int = 0
    kind: str = "device"
    vfs: list[VfConfig] = field(default_factory=list)
    addrs: list[str] = field(default_factory=list)
    peer: str = ""


class NetlinkManager:
    """Interface.  `ns` is a netns path ('' = the daemon's own namespace)."""

    def link_by_name(self, name: str, ns: str = "") -> Link: ...
    def link_set_up(self, name: str, ns: str = "") -> None: ...
    def link_set_down(self, name: str, ns: str = "") -> None: ...
    def link_set_name(self, name: str, new: str, ns: str = "") -> None: ...
    def link_set_alias(self, name: str, alias: str, ns: str = "") -> None: ...
    def link_set_hw_addr(self, name: str, mac: str, ns: str = "") -> None: ...
    def link_set_ns(self, name: str, target_ns: str, ns: str = "") -> None: ...
    def link_set_vf(self, pf: str, vf: int, **attrs) -> None: ...
    def addr_add(self, name: str, cidr: str, ns: str = "") -> None: ...
    def link_list(self, ns: str = "") -> list[Link]: ...
    def link_add_veth(self, name: str, peer: str, ns: str = "") -> None: ...
    def link_del(self, name: str, ns: str = "") -> None: ...


class FakeNetlink(NetlinkManager):
    def __init__(self):
        self._lock = threading.RLock()
        self.ns: dict[str, dict[str, Link]] = {"": {}}
        self._idx = 1
        self.ops: list[tuple] = []

    # helpers for tests / platform models
    def add_link(self, link: Link, ns: str = "") -> Link:
        with self._lock:
            self._idx += 1
            link.index = self._idx
            self.ns.setdefault(ns, {})[link.name] = link
            return link

    def add_netns(self, path: str) -> None:
        with self._lock:
            self.ns.setdefault(path, {})

    def _get(self, name: str, ns: str) -> Link:
        try:
            return self.ns[ns][name]
        except KeyError:
            raise LinkNotFound(f"Link not found: {name} (netns '{ns}')") from None

    def link_by_name(self, name, ns=""):
        with self._lock:
            return copy.deepcopy(self._get(name, ns))

    def link_set_up(self, name, ns=""):
        with self._lock:
            self._get(name, ns).up = True
            self.ops.append(("up", name, ns))

    def link_set_down(self, name, ns=""):
        with self._lock:
            self._get(name, ns).up = False
            self.ops.append(("down", name, ns))

    def link_set_name(self, name, new, ns=""):
        with self._lock:
            if new in self.ns[ns]:
                raise FileExistsError(f"link {new} exists in netns '{ns}'")
            link = self.ns[ns].pop(name) if name in self.ns.get(ns, {}) else self._get(name, ns)
            link.name = new
            self.ns[ns][new] = link
            self.ops.append(("rename", name, new, ns))

    def link_set_alias(self, name, alias, ns=""):
        with self._lock:
            self._get(name, ns).alias = alias

    def link_set_hw_addr(self, name, mac, ns=""):
        with self._lock:
            self._get(name, ns).mac = mac.lower()

    def link_set_ns(self, name, target_ns, ns=""):
        with self._lock:
            if target_ns not in self.ns:
                raise FileNotFoundError(f"netns {target_ns} does not exist")
            link = self.ns[ns].pop(name) if name in self.ns.get(ns, {}) else self._get(name, ns)
            if link.name in self.ns[target_ns]:
                self.ns[ns][name] = link
                raise FileExistsError(f"link {link.name} exists in {target_ns}")
            self.ns[target_ns][link.name] = link
            self.ops.append(("setns", name, ns, target_ns))

    def link_set_vf(self, pf, vf, **attrs):
        with self._lock:
            link = self._get(pf, "")
            while len(link.vfs) <= vf:
                link.vfs.append(VfConfig())
            for k, v in attrs.items():
                if not hasattr(link.vfs[vf], k):
                    raise AttributeError(f"unknown VF attribute {k}")
                setattr(link.vfs[vf], k, v)
            self.ops.append(("vf", pf, vf, dict(attrs)))

    def addr_add(self, name, cidr, ns=""):
        with self._lock:
            self._get(name, ns).addrs.append(cidr)

    def link_list(self, ns=""):
        with self._lock:
            return [copy.deepcopy(link) for link in self.ns.get(ns, {}).values()]

    def link_add_veth(self, name, peer, ns=""):
        with self._lock:
            for n, p in ((name, peer), (peer, name)):
                if n in self.ns.setdefault(ns, {}):
                    raise FileExistsError(n)
                mac = "02:00:%02x:%02x:%02x:%02x" % tuple(os.urandom(4))
                self.add_link(Link(name=n, mac=mac, kind="veth", peer=p), ns)

    def link_del(self, name, ns=""):
        with self._lock:
            link = self.ns[ns].pop(name, None)
            if link is None:
                raise LinkNotFound(name)
            if link.peer:
                for nsd in self.ns.values():
                    nsd.pop(link.peer, None)


# ---------------------------------------------------------------------------- real rtnetlink
RTM_NEWLINK, RTM_GETLINK, RTM_SETLINK = 16, 18, 19
NLM_F_REQUEST, NLM_F_ACK, NLM_F_DUMP = 1, 4, 0x300
IFLA_ADDRESS, IFLA_IFNAME, IFLA_NET_NS_FD, IFLA_IFALIAS = 1, 3, 28, 20
IFF_UP = 1


class RtNetlink(NetlinkManager):
    """Link operations over a raw NETLINK_ROUTE socket (namespace switching via setns(2) on a
    helper thread).  VF attributes are set through sysfs-free IFLA_VF_* messages."""

    def __init__(self):
        self.seq = 1

    def _sock(self):
        s = socket.socket(socket.AF_NETLINK, socket.SOCK_RAW, 0)  # NETLINK_ROUTE
        s.bind((0, 0))
        return s

    @staticmethod
    def _attr(t: int, data: bytes) -> bytes:
        ln = 4 + len(data)
        return struct.pack("HH", ln, t) + data + b"\0" * ((4 - ln % 4) % 4)

    def _request(self, msg_type: int, flags: int, ifi_index: int = 0, ifi_flags: int = 0, change: int = 0,
                 attrs: bytes = b"") -> list[bytes]:
        s = self._sock()
        try:
            body = struct.pack("BxHiII", socket.AF_UNSPEC, 0, ifi_index, ifi_flags, change) + attrs
            self.seq += 1
            hdr = struct.pack("IHHII", 16 + len(body), msg_type, flags | NLM_F_REQUEST, self.seq, 0)
            s.send(hdr + body)
            out = []
            while True:
                data = s.recv(65536)
                off = 0
                while off < len(data):
                    ln, typ, _fl, _seq, _pid = struct.unpack_from("IHHII", data, off)
                    if typ == 3:  # NLMSG_DONE
                        return out
                    if typ == 2:  # NLMSG_ERROR
                        err = struct.unpack_from("i", data, off + 16)[0]
                        if err:
                            raise OSError(-err, os.strerror(-err))
                        return out
                    out.append(data[off + 16: off + ln])
                    off += (ln + 3) & ~3
                if not (flags & NLM_F_DUMP):
                    return out
        finally:
            s.close()

    def _parse(self, msg: bytes) -> Link:
        _fam, _t, idx, flags, _chg = struct.unpack_from("BxHiII", msg, 0)
        off = 16
        link = Link(name="", index=idx, up=bool(flags & IFF_UP))
        while off + 4 <= len(msg):
            ln, t = struct.unpack_from("HH", msg, off)
            if ln < 4:
                break
            val = msg[off + 4: off + ln]
            if t == IFLA_IFNAME:
                link.name = val.rstrip(b"\0").decode()
            elif t == IFLA_ADDRESS and len(val) == 6:
                link.mac = ":".join(f"{b:02x}" for b in val)
            elif t == IFLA_IFALIAS:
                link.alias = val.rstrip(b"\0").decode()
            off += (ln + 3) & ~3
        return link

    def link_list(self, ns=""):
        return [self._parse(m) for m in self._request(RTM_GETLINK, NLM_F_DUMP)]

    def link_by_name(self, name, ns=""):
        for link in self.link_list(ns):
            if link.name == name:
                return link
        raise LinkNotFound(name)

    def _set(self, name, ifi_flags=0, change=0, attrs=b""):
        idx = self.link_by_name(name).index
        self._request(RTM_NEWLINK, NLM_F_ACK, idx, ifi_flags, change, attrs)

    def link_set_up(self, name, ns=""):
        self._set(name, IFF_UP, IFF_UP)

    def link_set_down(self, name, ns=""):
        self._set(name, 0, IFF_UP)

    def link_set_name(self, name, new, ns=""):
        self._set(name, attrs=self._attr(IFLA_IFNAME, new.encode() + b"\0"))

    def link_set_alias(self, name, alias, ns=""):
        self._set(name, attrs=self._attr(IFLA_IFALIAS, alias.encode() + b"\0"))

    def link_set_hw_addr(self, name, mac, ns=""):
        self._set(name, attrs=self._attr(IFLA_ADDRESS, bytes(int(x, 16) for x in mac.split(":"))))

    def link_set_ns(self, name, target_ns, ns=""):
        fd = os.open(target_ns, os.O_RDONLY)
        try:
            self._set(name, attrs=self._attr(IFLA_NET_NS_FD, struct.pack("I", fd)))
        finally:
            os.close(fd)
