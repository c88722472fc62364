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
    """Interface.  `ns` is a netns path ('' = the daemon's own namespace).  Every operation must
    be implemented (a silent no-op would let a CNI ADD "succeed" without doing anything)."""

    def link_by_name(self, name: str, ns: str = "") -> Link:
        raise NotImplementedError
    def link_set_up(self, name: str, ns: str = "") -> None:
        raise NotImplementedError
    def link_set_down(self, name: str, ns: str = "") -> None:
        raise NotImplementedError
    def link_set_name(self, name: str, new: str, ns: str = "") -> None:
        raise NotImplementedError
    def link_set_alias(self, name: str, alias: str, ns: str = "") -> None:
        raise NotImplementedError
    def link_set_hw_addr(self, name: str, mac: str, ns: str = "") -> None:
        raise NotImplementedError
    def link_set_mtu(self, name: str, mtu: int, ns: str = "") -> None:
        raise NotImplementedError
    def link_set_ns(self, name: str, target_ns: str, ns: str = "") -> None:
        raise NotImplementedError
    def link_set_vf(self, pf: str, vf: int, **attrs) -> None:
        raise NotImplementedError
    def addr_add(self, name: str, cidr: str, ns: str = "") -> None:
        raise NotImplementedError
    def addr_list(self, name: str, ns: str = "") -> list[str]:
        raise NotImplementedError
    def link_list(self, ns: str = "") -> list[Link]:
        raise NotImplementedError
    def link_add_veth(self, name: str, peer: str, ns: str = "") -> None:
        raise NotImplementedError
    def link_del(self, name: str, ns: str = "") -> None:
        raise NotImplementedError
    def run_in_ns(self, ns: str, fn):
        """Run fn() with the calling context inside netns `ns` (sockets it opens live there)."""
        raise NotImplementedError


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

    def addr_list(self, name, ns=""):
        with self._lock:
            return list(self._get(name, ns).addrs)

    def link_set_mtu(self, name, mtu, ns=""):
        with self._lock:
            self._get(name, ns).mtu = int(mtu)

    def run_in_ns(self, ns, fn):
        with self._lock:
            if ns not in self.ns:
                raise FileNotFoundError(f"netns {ns} does not exist")
        return fn()

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
RTM_NEWLINK, RTM_DELLINK, RTM_GETLINK = 16, 17, 18
RTM_NEWADDR, RTM_DELADDR, RTM_GETADDR = 20, 21, 22
NLM_F_REQUEST, NLM_F_ACK, NLM_F_EXCL, NLM_F_CREATE, NLM_F_DUMP = 1, 4, 0x200, 0x400, 0x300
NLA_F_NESTED = 0x8000
IFLA_ADDRESS, IFLA_IFNAME, IFLA_MTU, IFLA_LINKINFO, IFLA_IFALIAS = 1, 3, 4, 18, 20
IFLA_VFINFO_LIST, IFLA_NET_NS_FD = 22, 28
IFLA_MASTER = 10
IFLA_INFO_KIND, IFLA_INFO_DATA, VETH_INFO_PEER = 1, 2, 1
IFLA_VF_INFO = 1
IFLA_VF_MAC, IFLA_VF_VLAN, IFLA_VF_SPOOFCHK, IFLA_VF_LINK_STATE, IFLA_VF_RATE, IFLA_VF_TRUST = 1, 2, 4, 5, 6, 9
IFLA_VF_VLAN_LIST, IFLA_VF_VLAN_INFO = 12, 1
IFA_ADDRESS, IFA_LOCAL = 1, 2
IFF_UP = 1
CLONE_NEWNET = 0x40000000


def _libc():
    import ctypes

    return ctypes.CDLL(None, use_errno=True)


def setns_current_thread(ns_path: str) -> None:
    """Move the calling THREAD into the network namespace at `ns_path` (setns(2))."""
    import ctypes

    fd = os.open(ns_path, os.O_RDONLY)
    try:
        if _libc().setns(fd, CLONE_NEWNET) != 0:
            e = ctypes.get_errno()
            raise OSError(e, f"setns({ns_path}): {os.strerror(e)}")
    finally:
        os.close(fd)


def in_netns(ns: str, fn):
    """fn() on a helper thread that setns()'d into `ns` ('' = here).  Network namespaces are
    per thread, so the caller's own namespace never changes."""
    if not ns:
        return fn()
    box: dict = {}

    def run():
        try:
            setns_current_thread(ns)
            box["v"] = fn()
        except BaseException as e:  # noqa: BLE001 - re-raised in the caller
            box["e"] = e

    t = threading.Thread(target=run, name="netns-op")
    t.start()
    t.join()
    if "e" in box:
        raise box["e"]
    return box.get("v")


def create_netns(path: str) -> str:
    """Create a persistent network namespace bound at `path` (what `ip netns add` does)."""
    import ctypes

    os.makedirs(os.path.dirname(path), exist_ok=True)
    if not os.path.exists(path):
        open(path, "w").close()

    def run():
        lc = _libc()
        if lc.unshare(CLONE_NEWNET) != 0:
            e = ctypes.get_errno()
            raise OSError(e, f"unshare(CLONE_NEWNET): {os.strerror(e)}")
        src = f"/proc/self/task/{threading.get_native_id()}/ns/net"
        if lc.mount(src.encode(), path.encode(), None, 4096, None) != 0:  # MS_BIND
            e = ctypes.get_errno()
            raise OSError(e, f"bind mount {src} -> {path}: {os.strerror(e)}")

    box: dict = {}

    def wrapped():
        try:
            run()
        except BaseException as e:  # noqa: BLE001
            box["e"] = e

    t = threading.Thread(target=wrapped, name="netns-create")
    t.start()
    t.join()
    if "e" in box:
        try:
            os.unlink(path)
        except OSError:
            pass
        raise box["e"]
    return path


def delete_netns(path: str) -> None:
    lc = _libc()
    lc.umount2(path.encode(), 2)  # MNT_DETACH
    try:
        os.unlink(path)
    except OSError:
        pass


class RtNetlink(NetlinkManager):
    """rtnetlink over a raw NETLINK_ROUTE socket.  Operations on another network namespace run on
    a helper thread that setns()'d into it (the socket then talks to that namespace's kernel
    state), the way the reference's netns.Do + netlink calls work (networkfn.go:233-317,
    sriov.go:75-140, netlink_manager.go:12-90).  VF attributes use IFLA_VFINFO_LIST."""

    def __init__(self):
        self.seq = 1
        self._seq_lock = threading.Lock()

    def _sock(self):
        s = socket.socket(socket.AF_NETLINK, socket.SOCK_RAW, 0)  # NETLINK_ROUTE
        s.bind((0, 0))
        return s

    @staticmethod
    def _attr(t: int, data: bytes) -> bytes:
        ln = 4 + len(data)
        return struct.pack("HH", ln, t) + data + b"\0" * ((4 - ln % 4) % 4)

    @classmethod
    def _nest(cls, t: int, *children: bytes) -> bytes:
        return cls._attr(t | NLA_F_NESTED, b"".join(children))

    def _raw(self, msg_type: int, flags: int, body: bytes) -> list[bytes]:
        s = self._sock()
        try:
            with self._seq_lock:
                self.seq += 1
                seq = self.seq
            hdr = struct.pack("IHHII", 16 + len(body), msg_type, flags | NLM_F_REQUEST, seq, 0)
            s.send(hdr + body)
            out = []
            while True:
                data = s.recv(1 << 16)
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

    def _link_msg(self, msg_type: int, flags: int, ifi_index: int = 0, ifi_flags: int = 0, change: int = 0,
                  attrs: bytes = b"") -> list[bytes]:
        return self._raw(msg_type, flags, struct.pack("BxHiII", socket.AF_UNSPEC, 0, ifi_index, ifi_flags, change) + attrs)

    @staticmethod
    def _attrs(msg: bytes, off: int):
        while off + 4 <= len(msg):
            ln, t = struct.unpack_from("HH", msg, off)
            if ln < 4:
                break
            yield t & ~NLA_F_NESTED, msg[off + 4: off + ln]
            off += (ln + 3) & ~3

    def _parse(self, msg: bytes) -> Link:
        _fam, _t, idx, flags, _chg = struct.unpack_from("BxHiII", msg, 0)
        link = Link(name="", index=idx, up=bool(flags & IFF_UP))
        for t, val in self._attrs(msg, 16):
            if t == IFLA_IFNAME:
                link.name = val.rstrip(b"\0").decode()
            elif t == IFLA_ADDRESS and len(val) == 6:
                link.mac = ":".join(f"{b:02x}" for b in val)
            elif t == IFLA_IFALIAS:
                link.alias = val.rstrip(b"\0").decode()
            elif t == IFLA_MTU and len(val) >= 4:
                link.mtu = struct.unpack("I", val[:4])[0]
            elif t == IFLA_LINKINFO:
                for t2, v2 in self._attrs(val, 0):
                    if t2 == IFLA_INFO_KIND:
                        link.kind = v2.rstrip(b"\0").decode()
        return link

    def run_in_ns(self, ns, fn):
        return in_netns(ns, fn)

    # ------------------------------------------------------------------ links
    def link_list(self, ns=""):
        return in_netns(ns, lambda: [self._parse(m) for m in self._link_msg(RTM_GETLINK, NLM_F_DUMP)])

    def link_by_name(self, name, ns=""):
        for link in self.link_list(ns):
            if link.name == name:
                return link
        raise LinkNotFound(f"Link not found: {name} (netns '{ns}')")

    def _set(self, name, ns="", ifi_flags=0, change=0, attrs=b""):
        def op():
            idx = self.link_by_name(name).index
            self._link_msg(RTM_NEWLINK, NLM_F_ACK, idx, ifi_flags, change, attrs)

        in_netns(ns, op)

    def link_set_up(self, name, ns=""):
        self._set(name, ns, IFF_UP, IFF_UP)

    def link_set_down(self, name, ns=""):
        self._set(name, ns, 0, IFF_UP)

    def link_set_name(self, name, new, ns=""):
        self._set(name, ns, attrs=self._attr(IFLA_IFNAME, new.encode() + b"\0"))

    def link_set_alias(self, name, alias, ns=""):
        self._set(name, ns, attrs=self._attr(IFLA_IFALIAS, alias.encode() + b"\0"))

    def link_set_hw_addr(self, name, mac, ns=""):
        self._set(name, ns, attrs=self._attr(IFLA_ADDRESS, bytes(int(x, 16) for x in mac.split(":"))))

    def link_set_mtu(self, name, mtu, ns=""):
        self._set(name, ns, attrs=self._attr(IFLA_MTU, struct.pack("I", int(mtu))))

    def link_set_ns(self, name, target_ns, ns=""):
        # "" = this process's own namespace (the daemon's: host network), as elsewhere in this API
        fd = os.open(target_ns or "/proc/self/ns/net", os.O_RDONLY)
        try:
            self._set(name, ns, attrs=self._attr(IFLA_NET_NS_FD, struct.pack("I", fd)))
        finally:
            os.close(fd)

    def link_add_veth(self, name, peer, ns=""):
        peer_msg = struct.pack("BxHiII", socket.AF_UNSPEC, 0, 0, 0, 0) + self._attr(IFLA_IFNAME, peer.encode() + b"\0")
        info = self._nest(IFLA_LINKINFO, self._attr(IFLA_INFO_KIND, b"veth\0"),
                          self._nest(IFLA_INFO_DATA, self._nest(VETH_INFO_PEER, peer_msg)))
        attrs = self._attr(IFLA_IFNAME, name.encode() + b"\0") + info
        in_netns(ns, lambda: self._link_msg(RTM_NEWLINK, NLM_F_ACK | NLM_F_CREATE | NLM_F_EXCL, attrs=attrs))

    def link_del(self, name, ns=""):
        def op():
            idx = self.link_by_name(name).index
            self._link_msg(RTM_DELLINK, NLM_F_ACK, idx)

        in_netns(ns, op)

    def link_add_bridge(self, name, ns=""):
        """A Linux bridge netdev (`ip link add NAME type bridge`)."""
        info = self._nest(IFLA_LINKINFO, self._attr(IFLA_INFO_KIND, b"bridge\0"))
        attrs = self._attr(IFLA_IFNAME, name.encode() + b"\0") + info
        in_netns(ns, lambda: self._link_msg(RTM_NEWLINK, NLM_F_ACK | NLM_F_CREATE | NLM_F_EXCL, attrs=attrs))

    def link_set_master(self, name, master, ns=""):
        """Enslave `name` to the bridge `master` (`ip link set NAME master MASTER`)."""
        def op():
            m = self.link_by_name(master).index
            idx = self.link_by_name(name).index
            self._link_msg(RTM_NEWLINK, NLM_F_ACK, idx, 0, 0, self._attr(IFLA_MASTER, struct.pack("I", m)))

        in_netns(ns, op)

    # ------------------------------------------------------------------ addresses
    def addr_add(self, name, cidr, ns=""):
        import ipaddress

        net = ipaddress.ip_interface(cidr)
        fam = socket.AF_INET if net.version == 4 else socket.AF_INET6
        raw = net.ip.packed

        def op():
            idx = self.link_by_name(name).index
            body = struct.pack("BBBBI", fam, net.network.prefixlen, 0, 0, idx)
            body += self._attr(IFA_LOCAL, raw) + self._attr(IFA_ADDRESS, raw)
            self._raw(RTM_NEWADDR, NLM_F_ACK | NLM_F_CREATE | NLM_F_EXCL, body)

        in_netns(ns, op)

    def addr_list(self, name, ns=""):
        import ipaddress

        def op():
            idx = self.link_by_name(name).index
            out = []
            for m in self._raw(RTM_GETADDR, NLM_F_DUMP, struct.pack("BBBBI", socket.AF_UNSPEC, 0, 0, 0, 0)):
                fam, plen, _fl, _sc, ai = struct.unpack_from("BBBBI", m, 0)
                if ai != idx:
                    continue
                for t, v in self._attrs(m, 8):
                    if t == IFA_ADDRESS:
                        out.append(f"{ipaddress.ip_address(v)}/{plen}")
            return out

        return in_netns(ns, op)

    # ------------------------------------------------------------------ SR-IOV VFs
    def link_set_vf(self, pf, vf, **attrs):
        """IFLA_VF_* on the PF (sriov.go:200-282): mac, vlan / qos / vlan_proto, spoofchk, trust,
        min_tx_rate / max_tx_rate, link_state."""
        known = {"mac", "vlan", "qos", "vlan_proto", "spoofchk", "trust", "min_tx_rate", "max_tx_rate", "link_state"}
        bad = set(attrs) - known
        if bad:
            raise AttributeError(f"unknown VF attribute(s) {sorted(bad)}")
        parts = []
        if "mac" in attrs:
            mac = bytes(int(x, 16) for x in attrs["mac"].split(":"))
            parts.append(self._attr(IFLA_VF_MAC, struct.pack("I", vf) + mac + b"\0" * (32 - len(mac))))
        if "vlan" in attrs or "qos" in attrs or "vlan_proto" in attrs:
            vlan, qos = int(attrs.get("vlan", 0)), int(attrs.get("qos", 0))
            proto = int(attrs.get("vlan_proto", 0x8100))
            if proto == 0x8100:
                parts.append(self._attr(IFLA_VF_VLAN, struct.pack("III", vf, vlan, qos)))
            else:
                info = self._attr(IFLA_VF_VLAN_INFO, struct.pack("III", vf, vlan, qos) + struct.pack(">H", proto) + b"\0\0")
                parts.append(self._nest(IFLA_VF_VLAN_LIST, info))
        if "spoofchk" in attrs:
            parts.append(self._attr(IFLA_VF_SPOOFCHK, struct.pack("II", vf, 1 if attrs["spoofchk"] else 0)))
        if "trust" in attrs:
            parts.append(self._attr(IFLA_VF_TRUST, struct.pack("II", vf, 1 if attrs["trust"] else 0)))
        if "min_tx_rate" in attrs or "max_tx_rate" in attrs:
            parts.append(self._attr(IFLA_VF_RATE, struct.pack("III", vf, int(attrs.get("min_tx_rate", 0)),
                                                               int(attrs.get("max_tx_rate", 0)))))
        if "link_state" in attrs:
            parts.append(self._attr(IFLA_VF_LINK_STATE, struct.pack("II", vf, int(attrs["link_state"]))))
        if parts:
            self._set(pf, "", attrs=self._nest(IFLA_VFINFO_LIST, self._nest(IFLA_VF_INFO, *parts)))
