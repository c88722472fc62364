"""OpenFlow-subset software bridge compiled onto the MI355X data plane.

The Marvell and NetSec VSPs of the reference program Open vSwitch with `ovs-vsctl` / `ovs-ofctl`
(internal/daemon/vendor-specific-plugins/marvell/ovs-dp/ovsdp.go:47-161, intel-netsec/main.go,
vspnetutils.go:261-282).  `OvsBridge` keeps the same vocabulary —
bridges, ports, `priority=..,in_port=..,dl_dst=..,actions=..` flows, `del-flows` with
non-strict matching, `dump-flows` — and compiles the rule set into the GPU tables instead of an
OvS datapath:

* a port whose highest-priority in_port-only flow is `output:Y` gets `default_out = Y` (K11);
* `in_port=X,dl_dst=M,actions=output:Y` becomes a (bridge_X, M) -> Y entry in the MAC table (K12),
  `actions=in_port` a (bridge_X, M) -> X entry (the hairpin of K13), `actions=drop` an entry to
  the invalid port (counted as a bad-port drop);
* `actions=normal` puts the port on the bridge's learning domain (MAC entries of every port whose
  MAC is known / learned);
* every port that has dl_dst-specific flows gets its own bridge id, so the MAC table lookup of the
  fused kernel is exactly OvS's (in_port, dl_dst) match; specific entries beat the port default
  because the kernel consults the MAC table first.
A dl_dst flow with LOWER priority than the port's in_port-only flow can never match in OvS and is
therefore not compiled.  Flows without in_port apply to every port (at their priority).
"""
from __future__ import annotations

import itertools
import re
import threading
from dataclasses import dataclass, field

from . import tables as T

DEFAULT_PRIORITY = 32768
_bridge_ids = itertools.count(1000)
_bid_lock = threading.Lock()


def _next_bid() -> int:
    with _bid_lock:
        return next(_bridge_ids)


@dataclass
class Flow:
    priority: int
    in_port: str | None
    dl_dst: str | None
    action: str          # "output:<port>" | "in_port" | "drop" | "normal"

    def text(self) -> str:
        m = [f"priority={self.priority}"]
        if self.in_port is not None:
            m.append(f"in_port={self.in_port}")
        if self.dl_dst is not None:
            m.append(f"dl_dst={self.dl_dst}")
        return ",".join(m) + f" actions={self.action}"


@dataclass
class OvsPort:
    name: str
    index: int                    # data-plane port
    mac: str | None = None
    pci: str | None = None
    dpdk: bool = False
    ptype: str = "system"


def _norm_mac(m: str) -> str:
    b = bytes(int(x, 16) for x in m.split(":"))
    if len(b) != 6:
        raise ValueError(f"bad MAC {m!r}")
    return ":".join(f"{x:02x}" for x in b)


def parse_flow(spec: str) -> Flow:
    """`priority=100,in_port=X,dl_dst=M,actions=in_port` (ovs-ofctl add-flow syntax subset)."""
    spec = spec.strip()
    m = re.search(r"(?:^|,|\s)actions=(.+)$", spec)
    if not m:
        raise ValueError(f"flow without actions: {spec!r}")
    action = m.group(1).strip()
    match = spec[: m.start()].strip(" ,")
    prio, in_port, dl_dst = DEFAULT_PRIORITY, None, None
    for tok in filter(None, (t.strip() for t in re.split(r"[,\s]+", match))):
        k, _, v = tok.partition("=")
        if k == "priority":
            prio = int(v)
        elif k == "in_port":
            in_port = v
        elif k == "dl_dst":
            dl_dst = _norm_mac(v)
        else:
            raise ValueError(f"unsupported match field {k!r} (supported: priority, in_port, dl_dst)")
    action = action.lower() if action.lower() in ("in_port", "drop", "normal") else action
    if not (action in ("in_port", "drop", "normal") or re.fullmatch(r"output:\S+", action)):
        raise ValueError(f"unsupported action {action!r}")
    if not 0 <= prio <= 65535:
        raise ValueError("priority out of range")
    return Flow(prio, in_port, dl_dst, action)


class OvsBridge:
    def __init__(self, dp, name: str, datapath_type: str = "netdev"):
        self.dp = dp
        self.name = name
        self.datapath_type = datapath_type
        self.ports: dict[str, OvsPort] = {}
        self.flows: list[Flow] = []
        self.learned: dict[str, str] = {}    # mac -> port name (static "learning" for actions=normal)
        self.normal_bid = _next_bid()
        self._port_bid: dict[str, int] = {}
        self._lock = threading.RLock()
        self._owned_macs: list[tuple[int, str]] = []

    # ------------------------------------------------------------------ ovs-vsctl
    def add_port(self, name: str, index: int, mac: str | None = None, pci: str | None = None, dpdk: bool = False,
                 may_exist: bool = True) -> OvsPort:
        with self._lock:
            if name in self.ports:
                if may_exist:
                    return self.ports[name]
                raise ValueError(f"port {name} already exists on {self.name}")
            if any(p.index == index for p in self.ports.values()):
                raise ValueError(f"data-plane port {index} already used on {self.name}")
            p = OvsPort(name, index, _norm_mac(mac) if mac else None, pci, dpdk, "dpdk" if dpdk else "system")
            self.ports[name] = p
            if p.mac:
                self.learned[p.mac] = name
            self.dp.ports.set(index, flags=T.PORT_VALID, bridge_id=self.normal_bid, mac=p.mac or "00:00:00:00:00:00",
                              peer_mac=p.mac or "00:00:00:00:00:00")
            self.compile()
            return p

    def del_port(self, name: str, if_exists: bool = True) -> None:
        with self._lock:
            p = self.ports.pop(name, None)
            if p is None:
                if if_exists:
                    return
                raise KeyError(name)
            self.flows = [f for f in self.flows if f.in_port != name and f.action != f"output:{name}"]
            self.learned = {m: n for m, n in self.learned.items() if n != name}
            self.dp.ports.clear(p.index)
            self._port_bid.pop(name, None)
            self.compile()

    def list_ports(self) -> list[str]:
        return sorted(self.ports)

    def learn(self, mac: str, port: str) -> None:
        with self._lock:
            if port not in self.ports:
                raise KeyError(port)
            self.learned[_norm_mac(mac)] = port
            self.compile()

    # ------------------------------------------------------------------ ovs-ofctl
    def add_flow(self, spec: str | Flow) -> Flow:
        f = parse_flow(spec) if isinstance(spec, str) else spec
        with self._lock:
            for ref in (f.in_port, f.action[7:] if f.action.startswith("output:") else None):
                if ref is not None and ref not in self.ports:
                    raise KeyError(f"no port {ref} on bridge {self.name}")
            # same match + priority replaces (ovs-ofctl add-flow semantics)
            self.flows = [g for g in self.flows if not (g.priority == f.priority and g.in_port == f.in_port
                                                        and g.dl_dst == f.dl_dst)]
            self.flows.append(f)
            self.compile()
            return f

    def del_flows(self, spec: str = "") -> int:
        """Non-strict delete: removes every flow whose match includes all given fields."""
        want: dict[str, str] = {}
        for tok in filter(None, (t.strip() for t in re.split(r"[,\s]+", spec))):
            k, _, v = tok.partition("=")
            if k not in ("in_port", "dl_dst"):
                raise ValueError(f"unsupported match field {k!r}")
            want[k] = _norm_mac(v) if k == "dl_dst" else v
        with self._lock:
            keep = [f for f in self.flows
                    if not all(getattr(f, k) == v for k, v in want.items())]
            n = len(self.flows) - len(keep)
            self.flows = keep
            self.compile()
            return n

    def dump_flows(self) -> list[str]:
        with self._lock:
            return [f.text() for f in sorted(self.flows, key=lambda f: -f.priority)]

    # ------------------------------------------------------------------ compile
    def _target(self, f: Flow, in_port: str) -> int:
        if f.action == "in_port":
            return self.ports[in_port].index
        if f.action == "drop":
            return T.PORT_NONE
        return self.ports[f.action[7:]].index

    def compile(self) -> None:
        """Recompute this bridge's port defaults and MAC entries (idempotent)."""
        dp = self.dp
        with self._lock:
            for bid, mac in self._owned_macs:
                dp.macs.remove(bid, mac)
            self._owned_macs = []
            normal_entries = {m: self.ports[n].index for m, n in self.learned.items() if n in self.ports}
            for name, p in self.ports.items():
                rel = [f for f in self.flows if f.in_port in (None, name)]
                base = [f for f in rel if f.dl_dst is None]
                top = max(base, key=lambda f: f.priority) if base else None
                spec = [f for f in rel if f.dl_dst is not None and (top is None or f.priority >= top.priority)]
                normal = top is None or top.action == "normal"
                if spec:
                    bid = self._port_bid.setdefault(name, _next_bid())
                else:
                    bid = self.normal_bid if normal else self._port_bid.setdefault(name, _next_bid())
                dp.ports.update(p.index, bridge_id=bid)
                if top is not None and top.action != "normal":
                    dp.ports.update(p.index, default_out=self._target(top, name))
                else:
                    dp.ports.update(p.index, default_out=None)
                if bid != self.normal_bid:
                    entries: dict[str, tuple[int, int]] = {}
                    if normal:
                        for m, idx in normal_entries.items():
                            entries[m] = (-1, idx)
                    for f in spec:
                        if f.action == "normal":
                            tgt = normal_entries.get(f.dl_dst)
                            if tgt is None:
                                continue
                        else:
                            tgt = self._target(f, name)
                        if f.dl_dst not in entries or f.priority >= entries[f.dl_dst][0]:
                            entries[f.dl_dst] = (f.priority, tgt)
                    for m, (_, tgt) in entries.items():
                        dp.macs.insert(bid, m, tgt)
                        self._owned_macs.append((bid, m))
            for m, idx in normal_entries.items():
                dp.macs.insert(self.normal_bid, m, idx)
                self._owned_macs.append((self.normal_bid, m))


@dataclass
class OvsSwitch:
    """`ovs-vsctl` surface over a set of bridges sharing one data plane."""
    dp: object
    bridges: dict[str, OvsBridge] = field(default_factory=dict)

    def add_br(self, name: str, datapath_type: str = "netdev", may_exist: bool = True) -> OvsBridge:
        if name in self.bridges:
            if may_exist:
                return self.bridges[name]
            raise ValueError(f"bridge {name} exists")
        self.bridges[name] = OvsBridge(self.dp, name, datapath_type)
        return self.bridges[name]

    def del_br(self, name: str) -> None:
        br = self.bridges.pop(name, None)
        if br is not None:
            for p in list(br.ports):
                br.del_port(p)

    def br(self, name: str) -> OvsBridge:
        return self.bridges[name]
