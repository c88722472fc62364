"""P4Runtime-style table store for the linux-networking pipeline, compiled onto the GPU tables.

Reference: the Intel IPU VSP programs the FXP pipeline through `p4rt-ctl add-entry/del-entry br0
<table> <match,...,action=ctrl.act(args)>` (vendor/.../p4rtclient/p4rtclient.go:74-1155, SURVEY
V11/NAT11, kernels K1-K9).  `P4Runtime` accepts exactly those entry strings, validates them
against a P4Info (tables, match kinds, bit widths, action params, table sizes), keeps the entries
(INSERT of an existing key -> ALREADY_EXISTS, DELETE of a missing key -> NOT_FOUND, full table ->
RESOURCE_EXHAUSTED — the error vocabulary the VSP's retry logic keys on) and compiles the whole
entry set onto the MI355X data plane:

  K1 tx_source_port / rx_source_port      port -> source port (classification state)
  K2 tx_acc_vsi                           port default output, bridge bypassed
  K3 vsi_to_vsi_loopback                  (port bridge, MAC of the target VSI) -> port entries
  K4 source_port_to_pr_map                source port -> port-representor default output
  K5 l2_fwd_rx_table / l2_fwd_tx_table / sem_bypass   (bridge, dst MAC) -> port entries
  K6 handle_tx_* / vlan_push/pop_mod      per-source VLAN push (PORT_INGRESS_TAG), pop on the way
                                          back via (vid bridge, MAC) entries
  K7 source_port_to_bridge_map            port bridge id (vid-keyed entries: bridge = vid)
  K8 tx_lag_table                         LAG member table, hash[2:0]-indexed (PORT_LAG)
  K9 mir_prof + mirror_and_send           PORT_MIRROR with the profile's destination vport
A VSI is the second byte of its MAC and its vport is vsi + 16 (ipu-plugin utils.go:76-107); data-
plane port number == vport.  Physical ports 0..3 are data-plane ports PHY_BASE + n.
"""
from __future__ import annotations

import ipaddress
import re
import threading

import numpy as np
from dataclasses import dataclass, field

from . import tables as T
from .p4info import MI355X_P4INFO, P4Info

VSI_TO_VPORT = 16
PHY_BASE = 4000
TUNNEL_PORT_BASE = 3800      # data-plane ports of P4 tunnels (encap by destination, decap by tunnel_id)
STEER_BRIDGE_BASE = 0xF000   # per-port private bridges (bypass / loopback domains)


class P4Error(Exception):
    def __init__(self, code: str, msg: str):
        super().__init__(f"{code}: {msg}")
        self.code = code


# Actions of the reference's p4info whose semantics cannot be pinned from it (docs/DATAPLANE.md
# "L3 and tunnels"): refused at write time with UNIMPLEMENTED.
UNSUPPORTED_ACTIONS = {
    "tx_ipsec_tunnel_v6": "IPsec tunnels over an IPv6 underlay are not supported "
                          "(the p4info carries 80 of the 128 outer-destination bits)",
}


def vport_for_vsi(vsi: int) -> int:
    return vsi + VSI_TO_VPORT


def vsi_of_mac(mac: str | bytes) -> int:
    b = bytes.fromhex(mac.replace(":", "")) if isinstance(mac, str) else bytes(mac)
    return b[1]


_MAC_RE = re.compile(r"^[0-9a-fA-F]{2}(:[0-9a-fA-F]{2}){5}$")


def _int(v: str) -> int:
    v = v.strip()
    if v.count(".") == 3 and ":" not in v:      # dotted IPv4
        return int(ipaddress.IPv4Address(v))
    if _MAC_RE.match(v):                        # MAC
        return int(v.replace(":", ""), 16)
    if ":" in v:                                # IPv6 (incl. "::" forms)
        return int(ipaddress.IPv6Address(v))
    return int(v, 16) if v.lower().startswith("0x") else int(v)


@dataclass
class Entry:
    table: str
    key: tuple                  # ((field, value, mask), ...) in P4Info field order
    priority: int = 0
    action: str = ""
    params: dict = field(default_factory=dict)

    def text(self) -> str:
        parts = []
        for f, v, m in self.key:
            full = (1 << 64) - 1
            parts.append(f"{f}={v:#x}" + (f"/{m:#x}" if m != full and m is not None else ""))
        if self.priority:
            parts.append(f"priority={self.priority}")
        args = ",".join(f"{k}={v}" for k, v in self.params.items())
        parts.append(f"action={self.action}({args})")
        return ",".join(parts)


class P4Runtime:
    def __init__(self, dataplane=None, p4info: P4Info = MI355X_P4INFO, lag_ports: dict[int, int] | None = None):
        self.dp = dataplane
        self.p4info = p4info
        self.entries: dict[str, dict[tuple, Entry]] = {}
        self.lag_ports = dict(lag_ports or {})  # LAG group -> data-plane port that fronts it
        self._owned_ports: set[int] = set()
        self._owned_macs: list[tuple[int, str]] = []
        self._owned_routes: list[str] = []
        self._owned_nh: set[int] = set()
        self._owned_tunnels = False
        self._lock = threading.RLock()
        self.stats = {"writes": 0, "compiles": 0}

    # ------------------------------------------------------------------ parsing
    def _table(self, name: str):
        try:
            return self.p4info.table(name)
        except KeyError:
            raise P4Error("NOT_FOUND", f"table {name} not in the loaded pipeline") from None

    def parse(self, table: str, spec: str, need_action: bool = True) -> Entry:
        t = self._table(table)
        spec = spec.strip()
        action, args = "", ""
        m = re.search(r"(?:^|,)action=([\w.]+)(?:\((.*)\))?\s*$", spec)
        if m:
            action, args = m.group(1), m.group(2) or ""
            spec = spec[: m.start()]
        elif need_action:
            raise P4Error("INVALID_ARGUMENT", "entry has no action")
        given: dict[str, list[tuple[int, int | None]]] = {}
        priority = 0
        for tok in filter(None, (x.strip() for x in spec.split(","))):
            k, eq, v = tok.partition("=")
            if not eq:
                raise P4Error("INVALID_ARGUMENT", f"bad match token {tok!r}")
            if k == "priority":
                priority = _int(v)
                continue
            val, _, mask = v.partition("/")
            try:
                given.setdefault(k, []).append((_int(val), _int(mask) if mask else None))
            except ValueError:
                raise P4Error("INVALID_ARGUMENT", f"bad value in {tok!r}") from None
        key = []
        ternary = False
        for mf in t.match_fields:
            if not given.get(mf.name):
                raise P4Error("INVALID_ARGUMENT", f"missing match field {mf.name} for {t.name}")
            v, msk = given[mf.name].pop(0)  # repeated field names bind in order
            if not given[mf.name]:
                del given[mf.name]
            full = (1 << mf.bitwidth) - 1
            if v < 0 or v > full:
                raise P4Error("INVALID_ARGUMENT", f"{mf.name}={v} exceeds {mf.bitwidth} bits")
            if mf.match_type == "EXACT":
                if msk is not None and msk != full:
                    raise P4Error("INVALID_ARGUMENT", f"{mf.name} is an exact match; no mask allowed")
                msk = full
            elif mf.match_type == "LPM":       # value/prefix-length
                plen = mf.bitwidth if msk is None else msk
                if not 0 <= plen <= mf.bitwidth:
                    raise P4Error("INVALID_ARGUMENT", f"prefix length of {mf.name} out of range")
                msk = (full << (mf.bitwidth - plen)) & full
                v &= msk
            else:
                ternary = True
                msk = full if msk is None else msk
                if msk > full:
                    raise P4Error("INVALID_ARGUMENT", f"mask of {mf.name} exceeds {mf.bitwidth} bits")
                v &= msk
            key.append((mf.name, v, msk))
        if given:
            raise P4Error("INVALID_ARGUMENT", f"unknown match field(s) {sorted(given)} for {t.name}")
        if ternary and need_action and priority <= 0:
            raise P4Error("INVALID_ARGUMENT", f"ternary table {t.name} needs priority > 0")
        params: dict[str, int] = {}
        if action:
            try:
                a = self.p4info.action(action)
            except KeyError:
                raise P4Error("INVALID_ARGUMENT", f"unknown action {action}") from None
            if a.id not in t.action_ids:
                raise P4Error("INVALID_ARGUMENT", f"action {a.name} not allowed in {t.name}")
            vals = [x.strip() for x in args.split(",")] if args.strip() else []
            named = [x for x in vals if "=" in x]
            if named and len(named) != len(vals):
                raise P4Error("INVALID_ARGUMENT", "mixing positional and named action arguments")
            if named:
                for x in named:
                    k, _, v = x.partition("=")
                    p = next((p for p in a.params if p.name == k), None)
                    if p is None:
                        raise P4Error("INVALID_ARGUMENT", f"action {a.name} has no parameter {k}")
                    params[k] = _int(v)
            else:
                if len(vals) != len(a.params):
                    raise P4Error("INVALID_ARGUMENT", f"action {a.name} takes {len(a.params)} arguments, got {len(vals)}")
                params = {p.name: _int(v) for p, v in zip(a.params, vals)}
            for p in a.params:
                if p.name in params and params[p.name] >= (1 << p.bitwidth):
                    raise P4Error("INVALID_ARGUMENT", f"{p.name}={params[p.name]} exceeds {p.bitwidth} bits")
            action = a.name
        return Entry(t.name, tuple(key), priority, action, params)

    # ------------------------------------------------------------------ writes
    def add_entry(self, table: str, spec: str) -> Entry:
        with self._lock:
            e = self.parse(table, spec)
            tab = self.entries.setdefault(e.table, {})
            k = (e.key, e.priority)
            if k in tab:
                raise P4Error("ALREADY_EXISTS", f"entry already exists in {e.table}")
            if len(tab) >= self._table(e.table).size:
                raise P4Error("RESOURCE_EXHAUSTED", f"table {e.table} is full ({self._table(e.table).size})")
            if e.action and e.action.rsplit(".", 1)[-1] in UNSUPPORTED_ACTIONS:
                # refused before it is stored: a stored entry would make every later compile fail
                raise P4Error("UNIMPLEMENTED", UNSUPPORTED_ACTIONS[e.action.rsplit(".", 1)[-1]])
            tab[k] = e
            self.stats["writes"] += 1
            try:
                self.compile()
            except Exception:
                # transactional write: the entry that made the compile fail is taken back out and
                # the previous table state recompiled, so the runtime never stays stuck
                del tab[k]
                self.compile()
                raise
            return e

    def del_entry(self, table: str, spec: str) -> None:
        with self._lock:
            e = self.parse(table, spec, need_action=False)
            tab = self.entries.get(e.table, {})
            k = (e.key, e.priority)
            if k not in tab:
                raise P4Error("NOT_FOUND", f"no such entry in {e.table}")
            del tab[k]
            self.stats["writes"] += 1
            try:
                self.compile()
            except Exception:
                tab[k] = e
                self.compile()
                raise

    def get_entries(self, table: str | None = None) -> list[Entry]:
        with self._lock:
            if table is not None:
                return list(self.entries.get(self._table(table).name, {}).values())
            return [e for t in self.entries.values() for e in t.values()]

    def set_pipe(self, p4info: P4Info) -> None:
        with self._lock:
            self.p4info = p4info
            self.entries.clear()
            self.compile()

    # ------------------------------------------------------------------ compile
    def _rows(self, short: str) -> list[Entry]:
        name = short if "." in short else "linux_networking_control." + short
        rows = list(self.entries.get(name, {}).values())
        return sorted(rows, key=lambda e: -e.priority)

    @staticmethod
    def _k(e: Entry, i: int) -> tuple[int, int]:
        return e.key[i][1], e.key[i][2]

    def compile(self) -> None:
        """Recompute every P4-derived port attribute, MAC entry and LAG group (idempotent)."""
        if self.dp is None:
            return
        dp = self.dp
        self.stats["compiles"] += 1
        for bid, mac in self._owned_macs:
            dp.macs.remove(bid, mac)
        self._owned_macs = []
        keep = {"flags", "vlan", "mac_lo", "mac_hi", "gpu", "peer_mac_lo", "peer_mac_hi"}
        for p in self._owned_ports:
            f = int(dp.ports.a[p]["flags"]) & ~(T.PORT_HAS_DEFAULT | T.PORT_INGRESS_TAG | T.PORT_MIRROR | T.PORT_LAG |
                                                 T.PORT_VLAN_BRIDGE | T.PORT_VSI_LOOKUP)
            row = {k: dp.ports.a[p][k] for k in keep}
            dp.ports.a[p] = np.zeros((), T.PORT_DTYPE)
            for k, v in row.items():
                dp.ports.a[p][k] = v
            dp.ports.a[p]["flags"] = f
        dp.ports.version += 1
        owned: set[int] = set()

        def port(p: int) -> int:
            if 0 <= p < VSI_TO_VPORT:   # action port numbers below 16 name physical ports
                p = PHY_BASE + p
            if not 0 <= p < T.MAX_PORT_ID:
                raise P4Error("INVALID_ARGUMENT", f"port {p} outside the data plane")
            if not dp.ports.valid(p):
                dp.ports.set(p, flags=T.PORT_VALID)
            owned.add(p)
            return p

        def add_mac(bridge: int, mac: str, out: int) -> None:
            dp.macs.insert(bridge, mac, out)
            self._owned_macs.append((bridge, mac))

        # K1: source ports (a ternary VSI match applies to every VSI the pipeline references)
        src: dict[int, int] = {}
        known_vsis = {e.key[0][1] for t in ("tx_acc_vsi", "vsi_to_vsi_loopback", "handle_tx_from_host_to_ovs_and_ovs_to_wire_table",
                                          "handle_rx_loopback_from_host_to_ovs_table") for e in self._rows(t)}
        known_vsis |= {e.key[1][1] for e in self._rows("vsi_to_vsi_loopback")}
        for e in reversed(self._rows("tx_source_port")):  # lowest priority first, higher overrides
            v, m = self._k(e, 0)
            targets = [v] if m == 0x7FF else sorted(x for x in known_vsis if (x & m) == v)
            for vsi in targets:
                src[port(vport_for_vsi(vsi))] = e.params["source_port"]
        for e in self._rows("rx_source_port"):
            src[port(PHY_BASE + self._k(e, 0)[0])] = e.params["source_port"]
        # K7: bridge ids (highest priority wins per port)
        bridge: dict[int, int] = {}
        vlan_bridge: set[int] = set()
        for e in self._rows("source_port_to_bridge_map"):
            (sv, sm), (vv, vm) = self._k(e, 0), self._k(e, 1)
            for p, sp in src.items():
                if (sp & sm) == sv and p not in bridge:
                    if vm == 0 or vv == 0:   # wildcard or untagged-only
                        bridge[p] = e.params["bridge_id"]
                    else:
                        if vm != 0xFFF or vv != e.params["bridge_id"]:
                            raise P4Error("INVALID_ARGUMENT",
                                          "vid-keyed bridge mapping is supported as bridge_id == vid only")
                        vlan_bridge.add(p)
        for p, b in bridge.items():
            dp.ports.update(p, bridge_id=b)
        for p in vlan_bridge:
            dp.ports.a[p]["flags"] |= T.PORT_VLAN_BRIDGE
        # K4: source port -> port representor
        pr: dict[int, int] = {e.key[0][1]: e.params["port"] for e in self._rows("source_port_to_pr_map")
                              if e.action.endswith("fwd_to_vsi")}
        for p, sp in src.items():
            if sp in pr:
                dp.ports.update(p, default_out=port(pr[sp]))
        # K9 profiles + rx_phy_port_to_pr_map
        # mir_prof vport_id is a VSI when store_vsi=1 (p4rtclient.go:1033-1037)
        prof = {e.key[0][1]: (vport_for_vsi(e.params.get("vport_id", 0)) if e.params.get("store_vsi", 0)
                              else e.params.get("vport_id", 0)) for e in self._rows("mir_prof")}
        for e in self._rows("rx_phy_port_to_pr_map"):
            p = port(PHY_BASE + e.key[0][1])
            dp.ports.update(p, default_out=port(e.params["port"]))
            if e.action.endswith("mirror_and_send"):
                sess = e.params["mirror_session_id"]
                if sess not in prof:
                    raise P4Error("FAILED_PRECONDITION", f"mirror session {sess} has no mir_prof entry")
                dp.ports.set_mirror(p, port(prof[sess]))
        # K6: host <-> OvS VLAN handling (needs the vlan_push/pop mod blobs)
        push_ok = {e.key[0][1] for e in self._rows("vlan_push_mod_table")}
        pop_ok = {e.key[0][1] for e in self._rows("vlan_pop_mod_table")}
        for e in self._rows("handle_tx_from_host_to_ovs_and_ovs_to_wire_table"):
            p = port(vport_for_vsi(e.key[0][1]))
            if e.action.endswith("add_vlan_and_send_to_port"):
                dp.ports.update(p, default_out=port(e.params["port_id"]))
                if e.params["vlan_id"] in push_ok:
                    dp.ports.set_ingress_tag(p, e.params["vlan_id"])
            else:
                dp.ports.update(p, default_out=port(e.params["port_id"]))
        for e in self._rows("handle_rx_loopback_from_host_to_ovs_table"):
            p = port(vport_for_vsi(e.key[0][1]))
            if not dp.ports.a[p]["flags"] & T.PORT_HAS_DEFAULT:
                dp.ports.update(p, default_out=port(e.params["port_id"]))
        for e in self._rows("handle_tx_from_ovs_to_host_table"):
            mux = port(vport_for_vsi(e.key[0][1]))
            vid = e.key[1][1]
            dp.ports.a[mux]["flags"] |= T.PORT_VLAN_BRIDGE | T.PORT_VSI_LOOKUP
            out = port(e.params["port_id"])
            if e.params["vlan_id"] in pop_ok:
                add_mac(vid, vsi_mac(out - VSI_TO_VPORT), out)  # tag popped at ingress parse
        # K2: ACC bypass (overrides the PR map), on a private empty bridge
        for e in self._rows("tx_acc_vsi"):
            p = port(vport_for_vsi(e.key[0][1]))
            dp.ports.update(p, default_out=port(e.params["port"]), bridge_id=STEER_BRIDGE_BASE + p % 0x0FFF)
        # K3: VSI to VSI loopback: the source port looks up (its bridge, target VSI)
        for e in self._rows("vsi_to_vsi_loopback"):
            a, b = e.key[0][1], e.key[1][1]
            p = port(vport_for_vsi(a))
            if int(dp.ports.a[p]["bridge_id"]) == 0:
                dp.ports.update(p, bridge_id=STEER_BRIDGE_BASE + p % 0x0FFF)
            dp.ports.a[p]["flags"] |= T.PORT_VSI_LOOKUP
            add_mac(int(dp.ports.a[p]["bridge_id"]), vsi_mac(b), port(e.params["port"]))
        # K5: L2 forwarding
        for e in self._rows("l2_fwd_rx_table"):
            add_mac(e.key[0][1], _mac(e.key[1][1]), port(e.params["port"]))
        for e in self._rows("l2_fwd_tx_table"):
            add_mac(0, _mac(e.key[0][1]), port(e.params["port"]))
        for e in self._rows("sem_bypass"):
            add_mac(0, _mac(e.key[0][1]), port(e.params["port_id"]))
        # K8: LAG
        for grp, lag_port in self.lag_ports.items():
            members = [T.PORT_NONE] * T.LAG_WAYS
            any_member = False
            for h in range(T.LAG_WAYS):
                for e in self._rows("tx_lag_table"):
                    (gv, gm), (hv, hm) = self._k(e, 0), self._k(e, 1)
                    if (grp & gm) == gv and (h & hm) == hv:
                        if e.action.endswith("set_egress_port"):
                            members[h] = port(e.params["egress_port"])
                            any_member = True
                        break
            p = port(lag_port)
            if any_member:
                for h, mport in enumerate(members):
                    dp.lag.set_slot(grp, h, mport)
                dp.ports.set_lag(p, grp)
            else:
                dp.ports.set_lag(p, None)
        self._compile_l3_tunnels(dp, port, add_mac, src)
        self._compile_ipsec(dp)
        self._owned_ports = owned
        dp.ports.version += 1

    def _compile_ipsec(self, dp) -> None:
        """IPsec tables onto the ESP engine (dataplane/ipsec.py): ipsec_spd (protect with SA saidx /
        bypass), ipsec_tx_sa_classification_table (transport, or tunnel to dst_addr; drop),
        ipsec_tunnel_table + ipsec_tunnel_encap_mod_table (an SA's tunnel outer addresses),
        ipsec_rx_sa_classification_table (inbound (src, dst, SPI) -> SA) and
        ipv4_ipsec_tunnel_term_table (inbound SAs of those (src, dst) decapsulate a tunnel).  The SA
        key material itself comes from the IPsec control plane (`dp.ipsec.add_sa`), as the IPU's
        crypto SAD does; SA modes are applied to SAs that exist."""
        names = ("ipsec_spd", "ipsec_tx_sa_classification_table", "ipsec_tunnel_table", "ipsec_tunnel_encap_mod_table",
                 "ipv4_ipsec_tunnel_term_table", "MainControlDecrypt.ipsec_rx_sa_classification_table")
        rows = {n: self._rows(n) for n in names}
        if not any(rows.values()) and not getattr(self, "_owned_ipsec", False):
            return
        eng = dp.ipsec
        # Everything is validated and computed into locals first; the engine's rule sets are
        # swapped only once the whole compile succeeded (a half-applied SPD would let the kernel
        # protect traffic with a stale SPD while the host hands out sequence number 0).
        drops = set()
        modes: dict[tuple[int, int], tuple[int, int | None]] = {}
        for e in rows["ipsec_tx_sa_classification_table"]:
            d, p = e.key[0][1], e.key[1][1]
            if e.action.endswith("tx_ipsec_tunnel_v6"):
                raise P4Error("UNIMPLEMENTED", UNSUPPORTED_ACTIONS["tx_ipsec_tunnel_v6"])
            if e.action.endswith("drop"):
                drops.add((d, p))
            elif e.action.endswith("tx_ipsec_tunnel"):
                modes[(d, p)] = (2, e.params["dst_addr"])
            elif e.action.endswith(("tx_ipsec_transport", "tx_ipsec_transport_with_underlay")):
                modes[(d, p)] = (1, None)
        tun_of = {e.key[0][1]: e.params["tunnel_id"] for e in rows["ipsec_tunnel_table"] if e.action.endswith("set_ipsec_tunnel")}
        encap = {e.key[0][1]: e.params for e in rows["ipsec_tunnel_encap_mod_table"] if e.action.endswith("ipsec_tunnel_encap_mod")}
        from . import ipsec as I

        raw = lambda v: str(ipaddress.IPv4Address(v))  # noqa: E731
        spd: dict = {}
        sa_modes: list[tuple] = []
        for e in rows["ipsec_spd"]:
            d, p = e.key[0][1], e.key[1][1]
            if (d, p) in drops:
                spd[(raw(d), p)] = (I.DROP, 0)
            elif e.action.endswith("ipsec_protect_set_metadata"):
                sa = e.params["saidx"]
                spd[(raw(d), p)] = (I.PROTECT, sa)
                m = modes.get((d, p))
                if sa in eng.sa_info and m is not None:
                    if m[0] == 2:
                        enc = encap.get(tun_of.get(sa, -1), {})
                        sa_modes.append((sa, I.TUNNEL, raw(enc["ipsec_src_addr"]) if enc else None,
                                         raw(enc.get("ipsec_dst_addr", m[1])) if enc else raw(m[1])))
                    else:
                        sa_modes.append((sa, I.TRANSPORT, None, None))
            elif e.action.endswith("ipsec_bypass"):
                spd[(raw(d), p)] = (I.BYPASS, 0)
        terms = {(e.key[0][1], e.key[1][1]) for e in rows["ipv4_ipsec_tunnel_term_table"]}
        rx: dict = {}
        for e in rows["MainControlDecrypt.ipsec_rx_sa_classification_table"]:
            if not e.action.endswith("ipsec_decrypt"):
                continue
            s_, d_, spi = e.key[0][1], e.key[1][1], e.key[2][1]
            sa = e.params["saidx"]
            rx[(raw(s_), raw(d_), spi)] = sa
            if sa in eng.sa_info:
                sa_modes.append((sa, I.TUNNEL if (s_, d_) in terms else I.TRANSPORT, None, None))
        eng.replace_rules(spd, rx, sa_modes)
        self._owned_ipsec = any(rows.values())

    def _compile_tunnels_v6(self, dp, port, add_mac, bridges, mac_of) -> bool:
        """IPv6-underlay tunnels: l2_to_tunnel_v6 + {vxlan,geneve}_encap_v6[_vlan_pop]_mod_table onto
        PORT_TUNNEL6 ports (tunnels6), ipv6_tunnel_term_table + rx_ipv6_tunnel_source_port onto the
        local IPv6 VTEP (kernel recognition) and the host termination table (terms6)."""
        encap: dict[int, tuple[int, Entry]] = {}
        for kind, tab in ((T.TUN_VXLAN, "vxlan_encap_v6_mod_table"), (T.TUN_VXLAN, "vxlan_encap_v6_vlan_pop_mod_table"),
                          (T.TUN_GENEVE, "geneve_encap_v6_mod_table"), (T.TUN_GENEVE, "geneve_encap_v6_vlan_pop_mod_table")):
            for e in self._rows(tab):
                if e.params:
                    encap[e.params["dst_addr"]] = (kind, e)
        tunnels = [e for e in self._rows("l2_to_tunnel_v6") if e.action.endswith("set_tunnel_v6")]

        def dst_of(e: Entry) -> int:
            p = e.params
            return (p["ipv6_1"] << 96) | (p["ipv6_2"] << 64) | (p["ipv6_3"] << 32) | p["ipv6_4"]

        dsts = sorted({dst_of(e) for e in tunnels})
        if len(dsts) > 64:
            raise P4Error("RESOURCE_EXHAUSTED", "at most 64 IPv6-underlay tunnel destinations")
        terms = [e for e in self._rows("ipv6_tunnel_term_table") if "decap" in e.action]
        if not (tunnels or terms or self._owned_tunnels):
            return False            # tunnels6 / terms6 / vtep6 set outside P4Runtime stay as they are
        dp.tunnels6.n = 0
        dp.tunnels6.version += 1
        for k, d in enumerate(dsts):
            if d not in encap:
                raise P4Error("FAILED_PRECONDITION", f"tunnel to {ipaddress.IPv6Address(d)} has no v6 encap mod entry")
            kind, me = encap[d]
            tp = port(TUNNEL_PORT_BASE + 64 + k)
            r = dp.routes6.lookup(d) if len(dp.routes6) else 0
            nh = (r & 0xFFFF) if r & T.ROUTE_NH else None
            raw = lambda x: ":".join(f"{(x >> (8 * b)) & 0xFF:02x}" for b in range(6))  # noqa: E731
            if nh is not None and dp.nexthops.a[nh]["valid"]:
                n = dp.nexthops.a[nh]
                out = int(n["port"])
                dmac_s = raw(int(n["dmac_lo"]) | int(n["dmac_hi"]) << 32)
                smac_s = raw(int(n["smac_lo"]) | int(n["smac_hi"]) << 32)
            else:
                out, dmac_s, smac_s = port(PHY_BASE), "ff:ff:ff:ff:ff:ff", mac_of(0)
            p = me.params
            dp.tunnels6.set(k, src=p["src_addr"], dst=d, vni=p["vni"], out_port=out, smac=smac_s, dmac=dmac_s,
                            kind=kind, dport=p["dst_port"] or None, sport=p["src_port"],
                            traffic_class=(p["ds"] << 2) | p["ecn"], flow_label=p["flow_label"],
                            hop_limit=p["hop_limit"] or 64)
            dp.ports.a[tp]["flags"] |= T.PORT_VALID | T.PORT_TUNNEL | T.PORT_TUNNEL6
            dp.ports.a[tp]["lag"] = k
            for ent in tunnels:
                if dst_of(ent) == d:
                    for b in bridges:
                        add_mac(b, _mac(ent.key[0][1]), tp)
        # termination: recognised by the kernel against the local IPv6 VTEP, finished on the host
        dp.terms6.clear()
        sp_of = {(e.key[0][1], e.key[1][1]): e.params["source_port"] for e in self._rows("rx_ipv6_tunnel_source_port")
                 if e.action.endswith("set_source_port")}
        bm = {e2.key[0][1]: e2.params["bridge_id"] for e2 in self._rows("source_port_to_bridge_map")
              if e2.key[0][2] == 0xFFFF and e2.action.endswith("set_bridge_id")}
        for e in terms:
            s6, vni = e.key[0][1], e.key[1][1]
            tp = port(TUNNEL_PORT_BASE + 128 + (e.params["tunnel_id"] & 0x7F))
            dp.ports.a[tp]["flags"] |= T.PORT_VALID
            dp.terms6.insert(s6, vni, tp)
            if e.action.endswith("_and_push_vlan"):
                tab = "geneve_decap_and_push_vlan_mod_table" if "geneve" in e.action else "vxlan_decap_and_push_vlan_mod_table"
                me = next((m for m in self._rows(tab) if m.key[0][1] == e.params["tunnel_id"] and m.params), None)
                if me is None:
                    raise P4Error("FAILED_PRECONDITION", f"{e.action} for tunnel {e.params['tunnel_id']} has no {tab} entry")
                dp.ports.a[tp]["flags"] |= T.PORT_INGRESS_TAG
                dp.ports.a[tp]["ext"] = (int(dp.ports.a[tp]["ext"]) & ~0xFFF) | (me.params["vlan_id"] & 0xFFF)
            if sp_of.get((s6, vni)) in bm:
                dp.ports.update(tp, bridge_id=bm[sp_of[(s6, vni)]])
        local6 = {e.params["src_addr"] for _, e in encap.values()}
        if terms and local6:
            dp.vtep6.set(min(local6))
            for k in range(4):
                dp.ports.a[port(PHY_BASE + k)]["flags"] |= T.PORT_VTEP
        elif dp.vtep6.active:
            dp.vtep6.clear()
        return bool(tunnels or terms)

    def _compile_l3_tunnels(self, dp, port, add_mac, src: dict) -> None:
        """L3 (ipv4_table, ipv6_table, ecmp_hash_table, nexthop / ecmp_nexthop tables, rif_mod_table_*), tunnels
        (l2_to_tunnel_v4, *_encap_mod_table, ipv4_tunnel_term_table, rx_ipv4_tunnel_source_port),
        vm_{src,dst}_ip4_mac_map_table, rx_lag_table, l2_fwd_smac_table and always_trap_arp_table onto
        the GPU tables."""
        for cidr in self._owned_routes:
            (dp.routes6 if ":" in cidr else dp.routes).remove(cidr)
        self._owned_routes = []
        for nh in self._owned_nh:
            dp.nexthops.clear(nh)
        self._owned_nh = set()
        # router-interface MACs: start | mid | last 16-bit parts
        rif: dict[int, list[int]] = {}
        for i, part in enumerate(("start", "mid", "last")):
            for e in self._rows(f"rif_mod_table_{part}"):
                if e.action.endswith(f"set_src_mac_{part}"):
                    rif.setdefault(e.key[0][1], [0, 0, 0])[i] = e.params["arg"]

        def mac_of(v: int) -> str:
            return ":".join(f"{(v >> (8 * (5 - k))) & 0xFF:02x}" for k in range(6))

        def rif_mac(r: int) -> str:
            a = rif.get(r, [0, 0, 0])
            return mac_of((a[0] << 32) | (a[1] << 16) | a[2])

        def nexthop(nh: int, e: Entry) -> None:
            dmac = mac_of((e.params["dmac_high"] << 32) | e.params["dmac_low"])
            if e.action.endswith("set_nexthop_lag"):
                lagp = self.lag_ports.get(e.params["lag_group_id"])
                if lagp is None:
                    raise P4Error("FAILED_PRECONDITION", f"LAG group {e.params['lag_group_id']} has no port")
                dp.nexthops.set(nh, port(lagp), dmac=dmac, smac=mac_of(0))
            else:
                dp.nexthops.set(nh, port(e.params["egress_port"]), dmac=dmac, smac=rif_mac(e.params["router_interface_id"]))
            self._owned_nh.add(nh)

        for e in self._rows("ecmp_nexthop_table"):
            if e.action.endswith("ecmp_set_nexthop_info_dmac"):
                v, m = self._k(e, 0)
                for nh in ([v] if m == 0xFFFF else [x for x in range(dp.nexthops.a.shape[0]) if (x & m) == v]):
                    nexthop(nh, e)
        for e in self._rows("nexthop_table"):
            if e.action.endswith(("set_nexthop_info_dmac", "set_nexthop_lag")):
                nexthop(e.key[0][1], e)
        groups = set()
        for e in self._rows("ipv4_table"):
            net, msk = self._k(e, 1)
            plen = bin(msk).count("1")
            cidr = f"{ipaddress.IPv4Address(net)}/{plen}"
            if e.action.endswith("ipv4_set_nexthop_id"):
                dp.routes.add(cidr, nexthop=e.params["nexthop_id"])
            elif e.action.endswith("ecmp_hash_action"):
                dp.routes.add(cidr, ecmp_group=e.params["ecmp_group_id"])
                groups.add(e.params["ecmp_group_id"])
            else:
                continue
            self._owned_routes.append(cidr)
        for e in self._rows("ipv6_table"):
            net, msk = self._k(e, 1)
            plen = bin(msk).count("1")
            cidr = f"{ipaddress.IPv6Address(net)}/{plen}"
            if e.action.endswith("ipv6_set_nexthop_id"):
                dp.routes6.add(cidr, nexthop=e.params["nexthop_id"])
            elif e.action.endswith("ecmp_v6_hash_action"):
                dp.routes6.add(cidr, ecmp_group=e.params["ecmp_group_id"])
                groups.add(e.params["ecmp_group_id"])
            else:
                continue
            self._owned_routes.append(cidr)
        # VM IPv4 -> MAC maps: overrides applied to routed IPv4 after the nexthop's MACs
        vm_rows = [(kind, e) for kind, tab in ((T.VMMAC_SRC, "vm_src_ip4_mac_map"), (T.VMMAC_DST, "vm_dst_ip4_mac_map"))
                   for e in self._rows(f"{tab}_table") if e.action.endswith(f"{tab}_action")]
        if vm_rows or getattr(self, "_owned_vmmac", False):
            dp.vmmac.clear()
            for kind, e in vm_rows:
                x = "smac" if kind == T.VMMAC_SRC else "dmac"
                v = (e.params[f"{x}_high"] << 32) | (e.params[f"{x}_mid"] << 16) | e.params[f"{x}_low"]
                dp.vmmac.set(str(ipaddress.IPv4Address(e.key[0][1])), kind, mac_of(v))
        self._owned_vmmac = bool(vm_rows)
        for g in groups:
            for h in range(T.ECMP_WAYS):
                for e in self._rows("ecmp_hash_table"):  # highest priority first
                    (fv, fm), (hv, hm) = self._k(e, 0), self._k(e, 1)
                    if (g & fm) == fv and (h & hm) == hv:
                        if e.action.endswith("set_nexthop_id"):
                            dp.ecmp.set_slot(g, h, e.params["nexthop_id"])
                        break
        # tunnels: one tunnel port per destination VTEP; parameters from the encap mod tables
        encap: dict[int, tuple[int, Entry]] = {}
        for kind, tab in ((T.TUN_VXLAN, "vxlan_encap_mod_table"), (T.TUN_VXLAN, "vxlan_encap_vlan_pop_mod_table"),
                          (T.TUN_GENEVE, "geneve_encap_mod_table"), (T.TUN_GENEVE, "geneve_encap_vlan_pop_mod_table")):
            for e in self._rows(tab):
                if e.params:
                    encap[e.params["dst_addr"]] = (kind, e)
        tunnels = [e for e in self._rows("l2_to_tunnel_v4") if e.action.endswith("set_tunnel_v4")]
        local_vteps = {e.params["src_addr"] for _, e in encap.values()}
        bridges = {int(dp.ports.a[p]["bridge_id"]) for p in src} | {0}
        v4_dsts = sorted({e.params["dst_addr"] for e in tunnels})
        if len(v4_dsts) > 64:
            raise P4Error("RESOURCE_EXHAUSTED", "at most 64 IPv4-underlay tunnel destinations")
        for k, e in enumerate(v4_dsts):
            if e not in encap:
                raise P4Error("FAILED_PRECONDITION", f"tunnel to {ipaddress.IPv4Address(e)} has no encap mod entry")
            kind, me = encap[e]
            tp = port(TUNNEL_PORT_BASE + k)
            # underlay: routed like any IPv4 destination, else the first physical port
            r = dp.routes.lookup(e)
            nh = (r & 0xFFFF) if r & T.ROUTE_NH else None
            if nh is not None and dp.nexthops.a[nh]["valid"]:
                n = dp.nexthops.a[nh]
                out, dmac, smac = int(n["port"]), int(n["dmac_lo"]) | int(n["dmac_hi"]) << 32, int(n["smac_lo"]) | int(n["smac_hi"]) << 32
                raw = lambda x: ":".join(f"{(x >> (8 * b)) & 0xFF:02x}" for b in range(6))  # noqa: E731
                dmac_s, smac_s = raw(dmac), raw(smac)
            else:
                out, dmac_s, smac_s = port(PHY_BASE), "ff:ff:ff:ff:ff:ff", mac_of(0)
            dp.tunnels.set(k, src=me.params["src_addr"], dst=e, vni=me.params["vni"], out_port=out, smac=smac_s,
                           dmac=dmac_s, kind=kind, dport=me.params["dst_port"] or None, sport=me.params["src_port"])
            dp.ports.a[tp]["flags"] |= T.PORT_TUNNEL
            dp.ports.a[tp]["lag"] = k
            for ent in tunnels:
                if ent.params["dst_addr"] == e:
                    for b in bridges:
                        add_mac(b, _mac(ent.key[0][1]), tp)
        # termination: (outer src, vni) -> the tunnel_id's port, which is a source port
        sp_of = {(e.key[0][1], e.key[1][1]): e.params["source_port"] for e in self._rows("rx_ipv4_tunnel_source_port")
                 if e.action.endswith("set_source_port")}
        terms = [e for e in self._rows("ipv4_tunnel_term_table") if "decap" in e.action]
        if terms or self._owned_tunnels:
            dp.terms.a[:] = np.zeros((), T.TERM_DTYPE)
            dp.terms.n = 0
            dp.terms.version += 1
        for e in terms:
            s_ip, vni = e.key[0][1], e.key[1][1]
            tp = port(TUNNEL_PORT_BASE + 128 + (e.params["tunnel_id"] & 0x7F))
            dp.terms.insert(str(ipaddress.IPv4Address(s_ip)), vni, tp)
            if e.action.endswith("_and_push_vlan"):
                # decap + push VLAN (vxlan/geneve_decap_and_push_vlan_mod_table, blob = tunnel_id):
                # the inner frame leaves the termination port with that vid pushed (K6 semantics)
                tab = "geneve_decap_and_push_vlan_mod_table" if "geneve" in e.action else "vxlan_decap_and_push_vlan_mod_table"
                me = next((m for m in self._rows(tab) if m.key[0][1] == e.params["tunnel_id"] and m.params), None)
                if me is None:
                    raise P4Error("FAILED_PRECONDITION", f"{e.action} for tunnel {e.params['tunnel_id']} has no {tab} entry")
                dp.ports.a[tp]["flags"] |= T.PORT_INGRESS_TAG
                dp.ports.a[tp]["ext"] = (int(dp.ports.a[tp]["ext"]) & ~0xFFF) | (me.params["vlan_id"] & 0xFFF)
            if (s_ip, vni) in sp_of:
                bm = {e2.key[0][1]: e2.params["bridge_id"] for e2 in self._rows("source_port_to_bridge_map")
                      if e2.key[0][2] == 0xFFFF and e2.action.endswith("set_bridge_id")}
                if sp_of[(s_ip, vni)] in bm:
                    dp.ports.update(tp, bridge_id=bm[sp_of[(s_ip, vni)]])
        if terms and local_vteps:
            vtep = next(iter(local_vteps))
            for k in range(4):
                pp = port(PHY_BASE + k)
                dp.ports.a[pp]["flags"] |= T.PORT_VTEP
                dp.ports.a[pp]["ext"] = int(T.ip_raw(np.uint32(vtep))) if hasattr(T, "ip_raw") else int(
                    np.uint32(int.from_bytes(ipaddress.IPv4Address(vtep).packed, "little")))
        tun6 = self._compile_tunnels_v6(dp, port, add_mac, bridges, mac_of)
        self._owned_tunnels = bool(tunnels or terms or tun6)
        # rx LAG: frames from a member physical port enter as the LAG's vport
        for e in self._rows("rx_lag_table"):
            if e.action.endswith("fwd_to_vsi"):
                dp.ports.update(port(PHY_BASE + e.key[0][1]), default_out=port(e.params["port"]))
        # l2_fwd_smac_table present: its bridges learn (OvS-style, in the data plane)
        learn_bridges = {e.key[1][1] for e in self._rows("l2_fwd_smac_table")}
        trap = bool(self._rows("always_trap_arp_table"))
        for p in list(src) + [p for p in range(len(dp.ports.a)) if dp.ports.a[p]["flags"] & T.PORT_VALID and p in self._all_ports(dp)]:
            if int(dp.ports.a[p]["bridge_id"]) in learn_bridges:
                dp.ports.a[p]["flags"] |= T.PORT_LEARN
            if trap:
                dp.ports.a[p]["flags"] |= T.PORT_ARP_TRAP

    def _all_ports(self, dp) -> set:
        return set(self._owned_ports)


def vsi_mac(vsi: int) -> str:
    """The L2 key a VSI-lookup port matches: only byte 1 (the VSI) of the dst MAC is kept."""
    return f"00:{vsi & 0xFF:02x}:00:00:00:00"


def _mac(x: int) -> str:
    return ":".join(f"{(x >> (8 * (5 - i))) & 0xFF:02x}" for i in range(6))
