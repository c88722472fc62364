"""P4Info handling: a protobuf text-format reader and a P4Info helper.

The reference drives the Intel IPU pipeline through `p4rt-ctl` (cmd/intelvsp/p4rt-ctl, P4Info
helper :297-587) against the compiled pipeline's P4Info.  Here P4Info is
plain data: `parse_text` reads any protobuf text-format document (messages, repeated fields,
scalars, strings with escapes) into nested dicts/lists without needing the p4runtime protos, and
`P4Info` indexes tables / match fields / actions / params by name, alias and id.

`MI355X_P4INFO` is this framework's own P4Info for the linux-networking tables the GPU data
plane implements (generated from `TABLES` below, same table/field names and widths as the
reference pipeline so the same p4rt-ctl rule strings are accepted).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

_TOKEN = re.compile(r'\s*(?:(#[^\n]*)|([A-Za-z_][\w.]*)|("(?:[^"\\]|\\.)*")|(-?0x[0-9a-fA-F]+|-?\d+(?:\.\d+)?)|([{}:<>\[\],]))')


def _unescape(s: str) -> str:
    return bytes(s[1:-1], "utf-8").decode("unicode_escape")


def parse_text(text: str) -> dict:
    """Protobuf text format -> dict; every field maps to a list of values (repeated-safe)."""
    toks: list[tuple[str, str]] = []
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise ValueError(f"p4info text: unexpected input at offset {pos}: {text[pos:pos + 20]!r}")
        pos = m.end()
        if m.group(1):
            continue
        for kind, g in (("id", 2), ("str", 3), ("num", 4), ("p", 5)):
            if m.group(g) is not None:
                toks.append((kind, m.group(g)))
                break
    i = 0

    def message(end: str | None) -> dict:
        nonlocal i
        out: dict[str, list] = {}
        while i < len(toks):
            kind, v = toks[i]
            if kind == "p" and v == end:
                i += 1
                return out
            if kind != "id":
                raise ValueError(f"p4info text: expected a field name, got {v!r}")
            name = v
            i += 1
            if toks[i] == ("p", ":"):
                i += 1
            kind, v = toks[i]
            if kind == "p" and v in "{<":
                i += 1
                val = message("}" if v == "{" else ">")
            elif kind == "str":
                val = _unescape(v)
                i += 1
                while i < len(toks) and toks[i][0] == "str":  # adjacent literals concatenate
                    val += _unescape(toks[i][1])
                    i += 1
            elif kind == "num":
                val = int(v, 0) if re.fullmatch(r"-?(0x[0-9a-fA-F]+|\d+)", v) else float(v)
                i += 1
            else:  # enum identifier
                val = v
                i += 1
            out.setdefault(name, []).append(val)
        if end is not None:
            raise ValueError("p4info text: unterminated message")
        return out

    return message(None)


def _one(d: dict, k: str, default=None):
    v = d.get(k)
    return v[0] if v else default


@dataclass
class MatchField:
    id: int
    name: str
    bitwidth: int
    match_type: str  # EXACT / TERNARY / LPM / RANGE / OPTIONAL


@dataclass
class Param:
    id: int
    name: str
    bitwidth: int


@dataclass
class Action:
    id: int
    name: str
    alias: str
    params: list[Param] = field(default_factory=list)


@dataclass
class Table:
    id: int
    name: str
    alias: str
    match_fields: list[MatchField]
    action_ids: list[int]
    size: int
    const_default_action: int = 0

    def field(self, name: str) -> MatchField:
        for f in self.match_fields:
            if f.name == name:
                return f
        raise KeyError(f"table {self.name} has no match field {name!r}")


class P4Info:
    def __init__(self, doc: dict):
        self.tables: dict[str, Table] = {}
        self.actions: dict[str, Action] = {}
        self._tid: dict[int, Table] = {}
        self._aid: dict[int, Action] = {}
        for a in doc.get("actions", []):
            pre = _one(a, "preamble", {})
            act = Action(_one(pre, "id", 0), _one(pre, "name", ""), _one(pre, "alias", ""),
                         [Param(_one(p, "id", 0), _one(p, "name", ""), _one(p, "bitwidth", 0)) for p in a.get("params", [])])
            self.actions[act.name] = act
            if act.alias:
                self.actions.setdefault(act.alias, act)
            self._aid[act.id] = act
        for t in doc.get("tables", []):
            pre = _one(t, "preamble", {})
            mfs = [MatchField(_one(m, "id", 0), _one(m, "name", ""), _one(m, "bitwidth", 0), _one(m, "match_type", "EXACT"))
                   for m in t.get("match_fields", [])]
            tab = Table(_one(pre, "id", 0), _one(pre, "name", ""), _one(pre, "alias", ""), mfs,
                        [_one(r, "id", 0) for r in t.get("action_refs", [])], _one(t, "size", 0),
                        _one(t, "const_default_action_id", 0))
            self.tables[tab.name] = tab
            if tab.alias:
                self.tables.setdefault(tab.alias, tab)
            self._tid[tab.id] = tab

    @classmethod
    def from_text(cls, text: str) -> "P4Info":
        return cls(parse_text(text))

    def table(self, name_or_id) -> Table:
        t = self._tid.get(name_or_id) if isinstance(name_or_id, int) else self.tables.get(name_or_id)
        if t is None:
            raise KeyError(f"unknown table {name_or_id!r}")
        return t

    def action(self, name_or_id) -> Action:
        a = self._aid.get(name_or_id) if isinstance(name_or_id, int) else self.actions.get(name_or_id)
        if a is None:
            raise KeyError(f"unknown action {name_or_id!r}")
        return a

    def table_actions(self, table: Table) -> list[Action]:
        return [self._aid[i] for i in table.action_ids if i in self._aid]


# --------------------------------------------------------------------------------------------
# The MI355X data plane's linux-networking subset (table, [(field, width, match)], [actions], size)
C = "linux_networking_control."
TABLES = [
    ("tx_source_port", [("vmeta.common.vsi", 11, "TERNARY")], ["set_source_port", "drop"], 1024),
    ("rx_source_port", [("vmeta.common.port_id", 2, "EXACT"), ("zero_padding", 16, "EXACT")],
     ["set_source_port", "drop"], 1024),
    ("tx_acc_vsi", [("vmeta.common.vsi", 11, "EXACT"), ("zero_padding", 16, "EXACT")],
     ["l2_fwd_and_bypass_bridge", "drop"], 1024),
    ("vsi_to_vsi_loopback", [("vmeta.common.vsi", 11, "EXACT"), ("target_vsi", 11, "EXACT")], ["fwd_to_vsi", "drop"], 1024),
    ("source_port_to_pr_map", [("user_meta.cmeta.source_port", 16, "EXACT"), ("zero_padding", 8, "EXACT")],
     ["fwd_to_vsi", "drop"], 1024),
    ("rx_phy_port_to_pr_map", [("vmeta.common.port_id", 2, "EXACT"), ("zero_padding", 16, "EXACT")],
     ["fwd_to_vsi", "mirror_and_send", "drop"], 1024),
    ("source_port_to_bridge_map", [("user_meta.cmeta.source_port", 16, "TERNARY"),
                                   ("hdrs.vlan_ext[vmeta.common.depth].hdr.vid", 12, "TERNARY")],
     ["set_bridge_id", "drop"], 1024),
    ("l2_fwd_rx_table", [("user_meta.pmeta.bridge_id", 8, "EXACT"), ("dst_mac", 48, "EXACT")], ["l2_fwd"], 1024),
    # the reference VSP's l2_fwd_tx_table rule strings (p4rtclient.go:569) key on (dst_mac, tun_flag1_d0)
    ("l2_fwd_tx_table", [("dst_mac", 48, "EXACT"), ("user_meta.pmeta.tun_flag1_d0", 8, "EXACT")], ["l2_fwd"], 1024),
    ("sem_bypass", [("dst_mac", 48, "EXACT")], ["set_dest"], 1024),
    ("handle_tx_from_host_to_ovs_and_ovs_to_wire_table", [("vmeta.common.vsi", 11, "EXACT"),
                                                           ("user_meta.cmeta.bit32_zeros", 32, "EXACT")],
     ["add_vlan_and_send_to_port", "set_dest"], 1024),
    ("handle_rx_loopback_from_host_to_ovs_table", [("vmeta.common.vsi", 11, "EXACT"),
                                                   ("user_meta.cmeta.bit32_zeros", 32, "EXACT")], ["set_dest"], 1024),
    ("handle_tx_from_ovs_to_host_table", [("vmeta.common.vsi", 11, "EXACT"),
                                          ("hdrs.dot1q_tag[vmeta.common.depth].hdr.vid", 12, "EXACT")],
     ["remove_vlan_and_send_to_port", "set_dest"], 1024),
    ("handle_rx_loopback_from_ovs_to_host_table", [("vmeta.misc_internal.vm_to_vm_or_port_to_port[27:17]", 11, "EXACT"),
                                                   ("user_meta.cmeta.bit32_zeros", 32, "EXACT")], ["set_dest"], 1024),
    ("vlan_push_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["vlan_push"], 1024),
    ("vlan_pop_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["vlan_pop"], 1024),
    ("tx_lag_table", [("user_meta.cmeta.lag_group_id", 8, "TERNARY"), ("hash", 3, "TERNARY")],
     ["bypass", "set_egress_port", "drop"], 1024),
    ("ipv4_lpm_root_lut", [("user_meta.cmeta.bit16_zeros", 16, "TERNARY")], ["ipv4_lpm_root_lut_action"], 1),
    ("mir_prof", [("mirror_prof_key", 8, "EXACT")], ["mir_prof_action"], 256),
    # L3 (p4info.txt:696-871): LPM routes, nexthops, ECMP, router-interface MACs
    ("ipv4_table", [("ipv4_table_lpm_root", 32, "EXACT"), ("ipv4_dst_match", 32, "LPM")],
     ["ipv4_set_nexthop_id", "ecmp_hash_action", "NoAction"], 1024),
    ("ipv6_lpm_root_lut", [("user_meta.cmeta.bit16_zeros", 16, "TERNARY")], ["ipv6_lpm_root_lut_action"], 1),
    ("ipv6_table", [("ipv6_table_lpm_root", 32, "EXACT"), ("ipv6_dst_match", 128, "LPM")],
     ["ipv6_set_nexthop_id", "ecmp_v6_hash_action", "NoAction"], 1024),
    ("ecmp_hash_table", [("flex", 16, "TERNARY"), ("hash", 3, "TERNARY")], ["set_nexthop_id", "NoAction"], 1024),
    ("nexthop_table", [("user_meta.cmeta.nexthop_id", 16, "EXACT"), ("bit16_zeros", 8, "EXACT")],
     ["set_nexthop_info_dmac", "set_nexthop_lag", "drop", "NoAction"], 1024),
    ("ecmp_nexthop_table", [("user_meta.cmeta.nexthop_id", 16, "TERNARY")], ["ecmp_set_nexthop_info_dmac", "drop"], 1024),
    ("rif_mod_table_start", [("rif_mod_map_id0", 11, "EXACT")], ["set_src_mac_start", "NoAction"], 1024),
    ("rif_mod_table_mid", [("rif_mod_map_id1", 11, "EXACT")], ["set_src_mac_mid", "NoAction"], 1024),
    ("rif_mod_table_last", [("rif_mod_map_id2", 11, "EXACT")], ["set_src_mac_last", "NoAction"], 1024),
    # tunnels (p4info.txt:258-556, 930-1110)
    ("l2_to_tunnel_v4", [("hdrs.mac[vmeta.common.depth].da", 48, "EXACT")], ["set_tunnel_v4", "drop", "do_recirculate"], 1024),
    ("vxlan_encap_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["vxlan_encap", "NoAction"], 1024),
    ("vxlan_encap_vlan_pop_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["vxlan_encap_vlan_pop", "NoAction"], 1024),
    ("geneve_encap_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["geneve_encap", "NoAction"], 1024),
    ("geneve_encap_vlan_pop_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["geneve_encap_vlan_pop", "NoAction"], 1024),
    ("vxlan_decap_and_push_vlan_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")],
     ["vxlan_decap_and_push_vlan", "NoAction"], 1024),
    ("geneve_decap_and_push_vlan_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")],
     ["geneve_decap_and_push_vlan", "NoAction"], 1024),
    ("vxlan_decap_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["vxlan_decap_outer_hdr", "NoAction"], 1024),
    ("geneve_decap_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["geneve_decap_outer_hdr", "NoAction"], 1024),
    ("ipv4_tunnel_term_table", [("ipv4_src", 32, "EXACT"), ("vni", 24, "EXACT")],
     ["set_vxlan_decap_outer_hdr", "set_vxlan_decap_outer_and_push_vlan", "set_geneve_decap_outer_hdr",
      "set_geneve_decap_outer_and_push_vlan", "trap_enable"], 1024),
    ("rx_ipv4_tunnel_source_port", [("ipv4_src", 32, "EXACT"), ("vni", 24, "EXACT")], ["set_source_port", "drop"], 1024),
    # IPv6 underlay tunnels
    ("l2_to_tunnel_v6", [("hdrs.mac[vmeta.common.depth].da", 48, "EXACT")], ["set_tunnel_v6", "do_recirculate", "drop"], 1024),
    ("vxlan_encap_v6_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["vxlan_encap_v6", "NoAction"], 1024),
    ("vxlan_encap_v6_vlan_pop_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")],
     ["vxlan_encap_v6_vlan_pop", "NoAction"], 1024),
    ("geneve_encap_v6_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["geneve_encap_v6", "NoAction"], 1024),
    ("geneve_encap_v6_vlan_pop_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")],
     ["geneve_encap_v6_vlan_pop", "NoAction"], 1024),
    ("ipv6_tunnel_term_table", [("ipv6_src", 128, "EXACT"), ("vni", 24, "EXACT")],
     ["set_vxlan_decap_outer_hdr", "set_vxlan_decap_outer_and_push_vlan", "set_geneve_decap_outer_hdr",
      "set_geneve_decap_outer_and_push_vlan", "NoAction"], 1024),
    ("rx_ipv6_tunnel_source_port", [("ipv6_src", 128, "EXACT"), ("vni", 24, "EXACT")], ["set_source_port", "drop"], 1024),
    # IPsec (the IPU's inline crypto engine; here the ESP kernels, dataplane/ipsec.py)
    ("ipsec_spd", [("hdrs.ipv4[vmeta.common.depth].dst_ip", 32, "EXACT"), ("hdrs.ipv4[vmeta.common.depth].protocol", 8, "EXACT")],
     ["ipsec_protect_set_metadata", "ipsec_bypass", "NoAction"], 1024),
    ("ipsec_tx_sa_classification_table", [("hdrs.ipv4[vmeta.common.depth].dst_ip", 32, "EXACT"),
                                          ("hdrs.ipv4[vmeta.common.depth].protocol", 8, "EXACT"),
                                          ("user_meta.cmeta.is_tunnel", 1, "EXACT")],
     ["tx_ipsec_transport", "tx_ipsec_transport_with_underlay", "tx_ipsec_tunnel", "tx_ipsec_tunnel_v6", "drop",
      "NoAction"], 1024),
    ("ipsec_tunnel_table", [("vmeta.common.saidx", 24, "EXACT"), ("bit16_zeros", 13, "EXACT")],
     ["set_ipsec_tunnel", "NoAction"], 1024),
    ("ipsec_tunnel_encap_mod_table", [("vmeta.common.mod_blob_ptr", 24, "EXACT")], ["ipsec_tunnel_encap_mod", "NoAction"], 1024),
    ("ipv4_ipsec_tunnel_term_table", [("ipv4_src", 32, "EXACT"), ("ipv4_dst", 32, "EXACT")],
     ["decap_ipsec_tunnel_hdr", "do_recirculate"], 1024),
    ("MainControlDecrypt.ipsec_rx_sa_classification_table",
     [("hdrs.ipv4[vmeta.common.depth].src_ip", 32, "EXACT"), ("hdrs.ipv4[vmeta.common.depth].dst_ip", 32, "EXACT"),
      ("hdrs.esp.spi", 32, "EXACT")], ["MainControlDecrypt.ipsec_decrypt", "MainControlDecrypt.ipsec_bypass"], 1024),
    # keyless exact-match-engine housekeeping tables whose only action is NoAction (p4info.txt):
    # entries are accepted and, as in the pipeline, change nothing
    ("lem_exception", [], ["NoAction"], 1024),
    ("lem_clear", [], ["NoAction"], 1024),
    # LAG rx, smac learning check, ARP trap (p4info.txt:168, 783, 1011)
    ("rx_lag_table", [("vmeta.common.port_id", 2, "EXACT"), ("user_meta.cmeta.lag_group_id", 8, "EXACT")],
     ["fwd_to_vsi", "drop"], 1024),
    ("l2_fwd_smac_table", [("hdrs.mac[vmeta.common.depth].sa", 48, "EXACT"), ("user_meta.pmeta.bridge_id", 8, "EXACT")],
     ["NoAction", "fwd_to_cp"], 1024),
    # the compiled pipeline names both key fields hdrs.inval.data (p4info.txt:168-190): values bind in order
    ("always_trap_arp_table", [("hdrs.inval.data", 16, "EXACT"), ("hdrs.inval.data", 16, "EXACT")],
     ["do_trap_enable"], 1024),
    # RX recirculation (p4info.txt:189-212, const default do_recirculate, 0 SEM slots in the
    # compiled pipeline): the GPU pipeline recirculates terminated tunnel traffic by itself, so
    # entries are accepted and change nothing
    ("always_recirculate_table", [("hdrs.inval.data", 16, "EXACT"), ("hdrs.inval.data", 16, "EXACT")],
     ["do_recirculate"], 1024),
    # VM IPv4 -> MAC maps (p4info.txt:1393-1440): routed packets' source / destination MAC
    ("vm_src_ip4_mac_map_table", [("ipv4_src", 32, "EXACT")], ["vm_src_ip4_mac_map_action", "NoAction"], 1024),
    ("vm_dst_ip4_mac_map_table", [("ipv4_dst", 32, "EXACT")], ["vm_dst_ip4_mac_map_action", "NoAction"], 1024),
]
ACTIONS = {
    "vm_src_ip4_mac_map_action": [("smac_high", 16), ("smac_mid", 16), ("smac_low", 16)],
    "vm_dst_ip4_mac_map_action": [("dmac_high", 16), ("dmac_mid", 16), ("dmac_low", 16)],
    "set_source_port": [("source_port", 16)],
    "l2_fwd_and_bypass_bridge": [("port", 32)],
    "fwd_to_vsi": [("port", 32)],
    "mirror_and_send": [("port", 32), ("mirror_session_id", 16)],
    "set_bridge_id": [("bridge_id", 8)],
    "l2_fwd": [("port", 32)],
    "set_dest": [("port_id", 32)],
    "add_vlan_and_send_to_port": [("vlan_id", 12), ("port_id", 32)],
    "remove_vlan_and_send_to_port": [("vlan_id", 12), ("port_id", 32)],
    "vlan_push": [("pcp", 3), ("dei", 1), ("vlan_id", 12)],
    "vlan_pop": [],
    "bypass": [],
    "drop": [],
    "set_egress_port": [("router_interface_id", 16), ("egress_port", 32)],
    "ipv4_lpm_root_lut_action": [("ipv4_table_lpm_root", 32)],
    # subset of the pipeline's mirror profile parameters (the ones the VSP programs)
    "mir_prof_action": [("port_dest_type", 32), ("vport_id", 32), ("mode", 1), ("dest_id", 16), ("func_valid", 1),
                        ("store_vsi", 1)],
    "NoAction": [],
    "ipv4_set_nexthop_id": [("nexthop_id", 16)],
    "ipv6_set_nexthop_id": [("nexthop_id", 16)],
    "ecmp_v6_hash_action": [("ecmp_group_id", 16)],
    "ipv6_lpm_root_lut_action": [("ipv6_table_lpm_root", 32)],
    "ecmp_hash_action": [("ecmp_group_id", 16)],
    "set_nexthop_id": [("nexthop_id", 16)],
    "set_nexthop_info_dmac": [("router_interface_id", 16), ("egress_port", 32), ("dmac_high", 16), ("dmac_low", 32)],
    "set_nexthop_lag": [("lag_group_id", 8), ("dmac_high", 16), ("dmac_low", 32)],
    "ecmp_set_nexthop_info_dmac": [("router_interface_id", 16), ("egress_port", 32), ("dmac_high", 16), ("dmac_low", 32)],
    "set_src_mac_start": [("arg", 16)],
    "set_src_mac_mid": [("arg", 16)],
    "set_src_mac_last": [("arg", 16)],
    "set_tunnel_v4": [("dst_addr", 32)],
    "set_tunnel_v6": [("ipv6_1", 32), ("ipv6_2", 32), ("ipv6_3", 32), ("ipv6_4", 32)],
    **{a: [("src_addr", 128), ("dst_addr", 128), ("ds", 6), ("ecn", 2), ("flow_label", 20), ("hop_limit", 8),
           ("src_port", 16), ("dst_port", 16), ("vni", 24)]
       for a in ("vxlan_encap_v6", "vxlan_encap_v6_vlan_pop", "geneve_encap_v6", "geneve_encap_v6_vlan_pop")},
    "do_recirculate": [],
    "vxlan_encap": [("src_addr", 32), ("dst_addr", 32), ("src_port", 16), ("dst_port", 16), ("vni", 24)],
    "vxlan_encap_vlan_pop": [("src_addr", 32), ("dst_addr", 32), ("src_port", 16), ("dst_port", 16), ("vni", 24)],
    "geneve_encap": [("src_addr", 32), ("dst_addr", 32), ("src_port", 16), ("dst_port", 16), ("vni", 24)],
    "geneve_encap_vlan_pop": [("src_addr", 32), ("dst_addr", 32), ("src_port", 16), ("dst_port", 16), ("vni", 24)],
    "vxlan_decap_and_push_vlan": [("pcp", 3), ("dei", 1), ("vlan_id", 12)],
    "geneve_decap_and_push_vlan": [("pcp", 3), ("dei", 1), ("vlan_id", 12)],
    "set_vxlan_decap_outer_and_push_vlan": [("tunnel_id", 20)],
    "set_geneve_decap_outer_and_push_vlan": [("tunnel_id", 20)],
    "vxlan_decap_outer_hdr": [],
    "geneve_decap_outer_hdr": [],
    "set_vxlan_decap_outer_hdr": [("tunnel_id", 20)],
    "set_geneve_decap_outer_hdr": [("tunnel_id", 20)],
    "trap_enable": [],
    "fwd_to_cp": [],
    "do_trap_enable": [],
    "ipsec_protect_set_metadata": [("saidx", 24)],
    "ipsec_bypass": [],
    "tx_ipsec_transport": [],
    "tx_ipsec_transport_with_underlay": [],
    "tx_ipsec_tunnel": [("dst_addr", 32)],
    "tx_ipsec_tunnel_v6": [("dst_addr_1", 32), ("dst_addr_2", 32), ("dst_addr_3", 16)],
    "set_ipsec_tunnel": [("tunnel_id", 24)],
    "ipsec_tunnel_encap_mod": [("ipsec_src_addr", 32), ("ipsec_dst_addr", 32), ("proto", 8)],
    "decap_ipsec_tunnel_hdr": [],
    "MainControlDecrypt.ipsec_decrypt": [("saidx", 24)],
    "MainControlDecrypt.ipsec_bypass": [],
}


def _render_mi355x_p4info() -> str:
    lines = ['pkg_info {', '  arch: "mi355x-nfdp"', '}']
    aids = {}
    for k, (name, params) in enumerate(ACTIONS.items()):
        aid = 0x01000000 | (k + 1)
        aids[name] = aid
    for k, (tname, fields, acts, size) in enumerate(TABLES):
        full = tname if "." in tname else C + tname   # a name with a control prefix is used as is
        lines += ["tables {", "  preamble {", f"    id: {0x02000000 | (k + 1)}", f'    name: "{full}"',
                  f'    alias: "{tname.split(".")[-1]}"', "  }"]
        for j, (fname, width, mt) in enumerate(fields):
            lines += ["  match_fields {", f"    id: {j + 1}", f'    name: "{fname}"', f"    bitwidth: {width}",
                      f"    match_type: {mt}", "  }"]
        for a in acts:
            lines += ["  action_refs {", f"    id: {aids[a]}", "  }"]
        lines += [f"  size: {size}", "}"]
    for name, params in ACTIONS.items():
        full = name if "." in name else C + name
        lines += ["actions {", "  preamble {", f"    id: {aids[name]}", f'    name: "{full}"',
                  f'    alias: "{name.split(".")[-1]}"', "  }"]
        for j, (pname, width) in enumerate(params):
            lines += ["  params {", f"    id: {j + 1}", f'    name: "{pname}"', f"    bitwidth: {width}", "  }"]
        lines += ["}"]
    return "\n".join(lines) + "\n"


MI355X_P4INFO_TEXT = _render_mi355x_p4info()
MI355X_P4INFO = P4Info.from_text(MI355X_P4INFO_TEXT)
