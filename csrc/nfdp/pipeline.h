// pipeline.h — scalar per-packet stages shared by the GPU kernels and the CPU oracle.
//
// Stage order (one packet):
//   ingress_stage : port lookup, VLAN isolation (K10), spoof-check, bridge-id (K7), FlowKey
//   [hash + ACL   : done by the caller — MFMA on the GPU, scalar in the oracle]
//   flow lookup   : exact match, 2-choice bucketized cuckoo (1M+ flows)
//   chain_stage   : built-in NF hops (ACL verdict, SNAT, TTL, L2 steer, VLAN, hairpin) or the
//                   (bridge, dst-MAC) L2 table on a flow miss (K5); egress port tagging (K6)
#pragma once
#include <type_traits>

#include "nfdp.h"

namespace nfdp {

struct IngressState {
  uint32_t in_port;
  uint32_t bridge;
  uint32_t reason;    // != 0: already dropped
  uint32_t wire_len;  // ingress length (bytes counted on rx)
  uint32_t in_flags;  // ingress port flags (0 on a bad port)
  uint32_t in_ext;    // ingress port ext word (ingress-push vid, mirror port)
  FlowKey key;
};

// Table-access policy of the stages.  The oracle and the sharded kernels read the small tables
// straight from memory (DirectTables); the fused kernel passes a policy that serves them from
// LDS copies staged once per workgroup, so the per-packet path has no dependent global loads
// besides the frame and the flow bucket.
struct DirectTables {
  const TablesView& t;
  NFDP_HD PortEntry port(uint32_t i) const { return t.ports[i]; }
  NFDP_HD uint64_t chain_word(uint32_t c) const {  // nhops + 7 hop opcodes (first 8 B of the entry)
    return c < t.n_chains ? *reinterpret_cast<const uint64_t*>(&t.chains[c]) : 0ull;
  }
  NFDP_HD bool permit(int rule) const { return rule >= 0 ? t.acl_permit[rule] != 0 : t.acl_default_permit != 0; }
};

// IPv6 flow / ACL features in use: IPv6 packets get folded 5-tuple keys (make_key).
NFDP_HD bool v6_keys(const TablesView& t) { return t.flow6_on || t.n_acl6; }

// FOLD6 false: the caller fills IPv6 keys itself (the fused kernel takes them from v6_kernel, so
// the fold's registers stay out of its budget).
template <class TA, bool FOLD6 = true>
NFDP_HD void ingress_stage(const TablesView& t, const TA& ta, const uint32_t* d, uint32_t inmeta, Parsed& p,
                           IngressState& st) {
  st.in_port = inmeta & 0xFFFFu;
  uint32_t len = inmeta >> 16;  // whole frame; the slot holds its first min(len, 64) bytes
  st.wire_len = len;
  st.reason = kOk;
  if (len < 14 || len > kMaxFrame) { st.reason = kMalformed; len = len < 14 ? 14 : kMaxFrame; }
  parse(d, len, p);
  st.bridge = 0;
  st.in_flags = 0;
  st.in_ext = 0;
  if (st.in_port >= (uint32_t)kMaxPorts) {
    st.reason = kBadPort;
  } else {
    const PortEntry pe = ta.port(st.in_port);
    st.in_flags = pe.flags;
    st.in_ext = pe.ext;
    if ((pe.flags & (kPortValid | kPortLinkDown)) != kPortValid) st.reason = st.reason ? st.reason : kBadPort;
    const uint32_t vid = p.tci & 0xFFFu;
    if ((pe.flags & kPortVlanIsolate) && p.tagged && vid != pe.vlan)
      st.reason = st.reason ? st.reason : kVlanDrop;
    if ((pe.flags & kPortSpoofChk) &&
        (smac_lo(p.s) != pe.mac_lo || smac_hi(p.s) != pe.mac_hi))
      st.reason = st.reason ? st.reason : kSpoof;
    st.bridge = ((pe.flags & kPortVlanBridge) && p.tagged) ? vid : pe.bridge_id;
  }
  st.key = make_key(p, st.bridge, FOLD6 && v6_keys(t));
}
NFDP_HD void ingress_stage(const TablesView& t, const uint32_t* d, uint32_t inmeta, Parsed& p, IngressState& st) {
  ingress_stage(t, DirectTables{t}, d, inmeta, p, st);
}

// A packet that takes part in the exact-match flow stage: IPv4, or IPv6 when the flow table
// carries the IPv6 side array (its folded-key hits are verified against it: flow6_verify).
NFDP_HD bool flowable(const TablesView& t, const Parsed& p) { return p.ipv4 || (NFDP_IPV6 && p.ipv6 && t.flow6_on); }
// The ACL rule of a packet.  With IPv6 features in the tables (v6_keys), an IPv6 packet's rule
// comes from the IPv6 rules (acl6), never from the IPv4 TCAM over the folded key; without them
// its key (kKeyV6 set) goes through the IPv4 TCAM like any other, where AclTable's rules (which
// require kKeyV6 clear) never match it.
NFDP_HD int acl_rule_v6(const TablesView& t, const Parsed& p, const IngressState& st) {
  return t.n_acl6 ? acl6_first_match(t, p, st.bridge) : -1;
}
NFDP_HD int acl_rule_scalar(const TablesView& t, const Parsed& p, const IngressState& st) {
  return (p.ipv6 && v6_keys(t)) ? acl_rule_v6(t, p, st) : acl_first_match(t, st.key);
}

// ---- Wide header pairs: single-pass tunnel termination ----
// A frame on a VTEP (underlay) port may arrive as TWO consecutive slots: its bytes 0..63 (the
// head) and 64..127 (the continuation, in-meta port kPortCont, same length).  When the head is
// VXLAN / GENEVE (IPv4 or IPv6 underlay, an outer 802.1Q tag allowed) to the local VTEP, passes
// its port's ingress checks and (outer source, VNI) has a termination entry, the pipeline runs on
// the INNER frame in the same pass, as received on the tunnel port (P4 ipv4 / ipv6_tunnel_term_
// table + rx_*_tunnel_source_port, without the recirculation).  decap_pair returns that port and
// fills `inner` with the inner frame's first bytes: 64 over an IPv4 underlay, 58 / 54 over IPv6
// (untagged / tagged outer: the pair ends at byte 128) - `hv`; `strip` = the outer bytes.  -1:
// not terminated (the head goes through the pipeline as received).  Every rewrite stays in the
// first 56 bytes, so the egress takes the out slot's first hv (+ tag) bytes and the tail from
// in_frame + strip (nfdp.h out_tail).
// The tunnel header after the outer UDP header: VXLAN (4789) with its I flag (RFC 7348: the VNI is
// valid), or GENEVE (6081) version 0 with no options, not an OAM frame, carrying Ethernet (RFC
// 8926 protocol 0x6558).  b01: tunnel-header bytes 0 | 1 << 8 (raw), ptype: bytes 2..3 (raw).
NFDP_HD bool tunnel_hdr_ok(uint32_t dport, uint32_t b01, uint32_t ptype_raw) {
  if (dport == 4789u) return (b01 & 0x08u) != 0u;
  return dport == 6081u && (b01 & 0xFFu) == 0u && (b01 & 0x8000u) == 0u && ptype_raw == 0x5865u;
}

NFDP_HD uint32_t pair_dw(const uint32_t* d, const uint32_t* x, int j) {   // dword j of head ++ continuation
  return j < kSlotDwords ? d[j] : (j < 2 * kSlotDwords ? x[j - kSlotDwords] : 0u);
}
template <class TA>
NFDP_HD int decap_pair(const TablesView& t, const TA& ta, const uint32_t* d, const uint32_t* x, uint32_t inmeta,
                       uint32_t* inner, uint32_t& strip, uint32_t& hv) {
  strip = 0; hv = kSlotBytes;
  const uint32_t in_port = inmeta & 0xFFFFu, len = inmeta >> 16;
  if (in_port >= (uint32_t)kMaxPorts || len > kMaxFrame || len < 18) return -1;
  const PortEntry pe = ta.port(in_port);
  if ((pe.flags & (kPortValid | kPortLinkDown | kPortVtep)) != (kPortValid | kPortVtep)) return -1;
  const bool tg = be16_at(d, 12) == 0x8100u;
  // the outer frame's ingress checks (ingress_stage): a frame its port drops is not terminated
  if ((pe.flags & kPortVlanIsolate) && tg && (be16_at(d, 14) & 0xFFFu) != pe.vlan) return -1;
  if ((pe.flags & kPortSpoofChk) && (smac_lo(d) != pe.mac_lo || smac_hi(d) != pe.mac_hi)) return -1;
  // untagged view of the pair (dword j; constant j only: a run-time index would go to scratch)
  auto sn = [&](int j) -> uint32_t { return j < 3 ? d[j] : (tg ? pair_dw(d, x, j + 1) : pair_dw(d, x, j)); };
  auto a2 = [&](int b) -> uint32_t { return (sn(b >> 2) >> 16) | (sn((b >> 2) + 1) << 16); };   // raw32 at b = 2 mod 4
  auto sw = [](uint32_t v) -> uint32_t { return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu); };    // be16 of a raw half
  const uint32_t nlen = tg ? len - 4u : len;
  const uint32_t et = sw(sn(3));
  bool v6 = false;
  int tp = -1;
  if (et == 0x0800u) {
    // a whole datagram (neither MF nor a fragment offset), no options, UDP
    const bool ip_ok = ((sn(3) >> 16) & 0xFFu) == 0x45u && (sw(sn(5)) & 0x3FFFu) == 0u && (sn(5) >> 24) == 17u;
    if (!ip_ok || a2(30) != pe.ext || nlen < kEncapBytes + 14u) return -1;
    const uint32_t dport = sw(sn(9));
    if (!tunnel_hdr_ok(dport, sn(10) >> 16, sn(11) & 0xFFFFu)) return -1;
    const uint32_t vni = (((sn(11) >> 16) & 0xFFu) << 16) | ((sn(11) >> 24) << 8) | (sn(12) & 0xFFu);
    tp = term_lookup(t, a2(26), vni);
  } else if (et == 0x86DDu && t.vtep6_fold) {
    v6 = true;
    if (((sn(3) >> 20) & 0xFu) != 6u || (sn(5) & 0xFFu) != 17u || nlen < kEncap6Bytes + 14u) return -1;
    if (a2(38) != t.vtep6[0] || a2(42) != t.vtep6[1] || a2(46) != t.vtep6[2] || a2(50) != t.vtep6[3]) return -1;
    const uint32_t dport = sw(sn(14));
    if (!tunnel_hdr_ok(dport, sn(15) >> 16, sn(16) & 0xFFFFu)) return -1;
    const uint32_t vni = (((sn(16) >> 16) & 0xFFu) << 16) | ((sn(16) >> 24) << 8) | (sn(17) & 0xFFu);
    tp = term6_lookup(t, a2(22), a2(26), a2(30), a2(34), vni);
  } else {
    return -1;
  }
  if (tp < 0 || tp >= kMaxPorts) return -1;
  strip = (v6 ? kEncap6Bytes : kEncapBytes) + (tg ? 4u : 0u);
  hv = 2u * kSlotBytes - strip < (uint32_t)kSlotBytes ? 2u * kSlotBytes - strip : (uint32_t)kSlotBytes;
  // inner dword k = bytes strip + 4k .. of the pair; strip = 2 (mod 4): halves of two dwords
#pragma unroll
  for (int k = 0; k < kSlotDwords; ++k) {
    const uint32_t w12 = (pair_dw(d, x, 12 + k) >> 16) | (pair_dw(d, x, 13 + k) << 16);
    const uint32_t w13 = (pair_dw(d, x, 13 + k) >> 16) | (pair_dw(d, x, 14 + k) << 16);
    const uint32_t w17 = (pair_dw(d, x, 17 + k) >> 16) | (pair_dw(d, x, 18 + k) << 16);
    const uint32_t w18 = (pair_dw(d, x, 18 + k) >> 16) | (pair_dw(d, x, 19 + k) << 16);
    inner[k] = v6 ? (tg ? w18 : w17) : (tg ? w13 : w12);
  }
  return tp;
}

struct EgressDecision {
  uint32_t out_port;
  uint32_t reason;
  uint32_t push;      // 1 -> insert an 802.1Q tag with `tci`
  uint32_t tci;
  uint32_t mirror;    // 1 -> the ingress frame is also copied to the ingress port's mirror port (K9)
  uint32_t flood;     // bridge + 1 when the frame is flooded: out_port is the group's first member,
                      // side_stage emits a replica per further member
  uint32_t xhdr;      // outer-header bytes (50 IPv4 / 70 IPv6 underlay) when out_port is a tunnel port:
                      // the side pass writes them; 0 otherwise
  uint32_t inner_len; // kRecirc / kRecirc6: length of the decapsulated inner frame; kRemote from a
                      // kHopXfer: the hop the chain resumes at on the other GPU
};

// The resume word of a hand-off (EgressDecision::inner_len of a kRemote from a kHopXfer, HopState::hop):
// the hop the chain resumes at in the low byte, and the egress port the hops before the hand-off
// decided (bit 15 set) in the high half - resume_stage replays it for a route hop.
constexpr uint32_t kHopResumeHopMask = 0xFFu, kHopResumeHasPort = 0x8000u;
NFDP_HD uint32_t hop_resume_word(uint32_t hop, uint32_t port) {
  return port < 0xFFFFu ? (hop | kHopResumeHasPort | (port << 16)) : hop;
}

// Length of the frame that leaves (the meta word's len): inner frame for a recirculation, tag and
// outer-header bytes included otherwise, 0 for drops.
NFDP_HD uint32_t egress_len(const Parsed& p, const EgressDecision& e) {
  if (e.reason == kRecirc || e.reason == kRecirc6 || e.reason == kCont) return e.inner_len;
  if (e.reason) return 0u;
  return p.len + (e.push ? 4u : 0u) + e.xhdr;
}

NFDP_HD uint32_t byte_at(const uint32_t* s, int off) { return (s[off >> 2] >> (8 * (off & 3))) & 0xFFu; }

#ifndef NFDP_L3_ON
#define NFDP_L3_ON true   // build experiment knob: false compiles the routing / tunnel paths out
#endif
#ifndef NFDP_HOP_UNROLL
#define NFDP_HOP_UNROLL 1   // r2 A/B: the unrolled dispatch is 1-2 % faster despite ~100 more SGPR spills
#endif

// A port takes frames when it is configured, its link is up and its function's RX is enabled.
NFDP_HD bool port_can_egress(uint32_t flags) {
  return (flags & (kPortValid | kPortLinkDown | kPortRxOff)) == kPortValid;
}

// Final egress checks on a chosen port: LAG member (K8), validity, egress tag (K6), MTU.
// Returns a drop reason (0 = ok); `port`/`push`/`tci` are updated in place.
template <class TA>
NFDP_HD uint32_t finish_port(const TablesView& t, const TA& ta, uint32_t& port, uint32_t hash, bool vlan_done,
                             uint32_t& push, uint32_t& tci, uint32_t l2len, uint32_t* xhdr = nullptr) {
  if (port >= (uint32_t)kMaxPorts) return kBadPort;
  PortEntry pe = ta.port(port);
  if (pe.flags & kPortLag) {
    // LAG (K8): member = group[hash[2:0]] (tx_lag_table lag_group_id, hash/7)
    const uint32_t g = pe.lag;
    const uint32_t m = (t.lag_members && g < t.n_lag_groups) ? t.lag_members[g * kLagWays + (hash & 7u)] : kPortNone;
    if (m >= (uint32_t)kMaxPorts) return kBadPort;
    port = m;
    pe = ta.port(m);
  }
  if (!port_can_egress(pe.flags)) return kBadPort;
  if (!vlan_done && (pe.flags & kPortTagEgress) && pe.vlan) { push = 1; tci = pe.vlan & 0xFFFu; }
  // tunnel port (OvS vxlan / geneve port, P4 l2_to_tunnel_v4 / _v6): encapsulated by the side pass
  uint32_t enc = 0;
  if (NFDP_L3_ON && (pe.flags & kPortTunnel)) {
    const bool v6 = (pe.flags & kPortTunnel6) != 0;
    if (v6 ? (!t.tunnels6 || pe.lag >= t.n_tunnels6) : (!t.tunnels || pe.lag >= t.n_tunnels)) return kBadPort;
    enc = v6 ? kEncap6Bytes : kEncapBytes;
    if (xhdr) *xhdr = enc;
  }
  // l2len is untagged: the L3 size is l2len - 14 whatever the tagging
  if (l2len + (push ? 4u : 0u) + enc > kMaxFrame || (pe.mtu && l2len - 14u > pe.mtu)) return kTooBig;
  return kOk;
}

// IPv4 routing on the normalized frame (P4 ipv4_table LPM -> ecmp_hash_table -> nexthop_table,
// rif_mod_table for the source MAC): TTL - 1 with the checksum update, neighbour / router MACs,
// egress port.  Returns a drop reason (0 = routed, e.out_port set).  The
// vm_{src,dst}_ip4_mac_map_table overrides follow in chain_stage (vm_mac_map).
NFDP_HD uint32_t route_ipv4(const TablesView& t, Parsed& p, uint32_t hash, uint32_t& out_port) {
  if (!p.ipv4) return kNoRoute;
  const uint32_t dst = __builtin_bswap32(raw32_at2(p.s, 30));
  const int nh = route_nexthop(t, lpm_lookup(t, dst), hash);
  if (nh < 0) return kNoRoute;
  const NextHop n = t.nexthops[nh];
  if (!n.valid) return kNoRoute;
  if (!act_ttl(p)) return kTtlExpired;
  set_dmac(p.s, n.dmac_lo, n.dmac_hi);
  set_smac(p.s, n.smac_lo, n.smac_hi);
  out_port = n.port;
  return kOk;
}

// VM IPv4 -> MAC overrides of a routed IPv4 packet (P4 vm_src_ip4_mac_map_table /
// vm_dst_ip4_mac_map_table).  One call site per kernel (chain_stage's tail) keeps it to one
// inlined copy; callers test t.vmmac (wave-uniform) first.
NFDP_HD void vm_mac_map(const TablesView& t, Parsed& p) {
  for (uint32_t kind = kVmMacSrc; kind <= kVmMacDst; ++kind) {
    const int i = vmmac_lookup(t, raw32_at2(p.s, kind == kVmMacSrc ? 26 : 30), kind);
    if (i < 0) continue;
    const VmMacEntry m = t.vmmac[i];
    if (kind == kVmMacSrc) set_smac(p.s, m.mac_lo, m.mac_hi); else set_dmac(p.s, m.mac_lo, m.mac_hi);
  }
}

// IPv6 routing (P4 ipv6_table): LPM on the destination, hop limit - 1 (no header checksum in
// IPv6), neighbour / router MACs, egress port.  ECMP members are picked by a hash of the IPv6
// addresses and ports (the packet's Toeplitz hash covers IPv4 fields only).  Returns a drop
// reason (0 = routed).  Only the routed-interface miss path calls it (an IPv6 flow hit takes the chain).
NFDP_HD uint32_t route_ipv6(const TablesView& t, Parsed& p, uint32_t& out_port) {
  const uint32_t d0 = __builtin_bswap32(raw32_at2(p.s, 38)), d1 = __builtin_bswap32(raw32_at2(p.s, 42));
  const uint32_t d2 = __builtin_bswap32(raw32_at2(p.s, 46)), d3 = __builtin_bswap32(raw32_at2(p.s, 50));
  const uint32_t h6 = fmix32(d0 ^ d1 ^ d2 ^ d3 ^ raw32_at2(p.s, 22) ^ raw32_at2(p.s, 26) ^ raw32_at2(p.s, 30) ^
                             raw32_at2(p.s, 34) ^ (p.len >= 58 ? raw32_at2(p.s, 54) : 0u));
  const int nh = route_nexthop(t, lpm6_lookup(t, d0, d1, d2, d3), h6);
  if (nh < 0) return kNoRoute;
  const NextHop n = t.nexthops[nh];
  if (!n.valid) return kNoRoute;
  const uint32_t hl = byte_at(p.s, 21);
  if (hl <= 1u) return kTtlExpired;
  p.s[5] = (p.s[5] & ~(0xFFu << 8)) | ((hl - 1u) << 8);
  set_dmac(p.s, n.dmac_lo, n.dmac_hi);
  set_smac(p.s, n.smac_lo, n.smac_hi);
  out_port = n.port;
  return kOk;
}

// One chain hop (chain_stage and resume_stage).  Returns true when the hop ends the chain: a
// drop / punt (e.reason, e.out_port set) or a hand-off to another GPU (kHopXfer: e.reason =
// kRemote, e.out_port = that GPU's plane, e.inner_len = the hop the chain resumes at there).
// V6HOPS: the ttl hop also decrements an IPv6 hop limit.  A hop runs only on a flow hit and an
// IPv6 packet hits a flow only with IPv6 features in the tables, i.e. in the kernels' V6
// instances, so the IPv4-only instances compile it out (their register budget) with the same
// results as the oracle, which always has it.
// XFER: hand-offs are honoured (the oracle, the kernels' XFER instances, resume_stage); the other
// kernel instances never see split chains from the batch engine (DataPlane picks the XFER instances
// for tables that have them), and the persistent ring kernel runs a split chain whole on the GPU
// the frame entered (a kHopXfer hop is a no-op there), so their register budgets do not pay for it.
template <class TA, bool V6HOPS = true, bool XFER = true>
NFDP_HD bool apply_hop(const TablesView& t, const TA& ta, uint32_t op, int i, Parsed& p, const IngressState& st,
                       const FlowAction& act, int acl_rule, uint32_t hash, EgressDecision& e, bool& vlan_done) {
  if (op == kHopAcl) {
    if (!ta.permit(acl_rule)) { e.reason = kAclDeny; e.out_port = kPortNone; return true; }
  } else if (op == kHopNat) {
    if (p.ipv4) act_snat(p, act.nat_ip, act.nat_port);
  } else if (op == kHopL2Fwd) {
    e.out_port = act.out_port;
    if (e.out_port < (uint32_t)kMaxPorts) {
      const PortEntry pe = ta.port(e.out_port);
      set_dmac(p.s, pe.peer_mac_lo, pe.peer_mac_hi);
      set_smac(p.s, pe.mac_lo, pe.mac_hi);
    }
  } else if (op == kHopTtl) {
    if (p.ipv4 && !act_ttl(p)) { e.reason = kTtlExpired; e.out_port = kPortNone; return true; }
    if (V6HOPS && NFDP_IPV6 && p.ipv6) {   // hop limit - 1 (no IPv6 header checksum)
      const uint32_t hl = byte_at(p.s, 21);
      if (hl <= 1u) { e.reason = kTtlExpired; e.out_port = kPortNone; return true; }
      p.s[5] = (p.s[5] & ~(0xFFu << 8)) | ((hl - 1u) << 8);
    }
  } else if (op == kHopHairpin) {
    e.out_port = st.in_port;
    const uint32_t dl = dmac_lo(p.s), dh = dmac_hi(p.s);
    set_dmac(p.s, smac_lo(p.s), smac_hi(p.s));
    set_smac(p.s, dl, dh);
  } else if (op == kHopVlan) {
    if (act.vlan == 0xFFFFu) { e.push = 0; vlan_done = true; }
    else if (act.vlan) { e.push = 1; e.tci = act.vlan & 0xFFFu; vlan_done = true; }
  } else if (op == kHopDrop) {
    e.reason = kChainDrop; e.out_port = kPortNone; return true;
  } else if (op == kHopPunt) {
    e.reason = kNoRoute; e.out_port = kPortPunt; return true;
  } else if (NFDP_L3_ON && op == kHopRoute) {
    uint32_t rp = kPortNone;
    const uint32_t r = route_ipv4(t, p, hash, rp);
    if (r) { e.reason = r; e.out_port = r == kNoRoute ? kPortPunt : kPortNone; return true; }
    e.out_port = rp;
  } else if (XFER && op >= kHopXfer) {
    // the rest of the chain runs on another GPU (resume_stage there): the frame leaves with the
    // header as the hops so far left it, untagged (a vlan hop's push is replayed at the end).  The
    // egress port the hops so far decided travels in the resume word (hop_resume_word): a route
    // hop's port depends on the header it rewrote, so the resuming GPU cannot recompute it
    e.inner_len = hop_resume_word((uint32_t)i + 1u, e.out_port);
    e.reason = kRemote; e.out_port = op & kHopXferPlanes; e.push = 0;
    return true;
  }
  return false;
}

// `hit`: flow entry found; `act`: its action; `acl_rule`: first matching ACL rule or -1;
// `hash`: the packet's Toeplitz hash (LAG member selection uses hash[2:0], K8).
template <class TA, bool V6HOPS = true, bool XFER = true>
NFDP_HD EgressDecision chain_stage(const TablesView& t, const TA& ta, Parsed& p, const IngressState& st,
                                   bool hit, const FlowAction& act, int acl_rule, uint32_t hash) {
  EgressDecision e;
  e.out_port = kPortNone; e.reason = st.reason; e.push = 0; e.tci = 0; e.mirror = 0; e.flood = 0;
  e.xhdr = 0; e.inner_len = 0;
  if (e.reason) {
    // continuation slot: the meta carries the head's strip / valid bytes (set in st.in_ext)
    if (e.reason == kCont) { e.out_port = st.in_ext & 0xFFu; e.inner_len = st.in_ext >> 8; }
    return e;
  }
  bool vlan_done = false;
  if (!hit) {
    // tunnel termination on an underlay port (ipv4_tunnel_term_table + rx_ipv4_tunnel_source_port):
    // UDP 4789 (VXLAN) / 6081 (GENEVE, no options) to the local VTEP -> recirculate the inner
    // frame as received on the tunnel's port (P4 do_recirculate; the I/O layer re-injects it).
    // IPv6 underlay (ipv6_tunnel_term_table): the VNI (frame bytes 66..68) lies past the 64-B
    // header slot, so the kernel recognises the tunnel (destination folded against the local IPv6
    // VTEP) and the I/O layer finishes the (source, VNI) lookup and the decap (kRecirc6).  One
    // block for both families: offsets by family, so the cold path stays one region.
    if (NFDP_L3_ON && (st.in_flags & kPortVtep) && (p.ipv4 || (p.ipv6 && t.vtep6_fold))) {
      const bool v6 = p.ipv6;
      const uint32_t enc = v6 ? kEncap6Bytes : kEncapBytes;
      const bool to_me = v6 ? vtep6_fold(raw32_at2(p.s, 38), raw32_at2(p.s, 42), raw32_at2(p.s, 46),
                                         raw32_at2(p.s, 50)) == t.vtep6_fold
                            : raw32_at2(p.s, 30) == st.in_ext;
      const uint32_t proto = v6 ? byte_at(p.s, 20) : (p.s[5] >> 24);
      // (IPv4: parse() took offset 0 only; a first fragment, MF set, is not a whole datagram either)
      const bool whole = v6 || (be16_at(p.s, 20) & 0x2000u) == 0u;
      if (to_me && whole && proto == 17u && p.len >= enc + 14u) {
        // constant offsets only (a run-time index into p.s would move the header to scratch)
        const uint32_t dport = v6 ? be16_at(p.s, 56) : be16_at(p.s, 36);
        // IPv4: the tunnel header is in the slot; IPv6: it may lie past it (a tagged outer frame), so
        // the I/O layer checks it with the VNI on the whole frame (resolve_recirc6)
        const bool hdr_ok = v6 ? (dport == 4789u || dport == 6081u)
                               : tunnel_hdr_ok(dport, byte_at(p.s, 42) | (byte_at(p.s, 43) << 8),
                                               byte_at(p.s, 44) | (byte_at(p.s, 45) << 8));
        if (hdr_ok) {
          if (v6) {
            e.reason = kRecirc6; e.out_port = kPortNone; e.inner_len = p.len - kEncap6Bytes;
            return e;
          }
          const uint32_t vni = (byte_at(p.s, 46) << 16) | (byte_at(p.s, 47) << 8) | byte_at(p.s, 48);
          const int tp = term_lookup(t, raw32_at2(p.s, 26), vni);
          if (tp >= 0) {
            e.reason = kRecirc; e.out_port = (uint32_t)tp; e.inner_len = p.len - kEncapBytes;
            return e;
          }
        }
      }
    }
    // router interface (kPortRouted): IPv4 addressed to the port's own MAC is routed
    if (NFDP_L3_ON && (st.in_flags & kPortRouted) && (p.ipv4 || p.ipv6)) {
      const PortEntry ip = ta.port(st.in_port);
      if (dmac_lo(p.s) == ip.mac_lo && dmac_hi(p.s) == ip.mac_hi) {
        uint32_t op = kPortNone;
        const uint32_t r = p.ipv6 ? route_ipv6(t, p, op) : route_ipv4(t, p, hash, op);
        if (r) { e.reason = r; e.out_port = r == kNoRoute ? kPortPunt : kPortNone; return e; }
        e.out_port = op;
        if (t.vmmac && p.ipv4) vm_mac_map(t, p);
        const uint32_t r2 = finish_port(t, ta, e.out_port, hash, false, e.push, e.tci, p.len, &e.xhdr);
        if (r2) { e.reason = r2; e.out_port = kPortNone; e.xhdr = 0; return e; }
        e.mirror = (st.in_flags & kPortMirror) ? 1u : 0u;
        return e;
      }
    }
    // (bridge, dst MAC) table = OvS `in_port=X,dl_dst=M` / P4 l2_fwd; output == in_port is the
    // OvS hairpin.  A miss falls back to the ingress port's default output (`in_port=X ->
    // output:Y`, priority 10 in ovsdp.go:133-139) or is punted to the slow path.
    // P4 vsi_to_vsi_loopback (K3): the target VSI is the dst MAC's second byte, so those ports
    // look up (bridge, 00:VSI:00:00:00:00).
    const bool vsi_key = (st.in_flags & kPortVsiLookup) != 0;
    const int op = mac_lookup(t, st.bridge, vsi_key ? (dmac_lo(p.s) & 0xFF00u) : dmac_lo(p.s),
                              vsi_key ? 0u : dmac_hi(p.s));
    if (op >= 0) {
      e.out_port = (uint32_t)op;
    } else {
      const PortEntry ip = ta.port(st.in_port < (uint32_t)kMaxPorts ? st.in_port : 0);
      if (ip.flags & kPortHasDefault) {
        e.out_port = ip.default_out;  // OvS in_port=X,actions=output:Y outranks NORMAL
      } else if (st.bridge < t.n_flood && t.flood) {
        // broadcast / multicast / unknown unicast: flood to the bridge's members except the
        // ingress port (OvS NORMAL, ovsdp.go:40-74); the first member carries the frame
        const uint16_t* fg = t.flood + (size_t)st.bridge * kFloodWays;
        uint32_t first = kPortNone;
        for (int j = 0; j < kFloodWays; ++j) {
          const uint32_t m = fg[j];
          if (m >= kFloodLink) break;   // end of the group (or a link: never before two members)
          if (m != st.in_port) { first = m; break; }
        }
        if (first == kPortNone) { e.reason = kNoRoute; e.out_port = kPortNone; return e; }
        e.out_port = first;
        e.flood = st.bridge + 1;
      } else {
        e.out_port = kPortPunt; e.reason = kNoRoute; return e;
      }
    }
    // P4 add_vlan_and_send_to_port (K6): the source port's frames leave with its vid pushed.
    if (st.in_flags & kPortIngressTag) { e.push = 1; e.tci = st.in_ext & 0xFFFu; vlan_done = true; }
  } else {
    e.out_port = act.out_port;
    // nhops + 7 hop opcodes = the chain entry's first 8 bytes, read as one word; hop i is the
    // word shifted right by 8 (i + 1) (a shift, not an index into a private hop[] array, which
    // would live in scratch).  Unrolled by default (NFDP_HOP_UNROLL=0 keeps one copy of the hop
    // dispatch: ~100 fewer SGPR spills, but measured 1-2 % slower).
    const uint64_t hw = ta.chain_word(act.chain_id);
    const uint32_t nh = (uint32_t)(hw & 0xFFu);
#if NFDP_HOP_UNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int i = 0; i < kMaxHops; ++i) {
      if ((uint32_t)i >= nh) break;
      const uint32_t op = (uint32_t)((hw >> (8 * (i + 1))) & 0xFFu);
      if (apply_hop<TA, V6HOPS, XFER>(t, ta, op, i, p, st, act, acl_rule, hash, e, vlan_done)) return e;
    }
  }
  const uint32_t r = finish_port(t, ta, e.out_port, hash, vlan_done, e.push, e.tci, p.len, &e.xhdr);
  if (r) { e.reason = r; e.out_port = kPortNone; e.flood = 0; e.xhdr = 0; return e; }
  e.mirror = (st.in_flags & kPortMirror) ? 1u : 0u;  // mirror_and_send (K9)
  return e;
}

// The rest of a chain on the GPU a kHopXfer handed the frame to (the SFC hop pipeline across
// GPUs).  The frame arrives as the earlier hops left it (`p`, parsed from the handed-over slot);
// `st` carries its ingress port (flags from this GPU's replicated port table) and `act`, `acl_rule`,
// `hash` travel with it from the first GPU.  Hops before `hop0` already ran: their effects on the
// header are in the slot, and what they decided about the egress (the l2fwd / hairpin port, a vlan
// push / pop) is replayed from the chain word, which is the same on every GPU; a route hop's port
// (it depends on the header the route rewrote) comes with the frame, in the resume word's high half.
// Frames of split chains are not mirrored (K9 copies the ingress frame, which stayed on the first GPU).
template <class TA, bool V6HOPS = true>
NFDP_HD EgressDecision resume_stage(const TablesView& t, const TA& ta, Parsed& p, const IngressState& st,
                                    const FlowAction& act, int acl_rule, uint32_t hash, uint32_t resume) {
  const uint32_t hop0 = resume & kHopResumeHopMask;
  EgressDecision e;
  e.out_port = act.out_port; e.reason = st.reason; e.push = 0; e.tci = 0; e.mirror = 0; e.flood = 0;
  e.xhdr = 0; e.inner_len = 0;
  if (e.reason) { e.out_port = kPortNone; return e; }
  bool vlan_done = false;
  const uint64_t hw = ta.chain_word(act.chain_id);
  const uint32_t nh = (uint32_t)(hw & 0xFFu);
  if (hop0 == 0u || hop0 > nh) { e.reason = kChainDrop; e.out_port = kPortNone; return e; }
  for (int i = 0; i < kMaxHops; ++i) {
    if ((uint32_t)i >= nh) break;
    const uint32_t op = (uint32_t)((hw >> (8 * (i + 1))) & 0xFFu);
    if ((uint32_t)i < hop0) {   // replay what the earlier GPU's hops decided about the egress
      if (op == kHopL2Fwd) e.out_port = act.out_port;
      else if (op == kHopHairpin) e.out_port = st.in_port;
      else if (op == kHopVlan) {
        if (act.vlan == 0xFFFFu) { e.push = 0; vlan_done = true; }
        else if (act.vlan) { e.push = 1; e.tci = act.vlan & 0xFFFu; vlan_done = true; }
      } else if (op == kHopRoute) {
        if (!(resume & kHopResumeHasPort)) { e.reason = kChainDrop; e.out_port = kPortNone; return e; }
        e.out_port = resume >> 16;
      }
      continue;
    }
    if (apply_hop<TA, V6HOPS>(t, ta, op, i, p, st, act, acl_rule, hash, e, vlan_done)) return e;
  }
  const uint32_t r = finish_port(t, ta, e.out_port, hash, vlan_done, e.push, e.tci, p.len, &e.xhdr);
  if (r) { e.reason = r; e.out_port = kPortNone; e.xhdr = 0; return e; }
  return e;
}
NFDP_HD EgressDecision chain_stage(const TablesView& t, Parsed& p, const IngressState& st, bool hit,
                                   const FlowAction& act, int acl_rule, uint32_t hash = 0) {
  return chain_stage(t, DirectTables{t}, p, st, hit, act, acl_rule, hash);
}

// A handed-over frame on the GPU that resumes its chain: parse the slot as it stands and take the
// ingress port's flags from this GPU's (replicated) port table.  The ingress checks (VLAN
// isolation, spoof check) ran on the first GPU against the frame as received; they are not
// repeated against the rewritten header.
template <class TA>
NFDP_HD void resume_ingress(const TA& ta, const uint32_t* d, uint32_t inmeta, Parsed& p, IngressState& st) {
  st.in_port = inmeta & 0xFFFFu;
  uint32_t len = inmeta >> 16;
  st.wire_len = len;
  st.reason = kOk;
  if (len < 14 || len > kMaxFrame) { st.reason = kMalformed; len = len < 14 ? 14 : kMaxFrame; }
  parse(d, len, p);
  st.bridge = 0; st.in_flags = 0; st.in_ext = 0;
  if (st.in_port >= (uint32_t)kMaxPorts) {
    st.reason = kBadPort;
  } else {
    const PortEntry pe = ta.port(st.in_port);
    st.in_flags = pe.flags;
    st.in_ext = pe.ext;
  }
  st.key = FlowKey{0u, 0u, 0u, 0u};
}

// The hand-off record of a frame whose chain continues on another GPU (e.reason == kRemote from a
// kHopXfer): the state resume_stage needs there.
NFDP_HD HopState hop_state_of(const Parsed& p, const IngressState& st, const EgressDecision& e, const FlowAction& act,
                              int acl_rule, uint32_t hash) {
  HopState h;
  h.inmeta = st.in_port | (p.len << 16);
  h.hash = hash;
  h.acl_rule = acl_rule;
  h.hop = e.inner_len;
  h.act = act;
  return h;
}
// meta len of a frame: a hand-off carries the frame as it stands (egress_len says 0 for reasons)
NFDP_HD uint32_t out_len(const Parsed& p, const EgressDecision& e) {
  return (e.reason == kRemote && e.inner_len) ? p.len : egress_len(p, e);
}

// Outer headers of a tunnel port for an inner frame of `inner_len` bytes (50 B: Ethernet,
// IPv4 with DF and its checksum, UDP with the entropy source port and checksum 0, VXLAN flags
// 0x08 + VNI or GENEVE 0x6558 + VNI), as 16 LE dwords.
NFDP_HD void make_outer(const TunnelEntry& te, uint32_t inner_len, uint32_t hash, uint32_t* x) {
  // built as dwords (a byte array here went to scratch memory on the GPU: ~30 private loads and
  // stores per packet in the side pass, r5 s32)
  auto bs16 = [](uint32_t v) { return ((v >> 8) & 0xFFu) | ((v & 0xFFu) << 8); };   // 16-bit byte swap
  const uint32_t tl = 20u + 8u + 8u + inner_len, ul = 8u + 8u + inner_len;
  const uint32_t sp = te.sport ? (uint32_t)te.sport : bs16(0xC000u | (hash & 0x3FFFu));   // raw (wire order)
  // IPv4 header checksum over the 16-bit big-endian words of bytes 14..33 (its own field 0)
  uint32_t c = 0x4500u + (tl & 0xFFFFu) + 0x4000u + 0x4011u + bs16(te.src_ip & 0xFFFFu) + bs16(te.src_ip >> 16) +
               bs16(te.dst_ip & 0xFFFFu) + bs16(te.dst_ip >> 16);
  c = (c & 0xFFFFu) + (c >> 16);
  c = (c & 0xFFFFu) + (c >> 16);
  const uint32_t ck = bs16(~c & 0xFFFFu);
  const bool gen = te.type == kTunGeneve;
  x[0] = te.dmac_lo;
  x[1] = (uint32_t)te.dmac_hi | (te.smac_lo << 16);
  x[2] = (te.smac_lo >> 16) | ((uint32_t)te.smac_hi << 16);
  x[3] = 0x00450008u;                                   // EtherType 0x0800, version / IHL 0x45, TOS 0
  x[4] = bs16(tl & 0xFFFFu);                            // total length, id 0
  x[5] = 0x11400040u;                                   // DF, TTL 64, protocol UDP
  x[6] = ck | ((te.src_ip & 0xFFFFu) << 16);
  x[7] = (te.src_ip >> 16) | ((te.dst_ip & 0xFFFFu) << 16);
  x[8] = (te.dst_ip >> 16) | (sp << 16);
  x[9] = (uint32_t)te.dport | (bs16(ul & 0xFFFFu) << 16);
  x[10] = gen ? 0u : 0x00080000u;                       // UDP checksum 0; VXLAN flags 0x08
  x[11] = (gen ? 0x5865u : 0u) | (((te.vni >> 16) & 0xFFu) << 16) | (((te.vni >> 8) & 0xFFu) << 24);   // GENEVE 0x6558
  x[12] = te.vni & 0xFFu;
  for (int i = 13; i < kSlotDwords; ++i) x[i] = 0u;
}

// IPv6-underlay outer headers (70 B: Ethernet, IPv6 with next header UDP, UDP with the entropy
// source port and a zero checksum as RFC 6935 / 6936 allow for tunnel encapsulations, VXLAN or
// GENEVE + VNI).  The flow label is the entry's or, if 0, 20 bits of the packet hash (RFC 6438).
// `x` holds kXhdrBytes / 4 LE dwords.
NFDP_HD void make_outer6(const Tunnel6Entry& te, uint32_t inner_len, uint32_t hash, uint32_t* x) {
  // built as dwords, like make_outer (no byte array: scratch memory on the GPU)
  auto bs16 = [](uint32_t v) { return ((v >> 8) & 0xFFu) | ((v & 0xFFu) << 8); };
  const uint32_t fl = (te.tc_flow & 0xFFFFFu) ? (te.tc_flow & 0xFFFFFu) : (hash & 0xFFFFFu);
  const uint32_t vtf = (6u << 28) | (((te.tc_flow >> 20) & 0xFFu) << 20) | fl;
  const uint32_t ul = (8u + 8u + inner_len) & 0xFFFFu;
  const uint32_t hl = (te.hop_limit & 0xFFu) ? (te.hop_limit & 0xFFu) : 64u;
  const uint32_t sp = te.sport ? (uint32_t)te.sport : bs16(0xC000u | (hash & 0x3FFFu));
  const bool gen = te.type == kTunGeneve;
  x[0] = te.dmac_lo;
  x[1] = (uint32_t)te.dmac_hi | (te.smac_lo << 16);
  x[2] = (te.smac_lo >> 16) | ((uint32_t)te.smac_hi << 16);
  x[3] = 0xDD86u | (bs16(vtf >> 16) << 16);             // EtherType 0x86DD, version / class / label
  x[4] = bs16(vtf & 0xFFFFu) | (bs16(ul) << 16);        // payload length
  x[5] = 17u | (hl << 8) | ((te.src[0] & 0xFFFFu) << 16);
  for (int k = 0; k < 3; ++k) x[6 + k] = (te.src[k] >> 16) | ((te.src[k + 1] & 0xFFFFu) << 16);
  x[9] = (te.src[3] >> 16) | ((te.dst[0] & 0xFFFFu) << 16);
  for (int k = 0; k < 3; ++k) x[10 + k] = (te.dst[k] >> 16) | ((te.dst[k + 1] & 0xFFFFu) << 16);
  x[13] = (te.dst[3] >> 16) | (sp << 16);
  x[14] = (uint32_t)te.dport | (bs16(ul) << 16);
  x[15] = gen ? 0u : 0x00080000u;                       // UDP checksum 0 (RFC 6935); VXLAN flags 0x08
  x[16] = (gen ? 0x5865u : 0u) | (((te.vni >> 16) & 0xFFu) << 16) | (((te.vni >> 8) & 0xFFu) << 24);
  x[17] = te.vni & 0xFFu;
  for (int i = 18; i < kXhdrBytes / 4; ++i) x[i] = 0u;
}

// Side outputs: flood replicas, the K9 mirror copy, the ARP slow-path copy and MAC-learn events.
// The per-packet kernels only FLAG the packets that need them (side_needed -> the packet's index
// is appended to a side list; a flooded frame's primary copy carries kMetaFlood) and a separate
// pass (side_stage: side_kernel on the GPU, sequential in the oracle) emits them from the
// packet's input slot + ingress meta and its output slot + egress meta.  The hot kernel keeps its
// register budget; replicas are rare (flooding, mirroring, ARP-trap and learning ports only).
// `Sink` provides rep(hdr, meta, src), learn(bridge, lo, hi, port) and xhdr(hdr, src) (the
// tunnel outer-header record of packet src).  Every replica follows the
// out_tail() rule against its source packet's input frame.
NFDP_HD bool side_needed(const IngressState& st, const Parsed& p, const EgressDecision& e) {
  return (!e.reason && (e.flood || e.mirror || e.xhdr)) ||
         (!st.reason && ((st.in_flags & kPortLearn) || (p.arp && (st.in_flags & kPortArpTrap))));
}

// The packet hash of the side pass (tunnel entropy port, flood LAG members): the Toeplitz hash of
// the ingress key, bit by bit (the oracle) or from byte tables (side_kernel: LDS copies).
struct ScalarToeplitz {
  const uint8_t* rss_key;
  NFDP_HD uint32_t operator()(const FlowKey& k) const { return toeplitz_scalar(k, rss_key); }
};

template <class TA, class Sink, class Hash = ScalarToeplitz>
NFDP_HD void side_stage(const TablesView& t, const TA& ta, const uint32_t* d_in, uint32_t inmeta, const uint32_t* o,
                        uint32_t ometa, uint32_t src, Sink& sink, Hash hasher = Hash{nullptr}) {
  Parsed p;
  IngressState st;
  ingress_stage(t, ta, d_in, inmeta, p, st);
  if (st.reason) return;
  auto khash = [&]() -> uint32_t {
    if constexpr (std::is_same<Hash, ScalarToeplitz>::value) return toeplitz_scalar(st.key, t.rss_key);
    else return hasher(st.key);
  };
  // MAC learning (OvS NORMAL): (bridge, src MAC) -> in_port when the table disagrees
  if (st.in_flags & kPortLearn) {
    const uint32_t lo = smac_lo(p.s), hi = smac_hi(p.s);
    if (!(lo & 1u) && mac_lookup(t, st.bridge, lo, hi) != (int)st.in_port) sink.learn(st.bridge, lo, hi, st.in_port);
  }
  // ARP to the slow path (P4 always_trap_arp_table): the ingress frame, punted
  if (p.arp && (st.in_flags & kPortArpTrap)) sink.rep(d_in, make_meta(kPortPunt, st.wire_len, kArpTrap), src);
  if (meta_reason(ometa)) return;
  // tunnel encap: the outer Ethernet / IPv4|IPv6 / UDP / VXLAN|GENEVE header record of this packet
  if (ometa & kMetaXhdr) {
    const uint32_t tp = meta_port(ometa);
    if (tp < (uint32_t)kMaxPorts) {
      const PortEntry pe = ta.port(tp);
      uint32_t x[kXhdrBytes / 4];
      if ((pe.flags & kPortTunnel) && (pe.flags & kPortTunnel6)) {
        if (t.tunnels6 && pe.lag < t.n_tunnels6) {
          make_outer6(t.tunnels6[pe.lag], meta_len(ometa) - kEncap6Bytes, khash(), x);
          sink.xhdr(x, src, (kEncap6Bytes + 15) / 16);
        }
      } else if ((pe.flags & kPortTunnel) && t.tunnels && pe.lag < t.n_tunnels) {
        for (int i = kSlotDwords; i < kXhdrBytes / 4; ++i) x[i] = 0;
        make_outer(t.tunnels[pe.lag], meta_len(ometa) - kEncapBytes, khash(), x);
        sink.xhdr(x, src, (kEncapBytes + 15) / 16);
      }
    }
  }
  // mirror_and_send (K9): the frame as it leaves, also to the ingress port's mirror port
  if (st.in_flags & kPortMirror) {
    const uint32_t mp = st.in_ext >> 16;
    if (mp < (uint32_t)kMaxPorts && port_can_egress(ta.port(mp).flags)) sink.rep(o, make_meta(mp, meta_len(ometa), kOk), src);
  }
  // flood: one replica per further member of the bridge's group (the frame itself went to the
  // first member).  Flooding happens on the L2 path only, where no NF rewrote the frame, so the
  // re-parsed ingress frame is what every member gets (plus its own egress tag).
  if ((ometa & kMetaFlood) && t.flood && st.bridge < t.n_flood) {
    const uint16_t* fg = t.flood + (size_t)st.bridge * kFloodWays;
    bool first = true;
    uint32_t hops = 0;   // rows followed (bounded: a corrupt chain cannot loop forever)
    for (int j = 0; j < kFloodWays; ++j) {
      uint32_t m = fg[j];
      if (m == kPortNone) break;
      if (m >= kFloodLink) {        // overflow row of a group beyond 15 members
        const uint32_t row = m - kFloodLink;
        if (row >= kFloodMaxRows || ++hops > kFloodMaxRows) break;
        fg = t.flood + (size_t)row * kFloodWays;
        j = -1;
        continue;
      }
      if (m == st.in_port) continue;
      if (first) { first = false; continue; }
      uint32_t push = (st.in_flags & kPortIngressTag) ? 1u : 0u;
      uint32_t tci = push ? (st.in_ext & 0xFFFu) : 0u;
      uint32_t xh = 0;  // tunnel members are not flooded: remote MACs come from l2_to_tunnel entries
      if (finish_port(t, ta, m, khash(), push != 0, push, tci, p.len, &xh) != kOk || xh)
        continue;
      uint32_t c[kSlotDwords];
      emit(p, tci, push != 0, c);
      sink.rep(c, make_meta(m, p.len + (push ? 4u : 0u), kOk), src);
    }
  }
}

// Counter record helpers: packed (pkts << 40) | bytes in one 64-bit word so a packet costs a
// single atomic.  The control plane harvests (read + reset) well before 2^24 packets.
NFDP_HD uint64_t ctr_inc(uint32_t bytes) { return (1ull << 40) | (uint64_t)bytes; }

}  // namespace nfdp
