// pipeline.h — scalar per-packet stages shared by the GPU kernels and the CPU oracle.
//
// Stage order (one packet):
//   ingress_stage : port lookup, VLAN isolation (K10), spoof-check, bridge-id (K7), FlowKey
//   [hash + ACL   : done by the caller — MFMA on the GPU, scalar in the oracle]
//   flow lookup   : exact match, 2-choice bucketized cuckoo (1M+ flows)
//   chain_stage   : built-in NF hops (ACL verdict, SNAT, TTL, L2 steer, VLAN, hairpin) or the
//                   (bridge, dst-MAC) L2 table on a flow miss (K5); egress port tagging (K6)
#pragma once
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

template <class TA>
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
    if (!(pe.flags & kPortValid)) st.reason = st.reason ? st.reason : kBadPort;
    const uint32_t vid = p.tci & 0xFFFu;
    if ((pe.flags & kPortVlanIsolate) && p.tagged && vid != pe.vlan)
      st.reason = st.reason ? st.reason : kVlanDrop;
    if ((pe.flags & kPortSpoofChk) &&
        (smac_lo(p.s) != pe.mac_lo || smac_hi(p.s) != pe.mac_hi))
      st.reason = st.reason ? st.reason : kSpoof;
    st.bridge = ((pe.flags & kPortVlanBridge) && p.tagged) ? vid : pe.bridge_id;
  }
  st.key = make_key(p, st.bridge);
}
NFDP_HD void ingress_stage(const TablesView& t, const uint32_t* d, uint32_t inmeta, Parsed& p, IngressState& st) {
  ingress_stage(t, DirectTables{t}, d, inmeta, p, st);
}

struct EgressDecision {
  uint32_t out_port;
  uint32_t reason;
  uint32_t push;      // 1 -> insert an 802.1Q tag with `tci`
  uint32_t tci;
  uint32_t mirror;    // 1 -> the ingress frame is also copied to the ingress port's mirror port (K9)
  uint32_t flood;     // bridge + 1 when the frame is flooded: out_port is the group's first member,
                      // side_stage emits a replica per further member
};

// Final egress checks on a chosen port: LAG member (K8), validity, egress tag (K6), MTU.
// Returns a drop reason (0 = ok); `port`/`push`/`tci` are updated in place.
template <class TA>
NFDP_HD uint32_t finish_port(const TablesView& t, const TA& ta, uint32_t& port, uint32_t hash, bool vlan_done,
                             uint32_t& push, uint32_t& tci, uint32_t l2len) {
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
  if (!(pe.flags & kPortValid)) return kBadPort;
  if (!vlan_done && (pe.flags & kPortTagEgress) && pe.vlan) { push = 1; tci = pe.vlan & 0xFFFu; }
  // l2len is untagged: the L3 size is l2len - 14 whatever the tagging
  if (l2len + (push ? 4u : 0u) > kMaxFrame || (pe.mtu && l2len - 14u > pe.mtu)) return kTooBig;
  return kOk;
}

// `hit`: flow entry found; `act`: its action; `acl_rule`: first matching ACL rule or -1;
// `hash`: the packet's Toeplitz hash (LAG member selection uses hash[2:0], K8).
template <class TA>
NFDP_HD EgressDecision chain_stage(const TablesView& t, const TA& ta, Parsed& p, const IngressState& st,
                                   bool hit, const FlowAction& act, int acl_rule, uint32_t hash) {
  EgressDecision e;
  e.out_port = kPortNone; e.reason = st.reason; e.push = 0; e.tci = 0; e.mirror = 0; e.flood = 0;
  if (e.reason) return e;
  bool vlan_done = false;
  if (!hit) {
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
          if (m == kPortNone) break;
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
    // nhops + 7 hop opcodes = the chain entry's first 8 bytes, read as one word and decoded with
    // compile-time shifts (indexing a private hop[] array at run time would spill to scratch).
    const uint64_t hw = ta.chain_word(act.chain_id);
    const uint32_t nh = (uint32_t)(hw & 0xFFu);
#pragma unroll
    for (int i = 0; i < kMaxHops; ++i) {
      if ((uint32_t)i >= nh) break;
      const uint8_t op = (uint8_t)((hw >> (8 * (i + 1))) & 0xFFu);
      if (op == kHopAcl) {
        if (!ta.permit(acl_rule)) { e.reason = kAclDeny; e.out_port = kPortNone; return e; }
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
        if (p.ipv4 && !act_ttl(p)) { e.reason = kTtlExpired; e.out_port = kPortNone; return e; }
      } else if (op == kHopHairpin) {
        e.out_port = st.in_port;
        const uint32_t dl = dmac_lo(p.s), dh = dmac_hi(p.s);
        set_dmac(p.s, smac_lo(p.s), smac_hi(p.s));
        set_smac(p.s, dl, dh);
      } else if (op == kHopVlan) {
        if (act.vlan == 0xFFFFu) { e.push = 0; vlan_done = true; }
        else if (act.vlan) { e.push = 1; e.tci = act.vlan & 0xFFFu; vlan_done = true; }
      } else if (op == kHopDrop) {
        e.reason = kChainDrop; e.out_port = kPortNone; return e;
      } else if (op == kHopPunt) {
        e.reason = kNoRoute; e.out_port = kPortPunt; return e;
      }
    }
  }
  const uint32_t r = finish_port(t, ta, e.out_port, hash, vlan_done, e.push, e.tci, p.len);
  if (r) { e.reason = r; e.out_port = kPortNone; e.flood = 0; return e; }
  e.mirror = (st.in_flags & kPortMirror) ? 1u : 0u;  // mirror_and_send (K9)
  return e;
}
NFDP_HD EgressDecision chain_stage(const TablesView& t, Parsed& p, const IngressState& st, bool hit,
                                   const FlowAction& act, int acl_rule, uint32_t hash = 0) {
  return chain_stage(t, DirectTables{t}, p, st, hit, act, acl_rule, hash);
}

// Side outputs: flood replicas, the K9 mirror copy, the ARP slow-path copy and MAC-learn events.
// The per-packet kernels only FLAG the packets that need them (side_needed -> the packet's index
// is appended to a side list; a flooded frame's primary copy carries kMetaFlood) and a separate
// pass (side_stage: side_kernel on the GPU, sequential in the oracle) emits them from the
// packet's input slot + ingress meta and its output slot + egress meta.  The hot kernel keeps its
// register budget; replicas are rare (flooding, mirroring, ARP-trap and learning ports only).
// `Sink` provides rep(hdr, meta, src) and learn(bridge, lo, hi, port).  Every replica follows the
// out_tail() rule against its source packet's input frame.
NFDP_HD bool side_needed(const IngressState& st, const Parsed& p, const EgressDecision& e) {
  return (!e.reason && (e.flood || e.mirror)) ||
         (!st.reason && ((st.in_flags & kPortLearn) || (p.arp && (st.in_flags & kPortArpTrap))));
}

template <class TA, class Sink>
NFDP_HD void side_stage(const TablesView& t, const TA& ta, const uint32_t* d_in, uint32_t inmeta, const uint32_t* o,
                        uint32_t ometa, uint32_t src, Sink& sink) {
  Parsed p;
  IngressState st;
  ingress_stage(t, ta, d_in, inmeta, p, st);
  if (st.reason) return;
  // MAC learning (OvS NORMAL): (bridge, src MAC) -> in_port when the table disagrees
  if (st.in_flags & kPortLearn) {
    const uint32_t lo = smac_lo(p.s), hi = smac_hi(p.s);
    if (!(lo & 1u) && mac_lookup(t, st.bridge, lo, hi) != (int)st.in_port) sink.learn(st.bridge, lo, hi, st.in_port);
  }
  // ARP to the slow path (P4 always_trap_arp_table): the ingress frame, punted
  if (p.arp && (st.in_flags & kPortArpTrap)) sink.rep(d_in, make_meta(kPortPunt, st.wire_len, kArpTrap), src);
  if (meta_reason(ometa)) return;
  // mirror_and_send (K9): the frame as it leaves, also to the ingress port's mirror port
  if (st.in_flags & kPortMirror) {
    const uint32_t mp = st.in_ext >> 16;
    if (mp < (uint32_t)kMaxPorts && (ta.port(mp).flags & kPortValid)) sink.rep(o, make_meta(mp, meta_len(ometa), kOk), src);
  }
  // flood: one replica per further member of the bridge's group (the frame itself went to the
  // first member).  Flooding happens on the L2 path only, where no NF rewrote the frame, so the
  // re-parsed ingress frame is what every member gets (plus its own egress tag).
  if ((ometa & kMetaFlood) && t.flood && st.bridge < t.n_flood) {
    const uint16_t* fg = t.flood + (size_t)st.bridge * kFloodWays;
    bool first = true;
    for (int j = 0; j < kFloodWays; ++j) {
      uint32_t m = fg[j];
      if (m == kPortNone) break;
      if (m == st.in_port) continue;
      if (first) { first = false; continue; }
      uint32_t push = (st.in_flags & kPortIngressTag) ? 1u : 0u;
      uint32_t tci = push ? (st.in_ext & 0xFFFu) : 0u;
      if (finish_port(t, ta, m, toeplitz_scalar(st.key, t.rss_key), push != 0, push, tci, p.len) != kOk) continue;
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
