// nfdp.h — MI355X network-function data plane: shared types + scalar per-packet logic.
//
// This header is compiled only by hipcc (one toolchain, gfx950 only).  Everything here is
// `__host__ __device__` so the same per-packet semantics run inside the GPU kernels
// (kernels.hip) and inside the scalar CPU oracle (oracle.cpp) that the tests use to check the
// GPU bit-exactly.
//
// What it replaces in the reference (Ximinhan/dpu-operator): the per-packet behaviour the
// reference *configures* in DPU silicon / OvS but never executes itself:
//   * VF VLAN isolation / spoof-check (intel-netsec/main.go:432-503, vspnetutils.go:249-258)
//   * source-port / bridge-id classification (p4rtclient.go:242-256, 674-691)
//   * (bridge, dst-MAC) L2 forwarding (p4rtclient.go:565-571; p4info.txt:600-692)
//   * VLAN push/pop on the way to/from a host VF (p4rtclient.go:553-564)
//   * OvS steering / hairpin used for SFC hops (ovsdp.go:113-142, marvell/main.go:490-563)
// plus exact-match 5-tuple flow state (1M+ flows, sharded across GPUs) and built-in NFs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NFDP_HD __host__ __device__ __forceinline__
#ifndef NFDP_IPV6
#define NFDP_IPV6 1
#endif

namespace nfdp {

// ----------------------------------------------------------------------------------------
// Constants
// ----------------------------------------------------------------------------------------
constexpr int kSlotBytes = 64;         // header slot in HBM: the first min(len, 64) bytes of a frame
constexpr int kSlotDwords = kSlotBytes / 4;
constexpr uint32_t kMaxFrame = 9600;   // longest L2 frame (jumbo 9216 + tags); 14-bit length fields
constexpr int kFloodWays = 16;         // entries per flood-group row (bridge head row or overflow row)
// A flood-group entry >= kFloodLink (and != kPortNone) links to overflow row (entry - kFloodLink)
// of the same table: groups of any size are chains of 16-entry rows, 15 members + a link each.
// The host keeps a group's first two members in its head row, so the hot kernel's first-member
// search never follows a link; the side pass walks the whole chain.
constexpr uint16_t kFloodLink = 0x8000;
constexpr uint32_t kFloodMaxRows = 0x7000;   // link targets (rows) below this
constexpr int kMaxPorts = 4094;        // vport table rows (VF / NF / wire / PR ports); 4094/4095 = meta sentinels
constexpr int kBucketSlots = 4;        // flow-table bucket = 4 x {key, action} = one 128-B line
constexpr uint32_t kSlotUsed = 0x100u; // occupied marker, stored in FlowKey.meta byte 1
constexpr uint32_t kKeyV6 = 0x200u;    // FlowKey.meta: an IPv6 key (folded addresses, see make_key)
constexpr uint16_t kPortNone = 0xFFFF; // dropped
constexpr uint16_t kPortPunt = 0xFFFE; // to slow path (control plane upcall)
constexpr uint32_t kPortCont = 0xFFFDu; // in-meta port of the continuation slot of a wide header pair
// (kMaxPorts real ports; the 12-bit egress meta port field keeps 0xFFF / 0xFFE for none / punt)
constexpr int kMaxHops = 7;
constexpr int kAclKeyBits = 128;       // ACL / hash key = the 16-byte FlowKey

// drop / disposition reasons (meta bits 24..31)
enum Reason : uint32_t {
  kOk = 0,
  kBadPort = 1,
  kVlanDrop = 2,
  kSpoof = 3,
  kAclDeny = 4,
  kNoRoute = 5,  // punted to slow path (flow miss + MAC miss)
  kTooBig = 6,
  kChainDrop = 7,
  kTtlExpired = 8,
  kMalformed = 9,
  kRemote = 10,    // not a drop: handed to the egress GPU over xGMI (multi-GPU path), or the rest of
                   // its chain runs on another GPU (kHopXfer: port = that GPU's plane, len = frame length)
  kOverflow = 11,  // exchange segment full (multi-GPU path)
  kArpTrap = 12,   // ARP copy trapped to the slow path (P4 always_trap_arp_table)
  kRecirc = 13,    // tunnel terminated: recirculate frame[len - olen:] with in_port = meta port (decap)
  kRecirc6 = 14,   // IPv6-underlay VXLAN / GENEVE to the local VTEP: the VNI lies past the header slot, so
                   // the I/O layer finishes ipv6_tunnel_term_table on the whole frame (decap, recirculate)
  kCont = 15,      // continuation slot of a wide (128-B) header pair (pipeline.h decap_pair): not a
                   // frame; its meta's port field = bytes the head's egress strips from the head's
                   // input frame (0: not terminated), len field = valid bytes of the head's out slot
  kNumReasons = 16,
};

// port flags
enum PortFlags : uint32_t {
  kPortValid = 1u << 0,
  kPortSpoofChk = 1u << 1,      // src MAC must equal port MAC (sriov spoofchk)
  kPortVlanIsolate = 1u << 2,   // tagged ingress must carry port.vlan (K10)
  kPortTagEgress = 1u << 3,     // push port.vlan on egress (K6 vlan_push to host VF)
  kPortVlanBridge = 1u << 4,    // ingress vid selects bridge id (K7)
  kPortTrust = 1u << 5,
  kPortHasDefault = 1u << 6,    // L2 miss -> default_out instead of punt (OvS in_port=X,actions=output:Y)
  kPortIngressTag = 1u << 7,    // frames from this port leave tagged with ext[11:0] (K6 add_vlan_and_send)
  kPortMirror = 1u << 8,        // forwarded frames from this port are also copied to ext[31:16] (K9)
  kPortLag = 1u << 9,           // egress to this port picks a LAG member by hash[2:0] (K8)
  kPortVsiLookup = 1u << 10,    // L2 lookup keys on the target VSI (dst MAC byte 1) only (K3)
  kPortLearn = 1u << 11,        // (bridge, src MAC) -> in_port is learned from this port's frames (OvS NORMAL)
  kPortArpTrap = 1u << 12,      // ARP frames from this port are also copied to the slow path
  kPortRouted = 1u << 13,       // router interface: IPv4 to this port's MAC is routed (LPM) on a flow miss
  kPortTunnel = 1u << 14,       // egress via this port = VXLAN / GENEVE encap with tunnel[lag] (OvS tunnel port)
  kPortVtep = 1u << 15,         // underlay port: UDP 4789 / 6081 to ext (local VTEP IPv4) is terminated
  kPortRxOff = 1u << 16,        // ctrl-net RX_STATE down: the function takes no frames (egress dropped)
  kPortLinkDown = 1u << 17,     // ctrl-net LINK_STATUS down / DEV_REMOVE: neither receives nor sends
  kPortTunnel6 = 1u << 18,      // with kPortTunnel: IPv6 underlay, the tunnel is tunnels6[lag]
};

constexpr int kLagWays = 8;                 // members per LAG group (hash[2:0])

// chain hop opcodes (built-in GPU network functions)
enum Hop : uint8_t {
  kHopNone = 0,
  kHopAcl = 1,      // stateless firewall: TCAM (priority/ternary) on the ingress FlowKey
  kHopNat = 2,      // SNAT: rewrite src ip/port from the flow entry, incremental checksums
  kHopL2Fwd = 3,    // steer to flow.out_port, rewrite MACs to the egress port's (mac, peer_mac)
  kHopTtl = 4,      // router hop: TTL-1, checksum
  kHopHairpin = 5,  // bounce back out of the ingress port, swap MACs (OvS in_port action)
  kHopVlan = 6,     // push (1..4094) / pop (0xFFFF) flow.vlan
  kHopDrop = 7,
  kHopPunt = 8,
  kHopRoute = 9,    // IPv4 LPM (ipv4_table) -> nexthop / ECMP group -> MACs, port; TTL - 1
  kHopXfer = 0x10,  // | plane (0..15): the rest of the chain runs on that GPU (pipeline.h resume_stage)
};
constexpr uint32_t kHopXferPlanes = 0xFu;

// ----------------------------------------------------------------------------------------
// Tables (all POD, 16-B aligned so the kernels use dwordx4 accesses)
// ----------------------------------------------------------------------------------------
struct alignas(16) PortEntry {   // 32 B
  uint32_t flags;
  uint16_t vlan;                 // VF vlan (vf+2 in the reference's convention)
  uint16_t bridge_id;
  uint32_t mac_lo;               // this port's MAC (raw network-order bytes 0..3)
  uint16_t mac_hi;               //                  bytes 4..5
  uint16_t gpu;                  // owning GPU rank (egress side)
  uint32_t peer_mac_lo;          // MAC of whatever is attached (pod / NF / next hop)
  uint16_t peer_mac_hi;
  uint16_t default_out;          // with kPortHasDefault: egress port on an L2 (flow + MAC) miss
  uint32_t ext;                  // [11:0] ingress-push vid (kPortIngressTag); [31:16] mirror port (kPortMirror)
  uint16_t lag;                  // LAG group index (kPortLag)
  uint16_t mtu;                  // egress MTU in L3 bytes (frame - 14, untagged); 0 = kMaxFrame only
};
static_assert(sizeof(PortEntry) == 32, "PortEntry");

struct alignas(16) FlowKey {     // 16 B; also the ACL / Toeplitz input (128 bits)
  uint32_t src_ip;               // raw network-order bytes (little-endian load of the header)
  uint32_t dst_ip;               // (IPv6: fold6 of the four raw address words)
  uint32_t ports;                // sport (raw) | dport (raw) << 16
  uint32_t meta;                 // proto | (zone << 16) [| kKeyV6]; kSlotUsed never set in a packet key
};
static_assert(sizeof(FlowKey) == 16, "FlowKey");

struct alignas(16) FlowAction {  // 16 B value of an exact-match flow entry
  uint16_t chain_id;             // index into the chain table
  uint16_t out_port;             // egress vport
  uint32_t nat_ip;               // raw network order (used by kHopNat)
  uint16_t nat_port;             // raw network order
  uint16_t vlan;                 // used by kHopVlan: 0 none, 1..4094 push, 0xFFFF pop
  uint32_t flow_id;              // stable id (control plane bookkeeping)
};
static_assert(sizeof(FlowAction) == 16, "FlowAction");

// One flow-table slot: key (meta |= kSlotUsed when occupied) + action.  A bucket is 4 slots =
// 128 B = one cache line, so a probe is ONE line fetch (the tag-row + key + value design needed
// three dependent fetches).
struct alignas(16) FlowSlot {
  FlowKey key;
  FlowAction act;
};
static_assert(sizeof(FlowSlot) == 32, "FlowSlot");

struct alignas(16) ChainEntry {  // 16 B
  uint8_t nhops;
  uint8_t hop[kMaxHops];
  uint16_t acl_id;
  uint16_t flags;
  uint32_t pad;
};
static_assert(sizeof(ChainEntry) == 16, "ChainEntry");

struct alignas(16) MacEntry {    // 16 B, (bridge, dst-mac) -> port  (K5)
  uint32_t mac_lo;
  uint16_t mac_hi;
  uint16_t bridge_id;
  uint16_t out_port;
  uint16_t valid;                // kMacEmpty / kMacStatic / kMacTomb / kMacLearned (kMacClaim while inserting)
  uint32_t stamp;                // learned entries: last-seen stamp (host aging); static: 0
};
enum MacValid : uint16_t { kMacEmpty = 0, kMacStatic = 1, kMacTomb = 2, kMacLearned = 3, kMacClaim = 0xFFFF };
static_assert(sizeof(MacEntry) == 16, "MacEntry");

// ---- L3 (P4 ipv4_table + nexthop_table + ecmp_hash_table + rif_mod_table) ----
// IPv4 LPM as DIR-24-8: tbl24[dst >> 8] is a result or (kLpmExt | g) = tbl8 group g, whose
// entry [dst & 0xFF] is the result.  Result: 0 = no route; kind[29:28] 1 = nexthop, 2 = ECMP
// group; id[15:0] (bit 31 stays free for the tbl24 extension flag).
constexpr uint32_t kLpmExt = 1u << 31;
constexpr uint32_t kRouteNh = 1u << 28, kRouteEcmp = 2u << 28;
constexpr int kEcmpWays = 8;            // members per ECMP group, selected by hash[2:0]
struct alignas(16) NextHop {     // 16 B
  uint32_t dmac_lo;              // neighbour MAC (raw bytes 0..3)
  uint16_t dmac_hi;
  uint16_t port;                 // egress port (a LAG / tunnel port resolves further)
  uint32_t smac_lo;              // router interface MAC (rif_mod_table)
  uint16_t smac_hi;
  uint16_t valid;
};
static_assert(sizeof(NextHop) == 16, "NextHop");

// ---- tunnels (VXLAN / GENEVE, IPv4 underlay) ----
enum TunnelType : uint16_t { kTunVxlan = 1, kTunGeneve = 2 };
struct alignas(16) TunnelEntry { // 32 B: the outer headers of one tunnel port
  uint32_t src_ip, dst_ip;       // raw (network order) underlay addresses
  uint16_t sport;                // raw; 0 = 0xC000 | hash (entropy, RFC 7348)
  uint16_t dport;                // raw (4789 / 6081)
  uint32_t vni;                  // host order, 24 bits
  uint32_t smac_lo; uint16_t smac_hi;
  uint16_t out_port;             // underlay port the encapsulated frame leaves on
  uint32_t dmac_lo; uint16_t dmac_hi;
  uint16_t type;                 // TunnelType
};
static_assert(sizeof(TunnelEntry) == 32, "TunnelEntry");
struct alignas(16) Tunnel6Entry { // 64 B: IPv6-underlay tunnel (P4 vxlan / geneve_encap_v6_mod_table)
  uint32_t src[4], dst[4];       // raw (network order) underlay addresses
  uint16_t sport;                // raw; 0 = 0xC000 | hash
  uint16_t dport;                // raw
  uint32_t vni;                  // host order, 24 bits
  uint32_t smac_lo; uint16_t smac_hi;
  uint16_t out_port;
  uint32_t dmac_lo; uint16_t dmac_hi;
  uint16_t type;                 // TunnelType
  uint32_t tc_flow;              // traffic class [27:20] | flow label [19:0] (0 = hash-derived label)
  uint32_t hop_limit;            // [7:0] (0 = 64)
};
static_assert(sizeof(Tunnel6Entry) == 64, "Tunnel6Entry");
struct alignas(16) TermEntry {   // 16 B: (outer src ip, vni) -> tunnel port (ipv4_tunnel_term_table)
  uint32_t src_ip;               // raw
  uint32_t vni;
  uint16_t port;
  uint16_t valid;
  uint32_t pad;
};
static_assert(sizeof(TermEntry) == 16, "TermEntry");
struct alignas(16) Term6Entry {  // 32 B: (outer IPv6 src, vni) -> tunnel port (ipv6_tunnel_term_table)
  uint32_t src[4];               // raw words (network-order bytes, little-endian loads)
  uint32_t vni;
  uint16_t port;
  uint16_t valid;
  uint32_t pad[2];
};
static_assert(sizeof(Term6Entry) == 32, "Term6Entry");
// VM IPv4 -> MAC maps (P4 vm_src_ip4_mac_map_table / vm_dst_ip4_mac_map_table): a routed
// packet from a mapped source gets that source MAC, one to a mapped destination that
// destination MAC.  Open addressing over (ip, kind); kind 0 = empty slot.
constexpr uint32_t kVmMacSrc = 1, kVmMacDst = 2;
struct alignas(16) VmMacEntry {  // 16 B
  uint32_t ip;                   // raw (network byte order as loaded)
  uint32_t kind;                 // kVmMacSrc | kVmMacDst, 0 = empty
  uint32_t mac_lo, mac_hi;       // set_smac / set_dmac operands
};
static_assert(sizeof(VmMacEntry) == 16, "VmMacEntry");
constexpr int kVmMacProbe = 8;

// Hand-off record of a split chain (kHopXfer, the SFC hop pipeline across GPUs): what the GPU that
// runs the rest of the chain needs besides the 64-B header slot as the earlier hops left it.
struct alignas(16) HopState {    // 32 B
  uint32_t inmeta;               // in_port | frame length << 16 (the frame as handed over)
  uint32_t hash;                 // the packet's Toeplitz hash (LAG members, ECMP)
  int32_t acl_rule;              // first matching ACL rule (-1: none), for acl hops after the split
  uint32_t hop;                  // the hop the chain resumes at
  FlowAction act;                // the flow's action (chain id, out port, NAT, vlan)
};
static_assert(sizeof(HopState) == 32, "HopState");

// Verdict returned by the flow owner to the ingress GPU (multi-GPU path).
struct alignas(16) Verdict {     // 16 B
  uint16_t chain_id;
  uint16_t out_port;
  uint32_t nat_ip;
  uint16_t nat_port;
  uint16_t vlan;
  uint32_t status;               // 1 = hit, 0 = miss
};
static_assert(sizeof(Verdict) == 16, "Verdict");

// ----------------------------------------------------------------------------------------
// Hashing
// ----------------------------------------------------------------------------------------
NFDP_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}

// IPv6 address -> one 32-bit FlowKey word (raw words, a0 = bytes 0..3).  Nested fmix32 so no
// word enters linearly; lookups stay exact through the flow6 side array (flow6_verify).
NFDP_HD uint32_t fold6(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  return fmix32(a0 ^ fmix32(a1 ^ fmix32(a2 ^ fmix32(a3 ^ 0x6b43a9b5u))));
}

// Standard (Microsoft RSS) Toeplitz over the 16 key bytes in memory order, MSB-first bits.
// `rss_key` is >= 20 bytes.  Its first 12 input bytes (src ip, dst ip, sport, dport) give the
// standard RSS 4-tuple hash contribution; proto/zone extend it.
NFDP_HD uint32_t toeplitz_scalar(const FlowKey& k, const uint8_t* rss_key) {
  const uint32_t w[4] = {k.src_ip, k.dst_ip, k.ports, k.meta};
  uint32_t v = ((uint32_t)rss_key[0] << 24) | ((uint32_t)rss_key[1] << 16) |
               ((uint32_t)rss_key[2] << 8) | rss_key[3];
  uint32_t h = 0;
  for (int byte = 0; byte < 16; ++byte) {
    const uint32_t b = (w[byte >> 2] >> (8 * (byte & 3))) & 0xFFu;
    const uint32_t next = rss_key[byte + 4];
    for (int bit = 7; bit >= 0; --bit) {
      if (b & (1u << bit)) h ^= v;
      v = (v << 1) | ((next >> bit) & 1u);
    }
  }
  return h;
}

// Flow-table geometry derived from the Toeplitz hash: two candidate buckets.
struct TableHash { uint32_t b1, b2; };
NFDP_HD TableHash table_hash(uint32_t h, uint32_t bucket_mask) {
  TableHash t;
  const uint32_t m = fmix32(h ^ 0x9e3779b9u);
  t.b1 = h & bucket_mask;
  t.b2 = (m ^ (m >> 7)) & bucket_mask;
  if (t.b2 == t.b1) t.b2 = (t.b1 + 1) & bucket_mask;  // two distinct choices
  return t;
}
// Shard (owner GPU) from the top bits of the hash: independent of the bucket (low) bits.
NFDP_HD uint32_t owner_of(uint32_t h, uint32_t nshards) {
  return (uint32_t)(((uint64_t)h * nshards) >> 32);
}

// ----------------------------------------------------------------------------------------
// Parsing.  A header slot is 16 little-endian dwords = the first min(len, 64) bytes of the
// frame; `len` is the whole frame's length (up to kMaxFrame).  The payload beyond the slot stays
// where the I/O layer put it: no stage reads it (every rewrite - MACs, tag, SNAT with RFC 1624
// incremental checksums, TTL - falls in the first 56 bytes of the normalized view).  `s` is the
// *normalized* (untagged) view: an 802.1Q tag (4 B at offset 12) is removed by a one-dword
// shift, since 4 B = 1 dword.
// ----------------------------------------------------------------------------------------
struct Parsed {
  uint32_t s[kSlotDwords];  // normalized header (untagged layout), bytes beyond len / the slot are junk
  uint32_t len;             // normalized length of the WHOLE frame in bytes (tag removed)
  uint32_t tci;             // 802.1Q TCI (0 if untagged)
  bool tagged;
  bool ipv4;                // IPv4 with IHL=5, first fragment, fully inside the slot
  bool l4;                  // TCP or UDP ports present
  bool arp;                 // EtherType 0x0806
  bool ipv6;                // EtherType 0x86DD, fixed header inside the slot (routed; L2 otherwise)
};

NFDP_HD uint32_t be16_at(const uint32_t* s, int byte) {  // byte offset must be even
  const uint32_t w = s[byte >> 2] >> (8 * (byte & 2));
  return ((w & 0xFFu) << 8) | ((w >> 8) & 0xFFu);
}
NFDP_HD uint32_t raw16_at(const uint32_t* s, int byte) {  // raw LE 16 (even offset)
  return (s[byte >> 2] >> (8 * (byte & 2))) & 0xFFFFu;
}
NFDP_HD void set_raw16(uint32_t* s, int byte, uint32_t v) {
  const int sh = 8 * (byte & 2);
  s[byte >> 2] = (s[byte >> 2] & ~(0xFFFFu << sh)) | ((v & 0xFFFFu) << sh);
}
NFDP_HD uint32_t raw32_at2(const uint32_t* s, int byte) {  // byte ≡ 2 (mod 4)
  return (s[byte >> 2] >> 16) | (s[(byte >> 2) + 1] << 16);
}
NFDP_HD void set_raw32_at2(uint32_t* s, int byte, uint32_t v) {
  s[byte >> 2] = (s[byte >> 2] & 0xFFFFu) | (v << 16);
  s[(byte >> 2) + 1] = (s[(byte >> 2) + 1] & 0xFFFF0000u) | (v >> 16);
}

NFDP_HD void parse(const uint32_t* d, uint32_t len, Parsed& p) {
  const uint32_t et = be16_at(d, 12);
  p.tagged = (et == 0x8100u) && len >= 18;
  p.tci = p.tagged ? be16_at(d, 14) : 0u;
#pragma unroll
  for (int i = 0; i < 3; ++i) p.s[i] = d[i];
#pragma unroll
  for (int i = 3; i < kSlotDwords - 1; ++i) p.s[i] = p.tagged ? d[i + 1] : d[i];
  p.s[kSlotDwords - 1] = p.tagged ? 0u : d[kSlotDwords - 1];
  p.len = p.tagged ? len - 4 : len;
  const uint32_t et2 = be16_at(p.s, 12);
  const uint32_t verihl = p.s[3] >> 16 & 0xFFu;
  const uint32_t frag = be16_at(p.s, 20);
  p.ipv4 = et2 == 0x0800u && verihl == 0x45u && p.len >= 34 && (frag & 0x1FFFu) == 0;
  const uint32_t proto = p.s[5] >> 24;
  p.l4 = p.ipv4 && (proto == 6 || proto == 17) && p.len >= 38;
  p.arp = et2 == 0x0806u;
#if NFDP_IPV6
  p.ipv6 = et2 == 0x86DDu && p.len >= 54 && (p.s[3] >> 20 & 0xFu) == 6u;
#else
  p.ipv6 = false;
#endif
}

NFDP_HD uint32_t dmac_lo(const uint32_t* s) { return s[0]; }
NFDP_HD uint32_t dmac_hi(const uint32_t* s) { return s[1] & 0xFFFFu; }
NFDP_HD uint32_t smac_lo(const uint32_t* s) { return (s[1] >> 16) | (s[2] << 16); }
NFDP_HD uint32_t smac_hi(const uint32_t* s) { return s[2] >> 16; }
NFDP_HD void set_dmac(uint32_t* s, uint32_t lo, uint32_t hi) {
  s[0] = lo; s[1] = (s[1] & 0xFFFF0000u) | (hi & 0xFFFFu);
}
NFDP_HD void set_smac(uint32_t* s, uint32_t lo, uint32_t hi) {
  s[1] = (s[1] & 0xFFFFu) | (lo << 16);
  s[2] = (lo >> 16) | (hi << 16);
}

// IPv6 (fixed header at 14..53 of the normalized view): next header at byte 20, addresses at
// 22 / 38, TCP / UDP ports at 54 when the slot holds them.
NFDP_HD uint32_t v6_nh(const Parsed& p) { return (p.s[5] >> 0) & 0xFFu; }
NFDP_HD uint32_t v6_ports(const Parsed& p) {
  const uint32_t nh = v6_nh(p);
  return ((nh == 6u || nh == 17u) && p.len >= 58) ? raw32_at2(p.s, 54) : 0u;
}

// `v6fold`: build IPv6 keys (the tables use IPv6 features: TablesView::v6_keys); otherwise an
// IPv6 packet keeps the IPv4-offset key (it takes no flow / ACL part then).
NFDP_HD FlowKey make_key(const Parsed& p, uint32_t zone, bool v6fold = true) {
  FlowKey k;
  k.src_ip = raw32_at2(p.s, 26);
  k.dst_ip = raw32_at2(p.s, 30);
  k.ports = p.l4 ? raw32_at2(p.s, 34) : 0u;
  k.meta = (p.s[5] >> 24) | (zone << 16);
#if NFDP_IPV6
  // an IPv6 packet's key always carries kKeyV6: IPv4 rules (AclTable: kKeyV6 clear) and IPv4
  // flows never match it
  k.meta |= p.ipv6 ? kKeyV6 : 0u;
  if (v6fold && p.ipv6) {
    k.src_ip = fold6(raw32_at2(p.s, 22), raw32_at2(p.s, 26), raw32_at2(p.s, 30), raw32_at2(p.s, 34));
    k.dst_ip = fold6(raw32_at2(p.s, 38), raw32_at2(p.s, 42), raw32_at2(p.s, 46), raw32_at2(p.s, 50));
    k.ports = v6_ports(p);
    k.meta = v6_nh(p) | kKeyV6 | (zone << 16);
  }
#endif
  return k;
}

// ----------------------------------------------------------------------------------------
// Checksums (RFC 1624 incremental update).  Works in the raw (byte-swapped) 16-bit domain:
// the one's-complement sum is byte-order independent as long as field and csum agree.
// ----------------------------------------------------------------------------------------
NFDP_HD uint32_t csum_fold(uint32_t x) {
  x = (x & 0xFFFFu) + (x >> 16);
  x = (x & 0xFFFFu) + (x >> 16);
  return x;
}
NFDP_HD uint32_t csum_update16(uint32_t csum, uint32_t old16, uint32_t new16) {
  // HC' = ~(~HC + ~m + m')
  uint32_t x = (~csum & 0xFFFFu) + (~old16 & 0xFFFFu) + (new16 & 0xFFFFu);
  return ~csum_fold(x) & 0xFFFFu;
}
NFDP_HD uint32_t csum_update32(uint32_t csum, uint32_t old32, uint32_t new32) {
  uint32_t x = (~csum & 0xFFFFu) + (~old32 & 0xFFFFu) + (~(old32 >> 16) & 0xFFFFu) +
               (new32 & 0xFFFFu) + (new32 >> 16);
  return ~csum_fold(x) & 0xFFFFu;
}
// full IPv4 header checksum over 20 bytes at offset 14 of the normalized view (raw domain)
NFDP_HD uint32_t ipv4_csum_full(const uint32_t* s) {
  uint32_t x = 0;
  for (int b = 14; b < 34; b += 2)
    if (b != 24) x += raw16_at(s, b);
  return ~csum_fold(x) & 0xFFFFu;
}

// ----------------------------------------------------------------------------------------
// Actions on the normalized view
// ----------------------------------------------------------------------------------------
NFDP_HD void act_snat(Parsed& p, uint32_t new_ip, uint32_t new_port) {
  const uint32_t old_ip = raw32_at2(p.s, 26);
  uint32_t ipc = raw16_at(p.s, 24);
  ipc = csum_update32(ipc, old_ip, new_ip);
  set_raw16(p.s, 24, ipc);
  set_raw32_at2(p.s, 26, new_ip);
  if (p.l4) {
    // TCP csum at L4+16 (byte 50), UDP at L4+6 (byte 40).  Both offsets are compile-time
    // constants on purpose: a runtime index into p.s[] would put the whole frame in scratch.
    const uint32_t proto = p.s[5] >> 24;
    const uint32_t old_port = raw16_at(p.s, 34);
    if (proto == 6) {
      if (52 <= p.len) {
        uint32_t c = raw16_at(p.s, 50);
        c = csum_update32(c, old_ip, new_ip);
        c = csum_update16(c, old_port, new_port);
        set_raw16(p.s, 50, c);
      }
    } else {
      uint32_t c = raw16_at(p.s, 40);
      if (c != 0) {                          // UDP csum 0 = disabled
        c = csum_update32(c, old_ip, new_ip);
        c = csum_update16(c, old_port, new_port);
        if (c == 0) c = 0xFFFFu;
        set_raw16(p.s, 40, c);
      }
    }
    set_raw16(p.s, 34, new_port);
  }
}

NFDP_HD bool act_ttl(Parsed& p) {  // returns false when the TTL expires
  const uint32_t w = raw16_at(p.s, 22);  // raw: low byte = ttl, high byte = proto
  const uint32_t ttl = w & 0xFFu;
  if (ttl <= 1) return false;
  const uint32_t nw = (w & 0xFF00u) | (ttl - 1);
  set_raw16(p.s, 24, csum_update16(raw16_at(p.s, 24), w, nw));
  set_raw16(p.s, 22, nw);
  return true;
}

// Serialize the normalized view back to a slot, optionally inserting an 802.1Q tag.
NFDP_HD void emit(const Parsed& p, uint32_t push_tci, bool push, uint32_t* out) {
#pragma unroll
  for (int i = 0; i < 3; ++i) out[i] = p.s[i];
  const uint32_t tagw = 0x0081u | (((push_tci >> 8) & 0xFFu) << 16) | ((push_tci & 0xFFu) << 24);
  out[3] = push ? tagw : p.s[3];
#pragma unroll
  for (int i = 4; i < kSlotDwords; ++i) out[i] = push ? p.s[i - 1] : p.s[i];
}

// Egress metadata word: port[11:0] (0xFFF none, 0xFFE punt) | olen[25:12] | reason[29:26] |
// xhdr[30] (prepend the packet's outer-header record: tunnel encap, x = 50 B for an IPv4 underlay, 70 B
// for IPv6, ethertype at record bytes 12..13) | flood[31].  The frame that leaves is
// xrec[0:x] ++ ohdr[0:hl] ++ in_frame[to:len]  with  d = olen - x - len,  hl = min(64, min(len, 64) + d),
// to = hl - d  (out_tail below): the payload is never copied by the pipeline.
// 32-bit fold of an IPv6 address (raw words): the hot kernel's cheap "to the local VTEP?" test.
// The exact address and the (source, VNI) key are checked by the termination resolver.
NFDP_HD uint32_t vtep6_fold(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3) {
  const uint32_t h = a0 ^ ((a1 << 8) | (a1 >> 24)) ^ ((a2 << 16) | (a2 >> 16)) ^ ((a3 << 24) | (a3 >> 8));
  return h ? h : 1u;
}
constexpr uint32_t kMetaXhdr = 1u << 30;
constexpr uint32_t kMetaFlood = 1u << 31;  // primary copy of a flooded frame (side pass emits the rest)
constexpr uint32_t kEncapBytes = 50;   // outer Ethernet + IPv4 + UDP + VXLAN/GENEVE (no options)
constexpr uint32_t kEncap6Bytes = 70;  // outer Ethernet + IPv6 + UDP + VXLAN/GENEVE (no options)
constexpr int kXhdrBytes = 128;        // one packet's outer-header record (side pass output)
NFDP_HD uint32_t make_meta(uint32_t out_port, uint32_t len, uint32_t reason, bool xhdr = false, bool flood = false) {
  return (out_port & 0xFFFu) | ((len & 0x3FFFu) << 12) | ((reason & 0xFu) << 26) | (xhdr ? kMetaXhdr : 0u) |
         (flood ? kMetaFlood : 0u);
}
NFDP_HD uint32_t meta_port(uint32_t m) {
  const uint32_t p = m & 0xFFFu;
  return p >= 0xFFEu ? (p | 0xF000u) : p;
}
NFDP_HD uint32_t meta_len(uint32_t m) { return (m >> 12) & 0x3FFFu; }
NFDP_HD uint32_t cont_meta(uint32_t strip, uint32_t hv) { return make_meta(strip, hv, kCont); }
// A continuation slot's in-meta: kPortCont | len << 16 from the producer; once its pair was
// resolved (kernels.hip pair_kernel / the ring kernel) the len field is strip | hv << 8 | kPairDone.
constexpr uint32_t kPairDone = 0x8000u;
NFDP_HD uint32_t pair_cinfo(uint32_t cont_inmeta) {   // strip | hv << 8 (no strip: not resolved / not terminated)
  const uint32_t f = cont_inmeta >> 16;
  return (f & kPairDone) ? (f & 0x7FFFu) : ((uint32_t)kSlotBytes << 8);
}
NFDP_HD uint32_t meta_reason(uint32_t m) { return (m >> 26) & 0xFu; }
// Header bytes `hl` of the out slot that are valid and the offset `to` in the input frame where the
// unchanged tail continues (both from the in/out lengths; the `xlen` outer-header bytes excluded).
// `hv`: valid bytes of the input view the out slot was built from (64; fewer for an IPv6-underlay
// terminated frame, see decap_pair).  A terminated frame passes in_len = len - strip and reads its
// tail from in_frame + strip.
NFDP_HD void out_tail(uint32_t in_len, uint32_t olen, uint32_t xlen, uint32_t& hl, uint32_t& to,
                      uint32_t hv = kSlotBytes) {
  const int d = (int)olen - (int)xlen - (int)in_len;
  const int h_in = in_len < hv ? (int)in_len : (int)hv;
  int h = h_in + d;
  if (h > kSlotBytes) h = kSlotBytes;
  hl = (uint32_t)h;
  to = (uint32_t)(h - d);
}

// ----------------------------------------------------------------------------------------
// Pipeline parameters (kernarg / oracle argument).  Raw pointers into HBM (or host memory
// for the oracle).  Everything is sized by the control plane; the kernels never allocate.
// ----------------------------------------------------------------------------------------
// One IPv6 route: prefix words in host order (a[0] = most significant 32 bits), already masked to
// `plen` bits; plen 0xFF = empty slot.  32 B.
struct Lpm6Entry {
  uint32_t a[4];
  uint32_t plen;
  uint32_t result;   // kRouteNh | nexthop or kRouteEcmp | group (as IPv4)
  uint32_t pad[2];
};
constexpr uint32_t kLpm6Empty = 0xFFu;
constexpr int kLpm6Probe = 16;

struct TablesView {
  const PortEntry* ports;        // kMaxPorts
  const ChainEntry* chains;      // n_chains
  uint32_t n_chains;
  const FlowSlot* flows;         // nbuckets * kBucketSlots (one 128-B line per bucket)
  uint32_t bucket_mask;          // nbuckets - 1 (power of two)
  const MacEntry* macs;          // n_mac (power of two)
  uint32_t mac_mask;
  const uint8_t* rss_key;        // 52 B
  // ACL (TCAM): rules in priority order; value/mask over the 128-bit FlowKey.
  const uint32_t* acl_value;     // n_acl * 4
  const uint32_t* acl_mask;      // n_acl * 4
  const uint8_t* acl_permit;     // n_acl (1 permit, 0 deny)
  uint32_t n_acl;
  uint32_t acl_default_permit;   // verdict when no rule matches
  const uint16_t* lag_members;   // n_lag_groups * kLagWays egress ports (K8)
  uint32_t n_lag_groups;
  const uint16_t* flood;         // n_flood head rows of kFloodWays entries per bridge (kPortNone padded),
                                 // then overflow rows reached through kFloodLink entries
  uint32_t n_flood;              // bridges [0, n_flood) have a flood group
  const uint32_t* lpm24;         // 1 << 24 entries (nullable: no routes)
  const uint32_t* lpm8;          // n_lpm8 * 256
  uint32_t n_lpm8;
  const NextHop* nexthops;       // n_nexthops
  uint32_t n_nexthops;
  const uint16_t* ecmp;          // n_ecmp * kEcmpWays nexthop ids
  uint32_t n_ecmp;
  const TunnelEntry* tunnels;    // n_tunnels (indexed by a tunnel port's `lag`)
  uint32_t n_tunnels;
  const Tunnel6Entry* tunnels6;  // n_tunnels6 (kPortTunnel6 ports' `lag`)
  uint32_t n_tunnels6;
  uint32_t vtep6_fold;           // vtep6_fold() of the local IPv6 VTEP address (0: no IPv6 VTEP)
  const TermEntry* terms;        // term_mask + 1 slots, open addressing (nullable)
  uint32_t term_mask;
  const Term6Entry* terms6;      // term6_mask + 1 slots, open addressing (nullable: no IPv6 terminations)
  uint32_t term6_mask;
  uint32_t vtep6[4];             // the local IPv6 VTEP address, raw words (with vtep6_fold != 0)
  const VmMacEntry* vmmac;       // vmmac_mask + 1 slots, open addressing (nullable: no VM MAC maps)
  uint32_t vmmac_mask;
  // IPv6 FIB (P4 ipv6_table): one open-addressing table over (prefix, length) and the distinct
  // prefix lengths present, longest first; a lookup probes the lengths in that order
  const Lpm6Entry* lpm6;         // lpm6_mask + 1 slots (nullable: no IPv6 routes)
  uint32_t lpm6_mask;
  const uint8_t* lpm6_lens;      // n_lpm6_lens lengths, descending
  uint32_t n_lpm6_lens;
  // IPv6 flows: the flow-table buffer carries, after its nbuckets * 128 B of buckets, a side
  // array of the same geometry holding each slot's full IPv6 addresses (2 x 16 B: src, dst raw
  // words).  An IPv6 packet probes the folded key (make_key) and a hit counts only when the side
  // entry equals the packet's addresses (flow6_verify), so every flow-table copy (the ring's
  // double buffer) carries its own side array and a lookup is exact.
  uint32_t flow6_on;
  // IPv6 ACL (TCAM over the 384-bit key6: src6, dst6, ports, proto | zone << 16, 0, 0): rules in
  // priority order, their verdicts at acl_permit[n_acl + j] (one rule index space).
  const uint32_t* acl6_value;    // n_acl6 * 12
  const uint32_t* acl6_mask;     // n_acl6 * 12
  uint32_t n_acl6;
};

NFDP_HD uint32_t lpm_lookup(const TablesView& t, uint32_t dst /* host order */) {
  if (!t.lpm24) return 0;
  const uint32_t e = t.lpm24[dst >> 8];
  if (!(e & kLpmExt)) return e;
  const uint32_t g = e & ~kLpmExt;
  return g < t.n_lpm8 ? t.lpm8[(size_t)g * 256 + (dst & 0xFFu)] : 0u;
}
// route result -> nexthop id (ECMP by hash[2:0]) or -1
NFDP_HD int route_nexthop(const TablesView& t, uint32_t r, uint32_t hash) {
  const uint32_t id = r & 0xFFFFu;
  if ((r & (3u << 28)) == kRouteNh) return id < t.n_nexthops ? (int)id : -1;
  if ((r & (3u << 28)) == kRouteEcmp && t.ecmp && id < t.n_ecmp) {
    const uint32_t nh = t.ecmp[id * kEcmpWays + (hash & (kEcmpWays - 1))];
    return nh < t.n_nexthops ? (int)nh : -1;
  }
  return -1;
}
NFDP_HD uint32_t term_hash(uint32_t src_ip, uint32_t vni) { return fmix32(src_ip ^ (vni * 0x9E3779B1u)); }
// (outer src ip raw, vni) -> tunnel port or -1
NFDP_HD uint32_t lpm6_hash(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t plen) {
  return fmix32(a0 ^ fmix32(a1 ^ fmix32(a2 ^ fmix32(a3 ^ (plen * 0x9E3779B9u)))));
}
NFDP_HD uint32_t lpm6_word_mask(uint32_t plen, int w) {
  const int bits = (int)plen - 32 * w;
  return bits >= 32 ? 0xFFFFFFFFu : (bits <= 0 ? 0u : ~(0xFFFFFFFFu >> bits));
}
// Longest-prefix match of an IPv6 destination (host-order words d0 = most significant): probe
// each present prefix length, longest first.  Returns the route result or 0.  Scalars only (no
// private arrays): this runs inside the hot kernels' register budget.
NFDP_HD uint32_t lpm6_lookup(const TablesView& t, uint32_t d0, uint32_t d1, uint32_t d2, uint32_t d3) {
  if (!t.lpm6 || !t.lpm6_lens) return 0;
  for (uint32_t li = 0; li < t.n_lpm6_lens; ++li) {
    const uint32_t plen = t.lpm6_lens[li];
    const uint32_t m0 = d0 & lpm6_word_mask(plen, 0), m1 = d1 & lpm6_word_mask(plen, 1);
    const uint32_t m2 = d2 & lpm6_word_mask(plen, 2), m3 = d3 & lpm6_word_mask(plen, 3);
    const uint32_t h = lpm6_hash(m0, m1, m2, m3, plen) & t.lpm6_mask;
    for (int probe = 0; probe < kLpm6Probe; ++probe) {
      const Lpm6Entry& e = t.lpm6[(h + probe) & t.lpm6_mask];
      if (e.plen == kLpm6Empty) break;
      if (e.plen == plen && e.a[0] == m0 && e.a[1] == m1 && e.a[2] == m2 && e.a[3] == m3) return e.result;
    }
  }
  return 0;
}

NFDP_HD uint32_t vmmac_hash(uint32_t ip, uint32_t kind) { return fmix32(ip ^ (kind * 0x85EBCA77u)); }
// (raw IPv4, kind) -> slot or -1
NFDP_HD int vmmac_lookup(const TablesView& t, uint32_t ip, uint32_t kind) {
  const uint32_t h = vmmac_hash(ip, kind);
  for (int q = 0; q < kVmMacProbe; ++q) {
    const uint32_t i = (h + (uint32_t)q) & t.vmmac_mask;
    const VmMacEntry& e = t.vmmac[i];
    if (!e.kind) return -1;
    if (e.ip == ip && e.kind == kind) return (int)i;
  }
  return -1;
}

NFDP_HD int term_lookup(const TablesView& t, uint32_t src_ip, uint32_t vni) {
  if (!t.terms) return -1;
  const uint32_t h = term_hash(src_ip, vni);
  for (uint32_t q = 0; q < 8; ++q) {
    const TermEntry& e = t.terms[(h + q) & t.term_mask];
    if (!e.valid) return -1;
    if (e.src_ip == src_ip && e.vni == vni) return e.port;
  }
  return -1;
}

NFDP_HD uint32_t term6_hash(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t vni) {
  return fmix32(a0 ^ fmix32(a1 ^ fmix32(a2 ^ fmix32(a3 ^ (vni * 0x9E3779B1u)))));
}
// (outer src IPv6 raw words, vni) -> tunnel port or -1
NFDP_HD int term6_lookup(const TablesView& t, uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t vni) {
  if (!t.terms6) return -1;
  const uint32_t h = term6_hash(a0, a1, a2, a3, vni);
  for (uint32_t q = 0; q < 8; ++q) {
    const Term6Entry& e = t.terms6[(h + q) & t.term6_mask];
    if (!e.valid) return -1;
    if (e.src[0] == a0 && e.src[1] == a1 && e.src[2] == a2 && e.src[3] == a3 && e.vni == vni) return e.port;
  }
  return -1;
}

// Side outputs of a batch (pipeline.h side_stage): replicas (flood members, mirror copies, ARP
// slow-path copies) and MAC-learn events, appended at positions claimed with one atomic each.
// cnt: [0] replicas, [1] learn events, [2] replicas dropped (full), [3] learn events dropped,
// [4] learn events with no free slot (learn kernel), [5] side-list entries, [6] side-list dropped.
struct SideOut {
  uint32_t* rep_hdr;             // cap_rep x 64-B header slots
  uint32_t* rep_meta;            // cap_rep egress meta words
  uint32_t* rep_src;             // cap_rep source packet indices (whose input frame holds the tail)
  uint32_t cap_rep;
  uint32_t* learn;               // cap_learn x {mac_lo, mac_hi | bridge << 16, port, 0}
  uint32_t cap_learn;
  uint32_t* cnt;                 // 8 counters (nullptr: side outputs disabled); [5] side-list length
  uint32_t* list;                // packets flagged by the per-packet kernel for the side pass
  uint32_t cap_list;
  uint32_t* xhdr;                // [batch] x kXhdrBytes outer-header records of tunnel-encapsulated packets
  // Per-workgroup regions (fused kernel; null blk_cnt: one flat list claimed with a global
  // counter): workgroup b appends to list[b * blk_cap ...) with LDS claims and leaves its count in
  // blk_cnt[b]; set by the launcher (blk_cap, nblk) when the list holds every region.
  uint32_t* blk_cnt;
  uint32_t blk_cap;
  uint32_t nblk;
};

// Flow-table lookup (scalar).  Returns slot index or -1.
NFDP_HD int64_t flow_lookup(const TablesView& t, const FlowKey& k, uint32_t h) {
  const TableHash th = table_hash(h, t.bucket_mask);
  uint32_t bk[2] = {th.b1, th.b2};
  const uint32_t used = k.meta | kSlotUsed;
  for (int c = 0; c < 2; ++c) {
    for (int s = 0; s < kBucketSlots; ++s) {
      const FlowKey& e = t.flows[(size_t)bk[c] * kBucketSlots + s].key;
      if (e.src_ip == k.src_ip && e.dst_ip == k.dst_ip && e.ports == k.ports && e.meta == used)
        return (int64_t)bk[c] * kBucketSlots + s;
    }
  }
  return -1;
}

NFDP_HD uint32_t mac_hash(uint32_t bridge, uint32_t lo, uint32_t hi) {
  return fmix32(lo ^ (hi << 16) ^ (bridge * 0x9E3779B1u));
}

NFDP_HD int mac_lookup(const TablesView& t, uint32_t bridge, uint32_t lo, uint32_t hi) {
  if (!t.macs) return -1;
  const uint32_t h = mac_hash(bridge, lo, hi) & t.mac_mask;
  for (int probe = 0; probe < 16; ++probe) {
    const MacEntry& e = t.macs[(h + probe) & t.mac_mask];
    if (e.valid == kMacEmpty) return -1;
    if ((e.valid == kMacStatic || e.valid == kMacLearned) && e.mac_lo == lo && e.mac_hi == (hi & 0xFFFFu) &&
        e.bridge_id == bridge)
      return e.out_port;
  }
  return -1;
}

// The ACL key is the flow key with two port-class bits added to its meta word: "source port >=
// 1024" and "destination port >= 1024".  The range [1024, 65535] (the unprivileged / ephemeral
// ports, the most common range of real ACLs) is then ONE ternary entry instead of the six
// prefixes of a TCAM range expansion (AclTable.add).  Ports are raw (network order): a port's
// high byte is the low byte of its half, and port >= 1024 <=> high byte >= 4.  Never part of a
// flow key (bits 10 / 11 of meta are zero in every flow key and packet key).
constexpr uint32_t kAclSportHi = 0x400u, kAclDportHi = 0x800u;
NFDP_HD uint32_t acl_key_meta(uint32_t ports, uint32_t meta) {
  return meta | ((ports & 0xFCu) ? kAclSportHi : 0u) | ((ports & 0xFC0000u) ? kAclDportHi : 0u);
}

// Scalar ACL (priority order, first match).  Returns rule index or -1.
NFDP_HD int acl_first_match(const TablesView& t, const FlowKey& k) {
  const uint32_t w[4] = {k.src_ip, k.dst_ip, k.ports, acl_key_meta(k.ports, k.meta)};
  for (uint32_t r = 0; r < t.n_acl; ++r) {
    bool m = true;
    for (int i = 0; i < 4; ++i) m = m && ((w[i] ^ t.acl_value[4 * r + i]) & t.acl_mask[4 * r + i]) == 0;
    if (m) return (int)r;
  }
  return -1;
}

// IPv6 flows (TablesView::flow6_on): the side entry of flow slot `slot`.
NFDP_HD const uint32_t* flow6_side(const TablesView& t, int64_t slot) {
  return reinterpret_cast<const uint32_t*>(t.flows + (size_t)(t.bucket_mask + 1u) * kBucketSlots) + (size_t)slot * 8;
}
// Exact check of an IPv6 packet's folded-key hit: the slot's side entry holds its addresses.
NFDP_HD bool flow6_verify(const TablesView& t, const Parsed& p, int64_t slot) {
  const uint32_t* e = flow6_side(t, slot);
  bool ok = true;
#pragma unroll
  for (int k = 0; k < 8; ++k) ok = ok && e[k] == raw32_at2(p.s, 22 + 4 * k);
  return ok;
}

// The 12-word IPv6 ACL key: src6 (4 raw words), dst6 (4), ports, next header | zone << 16, 0, 0.
NFDP_HD uint32_t key6_word(const Parsed& p, uint32_t zone, int w) {
  return w < 8 ? raw32_at2(p.s, 22 + 4 * w) : (w == 8 ? v6_ports(p) : (w == 9 ? (v6_nh(p) | (zone << 16)) : 0u));
}
// Scalar IPv6 ACL (priority order, first match) -> index in the shared verdict space (n_acl + j)
// or -1.
NFDP_HD int acl6_first_match(const TablesView& t, const Parsed& p, uint32_t zone) {
  uint32_t kw[12];   // constant indices only (unrolled): stays in registers on the GPU
#pragma unroll
  for (int i = 0; i < 12; ++i) kw[i] = key6_word(p, zone, i);
  for (uint32_t r = 0; r < t.n_acl6; ++r) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) x |= (kw[i] ^ t.acl6_value[12 * r + i]) & t.acl6_mask[12 * r + i];
    if (!x) return (int)(t.n_acl + r);
  }
  return -1;
}

}  // namespace nfdp
