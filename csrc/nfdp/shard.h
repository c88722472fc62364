// shard.h — multi-GPU (flow-sharded) pipeline: shared geometry, descriptor/verdict formats and
// argument blocks for the four stage kernels (shard.hip) and their CPU twins (shard_cpu.cpp).
//
// One step on rank r of N (per batch of B packets):
//   1. ingress  : parse, port checks, MFMA hash + TCAM ACL, owner = hash shard;
//                 write a 32-B descriptor (the FlowKey + wire length) into segment[owner]
//   2. all-to-all(descriptors)                          [RCCL over xGMI]
//   3. owner    : exact-match lookup in the local 1/N of the flow table, per-flow counters,
//                 16-B verdict into the mirrored position
//   4. all-to-all(verdicts)                             [RCCL over xGMI]
//   5. apply    : NF chain (ACL verdict, SNAT, L2 steer, VLAN...) on the packet that never left
//                 the ingress GPU; local egress written in place, remote egress into
//                 segment[egress gpu] (64-B slot + 4-B meta)
//   6. all-to-all(packets)                              [RCCL over xGMI]
//   7. egress   : tx counters + latency stamps for packets received from peers
// Only 32 + 16 B per packet cross xGMI for the flow state; the 64-B payload crosses once, and
// only when the destination pod lives on another GPU.  All segments are fixed capacity so the
// collectives have static splits (no host round trip per step); segment slot 0 is a header
// carrying the fill count.
#pragma once
#include "pipeline.h"

namespace nfdp {

struct ShardGeom {
  uint32_t nranks;
  uint32_t rank;
  uint32_t cap_desc;  // descriptors per destination segment
  uint32_t cap_pkt;   // packets per destination segment
};

// Descriptor = 32 B {FlowKey, wire_len, 0, 0, 0} (a 16-bit frame length no longer fits the key's
// spare byte); verdict = 16 B.  Slot 0 of every segment is the {count, cap} header.
NFDP_HD size_t desc_seg_bytes(uint32_t cap) { return (size_t)(cap + 1) * 32; }
NFDP_HD size_t verdict_seg_bytes(uint32_t cap) { return (size_t)(cap + 1) * 16; }
NFDP_HD size_t pkt_meta_off(uint32_t cap) { return 64 + (size_t)cap * 64; }
NFDP_HD size_t pkt_seg_bytes(uint32_t cap) {
  return pkt_meta_off(cap) + (((size_t)cap * 4 + 63) & ~(size_t)63);
}

constexpr uint32_t kRefNone = 0xFFFFFFFFu;      // no flow lookup (non-IP / dropped at ingress)
constexpr uint32_t kRefOverflow = 0xFFFFFFFEu;  // descriptor segment was full


NFDP_HD Verdict make_verdict(bool hit, const FlowAction& a) {
  Verdict v;
  v.chain_id = a.chain_id; v.out_port = a.out_port; v.nat_ip = a.nat_ip;
  v.nat_port = a.nat_port; v.vlan = a.vlan; v.status = hit ? 1u : 0u;
  return v;
}
NFDP_HD FlowAction verdict_action(const Verdict& v) {
  FlowAction a;
  a.chain_id = v.chain_id; a.out_port = v.out_port; a.nat_ip = v.nat_ip;
  a.nat_port = v.nat_port; a.vlan = v.vlan; a.flow_id = 0;
  return a;
}

struct IngressArgs {
  TablesView t;
  const uint4* pkts;
  const uint32_t* inmeta;
  uint32_t n;
  ShardGeom g;
  uint8_t* send_desc;        // nranks segments of desc_seg_bytes(cap_desc)
  uint32_t* cnt;             // nranks fill counters (zeroed per step)
  uint32_t* ref;             // per packet: owner << 24 | pos, or kRef*
  uint32_t* aux;             // per packet: acl rule + 1 (0 = no match)
  const void* acl_wfrag; const void* acl_cinit; uint32_t acl_tiles;
  const void* toep_frag; const uint32_t* toep_tab;
};

struct OwnerArgs {
  TablesView t;
  ShardGeom g;
  const uint8_t* recv_desc;  // nranks segments (from every source rank)
  uint8_t* send_verdict;     // nranks segments, mirrored positions
  unsigned long long* flow_ctr;
  const uint32_t* toep_tab;  // [16][256]
};

struct ApplyArgs {
  TablesView t;
  const uint4* pkts;
  const uint32_t* inmeta;
  uint32_t n;
  ShardGeom g;
  const uint32_t* ref;
  const uint32_t* aux;
  const uint8_t* recv_verdict;
  uint4* out;                // local egress, in place (slot i)
  uint32_t* out_meta;        // reason kRemote for packets handed to a peer
  uint8_t* send_pkt;         // nranks packet segments
  uint32_t* pcnt;            // nranks fill counters (zeroed per step)
  unsigned long long* port_ctr;
  unsigned long long* drop_ctr;
  const unsigned long long* t0;
  uint32_t* lat;             // n/16 samples
};

struct EgressArgs {
  ShardGeom g;
  const uint8_t* recv_pkt;   // nranks packet segments received from peers
  unsigned long long* port_ctr;
  const unsigned long long* t0;
  uint32_t* lat;             // nranks * cap_pkt / 16 samples
};

// ---- CPU twins (shard_cpu.cpp) ----
void ingress_cpu(const IngressArgs& a);
void owner_cpu(const OwnerArgs& a);
void apply_cpu(const ApplyArgs& a);
void egress_cpu(const EgressArgs& a);
// ---- GPU launchers (shard.hip) ----
hipError_t launch_ingress(const IngressArgs& a, int hash_mode, int acl_mode, int num_cus, hipStream_t s);
hipError_t launch_seg_headers(const uint32_t* cnt, uint8_t* buf, uint32_t nranks, size_t seg_bytes,
                              uint32_t cap, hipStream_t s);
hipError_t launch_owner(const OwnerArgs& a, int num_cus, hipStream_t s);
hipError_t launch_apply(const ApplyArgs& a, int num_cus, hipStream_t s);
hipError_t launch_egress(const EgressArgs& a, int num_cus, hipStream_t s);

}  // namespace nfdp
