// host.h — host-side control structures for the data plane (authoritative flow table,
// classification-table builders, CPU oracle, kernel launchers).
#pragma once
#include <cstring>
#include <random>
#include <stdexcept>
#include <unordered_set>
#include <vector>

#include "pipeline.h"

namespace nfdp {

// ACL rule tiles per prefilter group (device.h kAclGroup; host.cpp build_acl_frags).
#ifndef NFDP_ACL_GROUP
#define NFDP_ACL_GROUP 8
#endif
constexpr uint32_t kAclGroupTiles = NFDP_ACL_GROUP;

// Authoritative host copy of the exact-match flow table.  Bucketized (8 slots) 2-choice cuckoo
// with eviction; every mutation records the touched bucket so the device copy is kept in sync by
// re-sending whole buckets (bucket_update_kernel), ordered on the data-plane stream between
// batches.  Replaces the reference's per-rule `p4rt-ctl add-entry` round trips
// (vendor/.../p4rtclient/p4rtclient.go:74-101) with batched HBM row writes.
class FlowTableHost {
 public:
  FlowTableHost(uint32_t nbuckets_pow2, const std::vector<uint8_t>& rss_key);
  uint32_t nbuckets() const { return nb_; }
  uint32_t mask() const { return nb_ - 1; }
  size_t size() const { return count_; }
  // returns slot index; throws when the table is full (after max kicks)
  int64_t insert(const FlowKey& k, const FlowAction& a);
  bool erase(const FlowKey& k);
  int64_t find(const FlowKey& k) const;
  uint32_t hash(const FlowKey& k) const { return toeplitz_scalar(k, rss_.data()); }
  const std::vector<FlowSlot>& slots() const { return slots_; }
  // dirty tracking
  std::vector<uint32_t> take_dirty();
  // slot moves performed by evictions since the last take (from, to), for counter migration
  std::vector<std::pair<int64_t, int64_t>> take_moves();
  void clear_dirty() { dirty_.clear(); moves_.clear(); }
  const std::vector<uint8_t>& rss_key() const { return rss_; }

 private:
  int find_in_bucket(uint32_t b, const FlowKey& k) const;
  uint32_t nb_;
  size_t count_ = 0;
  std::vector<uint8_t> rss_;
  std::vector<FlowSlot> slots_;
  std::unordered_set<uint32_t> dirty_;
  std::vector<std::pair<int64_t, int64_t>> moves_;
  std::mt19937 rng_{12345};
};

// Device-layout classification tables.
struct AclFrags {
  std::vector<int8_t> wfrag;   // [tiles][64][16]: FP4 (e2m1) A fragments, 32 nibbles per lane
  std::vector<int32_t> cinit;  // [tiles][4][4] f32 C init (bias * 4096 + rule) | [tiles][8] tile
                               // prefilters | [groups of 8 tiles][8] group prefilters | [ptiles][4][4]
                               // C init of the prefilter tiles (IPv4 tables; A fragments after the tiles')
  uint32_t tiles = 0;
  uint32_t ptiles = 0;         // prefilter tiles: tile t's prefilter is row t % 16 of prefilter tile t / 16
};
AclFrags build_acl_frags(const uint32_t* value, const uint32_t* mask, uint32_t n);
// IPv6 ACL tiles: 16 rules x 3 K-blocks of 128 key6 bits ([tiles][3][64] A fragments, [tiles][16]
// C init); rules keep their order (the rule index rides in the accumulator).
AclFrags build_acl6_frags(const uint32_t* value, const uint32_t* mask, uint32_t n);
std::vector<int8_t> build_toeplitz_frags(const uint8_t* rss_key);   // [2][2][64][16]
std::vector<uint32_t> build_toeplitz_table(const uint8_t* rss_key); // [16][256]

// CPU oracle of the fused pipeline (bit-exact reference for the GPU kernels).
struct OracleOut {
  std::vector<uint64_t> port_ctr;  // kMaxPorts * 2
  std::vector<uint64_t> drop_ctr;  // kNumReasons
};
void oracle_run(const TablesView& t, const uint32_t* pkts, const uint32_t* inmeta, uint32_t n,
                uint32_t* out, uint32_t* out_meta, uint64_t* flow_ctr, uint64_t* port_ctr,
                uint64_t* drop_ctr, uint32_t* hashes, int32_t* acl_rules, const SideOut* side = nullptr,
                HopState* hop_state = nullptr);
// The SFC hop pipeline across GPUs: the rest of split chains (kHopXfer) over handed-over frames
// (`hdr` slots + their HopState records); a frame its chain hands on again gets a record in
// `out_state` (nullable) and meta reason kRemote.  Counts tx / drops in port_ctr / drop_ctr.
// GPU twin: launch_resume.
void oracle_resume(const TablesView& t, const uint32_t* hdr, const HopState* state, uint32_t n, uint32_t* out,
                   uint32_t* out_meta, HopState* out_state, uint64_t* port_ctr, uint64_t* drop_ctr);
// MAC learning: apply learn events {mac_lo, mac_hi | bridge << 16, port, 0} to the MAC table
// (learned entries carry `stamp`; static entries are never overridden).  Returns the number of
// events that found no slot within the probe limit.  GPU twin: launch_mac_learn.
uint32_t mac_learn_cpu(MacEntry* macs, uint32_t mac_mask, const uint32_t* events, uint32_t n, uint32_t stamp);
hipError_t launch_mac_learn(MacEntry* macs, uint32_t mac_mask, const uint32_t* events, const uint32_t* n_events,
                            uint32_t cap, uint32_t stamp, uint32_t* dropped, hipStream_t s);
// Replicated multi-GPU twin of the fused REMOTE kernel: frames whose egress port belongs to
// another rank are written to send_pkt segment[egress rank] (positions in arrival order, fill
// counts in pcnt, headers written at the end), out_meta says kRemote for them.
struct RemoteOut {
  uint32_t nranks, rank, cap_pkt;
  uint8_t* send_pkt;
  uint32_t* pcnt;
  uint32_t steer = 0;  // 1: flow-owner steering (input header + ingress meta to the owner)
};
// Receive side of flow-owner steering (GPU: launch_gather): segments -> dense batch; returns n.
uint32_t gather_cpu(const uint8_t* recv, uint32_t nranks, uint32_t rank, uint32_t cap, uint32_t seg_bytes,
                    uint32_t meta_off, uint32_t* pkts, uint32_t* inmeta);
hipError_t launch_gather(const uint8_t* recv, uint32_t nranks, uint32_t rank, uint32_t cap, uint32_t seg_bytes,
                         uint32_t meta_off, void* pkts, uint32_t* inmeta, uint32_t* n_dev, hipStream_t s);
void oracle_run_remote(const TablesView& t, const uint32_t* pkts, const uint32_t* inmeta, uint32_t n,
                       uint32_t* out, uint32_t* out_meta, uint64_t* flow_ctr, uint64_t* port_ctr,
                       uint64_t* drop_ctr, const RemoteOut& r);

// ---- GPU launchers (kernels.hip) ----
struct LaunchCfg {
  int hash_mode = 2;
  int acl_mode = 1;
  int num_cus = 256;
};
struct FusedLaunch {
  TablesView t;
  const void* pkts; const uint32_t* inmeta; void* out; uint32_t* out_meta; uint32_t n;
  unsigned long long* flow_ctr; unsigned long long* port_ctr; unsigned long long* drop_ctr;
  const unsigned long long* t0; uint32_t* lat;
  const void* acl_wfrag; const void* acl_cinit; uint32_t acl_tiles;
  const void* toep_frag; const uint32_t* toep_tab;
  uint32_t flags = 0;
  // replicated multi-GPU mode (nranks > 1): remote-egress frames go to per-GPU send segments
  uint8_t* send_pkt = nullptr; uint32_t* pcnt = nullptr;
  uint32_t nranks = 0, rank = 0, cap_pkt = 0;
  SideOut side{};  // side outputs (flood / mirror / ARP replicas, learn events); cnt null = off
  uint32_t steer = 0;              // REMOTE: 1 = send packets of other GPUs' flow shards to their owner
  const uint32_t* n_dev = nullptr; // device-side count (<= n)
  // steer-by-list (1-GPU instances with nranks > 1): other GPUs' packets listed, not processed
  uint32_t* steer_list = nullptr;
  uint32_t* steer_cnt = nullptr;   // 2 + 4 * num_cus words: {grid, region size, count per workgroup}
  uint32_t steer_cap = 0;          // steer_list entries (>= steer_list_len(n, num_cus))
  // IPv6 ACL (t.n_acl6 > 0): acl6_kernel classifies the batch's IPv6 packets first (into out_meta)
  const void* acl6_wfrag = nullptr; const void* acl6_cinit = nullptr; uint32_t acl6_tiles = 0;
  // split chains (kHopXfer): each handed-off frame's HopState (n records, nullable: the XFER
  // instances run only when it is given)
  HopState* hop_state = nullptr;
  // IPv6 tables: v6_kernel's folded keys, one 16-B row per slot (coalesced for the fused V6
  // instances); null: parked in the first 16 B of each out slot (a strided read, 1/4 of its lines)
  void* v6_keys = nullptr;
};
// The hand-off itself (kernels.hip): frames of `meta` with reason kRemote and port `plane` (and
// their HopState records) -> the inbox on the GPU that resumes them, written there by this GPU
// (peer stores over xGMI; the same code when both planes share a device).  Inbox: count word
// (written by the publish step, <= cap), hdr [cap][64 B], state [cap], idx [cap] (source index).
struct HopInbox {
  uint32_t* count; uint4* hdr; HopState* state; uint32_t* idx; uint32_t cap;
};
hipError_t launch_hop_pack(const void* out, const uint32_t* meta, const HopState* state, uint32_t n,
                           const uint32_t* n_dev, uint32_t plane, uint32_t* fill, const HopInbox& dst,
                           hipStream_t s);
// resume_kernel over an inbox (count from the device): results + next hand-offs
hipError_t launch_resume(const TablesView& t, const HopInbox& in, void* out, uint32_t* out_meta, HopState* out_state,
                         unsigned long long* port_ctr, unsigned long long* drop_ctr, uint32_t flags, int num_cus,
                         hipStream_t s);
// Second half of steer-by-list: listed packets -> their owners' exchange segments (count-first,
// segments sized for the whole batch).
hipError_t launch_steer(const void* pkts, const uint32_t* inmeta, const uint32_t* list, const uint32_t* list_cnt,
                        uint32_t cap_list, uint32_t cnt_len, uint8_t* send, uint32_t* pcnt, uint32_t nranks,
                        uint32_t cap, hipStream_t s);
// steer_list entries a LIST launch over n packets can need
uint32_t steer_list_len(uint32_t n, int num_cus);
hipError_t launch_fused(const FusedLaunch& f, const LaunchCfg& cfg, hipStream_t s);
// Side pass alone (flood / mirror / ARP replicas, learn events, tunnel headers) over a side list
// another kernel filled (the persistent ring kernel): slots / meta are that kernel's buffers.
// IPsec ESP engine (ipsec.h / ipsec.hip / ipsec_cpu.cpp)
struct EspBatch;
struct EspSa;
struct EspTables;
hipError_t launch_esp(const EspBatch& a, bool enc, const uint32_t* te0, const uint8_t* sbox, const uint64_t* rem,
                      int num_cus, hipStream_t s);
EspTables esp_host_tables();
EspSa esp_build_sa(const uint8_t* key, size_t key_len, const uint8_t* salt, uint32_t spi, uint32_t mode,
                   uint32_t src_ip, uint32_t dst_ip, uint32_t smac_lo, uint16_t smac_hi, uint32_t dmac_lo,
                   uint16_t dmac_hi);
void esp_run_cpu(const EspBatch& a, bool enc);

hipError_t launch_side(const TablesView& t, const void* pkts, const uint32_t* inmeta, const void* out,
                       const uint32_t* out_meta, const SideOut& side, unsigned long long* port_ctr,
                       unsigned long long* drop_ctr, hipStream_t s,
                       uint32_t n_slots = 0, bool wrap = false, const uint32_t* toep_tab = nullptr);
size_t fused_lds_bytes(int hash_mode, int acl_mode, uint32_t acl_tiles);
// Wide header pairs of a batch resolved in place (kernels.hip pair_kernel; launch_fused runs it
// under launch flag 1 << 10).
hipError_t launch_pairs(void* pkts, uint32_t* inmeta, uint32_t n, const TablesView& t, unsigned long long* port_ctr,
                        bool count, hipStream_t s);
// ... and afterwards: continuation slots' metas -> kCont with the pair's strip / hv (pair_fix_kernel)
hipError_t launch_pair_fix(const uint32_t* inmeta, uint32_t* out_meta, uint32_t n, unsigned long long* drop_ctr,
                           bool count, hipStream_t s);
hipError_t launch_stamp(unsigned long long* dst, hipStream_t s);
hipError_t launch_bucket_update(const uint32_t* idx, uint32_t nb, const void* rows, void* flows,
                                uint32_t bucket_mask, hipStream_t s);
hipError_t launch_harvest(unsigned long long* ctr, unsigned long long* out, uint32_t n, hipStream_t s);

}  // namespace nfdp
