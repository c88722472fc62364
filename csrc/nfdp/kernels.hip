// kernels.hip — CDNA4 (gfx950) data-plane kernels.
//
// Design (MI355X-first, see docs/DATAPLANE.md):
//  * one packet per lane, 8 waves per workgroup, grid sized to the CU count x the LDS-admitted
//    blocks per CU, grid-stride over the batch; a wave's 64 slots are one 4-KiB run moved with
//    lane-contiguous dwordx4 loads/stores and transposed through LDS (coalesced frame I/O);
//  * classification is MFMA GEMMs over the bit-expanded 128-bit FlowKey (rules / hash bits are
//    the M rows, 16 packets the N columns, fragments staged once per workgroup in LDS):
//      - TCAM / priority ACL = key_bits x W[128 x R] + bias, W in {-1,0,+1}; a rule matches
//        iff its mismatch count is 0; first match by min((mismatch << 10) | rule); block-scaled
//        FP4 v_mfma_scale_f32_16x16x128_f8f6f4, the whole key in one instruction (device.h)
//      - Toeplitz RSS hash = LDS byte tables, or GF(2) product key_bits x T[128 x 32] with
//        parity (&1) on v_mfma_i32_16x16x64_i8
//  * exact-match flow lookup: 2-choice cuckoo, a bucket = 4 x {16-B key, 16-B action} = one
//    128-B line fetched wave-cooperatively (8 lanes per line), so a hit in the first bucket is
//    ONE dependent fetch (1M flows = 64 MB of HBM);
//  * per-port counters aggregated in LDS, flushed once per workgroup; per-flow counters are one
//    packed 64-bit atomic per packet.
// The persistent low-latency variant of the same stages lives in ring.hip.
#include "device.h"
#include "shard.h"

namespace nfdp {

// Fused-kernel geometry (overridable at build time for occupancy experiments).
#ifndef NFDP_FUSED_BLOCK
#define NFDP_FUSED_BLOCK 512
#endif
// Early bucket fetch (EARLY instances): the flow-bucket loads are issued between the hash and the
// ACL, so their latency runs under the rule-tile MFMA chain.  Holding the eight bucket lines
// through the ACL needs ~170 VGPRs, i.e. 2 waves / SIMD instead of 4: it pays when the ACL is
// long (many rule tiles survive the prefilter) and loses when it is short, so the launcher picks
// it from the rule-tile count (kEarlyAclTiles).
#ifndef NFDP_EARLY_WAVES_PER_EU
#define NFDP_EARLY_WAVES_PER_EU 2
#endif
#ifndef NFDP_EARLY_ACL_TILES
#define NFDP_EARLY_ACL_TILES 33   // > 512 rules (r2 A/B: -9 % at 256 rules, +13-17 % at 1024)
#endif
constexpr uint32_t kEarlyAclTiles = NFDP_EARLY_ACL_TILES;
constexpr uint32_t kFlagNoEarly = 1u << 8;     // launch flag: never the early-fetch instance (A/B)
constexpr uint32_t kFlagForceEarly = 1u << 9;  // launch flag: the early-fetch instance at any rule count (A/B)
constexpr uint32_t kFlagPairs = 1u << 10;      // launch flag: the batch may hold wide header pairs (pair_kernel first)

#ifndef NFDP_FUSED_WAVES_PER_EU
#define NFDP_FUSED_WAVES_PER_EU 4
#endif
constexpr int kFB = NFDP_FUSED_BLOCK;
#ifndef NFDP_FUSED_MAX_PER_CU
#define NFDP_FUSED_MAX_PER_CU 4   // grid: workgroups per CU the LDS allows, capped here (A/B)
#endif
#ifndef NFDP_KARG_RELOAD
#define NFDP_KARG_RELOAD 1
#endif
constexpr int kFWaves = kFB / 64;

struct FusedArgs {
  TablesView t;
  const uint4* pkts;              // n slots of 64 B
  const uint32_t* inmeta;         // in_port | len << 16
  uint4* out;                     // n slots
  uint32_t* out_meta;             // out_port | len << 16 | reason << 24
  uint32_t n;
  unsigned long long* flow_ctr;   // nbuckets * 8 packed counters (nullable)
  unsigned long long* port_ctr;   // kMaxPorts * 2 packed (rx, tx)
  unsigned long long* drop_ctr;   // kNumReasons
  const unsigned long long* t0;   // batch-release stamp (s_memrealtime ticks, 100 MHz)
  uint32_t* lat;                  // n/16 latency samples (ticks) (nullable)
  const v4i* acl_wfrag;           // [tiles][2][64] A fragments (int8 x16)
  const v4i* acl_cinit;           // [tiles][4] C init (bias) for rows 4g..4g+3
  const v4i* toep_frag;           // [2][2][64] A fragments of the Toeplitz matrix
  const uint32_t* toep_tab;       // [16][256] byte tables (LDS hash variant)
  uint32_t acl_tiles;             // ceil(n_acl / 16)
  uint32_t flags;                 // bit0 no port/drop counters, bit1 no latency samples, bit2 no flow counts, bit8 no early fetch
  // REMOTE variant (replicated tables, N GPUs): frames whose egress port lives on another GPU
  // go to segment[egress gpu] of send_pkt (64-B slot + 4-B meta, fill count in pcnt) instead of
  // out[i]; out_meta[i] then says kRemote.
  uint8_t* send_pkt;
  uint32_t* pcnt;
  uint32_t nranks, rank, cap_pkt;
  SideOut side;                   // flood / mirror / ARP replicas + learn events (side.cnt null: off)
  uint32_t steer;                 // REMOTE: 0 = by egress GPU (after the chain), 1 = by flow owner
                                  // (owner_of(hash) right after classification: the INPUT header +
                                  // ingress meta go to the owner, which runs the whole pipeline)
  const uint32_t* n_dev;          // optional device-side packet count (<= n): batches whose size only
                                  // the GPU knows (packets gathered from the exchange)
  // Flow-owner steering by list (1-GPU instances, nranks > 1): a packet of another GPU's flow
  // shard is not probed / chained / counted here; its index | owner << 26 is appended to this
  // workgroup's region of steer_list (steer_cap_blk entries per workgroup: every packet it could
  // see; the claim is an LDS atomic per wave, no global counter) and steer_kernel copies it to
  // the owner's exchange segment afterwards.  steer_cnt = {grid, steer_cap_blk, count[grid]}.
  // The hot instance keeps its register budget and its fixed-count store tail.
  uint32_t* steer_list;
  uint32_t* steer_cnt;
  uint32_t steer_cap_blk;
  // XFER instances (split chains, kHopXfer): a handed-off frame's HopState record (n x 32 B)
  HopState* hop_state;
  // V6 instances: the folded keys (v6_kernel): row i * v6_key_stride (1: the compact buffer, 4: the
  // out slots)
  const uint4* v6_key;
  uint32_t v6_key_stride;
};

__device__ __forceinline__ size_t lds_align16(size_t x) { return (x + 15) & ~(size_t)15; }

struct LdsLayout {
  size_t acl_w, acl_c, toep_f, toep_t, kx, pc, drops, tports, tchain, tperm, pt_w, pt_c, total;
  uint32_t ltiles, ctiles;  // ACL tiles whose A fragments / C init are staged
  uint32_t ptiles;          // one_block layouts: the prefilter tiles (device.h classify_wave), staged whole
  bool tabs;  // small tables (ports < kLdsPorts, chain words, ACL verdicts) staged in LDS
};
// `one_block`: the instance runs one workgroup per CU (EARLY: 2 waves / SIMD), so the rule tiles
// may use the LDS the second block would have had: every tile's C init and as many A fragments
// as fit (ClassBench-sized rule sets: ~100 of 199 tiles instead of 64).
__host__ __device__ inline LdsLayout lds_layout(int hash_mode, int acl_mode, uint32_t acl_tiles, bool one_block = false) {
  LdsLayout L;
  size_t o = 0;
  uint32_t lt = acl_tiles < kLdsAclTiles ? acl_tiles : kLdsAclTiles, ct = lt;
  const uint32_t pt = (one_block && acl_mode == kAclMfma && NFDP_ACL_PTILES) ? (acl_tiles + 15) / 16 : 0u;
  if (one_block && acl_mode == kAclMfma && acl_tiles > kLdsAclTiles) {
    const size_t rest = (hash_mode == kHashMfma ? 2 * 2 * 64 * 16 : 0) + (hash_mode == kHashLds ? kToepLdsWords * 4 : 0) +
                        kFWaves * 64 * 16 + kLdsPorts * 4 * 4 + kNumReasons * 4 + 16 + kLdsTabBytes +
                        (size_t)pt * (1024 + 64);
    const size_t budget = 160 * 1024 - 2048;   // static LDS + alignment margin
    ct = acl_tiles;
    const size_t room = budget > rest + (size_t)ct * 64 ? budget - rest - (size_t)ct * 64 : 0;
    const uint32_t fit = (uint32_t)(room / 1024) & ~(kAclGroup - 1);
    lt = fit > lt ? (fit < acl_tiles ? fit : acl_tiles) : lt;
  }
  L.ltiles = lt; L.ctiles = ct; L.ptiles = pt;
  L.acl_w = o; if (acl_mode == kAclMfma) o += (size_t)lt * 64 * 16;
  L.acl_c = o; if (acl_mode == kAclMfma) o += (size_t)ct * 4 * 16;
  L.pt_w = o; o += (size_t)pt * 64 * 16;
  L.pt_c = o; o += (size_t)pt * 4 * 16;
  L.toep_f = o; if (hash_mode == kHashMfma) o += 2 * 2 * 64 * 16;
  L.toep_t = o; if (hash_mode == kHashLds) o += kToepLdsWords * 4;
  L.kx = o; o += kFWaves * 64 * 16;
  L.pc = o; o += kLdsPorts * 4 * 4;
  L.drops = o; o += kNumReasons * 4;
  o = (o + 15) & ~(size_t)15;
  // The staged tables must not cost a resident block: within 80 KiB (two blocks per CU, the
  // VGPR-bound maximum) or, for layouts already at one block per CU, within the 160 KiB.
  const size_t with = o + kLdsTabBytes;
  L.tabs = (o <= 80 * 1024) ? (with <= 80 * 1024) : (with <= 160 * 1024 - 1024);
  L.tports = o; L.tchain = o + kLdsPorts * sizeof(PortEntry); L.tperm = L.tchain + kLdsChains * 8;
  if (L.tabs) o = with;
  L.total = (o + 15) & ~(size_t)15;
  return L;
}

// Per-flow packed counter add (no return).  The ablation forms are cost attribution only: without
// the add the headline kernel runs 0.219 instead of 0.273 ms per 4M packets; the same add at
// workgroup scope costs the same; issued one iteration later (after the next bucket loads, state
// in LDS) it is slower, 0.292 ms (r3 s13 A/B, profiles/r3_s13_flowctr_ab.txt): the cost is the
// random read-modify-write itself, not the wait behind it.
__device__ __forceinline__ void flow_ctr_add(unsigned long long* p, unsigned long long v) {
#if defined(NFDP_ABL_NO_FLOWCTR)     // no per-flow counts at all (wrong counters)
  (void)p; (void)v;
#elif defined(NFDP_ABL_FLOWCTR_WG)   // workgroup scope (not coherent across XCDs)
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#else
  atomicAdd(p, v);
#endif
}

constexpr int kBufCfg = 0x00020000;  // buffer resource word 3 (gfx9 family raw buffer)
constexpr int kStreamAux = 2;        // nt: frames are read once / written once (streaming)

// V6: the instances for tables with IPv6 flows / rules (1-GPU, not REMOTE / LIST): IPv6 keys,
// rules and flow checks come from v6_kernel.  Overriding the key costs its rematerialisation
// (the key words are otherwise recomputed from the header), so these instances load the next
// frame after the tail instead of prefetching it under this slot's work: the IPv4-only
// instances keep their register budget untouched.
// XFER: the instances for tables with split chains (kHopXfer hops): a frame handed to another GPU
// leaves its HopState record in a.hop_state (two fixed-count stores in the tail, like the others).
#ifndef NFDP_V6_PREFETCH
#define NFDP_V6_PREFETCH 0   // 1: the V6 instances prefetch the next slot like the IPv4 ones, 2: after
                             // the flow probe (A/B)
#endif
#ifndef NFDP_XFER_WAVES_PER_EU
#define NFDP_XFER_WAVES_PER_EU 4   // the split-chain instances (r5 s9: 346 us / 4M frames with 30 spilled
                                   // VGPRs at 4 waves, 387 us spill-free at 3)
#endif
template <int HASH, int ACL, bool REMOTE, bool EARLY, bool LIST = false, bool V6 = false, bool XFER = false>
__global__ __launch_bounds__(kFB, EARLY ? NFDP_EARLY_WAVES_PER_EU : (XFER ? NFDP_XFER_WAVES_PER_EU : NFDP_FUSED_WAVES_PER_EU))
void fused_kernel(FusedArgs a) {
  static_assert(!V6 || (!REMOTE && !LIST), "IPv6 instances are 1-GPU instances");
  static_assert(!XFER || (!REMOTE && !LIST && !V6), "split-chain instances are 1-GPU IPv4 instances");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ uint32_t rcnt[REMOTE ? 2 * kMaxRanks : 1], rbase[REMOTE ? kMaxRanks : 1];  // rcnt double-buffered
  __shared__ uint32_t lst_n;                                  // LIST: entries of this workgroup's region
  __shared__ uint32_t side_n;                                 // side-list entries of this workgroup (regions)
  const LdsLayout L = lds_layout(HASH, ACL, a.acl_tiles, EARLY);
  v4i* lw = reinterpret_cast<v4i*>(smem + L.acl_w);
  v4i* lc = reinterpret_cast<v4i*>(smem + L.acl_c);
  v4i* lt = reinterpret_cast<v4i*>(smem + L.toep_f);
  uint32_t* ltab = reinterpret_cast<uint32_t*>(smem + L.toep_t);
  uint4* kx = reinterpret_cast<uint4*>(smem + L.kx) + (threadIdx.x >> 6) * 64;
  uint32_t* pc = reinterpret_cast<uint32_t*>(smem + L.pc);   // [4][256]: rx_pk rx_by tx_pk tx_by
  uint32_t* drops = reinterpret_cast<uint32_t*>(smem + L.drops);

  // ---- stage classification tables + zero counters ----
  if constexpr (ACL == kAclMfma) {
    const uint32_t nw = L.ltiles * 64, nc = L.ctiles * 4;
    for (uint32_t i = threadIdx.x; i < nw; i += kFB) lw[i] = a.acl_wfrag[i];
    for (uint32_t i = threadIdx.x; i < nc; i += kFB) lc[i] = a.acl_cinit[i];
  }
  // one_block (EARLY) layouts: the prefilter tiles after the rule tiles' fragments / the prefilters
  const v4i* pw = reinterpret_cast<const v4i*>(smem + L.pt_w);
  const v4i* pcw = reinterpret_cast<const v4i*>(smem + L.pt_c);
  if constexpr (ACL == kAclMfma && EARLY) {
    const v4i* gpw = a.acl_wfrag + (size_t)a.acl_tiles * 64;
    const v4i* gpc = a.acl_cinit + (size_t)a.acl_tiles * 6 + (size_t)acl_groups(a.acl_tiles) * 2;
    for (uint32_t i = threadIdx.x; i < L.ptiles * 64; i += kFB) const_cast<v4i*>(pw)[i] = gpw[i];
    for (uint32_t i = threadIdx.x; i < L.ptiles * 4; i += kFB) const_cast<v4i*>(pcw)[i] = gpc[i];
  }
  const AclView av{lw, lc, a.acl_wfrag, a.acl_cinit, a.acl_tiles, L.ltiles, L.ctiles, pw, pcw, L.ptiles};
  if constexpr (HASH == kHashMfma)
    for (uint32_t i = threadIdx.x; i < 256; i += kFB) lt[i] = a.toep_frag[i];
  if constexpr (HASH == kHashLds)
    stage_toep(ltab, a.toep_tab, threadIdx.x, kFB);
  for (uint32_t i = threadIdx.x; i < kLdsPorts * 4; i += kFB) pc[i] = 0;
  if (threadIdx.x < kNumReasons) drops[threadIdx.x] = 0;
  if constexpr (REMOTE)
    if (threadIdx.x < 2 * kMaxRanks) rcnt[threadIdx.x] = 0;
  if constexpr (LIST)
    if (threadIdx.x == 0) lst_n = 0;
  if (threadIdx.x == 0) side_n = 0;
  PortEntry* lport = reinterpret_cast<PortEntry*>(smem + L.tports);
  uint64_t* lchain = reinterpret_cast<uint64_t*>(smem + L.tchain);
  uint8_t* lperm = smem + L.tperm;
  const LdsTables ta = stage_lds_tables(a.t, lport, lchain, lperm, L.tabs, kFB);
  __syncthreads();

  const unsigned long long t0 = a.t0 ? *a.t0 : __builtin_amdgcn_s_memrealtime();
  const uint32_t n = a.n_dev ? min(a.n, *a.n_dev) : a.n;
  const uint32_t stride = gridDim.x * kFB;
  // Software pipeline over the grid-stride loop.  s_waitcnt vmcnt retires loads, stores and
  // atomics together in issue order, so the next slot's frame is loaded BEFORE this slot's
  // flow-counter atomic and output stores: waiting for the frame never waits for them, and the
  // atomic (a memory-side RMW, the longest trip of the iteration) completes under the next
  // slot's parse + classification.
  uint32_t dn[kSlotDwords];
  uint32_t imn;
  // raw buffer views (num_records = valid bytes; offsets past it read 0 / drop the store)
  const __amdgpu_buffer_rsrc_t r_pk = __builtin_amdgcn_make_buffer_rsrc((void*)a.pkts, (short)0, (int)(a.n * 64u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_im = __builtin_amdgcn_make_buffer_rsrc((void*)a.inmeta, (short)0, (int)(a.n * 4u), kBufCfg);
  // first 4-KiB run of this wave (prefetched frames arrive chunk-per-lane in cn)
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u;  // wave-uniform (SGPR)
  auto run_of = [&](uint32_t base) { return base + wave0 < n ? (base + wave0) * 64u : kNoRun; };
  v4u cn[4];
  {
    wave_frames_load<kStreamAux>(r_pk, run_of(blockIdx.x * kFB), cn);
    const uint32_t i0 = blockIdx.x * kFB + threadIdx.x;
    imn = __builtin_amdgcn_raw_buffer_load_b32(r_im, i0 < n ? i0 * 4u : kNoRun, 0, kStreamAux);
  }
  const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc((void*)a.out, (short)0, (int)(a.n * 64u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_meta = __builtin_amdgcn_make_buffer_rsrc((void*)a.out_meta, (short)0, (int)(a.n * 4u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_lat = __builtin_amdgcn_make_buffer_rsrc((void*)a.lat, (short)0,
                                                                          a.lat ? (int)(((a.n + 15u) >> 4) * 4u) : 0, kBufCfg);
  const uint32_t ctr_mask = min(a.t.bucket_mask * kBucketSlots + (kBucketSlots - 1), 4095u);
  // REMOTE: the per-peer segments (< 2 GiB in all, checked at launch)
  const __amdgpu_buffer_rsrc_t r_send = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.send_pkt, (short)0, REMOTE ? (int)(a.nranks * pkt_seg_bytes(a.cap_pkt)) : 0, kBufCfg);
  // LIST: the steer list (entries < 2^26, checked at launch: byte offsets fit 32 bits)
  const __amdgpu_buffer_rsrc_t r_list = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.steer_list, (short)0, LIST ? (int)(gridDim.x * a.steer_cap_blk * 4u) : 0, kBufCfg);
  // XFER: the hand-off records (n * 32 B < 2 GiB: n < 2^25, checked at launch)
  const __amdgpu_buffer_rsrc_t r_hop = __builtin_amdgcn_make_buffer_rsrc(
      (void*)a.hop_state, (short)0, XFER ? (int)(a.n * 32u) : 0, kBufCfg);
  uint32_t it = 0;  // loop iteration (REMOTE reservation buffers alternate)
#if NFDP_KARG_RELOAD
  // The tables' bases and sizes are read where a stage uses them, from the kernel's argument
  // block (constant address space: scalar loads that hit the scalar cache), through a pointer
  // laundered once per iteration so the loads cannot be hoisted out of the loop.  Hoisted, the
  // ~75 dwords of TablesView stay live in SGPRs across the whole loop and the allocator spills
  // ~330 of them into VGPR lanes (v_writelane / v_readlane: VALU work and VGPRs the hot instance
  // does not have).
  typedef const __attribute__((address_space(4))) FusedArgs KArgs;
  KArgs* const kargs0 = (KArgs*)__builtin_amdgcn_kernarg_segment_ptr();
#endif
  for (uint32_t base = blockIdx.x * kFB; base < n; base += stride, ++it) {
    const uint32_t i = base + threadIdx.x;
    const bool valid = i < n;
#if NFDP_KARG_RELOAD
    KArgs* ka = kargs0;
    // (the LIST instances keep their hoisted bases: laundered, their VGPR spills grew 16 -> 19)
    if constexpr (!LIST) asm volatile("" : "+s"(ka));
    const TablesView& TV = *(const TablesView*)&ka->t;
    const LdsTables ta_it{TV, ta.lport, ta.lchain, ta.lperm, ta.nport, ta.nchain, ta.lds_perm};
#else
    const TablesView& TV = a.t;
    const LdsTables& ta_it = ta;
#endif
    wave_frames_to_lanes(kx, cn, dn);
    Parsed p;
    IngressState st;
    ingress_stage<LdsTables, false>(TV, ta_it, dn, imn, p, st);  // copies the frame into p.s: dn is free for the prefetch
    // IPv6 keys (tables with IPv6 flows / rules): v6_kernel folded them into a.v6_key (the compact
    // buffer, or out[i], overwritten by this lane's egress slot in the tail)
    if constexpr (V6) {
      if (__builtin_expect(__any(p.ipv6), 0)) {
        if (p.ipv6 && valid) {
          const uint4 k6 = a.v6_key[(size_t)i * a.v6_key_stride];
          st.key.src_ip = k6.x; st.key.dst_ip = k6.y; st.key.ports = k6.z; st.key.meta = k6.w;
        }
      }
    }
    const bool flowp = V6 ? flowable(TV, p) : p.ipv4;   // takes part in the flow stage
    // (a continuation slot of a wide header pair is bad_port here - in-meta port kPortCont;
    // pair_fix_kernel turns its meta / counters into kCont afterwards: no pair code in this loop)

    if (!valid) st.reason = kMalformed;

    uint32_t hash = 0;
    int acl_rule = -1;
    uint4 bv[8];
    if constexpr (EARLY) {
      // the bucket fetch leaves as soon as the hash is known: its latency runs under the ACL
      auto issue = [&](uint32_t h) { flow_probe_issue(TV, h, bv); };
      classify_wave<HASH, ACL, decltype(issue), true>(st.key, kx, av, lt, ltab, TV, hash, acl_rule, 0, 1, nullptr, issue);
    } else {
      classify_wave<HASH, ACL>(st.key, kx, av, lt, ltab, TV, hash, acl_rule);
    }
    // IPv6: the rule comes from the IPv6 TCAM (v6_kernel ran over this batch), never from the
    // IPv4 rules over the folded key (wave-uniform skip for all-IPv4 waves)
    // (instances without V6 run only for tables with no IPv6 flows / rules: an IPv6 packet's key
    // carries kKeyV6, which no IPv4 rule or flow matches)
    bool v6ok = false;
    if constexpr (V6) {
      if (__builtin_expect(__any(p.ipv6), 0)) {
        // (v6_kernel parks each IPv6 packet's rule + 1 | verified-hit << 31 in its out_meta word,
        // which this lane overwrites with the egress meta in the tail)
        if (p.ipv6) {
          const uint32_t w6 = valid ? a.out_meta[i] : 0u;
          acl_rule = (int)(w6 & 0xFFFFu) - 1;
          v6ok = (w6 >> 31) != 0;
        }
      }
    }
    // flow-owner steering (REMOTE steer = 1, or the 1-GPU instance's steer list): a packet of
    // another GPU's flow shard leaves now, as it came in; its owner runs the whole pipeline on it
    bool to_owner = false;
    uint32_t owner = a.rank;
    if constexpr (REMOTE) {
      if (a.steer) {
        owner = owner_of(hash, a.nranks);
        to_owner = valid && !st.reason && flowp && owner != a.rank;
        if (to_owner) st.reason = kRemote;  // no local probe / chain / counters
      }
    } else if constexpr (LIST) {   // separate instances: the 1-GPU hot kernel is untouched
      // the owner test only (the flag lives in st.reason: no probe / chain / counters); the list
      // append comes after the tail's stores, where the register pressure is lowest (placed
      // here, the same append cost the instance 15 more spilled VGPRs)
      if (valid && !st.reason && flowp && owner_of(hash, a.nranks) != a.rank) st.reason = kRemote;
    }
    if constexpr (!REMOTE && (!V6 || NFDP_V6_PREFETCH == 1)) {
      // prefetch the next slot now: it lands under this slot's probe and chain
      const uint32_t nx = i + stride;
      wave_frames_load<kStreamAux>(r_pk, run_of(base + stride), cn);
      imn = __builtin_amdgcn_raw_buffer_load_b32(r_im, nx < n ? nx * 4u : kNoRun, 0, kStreamAux);
    }

    bool hit = false;
    FlowAction act = {};
    int64_t slot = -1;
#ifndef NFDP_LANE_PROBE
    {
      uint4 v;
      if constexpr (EARLY) slot = flow_probe_finish(TV, st.key, hash, !st.reason && flowp, kx, bv, v);
      else slot = flow_probe_wave(TV, st.key, hash, !st.reason && flowp, kx, v);
#else
    if (!st.reason && flowp) {
      uint4 v;
      slot = flow_probe(TV, st.key, hash, v);
#endif
      // an IPv6 folded-key hit counts only if the slot's side entry holds this packet's addresses:
      // v6_kernel checked that before this kernel (bit 31 of the word it parked in out_meta[i])
      if (V6 && p.ipv6 && !v6ok) slot = -1;
      if (slot >= 0) {
        hit = true;
        act.chain_id = v.x & 0xFFFFu; act.out_port = v.x >> 16; act.nat_ip = v.y;
        act.nat_port = v.z & 0xFFFFu; act.vlan = v.z >> 16; act.flow_id = v.w;
      }
    }
    if constexpr (V6 && NFDP_V6_PREFETCH == 2) {   // the next slot under this one's chain, emit and tail
      const uint32_t nx = i + stride;
      wave_frames_load<kStreamAux>(r_pk, run_of(base + stride), cn);
      imn = __builtin_amdgcn_raw_buffer_load_b32(r_im, nx < n ? nx * 4u : kNoRun, 0, kStreamAux);
    }
#ifndef NFDP_ABL_NO_CHAIN
    const EgressDecision e = chain_stage<LdsTables, V6, XFER>(TV, ta_it, p, st, hit, act, acl_rule, hash);
#else  // cost attribution only (wrong results): no chain, the flow's port
    EgressDecision e{};
    e.out_port = hit ? act.out_port : kPortNone;
    e.reason = st.reason ? st.reason : (hit ? kOk : kNoRoute);   // a miss never egresses to kPortNone
#endif
    bool to_peer = false;
    uint32_t reason = e.reason;
    uint32_t eg = 0, pos = 0;
    if constexpr (REMOTE) {
      // egress GPU of the frame (or the flow owner when steering); block-aggregated slot in that
      // GPU's segment (all threads call)
      eg = a.steer ? owner : (e.reason ? a.rank : (uint32_t)ta_it.port(e.out_port).gpu);
      const bool remote = a.steer ? to_owner : (valid && !e.reason && eg != a.rank && eg < a.nranks);
      pos = reserve_block(a.pcnt, eg, remote, a.nranks, rcnt + (it & 1u) * kMaxRanks, rbase,
                          rcnt + (~it & 1u) * kMaxRanks);
      if (remote) {
        if (pos < a.cap_pkt) {
          uint8_t* segp = a.send_pkt + (size_t)eg * pkt_seg_bytes(a.cap_pkt);
          reinterpret_cast<uint32_t*>(segp + pkt_meta_off(a.cap_pkt))[pos] =
              a.steer ? imn : make_meta(e.out_port, egress_len(p, e), kOk, e.xhdr != 0);
          to_peer = true;
        } else {
          reason = kOverflow;
        }
      }
    }
    if (REMOTE && to_owner && !to_peer) reason = kOverflow;  // the owner's segment was full: dropped here
    // steer list: always delivered to the owner (kRemote is set only by the steer test here)
    const bool listed = LIST && e.reason == kRemote;
    const uint32_t olen = reason == e.reason ? (XFER ? out_len(p, e) : egress_len(p, e)) : 0u;
    const uint32_t meta = (to_peer || listed)
                              ? make_meta((a.steer || listed) ? kPortNone : e.out_port,
                                          (a.steer || listed) ? st.wire_len : olen, kRemote)
                              : make_meta(reason == kOverflow ? kPortNone : e.out_port, olen, reason,
                                          !reason && e.xhdr, !reason && e.flood);
    // port / drop counters: LDS, global only for ports >= kLdsPorts (issued before the tail)
    if (valid && !(a.flags & 1u) && !((to_owner && to_peer) || listed)) {  // a steered packet is counted by its owner
      if (st.in_port < kLdsPorts) {
        atomicAdd(&pc[st.in_port], 1u); atomicAdd(&pc[kLdsPorts + st.in_port], st.wire_len);
      } else if (st.in_port < (uint32_t)kMaxPorts) {
        atomicAdd(a.port_ctr + 2 * st.in_port, ctr_inc(st.wire_len));
      }
      if (reason) {
        atomicAdd(&drops[reason & (kNumReasons - 1)], 1u);
      } else if (to_peer) {
        // tx is counted where the frame leaves: the egress GPU's egress_kernel
      } else if (e.out_port < kLdsPorts) {
        atomicAdd(&pc[2 * kLdsPorts + e.out_port], 1u); atomicAdd(&pc[3 * kLdsPorts + e.out_port], olen);
      } else {
        atomicAdd(a.port_ctr + 2 * e.out_port + 1, ctr_inc(olen));
      }
    }
    uint32_t o[kSlotDwords];
    // a steered packet travels as it came in (p is untouched: the chain never ran on it); a listed
    // one is copied from the INPUT slot by steer_kernel (its out[] slot is not read)
#ifndef NFDP_ABL_NO_EMIT
    emit(p, to_owner ? p.tci : e.tci, to_owner ? p.tagged : e.push != 0, o);
#else  // cost attribution only (wrong results): the normalized header as is
#pragma unroll
    for (int q = 0; q < kSlotDwords; ++q) o[q] = p.s[q];
#endif
    if (a.side.cnt) {
      // flood / mirror / ARP-trap / learning packets go on the side list (side_kernel emits their
      // replicas and learn events after this kernel): a wave-uniform skip in the common case
      const bool sn = valid && side_needed(st, p, e);
      if (__builtin_expect(__any(sn), 0)) {
        // (the LIST instances keep the flat list: their register budget has no room for the
        // region form, and multi-GPU steering is where flagged packets are rare)
        if constexpr (LIST) side_list_append(a.side, sn, i);
        else side_list_append_blk(a.side, &side_n, sn, i);
      }
    }
    const bool sample = a.lat && !(a.flags & 2u) && (i & 15u) == 0 && !to_peer && !listed;
    const uint32_t lat_now = sample ? (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0) : 0u;
    if constexpr (!REMOTE) {
      // Fixed-count tail: every lane issues the same vector-memory instructions with no branch
      // around them (out-of-range buffer offsets are dropped by the hardware; a miss adds 0),
      // so the compiler can wait for the prefetched frame with vmcnt(N > 0) at the loop head
      // instead of draining this slot's atomic and stores.
      const uint32_t cslot = hit ? (uint32_t)slot : (i & ctr_mask);
      flow_ctr_add(a.flow_ctr + cslot, (hit && !(a.flags & 4u)) ? ctr_inc(st.wire_len) : 0ull);
      wave_frames_store<kStreamAux>(kx, o, r_out, run_of(base));
      __builtin_amdgcn_raw_buffer_store_b32(meta, r_meta, valid ? i * 4u : kNoRun, 0, kStreamAux);
      __builtin_amdgcn_raw_buffer_store_b32(lat_now, r_lat, sample ? (i >> 4) * 4u : kNoRun, 0, 0);
      if constexpr (LIST) {
        const unsigned long long m = __ballot(listed);
        uint32_t off = kNoRun;   // byte offset into the list; out of range = the lane stores nothing
        if (__builtin_expect(m != 0ull, 0)) {
          // rank among the wave's listed lanes (mbcnt: no 64-bit lane masks in VGPRs); the lowest
          // listed lane claims the wave's run with one LDS atomic, readlane broadcasts it (SGPR)
          const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          const int leader = __builtin_ctzll(m);
          uint32_t base = 0;
          if (listed && pre == 0) base = atomicAdd(&lst_n, (uint32_t)__builtin_popcountll(m));   // LDS: lgkmcnt only
          base = __builtin_amdgcn_readlane(base, leader);
          if (listed) off = (blockIdx.x * a.steer_cap_blk + base + pre) * 4u;
        }
        // one store per iteration whatever the ballot: the loop's vector-memory count stays fixed,
        // so the wait for the prefetched frame keeps its vmcnt(N > 0) (a store under a branch
        // would force vmcnt(0) at the loop head and expose this slot's tail)
        __builtin_amdgcn_raw_buffer_store_b32(i | (owner_of(hash, a.nranks) << 26), r_list, off, 0, 0);
      }
      if constexpr (XFER) {
        // a frame whose chain continues on another GPU: its record (hop_state_of), stored by every
        // lane (out-of-range offset: dropped) so the tail's memory-instruction count stays fixed
        const bool xf = valid && e.reason == kRemote && e.inner_len != 0u;
        const HopState hs = hop_state_of(p, st, e, act, acl_rule, hash);
        const uint32_t off = xf ? i * 32u : kNoRun;
        const v4u h0 = {hs.inmeta, hs.hash, (uint32_t)hs.acl_rule, hs.hop};
        const v4u h1 = {(uint32_t)act.chain_id | ((uint32_t)act.out_port << 16), act.nat_ip,
                        (uint32_t)act.nat_port | ((uint32_t)act.vlan << 16), act.flow_id};
        store_b128<kStreamAux>(h0, r_hop, off, 0);
        store_b128<kStreamAux>(h1, r_hop, off, 16);
      }
      if constexpr (V6 && NFDP_V6_PREFETCH == 0) {   // (no prefetch: the next slot is loaded here)
        const uint32_t nx = i + stride;
        wave_frames_load<kStreamAux>(r_pk, run_of(base + stride), cn);
        imn = __builtin_amdgcn_raw_buffer_load_b32(r_im, nx < n ? nx * 4u : kNoRun, 0, kStreamAux);
      }
    } else {
      if (hit && a.flow_ctr && !(a.flags & 4u)) atomicAdd(a.flow_ctr + slot, ctr_inc(st.wire_len));
      // frames for a peer: per lane into its segment slot; local frames: coalesced into out[]
      wave_segment_store<kStreamAux>(kx, o, r_send, to_peer, eg, pos, (uint32_t)pkt_seg_bytes(a.cap_pkt), a.cap_pkt);
      wave_frames_store<kStreamAux>(kx, o, r_out, run_of(base), __ballot(to_peer));
      if (valid) {
        a.out_meta[i] = meta;
        if (sample) a.lat[i >> 4] = lat_now;
      }
      const uint32_t nx = i + stride;
      wave_frames_load<kStreamAux>(r_pk, run_of(base + stride), cn);
      imn = __builtin_amdgcn_raw_buffer_load_b32(r_im, nx < n ? nx * 4u : kNoRun, 0, kStreamAux);
    }
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < kLdsPorts; q += kFB) {
    if (pc[q]) atomicAdd(a.port_ctr + 2 * q, ((unsigned long long)pc[q] << 40) | pc[kLdsPorts + q]);
    if (pc[2 * kLdsPorts + q])
      atomicAdd(a.port_ctr + 2 * q + 1, ((unsigned long long)pc[2 * kLdsPorts + q] << 40) | pc[3 * kLdsPorts + q]);
  }
  if (threadIdx.x < kNumReasons && drops[threadIdx.x])
    atomicAdd(a.drop_ctr + threadIdx.x, (unsigned long long)drops[threadIdx.x]);
  if (!LIST && a.side.cnt && threadIdx.x == 0) {
    // this workgroup's side-list region: its count for side_kernel, the batch total for the host
    const uint32_t c = side_n;
    a.side.blk_cnt[blockIdx.x] = c < a.side.blk_cap ? c : a.side.blk_cap;
    if (c) atomicAdd(a.side.cnt + 5, c);
    if (c > a.side.blk_cap) atomicAdd(a.side.cnt + 6, c - a.side.blk_cap);
  }
  if constexpr (LIST) {
    if (threadIdx.x == 0) {
      a.steer_cnt[2 + blockIdx.x] = lst_n;
      if (blockIdx.x == 0) { a.steer_cnt[0] = gridDim.x; a.steer_cnt[1] = a.steer_cap_blk; }
    }
  }
}

// Wide header pairs, batch form: one thread per continuation slot runs decap_pair on (head,
// continuation) and rewrites them in place - a terminated head's slot becomes its inner frame and
// its in-meta the tunnel port + inner length (its outer rx is counted on the VTEP port here); the
// continuation's in-meta keeps kPortCont and carries strip | hv << 8 | kPairDone.  The fused
// kernel then sees only ordinary slots (its register budget is untouched).  Idempotent: a pair
// already marked done is skipped, so a batch can be run again.
__global__ __launch_bounds__(256) void pair_kernel(uint4* pkts, uint32_t* inmeta, uint32_t n, TablesView t,
                                                   unsigned long long* port_ctr, uint32_t count) {
  // A wave owns a run of 64 consecutive slots: one coalesced 4-KiB load into its LDS tile (per-lane
  // 64-B slots at a 64-B stride ran at a quarter of the bandwidth), the pairs whose continuation
  // lies in the run are resolved from the tile, and only the head slots it rewrote are stored back
  // (coalesced, the other chunks masked off).  A head just before the run (the previous run's last
  // slot) belongs to this wave's lane 0 and is read / written in global memory: its own run never
  // stores an unmodified slot, so nothing races with that write.  Block-uniform trips; the VTEP rx
  // count is tallied per workgroup (every pair of a VTEP port adding to one counter word
  // serialised at the memory side: 25 ms per 2M pairs, r3 s23 trace).
  // The tile's 16-B chunks are XOR-swizzled per group of 4 slots (chunk q of slot s at 4s + (q ^
  // (s >> 2 & 3))): a lane reading its own 64-B slot otherwise hits the banks of lanes 4, 8, 12 on.
  __shared__ uint4 tile[4][256];
  __shared__ uint32_t vpk[kLdsPorts], vby[kLdsPorts];   // VTEP rx counts of this workgroup (ports < 256)
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint4* T = tile[wv];
  const uint32_t lsw = (lane >> 4) & 3u;   // swizzle of linear chunk q*64 + lane
  auto at = [](uint32_t s, int q) { return 4u * s + ((uint32_t)q ^ ((s >> 2) & 3u)); };
  for (uint32_t q = threadIdx.x; q < kLdsPorts; q += 256) { vpk[q] = 0; vby[q] = 0; }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r_pk = __builtin_amdgcn_make_buffer_rsrc((void*)pkts, (short)0, (int)(n * 64u), kBufCfg);
  for (uint32_t base = blockIdx.x * 256; base < n; base += gridDim.x * 256) {
    const uint32_t run0 = base + (wv << 6);
    const uint32_t soff = run0 < n ? run0 * 64u : kNoRun;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const v4u c = __builtin_amdgcn_raw_buffer_load_b128(r_pk, lane * 16u + q * 1024u, soff, 0);
      T[(q * 64 + lane) ^ lsw] = make_uint4(c.x, c.y, c.z, c.w);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const uint32_t i = run0 + lane;
    bool term = false, in_tile = false;
    uint32_t vport = 0, vlen = 0;
    const uint32_t cim = i < n ? inmeta[i] : 0u;
    if (i < n && (cim & 0xFFFFu) == kPortCont && !((cim >> 16) & kPairDone)) {
      uint32_t ci = (uint32_t)kSlotBytes << 8;
      const uint32_t him = i ? inmeta[i - 1] : kPortCont;
      if ((him & 0xFFFFu) != kPortCont) {
        uint32_t d[kSlotDwords], x[kSlotDwords], inner[kSlotDwords], strip, hv;
        in_tile = lane > 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 v = in_tile ? T[at(lane - 1, q)] : pkts[(size_t)(i - 1) * 4 + q];
          const uint4 w = T[at(lane, q)];
          d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
          x[4 * q] = w.x; x[4 * q + 1] = w.y; x[4 * q + 2] = w.z; x[4 * q + 3] = w.w;
        }
        const int tp = decap_pair(t, DirectTables{t}, d, x, him, inner, strip, hv);
        if (tp >= 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint4 o = make_uint4(inner[4 * q], inner[4 * q + 1], inner[4 * q + 2], inner[4 * q + 3]);
            if (in_tile) T[at(lane - 1, q)] = o;
            else pkts[(size_t)(i - 1) * 4 + q] = o;
          }
          inmeta[i - 1] = (uint32_t)tp | (((him >> 16) - strip) << 16);
          term = true; vport = him & 0xFFFFu; vlen = him >> 16;   // the outer frame, on its VTEP port
          ci = strip | (hv << 8);
        }
      }
      inmeta[i] = kPortCont | ((ci | kPairDone) << 16);
    }
    // slots of the run this wave rewrote: the head before each terminating lane > 0
    const unsigned long long mod = __ballot(term && in_tile) >> 1;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (mod) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = T[(q * 64 + lane) ^ lsw];
        const v4u w = {v.x, v.y, v.z, v.w};
        const bool keep = (mod >> (16u * q + (lane >> 2))) & 1ull;   // chunk q*64+lane is part of slot 16q + lane/4
        store_b128<0>(w, r_pk, keep ? lane * 16u + q * 1024u : kNoRun, soff);
      }
    }
    __builtin_amdgcn_wave_barrier();   // the tile is reloaded next trip
    if (count) {
      // per-workgroup LDS tallies, one global atomic per port per workgroup at the end (a
      // per-wave atomic on the VTEP port's counter word still serialised 64K waves at the memory
      // side: 0.81 ms per 4M slots, r3 s27 trace).  A wave whose pairs all sit on one VTEP port
      // (the usual case) adds its sums with one LDS atomic each: 64 lanes on one word serialise.
      const bool tv = term && vport < (uint32_t)kLdsPorts;
      const unsigned long long tb = __ballot(tv);
      if (tb) {
        const int lead = __builtin_ctzll(tb);
        const uint32_t p0 = __shfl(vport, lead);
        if (!__ballot(tv && vport != p0)) {
          uint32_t sum = tv ? vlen : 0u;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
          if ((int)lane == lead) { atomicAdd(&vpk[p0], (uint32_t)__popcll(tb)); atomicAdd(&vby[p0], sum); }
        } else if (tv) {
          atomicAdd(&vpk[vport], 1u); atomicAdd(&vby[vport], vlen);
        }
      }
      wave_counter_add(port_ctr, 2 * vport, vlen, true, term && vport >= (uint32_t)kLdsPorts);
    }
  }
  if (count) {
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < kLdsPorts; q += 256)
      if (vpk[q]) atomicAdd(port_ctr + 2 * q, ((unsigned long long)vpk[q] << 40) | vby[q]);
  }
}

// After the fused kernel: each continuation slot's meta becomes kCont with its pair's strip / hv,
// and its bad_port count (in-meta port kPortCont) moves to kCont.
__global__ __launch_bounds__(256) void pair_fix_kernel(const uint32_t* inmeta, uint32_t* out_meta, uint32_t n,
                                                       unsigned long long* drop_ctr, uint32_t count) {
  __shared__ uint32_t c;
  if (threadIdx.x == 0) c = 0;
  __syncthreads();
  uint32_t mine = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t im = inmeta[i];
    if ((im & 0xFFFFu) != kPortCont) continue;
    const uint32_t ci = pair_cinfo(im);
    out_meta[i] = cont_meta(ci & 0xFFu, ci >> 8);
    ++mine;
  }
  if (mine) atomicAdd(&c, mine);
  __syncthreads();
  if (threadIdx.x == 0 && c && count) {
    atomicAdd(drop_ctr + kBadPort, 0ull - (unsigned long long)c);
    atomicAdd(drop_ctr + kCont, (unsigned long long)c);
  }
}

hipError_t launch_pair_fix(const uint32_t* inmeta, uint32_t* out_meta, uint32_t n, unsigned long long* drop_ctr,
                           bool count, hipStream_t s) {
  if (!inmeta || !out_meta || !drop_ctr) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  // (256 workgroups, fewer same-address counter atomics at the end, measured slower: 36 vs 24 us
  // per 4M slots, r3 s32 vs s27: the per-slot loop wants the parallelism)
  const uint32_t g = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(pair_fix_kernel, dim3(g), dim3(256), 0, s, inmeta, out_meta, n, drop_ctr, count ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_pairs(void* pkts, uint32_t* inmeta, uint32_t n, const TablesView& t, unsigned long long* port_ctr,
                        bool count, hipStream_t s) {
  if (!pkts || !inmeta || !port_ctr) return hipErrorInvalidValue;
  if (n >= (1u << 25)) return hipErrorInvalidValue;   // 32-bit buffer views of the slots
  if (n == 0) return hipSuccess;
  const uint32_t g = (n + 255) / 256 < 2048 ? (n + 255) / 256 : 2048;
  hipLaunchKernelGGL(pair_kernel, dim3(g), dim3(256), 0, s, reinterpret_cast<uint4*>(pkts), inmeta, n, t, port_ctr,
                     count ? 1u : 0u);
  return hipGetLastError();
}

// Side pass (pipeline.h side_stage) over the packets the per-packet kernel put on the side list:
// flood replicas, mirror and ARP copies, learn events.  Reads the list length on the device.
struct SideArgs {
  TablesView t;
  const uint4* pkts; const uint32_t* inmeta; const uint4* out; const uint32_t* out_meta;
  SideOut side;
  unsigned long long* port_ctr; unsigned long long* drop_ctr;
  uint32_t n_slots;   // slots of the batch / ring (0: no wide pairs); a pair's continuation is the next slot
  uint32_t wrap;      // 1: ring slots (the next slot wraps modulo n_slots)
  const uint32_t* toep_tab;   // [16][256] Toeplitz byte tables (null: bit-by-bit hash)
};
// Toeplitz from byte tables staged in LDS (the side pass's tunnel entropy / flood LAG hash; the
// bit-by-bit form was most of side_kernel's time with every packet encapsulated)
struct LdsToeplitz {
  const uint32_t* tab;
  __device__ uint32_t operator()(const FlowKey& k) const {
    const uint32_t w[4] = {k.src_ip, k.dst_ip, k.ports, k.meta};
    uint32_t h = 0;
#pragma unroll
    for (int b = 0; b < 16; ++b) h ^= tab[b * 256 + ((w[b >> 2] >> (8 * (b & 3))) & 0xFFu)];
    return h;
  }
};
#ifndef NFDP_SIDE_WAVES_PER_EU
#define NFDP_SIDE_WAVES_PER_EU 1
#endif
__global__ __launch_bounds__(256, NFDP_SIDE_WAVES_PER_EU) void side_kernel(SideArgs a) {
  __shared__ uint32_t stab[16 * 256];
  __shared__ __attribute__((aligned(16))) uint8_t ltabs[kLdsTabBytes];   // ports / chain words / verdicts
  if (a.toep_tab)
    for (uint32_t q = threadIdx.x; q < 16 * 256; q += 256) stab[q] = a.toep_tab[q];
  const LdsTables ta = stage_lds_tables(a.t, reinterpret_cast<PortEntry*>(ltabs),
                                        reinterpret_cast<uint64_t*>(ltabs + kLdsPorts * sizeof(PortEntry)),
                                        ltabs + kLdsPorts * sizeof(PortEntry) + kLdsChains * 8, true, 256);
  __syncthreads();
  // flat list [0, cnt[5]) or the fused kernel's per-workgroup regions (blk_cnt[b] entries each)
  const bool blk = a.side.blk_cnt != nullptr;
  const uint32_t n = blk ? a.side.nblk * a.side.blk_cap : min(a.side.cnt[5], a.side.cap_list);
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
    if (blk) {
      const uint32_t r = j / a.side.blk_cap;
      if (j - r * a.side.blk_cap >= a.side.blk_cnt[r]) continue;
    }
    const uint32_t i = a.side.list[j];
    uint32_t d[kSlotDwords];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 v = a.pkts[(size_t)i * 4 + q];
      d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
    }
    // the egress slot is read only where a replica copies it (mirroring): in place, not loaded for
    // every listed packet (an overlay egress lists all of them for their outer headers)
    const uint32_t* o = reinterpret_cast<const uint32_t*>(a.out + (size_t)i * 4);
    // a terminated pair head: its side work is on the inner frame (the same decap_pair decision
    // the pair pass / ring kernel took; a batch's pair pass already rewrote it: then decap_pair
    // sees an ordinary frame and returns -1)
    uint32_t im = a.inmeta[i];
    if (a.n_slots && (im & 0xFFFFu) != kPortCont) {
      const uint32_t j = a.wrap ? (i + 1) % a.n_slots : i + 1;
      if (j < a.n_slots && (a.inmeta[j] & 0xFFFFu) == kPortCont) {
        uint32_t x[kSlotDwords], inner[kSlotDwords], strip, hv;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint4 v = a.pkts[(size_t)j * 4 + q];
          x[4 * q] = v.x; x[4 * q + 1] = v.y; x[4 * q + 2] = v.z; x[4 * q + 3] = v.w;
        }
        const int tp = decap_pair(a.t, DirectTables{a.t}, d, x, im, inner, strip, hv);
        if (tp >= 0) {
#pragma unroll
          for (int k = 0; k < kSlotDwords; ++k) d[k] = inner[k];
          im = (uint32_t)tp | (((im >> 16) - strip) << 16);
        }
      }
    }
    GpuSideSink sk{a.side, a.port_ctr, a.drop_ctr};
    if (a.toep_tab) side_stage(a.t, ta, d, im, o, a.out_meta[i], i, sk, LdsToeplitz{stab});
    else side_stage(a.t, ta, d, im, o, a.out_meta[i], i, sk);
  }
}

// Exchange receive side of flow-owner steering: the segments peers filled (64-B header slots +
// ingress meta, count in each segment header) -> one dense batch; the total goes to *n_dev so the
// fused kernel that follows processes exactly what arrived, with no host round trip.
__global__ __launch_bounds__(256) void gather_kernel(const uint8_t* recv, uint32_t nranks, uint32_t rank, uint32_t cap,
                                                     uint32_t seg_bytes, uint32_t meta_off, uint4* pkts, uint32_t* inmeta,
                                                     uint32_t* n_dev) {
  // each segment's slots land as one contiguous run of the batch: copied as a flat array of 16-B
  // chunks (consecutive lanes, consecutive chunks), not one 64-B slot per lane
  __shared__ uint32_t sbase[kMaxRanks], scnt[kMaxRanks];
  if (threadIdx.x == 0) {
    uint32_t b = 0;
    for (uint32_t q = 0; q < nranks; ++q) {
      const uint32_t c = q == rank ? 0u : min(reinterpret_cast<const uint32_t*>(recv + (size_t)q * seg_bytes)[0], cap);
      sbase[q] = b; scnt[q] = c; b += c;
    }
  }
  __syncthreads();
  const uint32_t cap4 = cap * 4u, total4 = nranks * cap4;   // (< 2^32: checked at launch)
  for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < total4; idx += gridDim.x * 256) {
    const uint32_t s = idx / cap4, u = idx - s * cap4;
    if ((u >> 2) >= scnt[s]) continue;   // (the own segment has count 0)
    const uint4* src = reinterpret_cast<const uint4*>(recv + (size_t)s * seg_bytes + 64);
    pkts[(size_t)sbase[s] * 4 + u] = src[u];
  }
  for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < nranks * cap; idx += gridDim.x * 256) {
    const uint32_t s = idx / cap, j = idx - s * cap;
    if (j >= scnt[s]) continue;
    inmeta[sbase[s] + j] = reinterpret_cast<const uint32_t*>(recv + (size_t)s * seg_bytes + meta_off)[j];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t q = 0; q < nranks; ++q)
      if (q != rank) t += min(reinterpret_cast<const uint32_t*>(recv + (size_t)q * seg_bytes)[0], cap);
    *n_dev = t;
  }
}

// Steer-list mode, second half: every listed packet (index | owner << 26) goes to its owner's
// exchange segment - its input slot and ingress meta, as they came in.  One workgroup walks one fused workgroup's list region 256 entries at a time;
// positions are claimed per owner in LDS, then ONE global atomic per owner per 256 entries
// reserves the run in that owner's segment.  Segments are sized for the whole batch (count-first
// exchange: nothing can overflow).
__global__ __launch_bounds__(256) void steer_kernel(const uint4* pkts, const uint32_t* inmeta, const uint32_t* list,
                                                    const uint32_t* list_cnt, uint32_t cap_list, uint32_t max_blk,
                                                    uint8_t* send, uint32_t* pcnt, uint32_t nranks, uint32_t cap,
                                                    uint32_t seg_bytes, uint32_t meta_off) {
  __shared__ uint32_t oc[kMaxRanks], ob[kMaxRanks];
  __shared__ uint32_t ssrc[256];            // the pass's entries: source slot (~0: none) ...
  __shared__ unsigned long long sdst[256];  // ... and the byte offset of its destination slot
  const uint32_t G = min(list_cnt[0], max_blk), capb = list_cnt[1];
  if ((unsigned long long)G * capb > cap_list) return;   // a header this launch did not write
  for (uint32_t b = blockIdx.x; b < G; b += gridDim.x) {
    const uint32_t c = min(list_cnt[2 + b], capb);
    for (uint32_t j0 = 0; j0 < c; j0 += 256) {
      if (threadIdx.x < kMaxRanks) oc[threadIdx.x] = 0;
      __syncthreads();
      const uint32_t j = j0 + threadIdx.x;
      const uint32_t e = j < c ? list[(size_t)b * capb + j] : 0xFFFFFFFFu;
      const uint32_t i = e & ((1u << 26) - 1u), o = e >> 26;
      const bool ok = j < c && o < nranks;
      const uint32_t local = ok ? atomicAdd(&oc[o], 1u) : 0u;
      __syncthreads();
      if (threadIdx.x < nranks && oc[threadIdx.x]) ob[threadIdx.x] = atomicAdd(&pcnt[threadIdx.x], oc[threadIdx.x]);
      __syncthreads();
      ssrc[threadIdx.x] = 0xFFFFFFFFu;
      if (ok) {
        const uint32_t pos = ob[o] + local;
        if (pos < cap) {   // cannot fail with cap = batch (kept as a guard)
          uint8_t* seg = send + (size_t)o * seg_bytes;
          ssrc[threadIdx.x] = i;
          sdst[threadIdx.x] = (unsigned long long)o * seg_bytes + 64ull + (unsigned long long)pos * 64ull;
          reinterpret_cast<uint32_t*>(seg + meta_off)[pos] = inmeta[i];
        }
      }
      __syncthreads();
      // the slots: four lanes per slot (one 16-B chunk each), so an instruction moves 16 whole
      // 64-B slots instead of 64 scattered 16-B pieces
#pragma unroll
      for (uint32_t r = 0; r < 4; ++r) {
        const uint32_t q = r * 256u + threadIdx.x, e = q >> 2, k = q & 3u;
        if (ssrc[e] != 0xFFFFFFFFu)
          reinterpret_cast<uint4*>(send + sdst[e])[k] = pkts[(size_t)ssrc[e] * 4 + k];
      }
      __syncthreads();   // ob / oc / the stash are reused by the next 256 entries
    }
  }
}

__global__ void stamp_kernel(unsigned long long* dst) {
  if (threadIdx.x == 0) *dst = __builtin_amdgcn_s_memrealtime();
}

// Scatter whole bucket rows (control-plane updates: a modified bucket is re-sent entire).
__global__ void bucket_update_kernel(const uint32_t* idx, uint32_t nb, const uint4* rows, uint4* flows,
                                     uint32_t bucket_mask) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;  // one thread per 16 B of a 128-B row
  const uint32_t bi = j / (kBucketSlots * 2), q = j % (kBucketSlots * 2);
  if (bi >= nb) return;
  const uint32_t b = idx[bi];
  if (b > bucket_mask) return;
  flows[(size_t)b * kBucketSlots * 2 + q] = rows[(size_t)bi * kBucketSlots * 2 + q];
}

// MAC learning (OvS NORMAL) on the GPU: one thread per learn event, lock-free insert into the
// open-addressed (bridge, MAC) table.  An empty slot is claimed with a CAS on its port/valid word
// (-> kMacClaim), the key and stamp are written, and a release store publishes kMacLearned.  A
// thread that sees a claimed slot re-reads it (a claimer publishes within the same loop
// iteration, so lanes of one wave never wait on each other); a known key only refreshes the
// port and stamp of a learned entry (static entries win).  Lookups running concurrently (the
// persistent ring) skip claimed slots and continue probing.
__global__ __launch_bounds__(256) void mac_learn_kernel(MacEntry* macs, uint32_t mask, const uint4* ev,
                                                        const uint32_t* n_events, uint32_t cap, uint32_t stamp,
                                                        uint32_t* dropped) {
  const uint32_t n = min(*n_events, cap);
  uint32_t* base = reinterpret_cast<uint32_t*>(macs);
  for (uint32_t j = blockIdx.x * 256 + threadIdx.x; j < n; j += gridDim.x * 256) {
    const uint4 v = ev[j];
    const uint32_t lo = v.x, hi = v.y & 0xFFFFu, br = v.y >> 16, port = v.z & 0xFFFFu;
    const uint32_t key1 = hi | (br << 16);
    const uint32_t h = mac_hash(br, lo, hi) & mask;
    uint32_t probe = 0, spins = 0;
    bool done = false;
    while (!done && probe < 16) {
      uint32_t* w = base + (size_t)((h + probe) & mask) * 4;
      const uint32_t w2 = __hip_atomic_load(w + 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t valid = w2 >> 16;
      if (valid == kMacClaim) {  // another wave is inserting here: re-read
        if (++spins > (1u << 16)) break;
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      if (valid == kMacEmpty) {
        if (atomicCAS(w + 2, w2, (0xFFFFu << 16) | port) == w2) {
          __hip_atomic_store(w + 0, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(w + 1, key1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(w + 3, stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(w + 2, ((uint32_t)kMacLearned << 16) | port, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
          done = true;
        }
        continue;  // lost the race: the slot is claimed now, re-read it
      }
      const uint32_t k0 = __hip_atomic_load(w + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t k1 = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((valid == kMacStatic || valid == kMacLearned) && k0 == lo && k1 == key1) {
        if (valid == kMacLearned) {
          __hip_atomic_store(w + 3, stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(w + 2, ((uint32_t)kMacLearned << 16) | port, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
        done = true;
        continue;
      }
      ++probe;
    }
    if (!done) atomicAdd(dropped, 1u);
  }
}

// Read-and-reset packed counters (harvest); host accumulates into 64-bit totals.
__global__ void harvest_kernel(unsigned long long* ctr, unsigned long long* out, uint32_t n) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j < n) out[j] = atomicExch(ctr + j, 0ull);
}


// ------------------------------------------------------------------------------------------
// Launchers
// ------------------------------------------------------------------------------------------
size_t fused_lds_bytes(int hash_mode, int acl_mode, uint32_t acl_tiles) {
  return lds_layout(hash_mode, acl_mode, acl_tiles).total;
}

// IPv6 pre-pass (v6_kernel), run before the fused kernel when the tables hold IPv6 rules or
// IPv6 flows, so the hot kernel's register budget carries neither the 384-bit TCAM nor the
// address check.  Per IPv6 packet it leaves one word in the batch's out_meta[i] (the fused
// kernel reads it, then writes its egress meta there): rule + 1 in bits 0..15 (0 = no rule),
// bit 31 = its folded FlowKey hits a flow whose side entry holds the packet's addresses
// (flow6_verify; the fused kernel's own probe finds the same slot) - and the packet's folded
// FlowKey in the first 16 B of its out slot (the fused kernel's key for it).
//  * ACL: the FP4 MFMA tile of classify_wave with K = 3 x 128 over the key6 (pipeline.h
//    key6_word), the three products chained through one accumulator (C init = bias * 4096 +
//    rule, A scaled by 2^12: the accumulator is (mismatch << 12) | rule exactly); rule tiles
//    stream from the global copy (L2-resident).
//  * flow check: Toeplitz (LDS byte tables) of the folded key, the cuckoo probe, the 32-B side
//    entry compare.
// One packet per lane; a wave with no IPv6 packet skips all of it (wave-uniform), so an IPv4
// batch costs one header read.
struct V6Args {
  TablesView t;
  const uint4* pkts;
  const uint32_t* inmeta;
  uint32_t n;
  const v4i* wfrag;    // [tiles][3][64] A fragments
  const v4i* cinit;    // [tiles][4] C init
  uint32_t tiles;      // 0: no IPv6 rules
  const uint32_t* toep_tab;   // [16][256] byte tables (null: scalar Toeplitz)
  uint32_t* res;              // the batch's out_meta: rule + 1 | verified << 31
  uint4* keys;                // row i * key_stride: the packet's folded FlowKey (FusedLaunch::v6_keys)
  uint32_t key_stride;
};

// Latency layout (r5 s16: 307 us per 4M-slot dual-stack batch, as long as the fused kernel itself;
// one dependent chain per iteration - frame, four rule tiles read from L2, bucket line, side entry):
//  * the first kV6LdsTiles rule tiles (fragments + C init) are staged in LDS once per workgroup;
//  * the next run's frames and in-meta words are loaded right after this run's parse;
//  * the bucket lines leave as soon as the folded key's hash is known (IPv6 packets only: an IPv4
//    packet's lines are not loaded) and land under the ACL's MFMAs.
#ifndef NFDP_V6_WAVES_PER_EU
#define NFDP_V6_WAVES_PER_EU 2
#endif
#ifndef NFDP_V6_ABL
#define NFDP_V6_ABL 0
#endif
#ifndef NFDP_V6_EARLY_PROBE
#define NFDP_V6_EARLY_PROBE 1   // 0: the bucket lines leave after the ACL (fewer live VGPRs)
#endif
constexpr uint32_t kV6LdsTiles = 4;   // 64 IPv6 rules: 12.25 KiB of LDS
__global__ __launch_bounds__(256, NFDP_V6_WAVES_PER_EU) void v6_kernel(V6Args a) {
  __shared__ uint32_t kw[4][64 * 13];   // per wave: 64 key6 rows of 12 words (+1 pad: bank spread)
  __shared__ uint4 kxs[4][64];          // per wave: frame transposition / probe key exchange scratch
  __shared__ uint32_t ltab[16 * 256];
  __shared__ v4i lwf[kV6LdsTiles * 3 * 64];
  __shared__ v4i lci[kV6LdsTiles * 4];
  // the small tables (ports < kLdsPorts, chain words, verdicts) staged like the fused kernel's:
  // the ingress port lookup is an LDS read, not a dependent global load per run
  __shared__ __attribute__((aligned(16))) uint8_t ltabs[kLdsTabBytes];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t g = lane >> 4, col = lane & 15u;
  uint32_t* row = kw[wv];
  uint4* kx = kxs[wv];
  if (a.toep_tab)
    for (uint32_t q = threadIdx.x; q < 16 * 256; q += 256) ltab[q] = a.toep_tab[q];
  const uint32_t lt6 = a.tiles < kV6LdsTiles ? a.tiles : kV6LdsTiles;
  for (uint32_t q = threadIdx.x; q < lt6 * 3 * 64; q += 256) lwf[q] = a.wfrag[q];
  for (uint32_t q = threadIdx.x; q < lt6 * 4; q += 256) lci[q] = a.cinit[q];
  const LdsTables ta = stage_lds_tables(a.t, reinterpret_cast<PortEntry*>(ltabs),
                                        reinterpret_cast<uint64_t*>(ltabs + kLdsPorts * sizeof(PortEntry)),
                                        ltabs + kLdsPorts * sizeof(PortEntry) + kLdsChains * 8, true, 256);
  __syncthreads();
  // coalesced frame loads (the wave's 64 slots = one 4-KiB run, device.h wave_frames_load)
  const __amdgpu_buffer_rsrc_t r_pk = __builtin_amdgcn_make_buffer_rsrc((void*)a.pkts, (short)0, (int)(a.n * 64u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_im = __builtin_amdgcn_make_buffer_rsrc((void*)a.inmeta, (short)0, (int)(a.n * 4u), kBufCfg);
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u;
  const uint32_t stride = gridDim.x * 256u;
  auto run_of = [&](uint32_t base) { return base + wave0 < a.n ? (base + wave0) * 64u : kNoRun; };
  v4u cn[4];
  uint32_t imn;
  {
    const uint32_t i0 = blockIdx.x * 256u + threadIdx.x;
    wave_frames_load<0>(r_pk, run_of(blockIdx.x * 256u), cn);
    imn = __builtin_amdgcn_raw_buffer_load_b32(r_im, i0 < a.n ? i0 * 4u : kNoRun, 0, 0);
  }
  // The side-entry check of a hit is deferred by one iteration (r5 s20 ablation: the flow check was
  // 120 of the kernel's 252 us, its second dependent random load exposed): the 32-B entry is loaded
  // when the probe finishes and compared - with the result word stored - after the NEXT run's ACL.
  uint32_t pv_i = kNoRun, pv_word = 0, pv_addr[8];
  bool pv_v6 = false, pv_chk = false;
  uint4 pv_s0 = make_uint4(0u, 0u, 0u, 0u), pv_s1 = pv_s0;
  auto finish_prev = [&]() {
    const bool ok = pv_chk && eq16(pv_s0, make_uint4(pv_addr[0], pv_addr[1], pv_addr[2], pv_addr[3])) &&
                    eq16(pv_s1, make_uint4(pv_addr[4], pv_addr[5], pv_addr[6], pv_addr[7]));
    if (pv_i != kNoRun) a.res[pv_i] = pv_v6 ? (pv_word | (ok ? 0x80000000u : 0u)) : 0u;
  };
  for (uint32_t base = blockIdx.x * 256u; base < a.n; base += stride) {   // block-uniform trips
    const uint32_t i = base + threadIdx.x;
    const bool valid = i < a.n;
    uint32_t d[kSlotDwords];
    wave_frames_to_lanes<true>(kx, cn, d);
    Parsed p;
    IngressState st;
    ingress_stage<LdsTables, true>(a.t, ta, d, valid ? imn : 0u, p, st);   // (with the IPv6 key fold)
    {   // the next run: lands under this one's classification
      const uint32_t nx = i + stride;
      wave_frames_load<0>(r_pk, run_of(base + stride), cn);
      imn = __builtin_amdgcn_raw_buffer_load_b32(r_im, nx < a.n ? nx * 4u : kNoRun, 0, 0);
    }
    const bool v6 = valid && p.ipv6;
    const bool any6 = __any(v6);
    const bool probe = v6 && !st.reason && a.t.flow6_on;
    uint32_t h = 0;
    uint4 bv[8];
    int rule = -1;
    if (any6) {   // wave-uniform: EXEC full from here (MFMA, cross-lane reads, the wave probe)
      auto issue = [&]() {
        if (!a.t.flow6_on || NFDP_V6_ABL == 2) return;
        // the folded key's Toeplitz hash, then the first-choice bucket lines (flow_probe_issue's
        // wave-cooperative layout: lane 8j + q... loads line part c of packet 8j + q's bucket)
        if (a.toep_tab) {
          const uint32_t w[4] = {st.key.src_ip, st.key.dst_ip, st.key.ports, st.key.meta};
#pragma unroll
          for (int q = 0; q < 16; ++q) h ^= ltab[q * 256 + ((w[q >> 2] >> (8 * (q & 3))) & 0xFFu)];
        } else {
          h = toeplitz_scalar(st.key, a.t.rss_key);
        }
        // (flat loads under the lane mask: a multi-GB table is past a buffer's 32-bit offsets)
        const uint4* fl = reinterpret_cast<const uint4*>(a.t.flows);
        const uint32_t b1 = probe ? (h & a.t.bucket_mask) : kNoRun;
        const uint32_t c = lane & 7u, q = lane >> 3;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t bj = (uint32_t)__shfl((int)b1, 8 * j + (int)q);
          bv[j] = bj != kNoRun ? fl[(size_t)bj * (kBucketSlots * 2) + c] : make_uint4(0u, 0u, 0u, 0u);
        }
      };
      if (NFDP_V6_EARLY_PROBE) issue();
#if NFDP_V6_ABL == 1   // cost attribution only (wrong results): no ACL
      if (false) {
#else
      if (a.tiles) {
#endif
#pragma unroll
        for (int w = 0; w < 12; ++w) row[lane * 13 + w] = key6_word(p, st.bridge, w);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        v8i_t b[3][4];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const uint32_t w = row[(16 * tt + col) * 13 + 4 * k + g];
            b[k][tt] = v8i_t{(int)spread8_fp4(w & 0xFFu), (int)spread8_fp4((w >> 8) & 0xFFu),
                             (int)spread8_fp4((w >> 16) & 0xFFu), (int)spread8_fp4(w >> 24), 0, 0, 0, 0};
          }
        uint32_t best[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        auto tile = [&](const v4i* wf, const v4i* ci4, uint32_t t) {
          const v4i ci = ci4[t * 4 + g];
          const v4f_t cc = {__int_as_float(ci[0]), __int_as_float(ci[1]), __int_as_float(ci[2]), __int_as_float(ci[3])};
          v4f_t acc[4] = {cc, cc, cc, cc};
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            const v4i a4 = wf[((size_t)t * 3 + k) * 64 + lane];
            const v8i_t av = {a4[0], a4[1], a4[2], a4[3], 0, 0, 0, 0};
#pragma unroll
            for (int tt = 0; tt < 4; ++tt)
              acc[tt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, b[k][tt], acc[tt], 4, 4, 0, kE8M0Idx, 0, kE8M0One);
          }
#pragma unroll
          for (int tt = 0; tt < 4; ++tt)
            best[tt] = min(best[tt], min(min(__float_as_uint(acc[tt][0]), __float_as_uint(acc[tt][1])),
                                         min(__float_as_uint(acc[tt][2]), __float_as_uint(acc[tt][3]))));
        };
        for (uint32_t t = 0; t < lt6; ++t) tile(lwf, lci, t);          // staged (LDS)
        for (uint32_t t = lt6; t < a.tiles; ++t) tile(a.wfrag, a.cinit, t);   // the rest (L2)
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) {
          best[tt] = min(best[tt], (uint32_t)__shfl_xor(best[tt], 16));
          best[tt] = min(best[tt], (uint32_t)__shfl_xor(best[tt], 32));
        }
        const uint32_t bb = pick4(g, best[0], best[1], best[2], best[3]);
        const uint32_t bvv = bb == 0xFFFFFFFFu ? bb : (uint32_t)__uint_as_float(bb);
        const int r = acl_rule_of(bvv, a.t.n_acl6);
        rule = r >= 0 ? (int)(a.t.n_acl + (uint32_t)r) : -1;
        __builtin_amdgcn_wave_barrier();
      }
      if (!NFDP_V6_EARLY_PROBE) issue();
    }
    finish_prev();   // the previous run's side entries arrived under this run's ACL
    int64_t slot = -1;
    if (any6 && a.t.flow6_on && NFDP_V6_ABL != 2) {   // (2: cost attribution only, no flow check)
      uint4 act;
      slot = flow_probe_finish(a.t, st.key, h, probe, kx, bv, act);
    }
    // this run's check: the hit slot's side entry (flow6_side) leaves now, compared next iteration
    pv_chk = v6 && slot >= 0;
    const uint4* se = reinterpret_cast<const uint4*>(flow6_side(a.t, pv_chk ? slot : 0));
    pv_s0 = pv_chk ? se[0] : make_uint4(0u, 0u, 0u, 0u);
    pv_s1 = pv_chk ? se[1] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int k = 0; k < 8; ++k) pv_addr[k] = raw32_at2(p.s, 22 + 4 * k);
    pv_i = valid ? i : kNoRun;
    pv_v6 = v6;
    pv_word = (uint32_t)(rule + 1);
    if (v6) a.keys[(size_t)i * a.key_stride] = make_uint4(st.key.src_ip, st.key.dst_ip, st.key.ports, st.key.meta);
  }
  finish_prev();
}

// ---- SFC hop pipeline across GPUs (split chains, kHopXfer) ----
// hop_pack_kernel: this GPU's frames handed to `plane` (meta reason kRemote, port = plane, a
// HopState record beside them) -> that plane's inbox.  The inbox lives on the GPU that resumes the
// chain, so these are peer stores over xGMI (plain stores into a peer allocation; the same code
// when both planes share a device).  A workgroup packs a chunk of kPackChunk frames: it counts its
// chunk's hand-offs (ballots), claims their inbox run with ONE atomic on this GPU's fill counter
// (per-wave claims on one word serialised at the memory side: 774 us per 4M frames, r5 s9
// profile), then each wave writes its quarter of the chunk in arrival order.  The publish step
// hands the count over once the batch is packed.
constexpr uint32_t kPackChunk = 4096;   // frames per workgroup pass (4 waves x 1024) at full batches
__global__ __launch_bounds__(256) void hop_pack_kernel(const uint4* out, const uint32_t* meta, const HopState* state,
                                                       uint32_t n, const uint32_t* n_dev, uint32_t plane,
                                                       uint32_t* fill, HopInbox dst, uint32_t chunk) {
  __shared__ uint32_t wcnt[4];
  __shared__ uint32_t wbase[4];
  const uint32_t nn = n_dev ? min(n, *n_dev) : n;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  auto mine = [&](uint32_t i) -> bool {
    if (i >= nn) return false;
    const uint32_t m = meta[i];
    return ((m >> 26) & 0xFu) == kRemote && (m & 0xFFFu) == plane;
  };
  // block-uniform trip count: every wave reaches each ballot and barrier
  for (uint32_t c0 = blockIdx.x * chunk; c0 < nn; c0 += gridDim.x * chunk) {
    const uint32_t w0 = c0 + wave * (chunk / 4);   // this wave's quarter, 16 runs of 64
    uint32_t cnt = 0;
    for (uint32_t k = 0; k < chunk / 4; k += 64) cnt += (uint32_t)__builtin_popcountll(__ballot(mine(w0 + k + lane)));
    if (lane == 0) wcnt[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tot = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
      uint32_t b0 = tot ? atomicAdd(fill, tot) : 0u;
      for (int w = 0; w < 4; ++w) { wbase[w] = b0; b0 += wcnt[w]; }
    }
    __syncthreads();
    uint32_t pos0 = wbase[wave];
    for (uint32_t k = 0; k < chunk / 4 && cnt; k += 64) {
      const uint32_t i = w0 + k + lane;
      const bool my = mine(i);
      const unsigned long long bm = __ballot(my);
      if (bm == ~0ull && pos0 + 64u <= dst.cap) {
        // a whole run handed to this plane (a chain split for all its traffic: the common case):
        // contiguous 4-KiB header / 2-KiB record copies, lane-contiguous 16-B chunks, instead of
        // one 64-B slot per lane (every load and store instruction striding over 64 slots)
        const uint4* sh = out + (size_t)(w0 + k) * 4;
        uint4* dh = dst.hdr + (size_t)pos0 * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) dh[q * 64 + lane] = sh[q * 64 + lane];
        const uint4* ss = reinterpret_cast<const uint4*>(state + (w0 + k));
        uint4* ds = reinterpret_cast<uint4*>(dst.state + pos0);
#pragma unroll
        for (int q = 0; q < 2; ++q) ds[q * 64 + lane] = ss[q * 64 + lane];
        dst.idx[pos0 + lane] = i;
      } else if (my) {
        const uint32_t pos = pos0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        if (pos < dst.cap) {
#pragma unroll
          for (int q = 0; q < 4; ++q) dst.hdr[(size_t)pos * 4 + q] = out[(size_t)i * 4 + q];
          dst.state[pos] = state[i];
          dst.idx[pos] = i;
        }
      }
      pos0 += (uint32_t)__builtin_popcountll(bm);
    }
    __syncthreads();   // (wcnt / wbase are rewritten next pass)
  }
}

// publish: the inbox count (<= cap) for the resuming GPU; the fill counter is reset for the next
// batch (stream order: after the pack kernel)
__global__ void hop_publish_kernel(uint32_t* fill, uint32_t cap, uint32_t* count) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const uint32_t f = *fill;
    *count = f < cap ? f : cap;
    *fill = 0u;
  }
}

hipError_t launch_hop_pack(const void* out, const uint32_t* meta, const HopState* state, uint32_t n,
                           const uint32_t* n_dev, uint32_t plane, uint32_t* fill, const HopInbox& dst,
                           hipStream_t s) {
  if (!out || !meta || !state || !fill || !dst.count || !dst.hdr || !dst.state || !dst.idx || plane > kHopXferPlanes)
    return hipErrorInvalidValue;
  // chunk: 4096 frames per workgroup at full batches (few claims), down to 256 for small ones
  // (enough workgroups to spread a 64K batch over the CUs); a multiple of 256 (4 waves x 64)
  uint32_t chunk = kPackChunk;
  while (chunk > 256 && (n + chunk - 1) / chunk < 512) chunk >>= 1;
  uint32_t grid = (n + chunk - 1) / chunk;
  if (grid > 2048) grid = 2048;
  if (grid) hipLaunchKernelGGL(hop_pack_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint4*>(out),
                               meta, state, n, n_dev, plane, fill, dst, chunk);
  hipLaunchKernelGGL(hop_publish_kernel, dim3(1), dim3(64), 0, s, fill, dst.cap, dst.count);
  return hipGetLastError();
}

// resume_kernel: the rest of the split chains over an inbox (pipeline.h resume_stage), one frame
// per lane.  Egress counters per workgroup in LDS (ports < kLdsPorts), like the fused kernel's.
struct ResumeArgs {
  TablesView t;
  HopInbox in;
  uint4* out;
  uint32_t* out_meta;
  HopState* out_state;            // next hand-offs (nullable)
  unsigned long long* port_ctr;
  unsigned long long* drop_ctr;
  uint32_t flags;                 // bit0: no counters
};
__global__ __launch_bounds__(256) void resume_kernel(ResumeArgs a) {
  __shared__ uint32_t pc[2 * kLdsPorts];   // tx packets, tx bytes
  __shared__ uint32_t drops[kNumReasons];
  __shared__ uint4 kxs[4][64];   // per wave: the slot-run transposition (device.h wave_frames_*)
  __shared__ __attribute__((aligned(16))) uint8_t ltabs[kLdsTabBytes];   // ports / chain words / verdicts
  for (uint32_t q = threadIdx.x; q < 2 * kLdsPorts; q += 256) pc[q] = 0;
  if (threadIdx.x < kNumReasons) drops[threadIdx.x] = 0;
  const LdsTables ta = stage_lds_tables(a.t, reinterpret_cast<PortEntry*>(ltabs),
                                        reinterpret_cast<uint64_t*>(ltabs + kLdsPorts * sizeof(PortEntry)),
                                        ltabs + kLdsPorts * sizeof(PortEntry) + kLdsChains * 8, true, 256);
  __syncthreads();
  const uint32_t n = min(*a.in.count, a.in.cap);
  const bool count = !(a.flags & 1u);
  // header slots in and out as coalesced 4-KiB runs per wave (one slot per lane strides every load
  // and store instruction over 64 slots); block-uniform trips, EXEC full at the transpositions
  uint4* kx = kxs[threadIdx.x >> 6];
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u;
  const __amdgpu_buffer_rsrc_t r_in = __builtin_amdgcn_make_buffer_rsrc((void*)a.in.hdr, (short)0, (int)(n * 64u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc((void*)a.out, (short)0, (int)(n * 64u), kBufCfg);
  for (uint32_t base = blockIdx.x * 256u; base < n; base += gridDim.x * 256u) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t run = base + wave0 < n ? (base + wave0) * 64u : kNoRun;
    uint32_t d[kSlotDwords];
    {
      v4u cn[4];
      wave_frames_load<kStreamAux>(r_in, run, cn);
      wave_frames_to_lanes(kx, cn, d);
    }
    uint32_t o[kSlotDwords] = {};
    if (i < n) {
    const HopState hs = a.in.state[i];
    Parsed p;
    IngressState st;
    resume_ingress(ta, d, hs.inmeta, p, st);
    const EgressDecision e = resume_stage(a.t, ta, p, st, hs.act, hs.acl_rule, hs.hash, hs.hop);
    emit(p, e.tci, e.push != 0, o);
    const uint32_t olen = out_len(p, e);
    a.out_meta[i] = make_meta(e.out_port, olen, e.reason, !e.reason && e.xhdr, false);
    if (a.out_state && e.reason == kRemote && e.inner_len) a.out_state[i] = hop_state_of(p, st, e, hs.act, hs.acl_rule, hs.hash);
    if (count) {
      if (e.reason) {
        atomicAdd(&drops[e.reason & (kNumReasons - 1)], 1u);
      } else if (e.out_port < kLdsPorts) {
        atomicAdd(&pc[e.out_port], 1u); atomicAdd(&pc[kLdsPorts + e.out_port], olen);
      } else {
        atomicAdd(a.port_ctr + 2 * e.out_port + 1, ctr_inc(olen));
      }
    }
    }
    wave_frames_store<kStreamAux>(kx, o, r_out, run);   // (lanes past n: dropped by the buffer bounds)
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < kLdsPorts; q += 256)
    if (pc[q]) atomicAdd(a.port_ctr + 2 * q + 1, ((unsigned long long)pc[q] << 40) | pc[kLdsPorts + q]);
  if (threadIdx.x < kNumReasons && drops[threadIdx.x])
    atomicAdd(a.drop_ctr + threadIdx.x, (unsigned long long)drops[threadIdx.x]);
}

hipError_t launch_resume(const TablesView& t, const HopInbox& in, void* out, uint32_t* out_meta, HopState* out_state,
                         unsigned long long* port_ctr, unsigned long long* drop_ctr, uint32_t flags, int num_cus,
                         hipStream_t s) {
  if (!in.count || !in.hdr || !in.state || !out || !out_meta || !port_ctr || !drop_ctr) return hipErrorInvalidValue;
  if (in.cap >= (1u << 25)) return hipErrorInvalidValue;   // (32-bit buffer views of the slot runs)
  uint32_t grid = (in.cap + 255) / 256;
  const uint32_t lim = (uint32_t)(num_cus > 0 ? num_cus : 256) * 8u;
  if (grid > lim) grid = lim;
  if (grid == 0) return hipSuccess;
  ResumeArgs a{t, in, reinterpret_cast<uint4*>(out), out_meta, out_state, port_ctr, drop_ctr, flags};
  hipLaunchKernelGGL(resume_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

static hipError_t launch_v6(const FusedLaunch& f, int num_cus, hipStream_t s) {
  if (!f.pkts || !f.inmeta || !f.out_meta || !f.out) return hipErrorInvalidValue;
  if (f.t.n_acl6 && (!f.acl6_wfrag || !f.acl6_cinit || f.acl6_tiles == 0 || f.acl6_tiles > kAclMaxRules / 16 ||
                     f.t.n_acl6 > f.acl6_tiles * 16))
    return hipErrorInvalidValue;
  V6Args a{f.t, reinterpret_cast<const uint4*>(f.pkts), f.inmeta, f.n, reinterpret_cast<const v4i*>(f.acl6_wfrag),
           reinterpret_cast<const v4i*>(f.acl6_cinit), f.t.n_acl6 ? f.acl6_tiles : 0u, f.toep_tab, f.out_meta,
           reinterpret_cast<uint4*>(f.v6_keys ? f.v6_keys : f.out), f.v6_keys ? 1u : 4u};
  // one workgroup per SIMD-resident slot (NFDP_V6_WAVES_PER_EU 4-wave blocks per CU): every block
  // runs the same number of grid-stride trips, no second round of blocks behind the first
  uint32_t grid = (f.n + 255) / 256;
  const uint32_t cap = (uint32_t)num_cus * NFDP_V6_WAVES_PER_EU;
  if (grid > cap) grid = cap;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(v6_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int H, int A, bool R, bool E = false, bool LS = false, bool V6 = false, bool X = false>
static hipError_t launch_fused_t(const FusedArgs& a, int num_cus, hipStream_t s) {
  // static LDS (REMOTE reservation counters) + dynamic tables must fit 160 KiB
  // rcnt[2][..] + rbase + lst_n, with room for the compiler's alignment of the static block
  constexpr size_t kStatic = (3 * (R ? kMaxRanks : 1) + 1) * sizeof(uint32_t) + 64;
  constexpr size_t kMaxDyn = 160 * 1024 - kStatic;
  const size_t lds = lds_layout(H, A, a.acl_tiles, E).total;
  if (lds > kMaxDyn) return hipErrorInvalidValue;
  if (R && (a.nranks == 0 || a.nranks > kMaxRanks || a.rank >= a.nranks || !a.send_pkt || !a.pcnt ||
            (size_t)a.nranks * pkt_seg_bytes(a.cap_pkt) >= (1ull << 31) || a.n >= (1u << 25)))
    return hipErrorInvalidValue;
  // the 1-GPU variant's fixed-count tail: buffer views need n * 64 B < 2 GiB and a counter table
  if (!R && (a.n >= (1u << 25) || !a.flow_ctr || !a.out_meta)) return hipErrorInvalidValue;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&fused_kernel<H, A, R, E, LS, V6, X>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxDyn);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  int per_cu = (int)((160 * 1024) / (lds ? lds : 1));
  per_cu = per_cu < 1 ? 1 : (per_cu > NFDP_FUSED_MAX_PER_CU ? NFDP_FUSED_MAX_PER_CU : per_cu);
  const uint32_t need = (a.n + kFB - 1) / kFB;
  uint32_t grid = (uint32_t)(per_cu * num_cus);
  if (need < grid) grid = need;
  if (grid == 0) return hipSuccess;
  FusedArgs b = a;
  if (b.side.cnt && LS) b.side.blk_cnt = nullptr;   // LIST instances: one flat list
  if (b.side.cnt && !LS) {
    // side-list regions: a region holds every packet its workgroup's grid-stride loop visits, or
    // its share of a smaller list (entries past it are counted as dropped, cnt[6])
    if (!b.side.blk_cnt || grid > b.side.nblk) return hipErrorInvalidValue;
    const uint64_t stride = (uint64_t)grid * kFB;
    const uint64_t need = ((a.n + stride - 1) / stride) * kFB, share = b.side.cap_list / grid;
    b.side.blk_cap = (uint32_t)(need < share ? need : share);
    b.side.nblk = grid;
  }
  if constexpr (LS) {
    // each workgroup's list region holds every packet its grid-stride loop visits
    const uint64_t stride = (uint64_t)grid * kFB;
    b.steer_cap_blk = (uint32_t)(((a.n + stride - 1) / stride) * kFB);
    if ((uint64_t)grid * b.steer_cap_blk > a.steer_cap_blk || grid > (uint32_t)(4 * num_cus))
      return hipErrorInvalidValue;   // (steer_cap_blk carries the list's capacity in)
  }
  if (X && !a.hop_state) return hipErrorInvalidValue;
  hipLaunchKernelGGL((fused_kernel<H, A, R, E, LS, V6, X>), dim3(grid), dim3(kFB), lds, s, b);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !a.side.cnt || a.side.cap_list == 0) return e;
  return launch_side(a.t, a.pkts, a.inmeta, a.out, a.out_meta, b.side, a.port_ctr, a.drop_ctr, s, a.n, false, a.toep_tab);
}

hipError_t launch_side(const TablesView& t, const void* pkts, const uint32_t* inmeta, const void* out,
                       const uint32_t* out_meta, const SideOut& side, unsigned long long* port_ctr,
                       unsigned long long* drop_ctr, hipStream_t s, uint32_t n_slots, bool wrap,
                       const uint32_t* toep_tab) {
  if (!side.cnt || side.cap_list == 0) return hipSuccess;
  if (!pkts || !inmeta || !out || !out_meta || !side.list || !port_ctr || !drop_ctr) return hipErrorInvalidValue;
  SideArgs sa{t, reinterpret_cast<const uint4*>(pkts), inmeta, reinterpret_cast<const uint4*>(out), out_meta, side,
              port_ctr, drop_ctr, n_slots, wrap ? 1u : 0u, toep_tab};
  // grid for what the batch can put on the list (each workgroup stages the Toeplitz tables)
  const uint32_t lim = n_slots && n_slots < side.cap_list ? n_slots : side.cap_list;
  const uint32_t sg = (lim + 255) / 256 < 512 ? (lim + 255) / 256 : 512;
  hipLaunchKernelGGL(side_kernel, dim3(sg), dim3(256), 0, s, sa);
  return hipGetLastError();
}

static FusedArgs make_fused_args(const FusedLaunch& f) {
  FusedArgs a;
  a.t = f.t;
  a.pkts = reinterpret_cast<const uint4*>(f.pkts);
  a.inmeta = f.inmeta;
  a.out = reinterpret_cast<uint4*>(f.out);
  a.out_meta = f.out_meta;
  a.n = f.n;
  a.flow_ctr = f.flow_ctr; a.port_ctr = f.port_ctr; a.drop_ctr = f.drop_ctr;
  a.t0 = f.t0; a.lat = f.lat;
  a.acl_wfrag = reinterpret_cast<const v4i*>(f.acl_wfrag);
  a.acl_cinit = reinterpret_cast<const v4i*>(f.acl_cinit);
  a.acl_tiles = f.acl_tiles;
  a.toep_frag = reinterpret_cast<const v4i*>(f.toep_frag);
  a.toep_tab = f.toep_tab;
  a.flags = f.flags;
  a.send_pkt = f.send_pkt; a.pcnt = f.pcnt;
  a.nranks = f.nranks; a.rank = f.rank; a.cap_pkt = f.cap_pkt;
  a.side = f.side;
  a.steer = f.steer;
  a.n_dev = f.n_dev;
  a.steer_list = f.steer_list;
  a.steer_cnt = f.steer_cnt;
  a.steer_cap_blk = f.steer_cap;
  a.hop_state = f.hop_state;
  a.v6_key = reinterpret_cast<const uint4*>(f.v6_keys ? f.v6_keys : f.out);
  a.v6_key_stride = f.v6_keys ? 1u : 4u;
  return a;
}

static hipError_t launch_fused_body(const FusedLaunch& f, const LaunchCfg& cfg, hipStream_t s);

hipError_t launch_fused(const FusedLaunch& f, const LaunchCfg& cfg, hipStream_t s) {
  if (f.steer_list && (!f.steer_cnt || f.nranks < 2 || f.nranks > kMaxRanks || f.rank >= f.nranks || f.n >= (1u << 26)))
    return hipErrorInvalidValue;
  if (f.side.cnt && ((f.side.cap_rep && (!f.side.rep_hdr || !f.side.rep_meta || !f.side.rep_src)) ||
                     (f.side.cap_learn && !f.side.learn) || (f.side.cap_list && !f.side.list)))
    return hipErrorInvalidValue;
  if (f.t.n_acl6 && (!f.out_meta || !f.acl6_wfrag || !f.acl6_cinit || f.acl6_tiles == 0)) return hipErrorInvalidValue;
  const bool v6pass = f.t.n_acl6 || f.t.flow6_on;
  if (f.flags & kFlagPairs) {   // wide header pairs: resolved in place before the pipeline (pair_kernel)
    const hipError_t e = launch_pairs(const_cast<void*>(f.pkts), const_cast<uint32_t*>(f.inmeta), f.n, f.t, f.port_ctr,
                                      !(f.flags & 1u), s);
    if (e != hipSuccess) return e;
    if (v6pass) {
      const hipError_t e6 = launch_v6(f, cfg.num_cus, s);
      if (e6 != hipSuccess) return e6;
    }
    const hipError_t e2 = launch_fused_body(f, cfg, s);
    if (e2 != hipSuccess) return e2;
    return launch_pair_fix(f.inmeta, f.out_meta, f.n, f.drop_ctr, !(f.flags & 1u), s);
  }
  if (v6pass) {
    const hipError_t e6 = launch_v6(f, cfg.num_cus, s);
    if (e6 != hipSuccess) return e6;
  }
  return launch_fused_body(f, cfg, s);
}

static hipError_t launch_fused_body(const FusedLaunch& f, const LaunchCfg& cfg, hipStream_t s) {
  FusedArgs a = make_fused_args(f);
  const bool remote = f.nranks > 1 && !f.steer_list;   // steer list: the 1-GPU instances
  if (cfg.acl_mode == kAclMfma && (f.acl_tiles == 0 || f.acl_tiles > kAclMaxRules / 16)) return hipErrorInvalidValue;
  const int h = cfg.hash_mode, ac = cfg.acl_mode, cu = cfg.num_cus;
#ifdef NFDP_HEADLINE_ONLY   // register-budget experiments: compile the headline instance alone
  (void)h; (void)remote;
  return launch_fused_t<kHashLds, kAclMfma, false, false>(a, cu, s);
#else
  const bool early = ac == kAclMfma && !(f.flags & kFlagNoEarly) &&
                     (f.acl_tiles >= kEarlyAclTiles || (f.flags & kFlagForceEarly));
  if (f.hop_state) {   // split chains: the XFER instances (1 GPU, IPv4 tables, MFMA ACL)
    if (remote || f.steer_list || f.t.n_acl6 || f.t.flow6_on || ac != kAclMfma || h == kHashScalar)
      return hipErrorNotSupported;
    return h == kHashLds ? launch_fused_t<kHashLds, kAclMfma, false, false, false, false, true>(a, cu, s)
                         : launch_fused_t<kHashMfma, kAclMfma, false, false, false, false, true>(a, cu, s);
  }
  if (f.t.n_acl6 || f.t.flow6_on) {   // IPv6 flows / rules: the V6 instances (1 GPU, MFMA ACL)
    if (remote || f.steer_list || ac != kAclMfma || h == kHashScalar) return hipErrorNotSupported;
    if (h == kHashLds) return early ? launch_fused_t<kHashLds, kAclMfma, false, true, false, true>(a, cu, s)
                                    : launch_fused_t<kHashLds, kAclMfma, false, false, false, true>(a, cu, s);
    return early ? launch_fused_t<kHashMfma, kAclMfma, false, true, false, true>(a, cu, s)
                 : launch_fused_t<kHashMfma, kAclMfma, false, false, false, true>(a, cu, s);
  }
  if (f.steer_list) {   // flow-owner steering by list: the LIST instances (multi-GPU RSS)
#define NFDP_LCASE(HH, AA)                                                                 \
    if (h == HH && ac == AA)                                                               \
      return (early && AA == kAclMfma) ? launch_fused_t<HH, AA, false, true, true>(a, cu, s) \
                                       : launch_fused_t<HH, AA, false, false, true>(a, cu, s);
    NFDP_LCASE(1, 1) NFDP_LCASE(1, 2) NFDP_LCASE(2, 1) NFDP_LCASE(2, 2)
#undef NFDP_LCASE
    return hipErrorInvalidValue;   // (scalar hash / scalar ACL: the REMOTE steer instances)
  }
  if (early) {
    if (h == kHashLds) return remote ? launch_fused_t<kHashLds, kAclMfma, true, true>(a, cu, s)
                                     : launch_fused_t<kHashLds, kAclMfma, false, true>(a, cu, s);
    if (h == kHashMfma) return remote ? launch_fused_t<kHashMfma, kAclMfma, true, true>(a, cu, s)
                                      : launch_fused_t<kHashMfma, kAclMfma, false, true>(a, cu, s);
  }
#define NFDP_CASE(HH, AA)                                                                  \
  if (h == HH && ac == AA)                                                                 \
    return remote ? launch_fused_t<HH, AA, true>(a, cu, s) : launch_fused_t<HH, AA, false>(a, cu, s);
  NFDP_CASE(0, 0) NFDP_CASE(0, 1) NFDP_CASE(0, 2)
  NFDP_CASE(1, 0) NFDP_CASE(1, 1) NFDP_CASE(1, 2)
  NFDP_CASE(2, 0) NFDP_CASE(2, 1) NFDP_CASE(2, 2)
#undef NFDP_CASE
  return hipErrorInvalidValue;
#endif
}

hipError_t launch_gather(const uint8_t* recv, uint32_t nranks, uint32_t rank, uint32_t cap, uint32_t seg_bytes,
                         uint32_t meta_off, void* pkts, uint32_t* inmeta, uint32_t* n_dev, hipStream_t s) {
  if (!recv || !pkts || !inmeta || !n_dev || rank >= nranks || nranks > kMaxRanks) return hipErrorInvalidValue;
  if ((uint64_t)nranks * cap * 4u >= (1ull << 32)) return hipErrorInvalidValue;
  const uint32_t total = nranks * cap * 4u;
  uint32_t grid = (total + 255) / 256;
  if (grid > 1024) grid = 1024;
  if (grid == 0) grid = 1;
  hipLaunchKernelGGL(gather_kernel, dim3(grid), dim3(256), 0, s, recv, nranks, rank, cap, seg_bytes, meta_off,
                     reinterpret_cast<uint4*>(pkts), inmeta, n_dev);
  return hipGetLastError();
}

hipError_t launch_steer(const void* pkts, const uint32_t* inmeta, const uint32_t* list, const uint32_t* list_cnt,
                        uint32_t cap_list, uint32_t cnt_len, uint8_t* send, uint32_t* pcnt, uint32_t nranks,
                        uint32_t cap, hipStream_t s) {
  if (!pkts || !inmeta || !list || !list_cnt || !send || !pcnt || nranks < 2 || nranks > kMaxRanks || cnt_len < 3)
    return hipErrorInvalidValue;
  if (pkt_seg_bytes(cap) * nranks >= (1ull << 40)) return hipErrorInvalidValue;
  const uint32_t max_blk = cnt_len - 2;
  const uint32_t grid = max_blk < 1024 ? max_blk : 1024;
  hipLaunchKernelGGL(steer_kernel, dim3(grid), dim3(256), 0, s, reinterpret_cast<const uint4*>(pkts), inmeta, list,
                     list_cnt, cap_list, max_blk, send, pcnt, nranks, cap, (uint32_t)pkt_seg_bytes(cap),
                     (uint32_t)pkt_meta_off(cap));
  return hipGetLastError();
}

uint32_t steer_list_len(uint32_t n, int num_cus) {
  // what launch_fused_t's LIST regions can need: n rounded up per workgroup, <= 4 workgroups/CU
  return n + (uint32_t)(4 * num_cus) * (uint32_t)kFB;
}

hipError_t launch_stamp(unsigned long long* dst, hipStream_t s) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, s, dst);
  return hipGetLastError();
}

hipError_t launch_bucket_update(const uint32_t* idx, uint32_t nb, const void* rows, void* flows,
                                uint32_t bucket_mask, hipStream_t s) {
  if (nb == 0) return hipSuccess;
  const uint32_t threads = nb * kBucketSlots * 2;
  hipLaunchKernelGGL(bucket_update_kernel, dim3((threads + 255) / 256), dim3(256), 0, s, idx, nb,
                     reinterpret_cast<const uint4*>(rows), reinterpret_cast<uint4*>(flows), bucket_mask);
  return hipGetLastError();
}

hipError_t launch_mac_learn(MacEntry* macs, uint32_t mac_mask, const uint32_t* events, const uint32_t* n_events,
                            uint32_t cap, uint32_t stamp, uint32_t* dropped, hipStream_t s) {
  if (!macs || !events || !n_events || !dropped || ((mac_mask + 1) & mac_mask)) return hipErrorInvalidValue;
  if (cap == 0) return hipSuccess;
  const uint32_t grid = (cap + 255) / 256 < 256 ? (cap + 255) / 256 : 256;
  hipLaunchKernelGGL(mac_learn_kernel, dim3(grid), dim3(256), 0, s, macs, mac_mask,
                     reinterpret_cast<const uint4*>(events), n_events, cap, stamp, dropped);
  return hipGetLastError();
}

hipError_t launch_harvest(unsigned long long* ctr, unsigned long long* out, uint32_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(harvest_kernel, dim3((n + 255) / 256), dim3(256), 0, s, ctr, out, n);
  return hipGetLastError();
}

}  // namespace nfdp
