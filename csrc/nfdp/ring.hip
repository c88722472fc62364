// ring.hip — persistent ring kernel + host engine (see ring.h for the protocol).
#include "ring.h"

#include <cstddef>
#include <cstdlib>
#include <string>

#include <immintrin.h>

#include <chrono>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

#include "device.h"

namespace nfdp {

constexpr int kRingBlock = 256;            // 4 independent waves per workgroup
constexpr int kRingWaves = kRingBlock / 64;

struct RingArgs {
  TablesView t;
  const uint4* pkts; const uint32_t* inmeta; uint4* out; uint32_t* out_meta;
  uint32_t ring_mask;
  RingCtl* ctl; uint32_t* flags; RingDevState* st; uint32_t* svc;
  unsigned long long* flow_ctr; unsigned long long* port_ctr; unsigned long long* drop_ctr;
  const v4i* acl_wfrag; const v4i* acl_cinit; uint32_t acl_tiles;
  const v4i* toep_frag; const uint32_t* toep_tab;
  unsigned long long deadline;
  const void* flows2[2];  // flow-table copies by epoch parity (the same pointer twice if not double buffered)
  const RingTableSet* sets;  // coop: table sets by epoch bit 1
  uint32_t lds_tiles;        // coop: ACL tiles the LDS layout holds
  uint32_t epoch0;
  SideOut side;           // side list (cnt null = off): slots needing replicas / learn events / outer headers
  uint32_t flags_bits;  // bit2: no per-flow counts; bits 5/6: diagnostics (kRingTrace, kRingNoCounters)
  uint32_t nq;          // queues: workgroup b serves queue b % nq (ctl / st / flags / svc / slots per queue)
  RingCtrlRing* ctrl;   // control mailbox (pinned host memory, device view)
  const unsigned long long* faddr;   // zero-copy rx: per-slot frame addresses (null: in slots)
  GdeRing* gde;         // GPU-direct egress table [kMaxPorts][nq] (null: off; ring.h GdeRing)
  const XferPeer* xpeers;   // cross-GPU hops (ring.h XferEntry): every plane (null: off)
  // the same records by value: indexed by a wave-uniform plane they are scalar loads from the
  // kernarg segment, so every descriptor built from them is uniform (a record read from global
  // memory the kernel writes is a vector load, and each access through a descriptor built from it
  // a loop over the lanes: 26 such loops in the hand-off path, r6 tools/waterfall_scan.py)
  XferPeer xpv[kMaxXferPlanes];
  uint32_t xplane, nplanes, xfer_wgs;
  uint32_t* xpend;          // this ring's [nq][chunks] hand-offs not back yet (pinned host memory)
};
// Frames are read and written with system-coherent buffer ops (sc0 sc1): the loads never hit a
// stale L2 line of a slot a producer (host / NIC DMA) rewrote, and the stores write through to
// HBM, so completion needs only "my stores are done" (s_waitcnt) before the flag — no per-chunk
// L2 invalidate / writeback, which serialised the ring at ~1.5 Gpps under load.
constexpr int kSysAux = 1 | 16;  // cache-policy bits: sc0 | sc1 (gfx940+)
constexpr int kBufRaw = 0x00020000;
// Phase trace: drain the memory counters at each stage boundary and stamp it (svc[chunk][0..6];
// [7] is always the chunk's total service time).  Serialises the stages — attribution only.
constexpr uint32_t kRingTrace = 1u << 5;
constexpr int kSvcWords = 8;
constexpr uint32_t kRingNoCounters = 1u << 6;  // diagnostic: skip every counter update

struct RingLds { size_t acl_w, acl_c, toep_f, toep_t, kx, tports, tchain, tperm, pc, drops, total; };

// Port / drop counters of a workgroup accumulate in LDS (u32) and are moved to the global packed
// counters by whichever wave flushes (atomic exchange: every count moves exactly once).  A wave
// flushes when it runs out of published work and every kFlushChunks chunks; the last wave to
// exit flushes the rest, so the totals are exact once the grid has drained.
constexpr uint32_t kFlushChunks = 256;
__device__ __forceinline__ void flush_lds_counters(uint32_t* pc, uint32_t* drops, unsigned long long* port_ctr,
                                                   unsigned long long* drop_ctr) {
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t q = lane; q < kLdsPorts; q += 64) {
    const uint32_t rp = atomicExch(&pc[q], 0u), rb = atomicExch(&pc[kLdsPorts + q], 0u);
    if (rp | rb) atomicAdd(port_ctr + 2 * q, ((unsigned long long)rp << 40) | rb);
    const uint32_t tp = atomicExch(&pc[2 * kLdsPorts + q], 0u), tb = atomicExch(&pc[3 * kLdsPorts + q], 0u);
    if (tp | tb) atomicAdd(port_ctr + 2 * q + 1, ((unsigned long long)tp << 40) | tb);
  }
  if (lane < kNumReasons) {
    const uint32_t d = atomicExch(&drops[lane], 0u);
    if (d) atomicAdd(drop_ctr + lane, (unsigned long long)d);
  }
}
__host__ __device__ inline RingLds ring_lds(int hash_mode, int acl_mode, uint32_t acl_tiles) {
  RingLds L;
  size_t o = 0;
  const uint32_t lt = acl_tiles < kLdsAclTiles ? acl_tiles : kLdsAclTiles;
  L.acl_w = o; if (acl_mode == kAclMfma) o += (size_t)lt * 64 * 16;
  L.acl_c = o; if (acl_mode == kAclMfma) o += (size_t)lt * 4 * 16;
  L.toep_f = o; if (hash_mode == kHashMfma) o += 2 * 2 * 64 * 16;
  L.toep_t = o; if (hash_mode == kHashLds) o += kToepLdsWords * 4;
  L.kx = o; o += kRingWaves * 64 * 16;
  L.tports = o; o += kLdsPorts * sizeof(PortEntry);
  L.tchain = o; o += kLdsChains * 8;
  L.tperm = o; o += 1024;
  L.pc = o; o += kLdsPorts * 4 * 4;     // [rx_pk, rx_by, tx_pk, tx_by][kLdsPorts] u32
  L.drops = o; o += kNumReasons * 4;
  L.total = (o + 15) & ~(size_t)15;
  return L;
}

__device__ __forceinline__ unsigned long long rfl64(unsigned long long v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// Zero-copy rx: the chunk's 64 frames lie wherever the producer's ports hold them (one address
// per slot in fa[], pinned host memory).  Lane L loads 16-B piece L % 4 of frame q * 16 + L / 4
// in pass q — the same register layout as a contiguous run's loads (wave_frames_load), so the
// LDS transpose is shared, and the 4 lanes of a frame read one 64-B line together (one request
// per line, as for the run).  System-coherent (sc0 sc1): the producer rewrites the buffers.
__device__ __forceinline__ void ring_frames_gather(const unsigned long long* fa, uint32_t i, v4u c[4]) {
  const uint32_t lane = threadIdx.x & 63u;
  const unsigned long long mine = __hip_atomic_load(fa + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const int lo = (int)(uint32_t)mine, hi = (int)(uint32_t)(mine >> 32);
  unsigned long long p[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int src = q * 16 + (int)(lane >> 2);
    p[q] = (((unsigned long long)(uint32_t)__shfl(hi, src) << 32) | (uint32_t)__shfl(lo, src)) + (lane & 3u) * 16u;
  }
  asm volatile(
      "global_load_dwordx4 %0, %4, off sc0 sc1\n\t"
      "global_load_dwordx4 %1, %5, off sc0 sc1\n\t"
      "global_load_dwordx4 %2, %6, off sc0 sc1\n\t"
      "global_load_dwordx4 %3, %7, off sc0 sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(c[0]), "=&v"(c[1]), "=&v"(c[2]), "=&v"(c[3])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3])
      : "memory");
}

// Bytes at and past `len` read as zero (what a copied frame's in slot holds there).
__device__ __forceinline__ void frame_clip(uint32_t* d, uint32_t len) {
#pragma unroll
  for (int k = 0; k < kSlotDwords; ++k) {
    const int rem = (int)len - 4 * k;
    d[k] = rem >= 4 ? d[k] : rem <= 0 ? 0u : d[k] & ((1u << (8 * rem)) - 1u);
  }
}

// Claim the next chunk ticket and wait until it is published.  Returns false when the wave must
// exit (stop seen with nothing left for this ticket, or the device deadline passed).
//
// Polling uses RELAXED loads (scope bits only: they bypass the non-coherent caches without the
// cache invalidate an acquire load carries — polling waves must not flush the L2 that holds the
// flow table).  Waves far from the frontier back off
// (s_sleep grows with the distance in chunks), so ~1K waiting waves do not turn the prod mirror
// into a hot spot that slows the waves doing work.
template <class OnIdle>
__device__ __forceinline__ bool ring_wait_chunk(const RingArgs& a, RingCtl* ctl, RingDevState* st, uint32_t lane,
                                                unsigned long long t_begin, unsigned long long& tk_out,
                                                uint32_t& epoch_out, uint32_t& gen_out, OnIdle on_idle) {
  unsigned long long tk = 0;
  if (lane == 0) tk = atomicAdd(&st->claim, 1ull);
  tk = rfl64(tk);
  tk_out = tk;
  const unsigned long long first = tk * 64ull;
  const unsigned long long need = first + 64ull;
  for (;;) {
    unsigned long long v = 0;
    uint32_t g = 0;
    if (lane == 0) {
      // the control-mailbox generation rides along with the poll (two loads in flight together)
      g = __hip_atomic_load(&a.st->ctl_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      v = __hip_atomic_load(&st->dprod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ring_count(v) < need && ring_count(v) == first && !(v & kRingStop)) {
        // frontier wave (its chunk is the first unpublished one): the only PCIe poller
        const unsigned long long hv = __hip_atomic_load(&ctl->prod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (hv > v) {
          __hip_atomic_fetch_max(&st->dprod, hv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v = hv;
        }
      }
    }
    v = rfl64(v);
    const unsigned long long avail = ring_count(v);
    if (avail >= need) {
      // the word that published this chunk (or a later one) names the flow-table copy: a word
      // older than the last flip has count <= the flip point, so only chunks below it (the
      // grace period's) can still use the previous copy
      epoch_out = ring_epoch(v);
      gen_out = __builtin_amdgcn_readfirstlane(g);
      return true;
    }
    on_idle();                        // no published work for this wave: settle its bookkeeping
    if (v & kRingStop) return false;  // stop and final count come in one word: nothing more will arrive
    if (__builtin_amdgcn_s_memrealtime() - t_begin > a.deadline) return false;
    const unsigned long long dist = (first - avail) >> 6;  // chunks ahead of the frontier
    if (dist == 0) __builtin_amdgcn_s_sleep(1);
    else if (dist < 8) __builtin_amdgcn_s_sleep(4);
    else if (dist < 64) __builtin_amdgcn_s_sleep(32);
    else __builtin_amdgcn_s_sleep(127);
  }
}

// GPU-direct egress of one chunk (ring.h GdeRing).  Every lane calls it (EXEC full).  Two short
// sections taken in ticket order (a pod sees a queue's frames in arrival order) around the frame
// writes, which chunks do in parallel:
//   1. reserve (turn gde_turn): per egress port, the lanes' slots in the port's GPU ring (the pod's
//      tail re-read over PCIe only when the cached one says full); the rest stays with the host;
//   2. the frames (one full 64-B line each: 16 per pass through the wave's LDS scratch) and their
//      descriptors, system-coherent write-through stores, waited for;
//   3. commit (turn gde_commit): each port's head published (system scope), waited for before the
//      next chunk may publish a later one, so a head never goes back.
// Every access to the shared egress state is a relaxed agent-scope atomic (no fences: an acquire /
// release would invalidate / write back the XCD's L2 - the flow table - per chunk).  A wave still
// waiting for a turn at the device deadline (the grid is exiting) does not take it: the chunk's
// frames stay with the host path, and no head moves without the turn.
__device__ __forceinline__ bool gde_turn(uint64_t* turn, unsigned long long tk, uint32_t lane, const RingArgs& a,
                                         unsigned long long t_begin) {
  uint32_t ok = 1u;
  if (lane == 0) {
    while (__hip_atomic_load(turn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tk) {
      if (__builtin_amdgcn_s_memrealtime() - t_begin > a.deadline) { ok = 0u; break; }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return __builtin_amdgcn_readfirstlane(ok) != 0u;
}
__device__ __forceinline__ void gde_deliver(const RingArgs& a, RingDevState* qst, uint32_t qi, unsigned long long tk,
                                            uint32_t lane, unsigned long long t_begin, bool elig0, uint32_t port,
                                            uint32_t olen, const uint32_t* o, uint32_t& meta, uint4* kx) {
  bool elig = elig0 && port < (uint32_t)kMaxPorts;
  auto ld32 = [](const uint32_t* x) { return __hip_atomic_load(x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto ld64 = [](const uint64_t* x) { return __hip_atomic_load(x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  // each lane reads its port's ring geometry before any turn (it changes only while the entry is
  // not valid): the serialised sections then load nothing but the head / tail
  uint64_t m_ctl = 0, m_desc = 0, m_buf = 0;
  uint32_t m_mask = 0, m_bsz = 0;
  if (elig) {
    const GdeRing* g = a.gde + (size_t)port * a.nq + qi;
    elig = ld32(&g->valid) == 1u;
    m_ctl = ld64(&g->ctl); m_desc = ld64(&g->desc); m_buf = ld64(&g->buf);
    m_mask = ld32(&g->mask); m_bsz = ld32(&g->buf_size);
  }
  auto rl64 = [](uint64_t v, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  };
  const unsigned long long tw0 = __builtin_amdgcn_s_memrealtime();
  const bool t_res = gde_turn(&qst->gde_turn, tk, lane, a, t_begin);
  if (!t_res) elig = false;   // (deadline: nothing reserved, the turn is not ours to pass on)
  const unsigned long long tw1 = __builtin_amdgcn_s_memrealtime();
  // ---- 1. reserve ----
  bool go = false;
  uint32_t pos = 0, end = 0, n_frames = 0, n_full = 0;   // (end: the port's new head)
  unsigned long long rem = __ballot(elig);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const uint32_t P = __builtin_amdgcn_readlane(port, leader);
    const bool mine = elig && port == P;
    const unsigned long long bm = __ballot(mine);
    rem &= ~bm;
    GdeRing* g = a.gde + (size_t)P * a.nq + qi;
    const uint32_t mask = __builtin_amdgcn_readlane(m_mask, leader);
    uint32_t head = __builtin_amdgcn_readfirstlane(ld32(&g->head)), tc = __builtin_amdgcn_readfirstlane(ld32(&g->tail_cache));
    const uint32_t cnt = (uint32_t)__builtin_popcountll(bm);
    uint32_t room = mask + 1u - (head - tc);
    if (room < cnt) {   // full by the cached tail: what the pod has drained since (one PCIe read)
      const uint64_t ctl = rl64(m_ctl, leader);
      uint32_t t = 0;
      if (lane == 0)
        t = __hip_atomic_load(reinterpret_cast<uint32_t*>(ctl + 64), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      tc = __builtin_amdgcn_readfirstlane(t);
      room = mask + 1u - (head - tc);
      if (room > mask + 1u) room = 0;   // (a bogus tail from the pod: deliver nothing)
    }
    const uint32_t n_ok = cnt < room ? cnt : room;
    n_frames += n_ok;
    n_full += cnt - n_ok;
    const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    if (mine && pre < n_ok) { go = true; pos = (head + pre) & mask; end = head + n_ok; }
    if (lane == 0) {
      __hip_atomic_store(&g->head, head + n_ok, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&g->tail_cache, tc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);   // the reservations are in memory before the next chunk reserves
  if (lane == 0 && t_res) __hip_atomic_store(&qst->gde_turn, tk + 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long tw2 = __builtin_amdgcn_s_memrealtime();
  // ---- 2. frames and descriptors (parallel across chunks) ----
  // Each frame as ONE full 64-B line write: 16 frames per pass through the wave's LDS scratch, the
  // 4 lanes of a frame storing its 4 pieces in the same instruction (they coalesce).  Per-lane 16-B
  // stores were partial-line writes to host memory: ~11 us per chunk (r5 s12 diagnostics).
  unsigned long long rgo = __ballot(go);
  while (rgo) {
    const int leader = __builtin_ctzll(rgo);
    const uint32_t P = __builtin_amdgcn_readlane(port, leader);
    const bool mine = go && port == P;
    const unsigned long long bgo = __ballot(mine);
    rgo &= ~bgo;
    const uint64_t desc = rl64(m_desc, leader), buf = rl64(m_buf, leader);
    const uint32_t mask = __builtin_amdgcn_readlane(m_mask, leader);
    const uint32_t bsz = __builtin_amdgcn_readlane(m_bsz, leader);
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(buf), (short)0,
                                                                        (int)((mask + 1u) * bsz), kBufRaw);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(desc), (short)0,
                                                                        (int)((mask + 1u) * 8u), kBufRaw);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (((bgo >> (16 * q)) & 0xFFFFull) == 0ull) continue;   // (wave-uniform)
      if ((lane >> 4) == (uint32_t)q) {
#pragma unroll
        for (int k = 0; k < 4; ++k) kx[kx_at(lane & 15u, k)] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const uint4 v = kx[kx_at(lane >> 2, lane & 3u)];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const int src = 16 * q + (int)(lane >> 2);
      const uint32_t spos = (uint32_t)__shfl((int)pos, src);
      const bool sgo = ((bgo >> src) & 1ull) != 0ull;
      const v4u w = {v.x, v.y, v.z, v.w};
      store_b128<kSysAux>(w, rb, sgo ? spos * bsz + 16u * (lane & 3u) : kNoRun, 0);
    }
    // descriptors: consecutive positions are consecutive 8-B entries (full lines when 8 in a row)
    typedef unsigned int v2u_t __attribute__((ext_vector_type(2)));
    const v2u_t dv = {olen, 0u};
    __builtin_amdgcn_raw_buffer_store_b64(dv, rd, mine ? pos * 8u : kNoRun, 0, kSysAux);
  }
  __builtin_amdgcn_s_waitcnt(0);   // (write-through stores done: the frames are in host memory)
  // ---- 3. commit: heads in ticket order ----
  const unsigned long long tw3 = __builtin_amdgcn_s_memrealtime();
  const bool t_com = gde_turn(&qst->gde_commit, tk, lane, a, t_begin);
  // (deadline: the slots written stay unpublished - the pod never sees them - and the host path
  // delivers these frames: their meta is left as it was)
  if (!t_com) go = false;
  if (go) meta = make_meta(port, kMetaLenGde, kOk);
  const unsigned long long tw4 = __builtin_amdgcn_s_memrealtime();
  rgo = __ballot(go);
  while (rgo) {
    const int leader = __builtin_ctzll(rgo);
    const uint32_t P = __builtin_amdgcn_readlane(port, leader);
    const uint32_t E = __builtin_amdgcn_readlane(end, leader);
    rgo &= ~__ballot(go && port == P);
    const uint64_t ctl = rl64(m_ctl, leader);
    if (lane == 0) __hip_atomic_store(reinterpret_cast<uint32_t*>(ctl), E, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // (waited for: a later chunk's head landing first and then overwritten would go back.  A PCIe
  // atomic add of the count instead needs no wait, but measured slower: 28-32 vs 42-57 Mpps, r5 s14)
  __builtin_amdgcn_s_waitcnt(0);   // this chunk's heads are out before a later chunk's may be
  if (lane == 0 && t_com) {
    __hip_atomic_store(&qst->gde_commit, tk + 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long tw5 = __builtin_amdgcn_s_memrealtime();
    __hip_atomic_fetch_add(&qst->gde_wait, (uint64_t)((tw1 - tw0) + (tw4 - tw3)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&qst->gde_sect, (uint64_t)((tw2 - tw1) + (tw5 - tw4)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&qst->gde_chunks, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&qst->gde_frames, (uint64_t)n_frames, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&qst->gde_full, (uint64_t)n_full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- SFC hops across GPUs in the live path (ring.h XferEntry) ----------------------------------
__device__ __forceinline__ uint32_t lane_rank(unsigned long long bm) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
}
__device__ __forceinline__ void hs_pack(const HopState& h, uint32_t w[8]) {
  w[0] = h.inmeta; w[1] = h.hash; w[2] = (uint32_t)h.acl_rule; w[3] = h.hop;
  w[4] = (uint32_t)h.act.chain_id | ((uint32_t)h.act.out_port << 16); w[5] = h.act.nat_ip;
  w[6] = (uint32_t)h.act.nat_port | ((uint32_t)h.act.vlan << 16); w[7] = h.act.flow_id;
}
__device__ __forceinline__ HopState hs_unpack(const uint32_t w[8]) {
  HopState h;
  h.inmeta = w[0]; h.hash = w[1]; h.acl_rule = (int32_t)w[2]; h.hop = w[3];
  h.act.chain_id = (uint16_t)(w[4] & 0xFFFFu); h.act.out_port = (uint16_t)(w[4] >> 16); h.act.nat_ip = w[5];
  h.act.nat_port = (uint16_t)(w[6] & 0xFFFFu); h.act.vlan = (uint16_t)(w[6] >> 16); h.act.flow_id = w[7];
  return h;
}
// A hand-off op naming no plane of this node (or no hop to resume at) ends the chain as a drop.
__device__ __forceinline__ void xfer_check(EgressDecision& e, uint32_t nplanes) {
  if (e.reason == kRemote && (e.out_port >= nplanes || e.inner_len == 0u)) { e.reason = kChainDrop; e.out_port = kPortNone; }
}

// The `go` lanes' frames to the inboxes of their planes (`plane`).  EXEC full.  Per target plane:
// one system-scope add on its inbox tail reserves the run of entries; each lane waits until its
// entry of a ring ago was consumed, stores slot, record and way back (system-coherent stores into
// the peer's HBM), and once every store is done the entry's seq.
__device__ __forceinline__ void xfer_send(const RingArgs& a, bool go, uint32_t plane, const uint32_t* o, const HopState& hs,
                                       uint32_t origin, uint32_t pos, uint32_t lane, unsigned long long t_begin) {
  uint32_t hw[8];
  hs_pack(hs, hw);
  unsigned long long rem = __ballot(go);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const uint32_t P = __builtin_amdgcn_readlane(plane, leader);
    const bool mine = go && plane == P;
    const unsigned long long bm = __ballot(mine);
    rem &= ~bm;
    XferInbox* ib = a.xpv[P].inbox;
    XferEntry* ent = a.xpv[P].entries;
    const uint32_t cmask = a.xpv[P].cap_mask;
    unsigned long long base = 0;
    if (lane == 0)
      base = __hip_atomic_fetch_add(&ib->tail, (unsigned long long)__builtin_popcountll(bm), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_SYSTEM);
    base = rfl64(base);
    const unsigned long long idx = base + lane_rank(bm);
    XferEntry* en = ent + (idx & cmask);
    if (mine && idx > cmask) {   // the entry a ring of the inbox ago must have been consumed
      const unsigned long long want = (idx - cmask) | kXferDone;   // ((idx - cap) + 1) | done
      while (__hip_atomic_load(&en->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
        if (__builtin_amdgcn_s_memrealtime() - t_begin > a.deadline) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc((void*)ent, (short)0,
                                                                        (int)((cmask + 1u) * 128u), kBufRaw);
    const uint32_t off = mine ? (uint32_t)((idx & cmask) * 128u) : kNoRun;
#pragma unroll
    for (int k = 0; k < 4; ++k) store_b128<kSysAux>(v4u{o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]}, re, off + 16u * k, 0);
    store_b128<kSysAux>(v4u{hw[0], hw[1], hw[2], hw[3]}, re, off + 64u, 0);
    store_b128<kSysAux>(v4u{hw[4], hw[5], hw[6], hw[7]}, re, off + 80u, 0);
    store_b128<kSysAux>(v4u{origin, pos, (uint32_t)__builtin_amdgcn_s_memrealtime(), 0u}, re, off + 96u, 0);
    __builtin_amdgcn_s_waitcnt(0);   // the entry is in the peer's memory before its seq says so
    if (mine) __hip_atomic_store(&en->seq, idx + 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// One pass over the `rdy` lanes' inbox entries (EXEC full): the rest of their chains, then either
// on to the next plane or back to the entry ring's out slot, its chunk's pending count reduced.
template <bool COOP>
__device__ __forceinline__ void xfer_resume(const RingArgs& a, bool rdy, XferEntry* en, unsigned long long idx, uint32_t lane,
                                         unsigned long long t_begin, uint32_t& seen_ep, uint4* kx) {
  const uint32_t t_pick = (uint32_t)__builtin_amdgcn_s_memrealtime();
  unsigned long long v = 0;
  if (lane == 0) v = __hip_atomic_load(&a.st->dprod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t ep = ring_epoch(rfl64(v));
  if (ep != seen_ep) {   // the host changed a table: drop cached lines first (as the chunk waves do)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    seen_ep = ep;
  }
  const TablesView& T = COOP ? a.sets[(ep & kEpochSetBit) >> 1].t : a.t;
  const DirectTables ta{T};
  // the entry (system-coherent loads: a peer wrote it).  One descriptor over the whole inbox and a
  // per-lane offset: a descriptor built from each lane's own entry pointer is not wave-uniform and
  // compiles to a loop over the 64 lanes (r6: 17 us of a 22-us resume pass, unloaded)
  const uint32_t cmask = a.xpv[a.xplane].cap_mask;
  const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc((void*)a.xpv[a.xplane].entries, (short)0,
                                                                      (int)((cmask + 1u) * 128u), kBufRaw);
  const uint32_t eo = rdy ? (uint32_t)(idx & cmask) * 128u : kNoRun;
  uint32_t d[kSlotDwords], hw[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const v4u c = __builtin_amdgcn_raw_buffer_load_b128(re, eo, 16 * k, kSysAux);
    d[4 * k] = c[0]; d[4 * k + 1] = c[1]; d[4 * k + 2] = c[2]; d[4 * k + 3] = c[3];
  }
  {
    const v4u c0 = __builtin_amdgcn_raw_buffer_load_b128(re, eo, 64, kSysAux);
    const v4u c1 = __builtin_amdgcn_raw_buffer_load_b128(re, eo, 80, kSysAux);
    hw[0] = c0[0]; hw[1] = c0[1]; hw[2] = c0[2]; hw[3] = c0[3]; hw[4] = c1[0]; hw[5] = c1[1]; hw[6] = c1[2]; hw[7] = c1[3];
  }
  const v4u way = __builtin_amdgcn_raw_buffer_load_b128(re, eo, 96, kSysAux);
  const uint32_t origin = way[0], pos = way[1];
  const HopState hs = hs_unpack(hw);
  Parsed p;
  IngressState st;
  __builtin_amdgcn_s_waitcnt(0);   // (timing: the entry is in)
  const uint32_t t_ld = (uint32_t)__builtin_amdgcn_s_memrealtime();
  resume_ingress(ta, d, hs.inmeta, p, st);
  EgressDecision e = resume_stage<DirectTables, false>(T, ta, p, st, hs.act, hs.acl_rule, hs.hash, hs.hop);
  xfer_check(e, a.nplanes);
  const uint32_t t_sg = (uint32_t)__builtin_amdgcn_s_memrealtime() + (e.out_port & 0u);
  uint32_t o[kSlotDwords];
  emit(p, e.tci, e.push != 0, o);
  const uint32_t olen = out_len(p, e);
  const bool again = rdy && e.reason == kRemote;   // handed on: same way back, still pending
  const bool fin = rdy && !again;
  const uint32_t meta = make_meta(e.out_port, olen, e.reason, !e.reason && e.xhdr, false);
  if (__ballot(again)) xfer_send(a, again, e.out_port, o, hop_state_of(p, st, e, hs.act, hs.acl_rule, hs.hash),
                                 origin, pos, lane, t_begin);
  // back to the entry ring: final slot and meta into its out slot (pinned host memory).  Each slot
  // goes out as ONE full 64-B line write: 16 frames per pass through the wave's LDS scratch, the 4
  // lanes of a frame storing its 4 pieces in one instruction (per-lane 16-B stores are partial-line
  // PCIe writes, ~11 us per 64 frames: the GPU-direct egress measurements, r5 s12)
  const uint32_t oplane = origin & 0xFFu, oq = origin >> 8;
  unsigned long long rem = __ballot(fin);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const uint32_t O = __builtin_amdgcn_readlane(oplane, leader);
    const bool mine = fin && oplane == O;
    const unsigned long long bm = __ballot(mine);
    rem &= ~bm;
    const uint32_t slots = a.xpv[O].ring_mask + 1u, nq = a.xpv[O].nq;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)a.xpv[O].out, (short)0,
                                                                        (int)(nq * slots * 64u), kBufRaw);
    const __amdgpu_buffer_rsrc_t rm = __builtin_amdgcn_make_buffer_rsrc((void*)a.xpv[O].out_meta, (short)0,
                                                                        (int)(nq * slots * 4u), kBufRaw);
    const uint32_t at = oq * slots + (pos & (slots - 1u));
    const bool ok = mine && oq < nq;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (((bm >> (16 * q)) & 0xFFFFull) == 0ull) continue;   // (wave-uniform)
      if ((lane >> 4) == (uint32_t)q) {
#pragma unroll
        for (int k = 0; k < 4; ++k) kx[kx_at(lane & 15u, k)] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const uint4 v = kx[kx_at(lane >> 2, lane & 3u)];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const int src = 16 * q + (int)(lane >> 2);
      const uint32_t sat = (uint32_t)__shfl((int)at, src);
      const bool sok = __shfl(ok ? 1 : 0, src) != 0;
      store_b128<kSysAux>(v4u{v.x, v.y, v.z, v.w}, ro, sok ? sat * 64u + 16u * (lane & 3u) : kNoRun, 0);
    }
    __builtin_amdgcn_raw_buffer_store_b32(meta, rm, ok ? at * 4u : kNoRun, 0, kSysAux);
  }
  __builtin_amdgcn_s_waitcnt(0);   // (the slots are in host memory before their chunk's count moves)
  const uint32_t t_wb = (uint32_t)__builtin_amdgcn_s_memrealtime();
  // pending counts: one system-scope subtraction per (entry plane, queue, chunk)
  const uint32_t chunk = pos >> 6;
  rem = __ballot(fin);
  while (rem) {
    const int leader = __builtin_ctzll(rem);
    const uint32_t K0 = __builtin_amdgcn_readlane(origin, leader), K1 = __builtin_amdgcn_readlane(chunk, leader);
    const unsigned long long bm = __ballot(fin && origin == K0 && chunk == K1);
    rem &= ~bm;
    const uint32_t O = K0 & 0xFFu, Q = K0 >> 8;
    const uint32_t nch = (a.xpv[O].ring_mask + 1u) >> 6;
    if (lane == 0 && Q < a.xpv[O].nq)
      __hip_atomic_fetch_sub(a.xpv[O].xpend + (size_t)Q * nch + (K1 & (nch - 1u)), (uint32_t)__builtin_popcountll(bm),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // entries consumed (a producer a ring later may reuse them), counters of this plane
  if (rdy) __hip_atomic_store(&en->seq, (idx + 1ull) | kXferDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  {   // hand-off timing sample: this pass's first entry
    const unsigned long long rbm = __ballot(rdy);
    if (rbm && lane == 0) {
      XferInbox* ib = a.xpv[a.xplane].inbox;
      const uint32_t ts = __builtin_amdgcn_readlane(way[2], __builtin_ctzll(rbm));
      atomicAdd(&ib->t_wait, (unsigned long long)(t_pick - ts));
      atomicAdd(&ib->t_work, (unsigned long long)((uint32_t)__builtin_amdgcn_s_memrealtime() - t_pick));
      atomicAdd(&ib->n_timed, 1ull);
      atomicAdd(&ib->t_load, (unsigned long long)(t_ld - t_pick));
      atomicAdd(&ib->t_stage, (unsigned long long)(t_sg - t_ld));
      atomicAdd(&ib->t_wb, (unsigned long long)(t_wb - t_sg));
    }
  }
  if (rdy && !(a.flags_bits & kRingNoCounters)) {
    if (e.reason) atomicAdd(a.drop_ctr + (e.reason & (kNumReasons - 1)), 1ull);
    else if (e.out_port < (uint32_t)kMaxPorts) atomicAdd(a.port_ctr + 2 * e.out_port + 1, ctr_inc(olen));
  }
}

// The inbox service of an XF grid (its last xfer_wgs workgroups; every wave on its own): claim an
// inbox chunk of 64 entries by ticket, resume each entry as soon as its seq says it is written, and
// take the next ticket once all 64 are done.  One system-scope load of the inbox tail per poll
// says which of the ticket's entries are reserved at all (a ticket nobody reserved into sleeps
// longer; the entries' own seq words are read only when reserved).  On the stop word (queue 0's,
// mirrored by its frontier wave) a wave still finishes every reserved entry of its ticket, and
// keeps claiming tickets while reserved entries remain, so a producer never waits forever for room.
template <bool COOP>
__device__ __forceinline__ void xfer_serve(const RingArgs& a, uint32_t lane, unsigned long long t_begin, uint4* kx) {
  XferInbox* ib = a.xpv[a.xplane].inbox;
  XferEntry* ent = a.xpv[a.xplane].entries;
  const uint32_t cmask = a.xpv[a.xplane].cap_mask;
  uint32_t seen_ep = 0xFFFFFFFFu;
  auto tail_now = [&]() {
    unsigned long long tl = 0;
    if (lane == 0) tl = __hip_atomic_load(&ib->tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return rfl64(tl);
  };
  auto stopping = [&]() {
    unsigned long long v = 0;
    if (lane == 0) v = __hip_atomic_load(&a.st->dprod, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (rfl64(v) & kRingStop) != 0ull || __builtin_amdgcn_s_memrealtime() - t_begin > a.deadline;
  };
  for (;;) {
    unsigned long long tk = 0;
    if (lane == 0) tk = __hip_atomic_fetch_add(&ib->claim, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tk = rfl64(tk);
    const unsigned long long first = tk * 64ull;
    const unsigned long long idx = first + lane;
    XferEntry* en = ent + (idx & cmask);
    bool done = false;
    for (;;) {
      const unsigned long long tl = tail_now();
      const bool reserved = idx < tl;
      bool rdy = false;
      if (reserved && !done) {
        const unsigned long long sq = __hip_atomic_load(&en->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        done = sq == ((idx + 1ull) | kXferDone);   // (consumed before a restart of this grid)
        rdy = !done && sq == idx + 1ull;
      }
      const unsigned long long rb = __ballot(rdy);
      if (rb) {
        xfer_resume<COOP>(a, rdy, en, idx, lane, t_begin, seen_ep, kx);
        done = done || rdy;
      }
      if (__ballot(!done) == 0ull) break;   // the ticket's 64 entries are handled
      if (!rb) {
        // stopping: what is reserved of this ticket is handled - the rest will never come
        if (stopping() && __ballot(reserved && !done) == 0ull) return;
        if (tl <= first) __builtin_amdgcn_s_sleep(32);
        else __builtin_amdgcn_s_sleep(2);
      }
    }
  }
}

// COOP = false: the 4 waves of a workgroup claim and process chunks independently (throughput).
// COOP = true (latency): the workgroup processes ONE chunk at a time — wave 0 claims and polls,
// all 4 waves parse the chunk and each scans a quarter of the ACL rule tiles on its own SIMD
// (the single-wave MFMA chain is the longest stage of a chunk), wave 0 combines the partial
// first-match minima through LDS and finishes the chunk.
// V6: instances for tables with IPv6 flows / rules (the IPv6 key fold, the IPv6 TCAM and the
// address check inline); the others keep the IPv4 path's register budget (an IPv6 packet's key
// carries kKeyV6 there and takes no flow / ACL part).
// GDE: the GPU-direct egress instances (gde_deliver in the chunk's tail; 2 waves / SIMD, <= 256
// registers); the others keep the ring's code and register allocation as they were without it.
// XF: the instances for split chains across the node's GPU planes (hand-offs sent to the next
// plane's inbox; the grid's last xfer_wgs workgroups serve this plane's inbox).
template <int HASH, int ACL, bool COOP, bool V6 = false, bool GDE = false, bool XF = false>
__global__ __launch_bounds__(kRingBlock, (GDE || XF) ? 2 : 1) void ring_kernel(RingArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if constexpr (XF) {
    if (blockIdx.x >= gridDim.x - a.xfer_wgs) {   // (block-uniform: the whole workgroup serves the inbox)
      const RingLds Lx = ring_lds(HASH, ACL, COOP ? a.lds_tiles : a.acl_tiles);
      uint4* kxx = reinterpret_cast<uint4*>(smem + Lx.kx) + (threadIdx.x >> 6) * 64;
      xfer_serve<COOP>(a, threadIdx.x & 63u, __builtin_amdgcn_s_memrealtime(), kxx);
      return;
    }
  }
  __shared__ unsigned long long coop_tk;                      // ticket
  __shared__ uint32_t coop_ctl[4];                            // go, epoch, table-set serial, ctl gen
  __shared__ uint32_t coop_best[COOP ? kRingWaves : 1][64];   // per-wave ACL partial minima
  __shared__ RingTableSet lset;                               // coop: the table set in use (LDS copy)
  const RingLds L = ring_lds(HASH, ACL, COOP ? a.lds_tiles : a.acl_tiles);
  v4i* lw = reinterpret_cast<v4i*>(smem + L.acl_w);
  v4i* lc = reinterpret_cast<v4i*>(smem + L.acl_c);
  v4i* lt = reinterpret_cast<v4i*>(smem + L.toep_f);
  uint32_t* ltab = reinterpret_cast<uint32_t*>(smem + L.toep_t);
  PortEntry* lport = reinterpret_cast<PortEntry*>(smem + L.tports);
  uint64_t* lchain = reinterpret_cast<uint64_t*>(smem + L.tchain);
  uint8_t* lperm = smem + L.tperm;
  // (Re)stage the small tables of a table set into LDS: all threads of the workgroup call it.
  // Non-coop rings stage the launch tables once (a commit drains and relaunches them).
  uint32_t cur_set = 0, cur_serial = 0, nport = 0, nchain = 0;
  // control-mailbox generation the LDS copies reflect (read before the first staging)
  uint32_t cur_gen = __hip_atomic_load(&a.st->ctl_gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool lds_perm = false;
  auto stage = [&](const TablesView& t, const v4i* wf, const v4i* ci, uint32_t tiles, const v4i* tf,
                   const uint32_t* tt) {
    if constexpr (ACL == kAclMfma) {
      const uint32_t lt_ = min(tiles, kLdsAclTiles), nw = lt_ * 64, nc = lt_ * 4;
      for (uint32_t i = threadIdx.x; i < nw; i += kRingBlock) lw[i] = wf[i];
      for (uint32_t i = threadIdx.x; i < nc; i += kRingBlock) lc[i] = ci[i];
    }
    if constexpr (HASH == kHashMfma)
      for (uint32_t i = threadIdx.x; i < 256; i += kRingBlock) lt[i] = tf[i];
    if constexpr (HASH == kHashLds)
      stage_toep(ltab, tt, threadIdx.x, kRingBlock);
    // ports / chain words / ACL verdicts in LDS: the per-packet path's only global loads are the
    // frame and the flow bucket
    const LdsTables s0 = stage_lds_tables(t, lport, lchain, lperm, true, kRingBlock);
    nport = s0.nport; nchain = s0.nchain; lds_perm = s0.lds_perm;
  };
  auto stage_set = [&](uint32_t which) {
    __syncthreads();   // no wave still reads the previous copies
    // the set's buffers are fresh allocations that may reuse addresses this CU / XCD still caches
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.sets + which);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&lset);
    for (uint32_t i = threadIdx.x; i < sizeof(RingTableSet) / 4; i += kRingBlock) dst[i] = src[i];
    __syncthreads();
    stage(lset.t, static_cast<const v4i*>(lset.acl_wfrag), static_cast<const v4i*>(lset.acl_cinit), lset.acl_tiles,
          static_cast<const v4i*>(lset.toep_frag), lset.toep_tab);
    cur_set = which;
    cur_serial = lset.serial;
    __syncthreads();
  };
  if constexpr (COOP) {
    stage_set((a.epoch0 & kEpochSetBit) >> 1);
  } else {
    stage(a.t, a.acl_wfrag, a.acl_cinit, a.acl_tiles, a.toep_frag, a.toep_tab);
  }
  uint32_t* pc = reinterpret_cast<uint32_t*>(smem + L.pc);
  uint32_t* drops = reinterpret_cast<uint32_t*>(smem + L.drops);
  for (uint32_t i = threadIdx.x; i < kLdsPorts * 4; i += kRingBlock) pc[i] = 0;
  if (threadIdx.x < kNumReasons) drops[threadIdx.x] = 0;
  __syncthreads();

  // this workgroup's queue (wave-uniform): its control word, ticket state, flags and slot range
  const uint32_t nch_q = (a.ring_mask >> 6) + 1u;   // chunks per queue
  const uint32_t qi = a.nq > 1 ? blockIdx.x % a.nq : 0u;
  RingCtl* const qctl = a.ctl + qi;
  RingDevState* const qst = a.st + qi;
  uint32_t* const qflags = a.flags + (size_t)qi * nch_q;
  uint32_t* const qsvc = a.svc ? a.svc + (size_t)qi * nch_q * kSvcWords : nullptr;
  // raw buffer views over the queue's ring (capacity <= 2^24 slots: byte offsets fit 32 bits)
  const uint32_t rbytes = (a.ring_mask + 1u) * 64u;
  const size_t qslot0 = (size_t)qi * (a.ring_mask + 1u);
  const __amdgpu_buffer_rsrc_t r_pk = __builtin_amdgcn_make_buffer_rsrc((void*)(a.pkts + qslot0 * 4), (short)0, (int)rbytes, kBufRaw);
  const __amdgpu_buffer_rsrc_t r_im = __builtin_amdgcn_make_buffer_rsrc((void*)(a.inmeta + qslot0), (short)0, (int)(rbytes / 16), kBufRaw);
  const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc((void*)(a.out + qslot0 * 4), (short)0, (int)rbytes, kBufRaw);
  const __amdgpu_buffer_rsrc_t r_meta = __builtin_amdgcn_make_buffer_rsrc((void*)(a.out_meta + qslot0), (short)0, (int)(rbytes / 16), kBufRaw);
  const bool counters = !(a.flags_bits & kRingNoCounters);
  uint32_t since_flush = 0;  // chunks this wave added to the LDS counters since its last flush
  const uint32_t wave = threadIdx.x >> 6;
  uint4* kx = reinterpret_cast<uint4*>(smem + L.kx) + wave * 64;
  const uint32_t lane = threadIdx.x & 63u;

  // ---- control mailbox (ring.h RingCtrlRing): workgroup 0's wave 0 applies posted writes ----
#ifndef NFDP_NO_CTRL_POLL
  const bool poller = blockIdx.x == 0 && wave == 0 && a.ctrl != nullptr;
#else   // latency attribution only (control writes are never applied)
  const bool poller = false;
#endif
  unsigned long long ctrl_n = 0, ctrl_t = 0;
  uint32_t ctrl_tick = 0;
  if (poller) {
    unsigned long long d0 = 0;
    if (lane == 0) d0 = __hip_atomic_load(&a.ctrl->done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    ctrl_n = rfl64(d0);
  }
  auto poll_ctrl = [&]() {   // EXEC full; every lane reads the same words (one request per wave)
    const unsigned long long h = __hip_atomic_load(&a.ctrl->head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long n0 = ctrl_n;
    bool moved = false, restage = false;
    while (__builtin_amdgcn_readfirstlane((uint32_t)(ctrl_n < h && ctrl_n - n0 < kCtrlSlots))) {
      RingCtrlEntry* ent = a.ctrl->e + (ctrl_n % kCtrlSlots);
      const uint32_t sq = __hip_atomic_load(&ent->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if (__builtin_amdgcn_readfirstlane(sq) != (uint32_t)(ctrl_n + 1)) break;   // not visible yet: next poll
      const unsigned long long dst64 = __hip_atomic_load(&ent->dst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t nw = __hip_atomic_load(&ent->nwords, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint32_t n = min(nw & ~kCtrlNoRestage, kCtrlWords);
      restage = restage || !(nw & kCtrlNoRestage);
      if (lane < n) {
        const uint32_t v = __hip_atomic_load(&ent->data[lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(reinterpret_cast<uint32_t*>(dst64) + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#ifdef NFDP_CTRL_DEBUG
      if (lane == 0) printf("ctrl poll: h %llu n0 %llu entry %llu seq %u dst %llx words %u\n", h, n0, ctrl_n, sq, dst64, n);
#endif
      ++ctrl_n;
      moved = true;
    }
    if (!moved) return;
    // the writes reach every XCD before the generation moves; then the host hears it
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (lane == 0) {
      // (writes that no LDS copy holds - the table-set serial mirror - leave the copies alone)
      if (restage) __hip_atomic_fetch_add(&a.st->ctl_gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.ctrl->done, ctrl_n, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };
  auto on_idle = [&]() {
    if (since_flush) { flush_lds_counters(pc, drops, a.port_ctr, a.drop_ctr); since_flush = 0; }
    if (poller) {   // idle: look at the mailbox at most every microsecond (one PCIe read)
      const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
      if (tn - ctrl_t >= 100) { ctrl_t = tn; poll_ctrl(); }
    }
  };
  const uint32_t nch_mask = a.ring_mask >> 6;  // R/64 - 1
  const unsigned long long t_begin = __builtin_amdgcn_s_memrealtime();
  uint32_t seen_epoch = 0xFFFFFFFFu;  // epoch of this wave's previous chunk
  unsigned long long seen_t = 0;      // when this wave took its previous chunk
  uint32_t w0_epoch = 0xFFFFFFFFu;    // coop wave 0: epoch / time of the workgroup's previous chunk
  unsigned long long w0_t = 0;

  for (;;) {
    unsigned long long tk = 0;
    uint32_t epoch = 0;
    if constexpr (COOP) {
      if (wave == 0) {
        uint32_t gen = cur_gen;
        const bool go = ring_wait_chunk(a, qctl, qst, lane, t_begin, tk, epoch, gen, on_idle);
        // the serial of the set this epoch names, read only when the epoch moved (or the
        // workgroup idled long enough for the epoch value to have come round again)
        uint32_t ser = cur_serial;
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
#ifndef NFDP_NO_SERIAL_ALIAS
        if (go && (epoch != w0_epoch || tn - w0_t > kEpochAliasTicks)) {
#else   // latency attribution only (misses a set rewritten twice while idle)
        if (go && epoch != w0_epoch) {
#endif
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          ser = __hip_atomic_load(&a.st->set_serial[(epoch & kEpochSetBit) >> 1], __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);   // (device mirror: no PCIe round trip)
        }
        w0_epoch = epoch;
        w0_t = tn;
        if (lane == 0) { coop_tk = tk; coop_ctl[0] = go ? 1u : 0u; coop_ctl[1] = epoch; coop_ctl[2] = ser; coop_ctl[3] = gen; }
      }
      __syncthreads();
      tk = rfl64(coop_tk);
      epoch = __builtin_amdgcn_readfirstlane(coop_ctl[1]);
      if (!__builtin_amdgcn_readfirstlane(coop_ctl[0])) break;
    } else {
      uint32_t gen = 0;   // (non-coop rings stage their LDS copies at launch only)
      if (!ring_wait_chunk(a, qctl, qst, lane, t_begin, tk, epoch, gen, on_idle)) break;
    }
    const unsigned long long t_avail = __builtin_amdgcn_s_memrealtime();
#ifndef NFDP_NO_ALIAS_FENCE
    if (epoch != seen_epoch || t_avail - seen_t > kEpochAliasTicks) {
#else   // latency attribution only (stale table lines after 32 idle epoch changes)
    if (epoch != seen_epoch) {
#endif
      // A new epoch: the host rewrote a table this kernel reads with ordinary cached loads (the
      // flow-table copy it now names, the table set, or the MAC table after learning).  The
      // lines this wave's CU L1 and its XCD's L2 still hold may be stale - this grid never sees
      // the cache invalidate a kernel launch brings - so drop them (agent-scope acquire) first.
      // The generation is 5 bits: a wave idle through a multiple of 32 changes would see its old
      // value again.  The host spaces any 32 consecutive changes over >= kEpochAliasHostUs, so a
      // wave whose previous chunk is older than half of that invalidates regardless.
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      seen_epoch = epoch;
    }
    seen_t = t_avail;
    if constexpr (COOP) {
      // a new table set: every wave of the workgroup holds the same epoch (wave 0 broadcast it),
      // so the branch is uniform and the barriers inside are safe
      const uint32_t want = (epoch & kEpochSetBit) >> 1;
      if (want != cur_set || __builtin_amdgcn_readfirstlane(coop_ctl[2]) != cur_serial) stage_set(want);
      // control-mailbox writes applied since this workgroup staged its copies: restage the small
      // tables (ports, chain words, ACL verdicts) from the set's device buffers, which hold them
      const uint32_t gen = __builtin_amdgcn_readfirstlane(coop_ctl[3]);
      if (gen != cur_gen) {
#ifdef NFDP_CTRL_DEBUG
        if (threadIdx.x == 0) printf("restage: block %u gen %u -> %u ports %p\n", blockIdx.x, cur_gen, gen, (const void*)lset.t.ports);
#endif
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __syncthreads();   // no wave still reads the LDS copies
        const LdsTables s1 = stage_lds_tables(lset.t, lport, lchain, lperm, true, kRingBlock);
        nport = s1.nport; nchain = s1.nchain; lds_perm = s1.lds_perm;
        __syncthreads();
        cur_gen = gen;
      }
    }
    const TablesView& T = COOP ? lset.t : a.t;
    const LdsTables ta{T, lport, lchain, lperm, nport, nchain, lds_perm};
    const AclView av = COOP ? AclView{lw, lc, static_cast<const v4i*>(lset.acl_wfrag),
                                      static_cast<const v4i*>(lset.acl_cinit), lset.acl_tiles}
                            : AclView{lw, lc, a.acl_wfrag, a.acl_cinit, a.acl_tiles};
    const bool trace = (a.flags_bits & kRingTrace) != 0 && wave == 0;
    uint32_t tr0 = 0, tr1 = 0, tr2 = 0, tr3 = 0, tr4 = 0, tr5 = 0;
#define NFDP_RING_MARK(var)                                                 \
  if (trace) {                                                              \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");             \
    var = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_avail);          \
  }

    // ---- one packet per lane: the fused kernel's stages ----
    const uint32_t tk32 = (uint32_t)tk;  // slot / flag positions are modulo the ring (<= 2^24 slots)
    const uint32_t i = (tk32 * 64u + lane) & a.ring_mask;
    // the chunk's 64 slots are one 4-KiB run: lane-contiguous loads, transposed through LDS
    const uint32_t run = __builtin_amdgcn_readfirstlane(((tk32 * 64u) & a.ring_mask) * 64u);
    uint32_t d[kSlotDwords];
    const uint32_t im = __builtin_amdgcn_raw_buffer_load_b32(r_im, i * 4u, 0, kSysAux);
    {
      v4u c[4];
      if (a.faddr) {
        ring_frames_gather(a.faddr + qslot0, i, c);
      } else {
        wave_frames_load<kSysAux>(r_pk, run, c);
      }
      wave_frames_to_lanes(kx, c, d);
    }
    if (a.faddr) frame_clip(d, im >> 16);   // the bytes past the frame are not the producer's zeros
    NFDP_RING_MARK(tr0)
    Parsed p;
    IngressState st;
    ingress_stage<LdsTables, V6>(T, ta, d, im, p, st);
    uint32_t hash = 0;
    int acl_rule = -1;
    if constexpr (COOP && ACL == kAclMfma) {
      uint32_t b = 0xFFFFFFFFu;
      classify_wave<HASH, ACL>(st.key, kx, av, lt, ltab, T, hash, acl_rule, wave, kRingWaves, &b);
      coop_best[wave][lane] = b;
      __syncthreads();
      if (wave != 0) continue;  // helpers go back to wait for the next chunk
      b = min(min(coop_best[0][lane], coop_best[1][lane]), min(coop_best[2][lane], coop_best[3][lane]));
      acl_rule = acl_rule_of(b, T.n_acl);
    } else {
      if (COOP && wave != 0) continue;  // nothing to share without the MFMA ACL
      classify_wave<HASH, ACL>(st.key, kx, av, lt, ltab, T, hash, acl_rule);
    }
    // IPv6: the IPv6 TCAM (scalar here: the ring keeps its register budget for the IPv4 path)
    if constexpr (V6) {
      if (__builtin_expect(__any(p.ipv6 && v6_keys(T)), 0)) {
        if (p.ipv6 && v6_keys(T)) acl_rule = acl_rule_v6(T, p, st);
      }
    }
    NFDP_RING_MARK(tr1)
    bool hit = false;
    FlowAction act = {};
    int64_t slot = -1;
    if (!st.reason && (V6 ? flowable(T, p) : p.ipv4)) {
      uint4 v;
      TablesView tv = T;
      tv.flows = static_cast<const FlowSlot*>(a.flows2[epoch & 1u]);   // (its IPv6 side array follows it)
      slot = flow_probe(tv, st.key, hash, v);
      if (V6 && slot >= 0 && p.ipv6 && !flow6_verify(tv, p, slot)) slot = -1;
      if (slot >= 0) {
        hit = true;
        act.chain_id = v.x & 0xFFFFu; act.out_port = v.x >> 16; act.nat_ip = v.y;
        act.nat_port = v.z & 0xFFFFu; act.vlan = v.z >> 16; act.flow_id = v.w;
      }
    }
    NFDP_RING_MARK(tr2)
    EgressDecision e = chain_stage<LdsTables, V6, XF>(T, ta, p, st, hit, act, acl_rule, hash);
    if constexpr (XF) xfer_check(e, a.nplanes);
    const uint32_t olen = egress_len(p, e);
    uint32_t o[kSlotDwords];
    emit(p, e.tci, e.push != 0, o);
    const bool pad = im == kRingPadMeta;  // filler slot of a partial burst: no counters, no side work
    uint32_t meta = make_meta(e.out_port, olen, e.reason, !e.reason && e.xhdr, !e.reason && e.flood);
    if constexpr (GDE)   // GPU-direct egress: frames for memif vports straight into the pods' rings
      gde_deliver(a, qst, qi, tk, lane, t_begin, !pad && !e.reason && !e.xhdr && !e.flood && olen <= 64u,
                  e.out_port, olen, o, meta, kx);
    // split chains (XF): frames handed to another plane's grid (ring.h XferEntry) are not stored
    // here - their resumer writes their out slot and meta, so no ordering between the two is needed
    const unsigned long long bx = XF ? __ballot(!pad && e.reason == kRemote) : 0ull;
    wave_frames_store<kSysAux>(kx, o, r_out, run, bx);
    __builtin_amdgcn_raw_buffer_store_b32(meta, r_meta, ((bx >> lane) & 1ull) ? kNoRun : i * 4u, 0, kSysAux);
    if constexpr (XF) {
      if (bx) {
        // the chunk's pending count goes UP by the hand-offs (an add, not a store: a resumer's
        // decrement may land first; the word reads 0 only once both have, and the add is done
        // before the chunk's flag - the waitcnt below - so the host never sees an early 0)
        if (lane == 0)
          __hip_atomic_fetch_add(a.xpend + (size_t)qi * nch_q + (tk32 & nch_mask), (uint32_t)__builtin_popcountll(bx),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        xfer_send(a, ((bx >> lane) & 1ull) != 0ull, e.out_port, o, hop_state_of(p, st, e, act, acl_rule, hash),
                  a.xplane | (qi << 8), i, lane, t_begin);
      }
    }
    if (a.side.cnt) {
      // flood / mirror / ARP-trap / learning / tunnel packets go on the side list; the host runs
      // the side pass over them once the chunk's flag is seen (before the flag: vmcnt covers it)
      const bool sn = !pad && side_needed(st, p, e);
      if (__builtin_expect(__any(sn), 0)) side_list_append(a.side, sn, i);
    }
    NFDP_RING_MARK(tr3)

    // ---- completion: the chunk's write-through stores are done before its flag is written ----
    __builtin_amdgcn_s_waitcnt(0);
    NFDP_RING_MARK(tr4)
    if (lane == 0) {
      if (qsvc) qsvc[(size_t)(tk32 & nch_mask) * kSvcWords + 7] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_avail);
      __hip_atomic_store(&qflags[tk32 & nch_mask], tk32 + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }

    // ---- counters, off the latency path (after the flag): port / drop counters into the
    // workgroup's LDS (flushed when idle, every kFlushChunks chunks and at exit), per-flow words
    // (nearly distinct per packet) straight to the global table.
    if (counters && !pad) {   // (per lane: filler lanes count nothing)
      if (st.in_port < (uint32_t)kLdsPorts) {
        atomicAdd(&pc[st.in_port], 1u); atomicAdd(&pc[kLdsPorts + st.in_port], st.wire_len);
      } else if (st.in_port < (uint32_t)kMaxPorts) {
        atomicAdd(a.port_ctr + 2 * st.in_port, ctr_inc(st.wire_len));
      }
      if (e.reason) {
        atomicAdd(&drops[e.reason & (kNumReasons - 1)], 1u);
      } else if (e.out_port < (uint32_t)kLdsPorts) {
        atomicAdd(&pc[2 * kLdsPorts + e.out_port], 1u); atomicAdd(&pc[3 * kLdsPorts + e.out_port], olen);
      } else {
        atomicAdd(a.port_ctr + 2 * e.out_port + 1, ctr_inc(olen));
      }
      if (hit && a.flow_ctr && !(a.flags_bits & 4u)) atomicAdd(a.flow_ctr + slot, ctr_inc(st.wire_len));
    }
    // Wave-uniform: the flush moves every port's tally with the lane that owns that port index
    // (flush_lds_counters), whatever lane counted the packet, so it must run with EXEC full.  (A
    // per-lane count inside the branch above left a port's tallies behind for good whenever its
    // lane had been a filler lane of every chunk since its last flush.)
    if (counters && ++since_flush >= kFlushChunks) on_idle();
    if (poller && (++ctrl_tick & 15u) == 0) poll_ctrl();   // busy: the mailbox every 16 chunks
    NFDP_RING_MARK(tr5)
#undef NFDP_RING_MARK
    if (trace && lane == 0 && qsvc) {
      uint32_t* sv = qsvc + (size_t)(tk32 & nch_mask) * kSvcWords;
      sv[0] = tr0; sv[1] = tr1; sv[2] = tr2; sv[3] = tr3; sv[4] = tr4; sv[5] = tr5; sv[6] = 0;
    }
  }
  on_idle();  // exit: whatever this wave counted since its last flush reaches the global table
}

// why the last launch_ring on this thread refused its arguments (RingEngine::start's message)
thread_local const char* g_ring_why = "";
static hipError_t ring_bad(const char* why) {
  g_ring_why = why;
  return hipErrorInvalidValue;
}

template <int H, int A, bool C, bool V6 = false, bool G = false, bool X = false>
static hipError_t launch_ring_t(const RingArgs& a, int num_cus, int wgs, hipStream_t s) {
  const size_t lds = ring_lds(H, A, C ? a.lds_tiles : a.acl_tiles).total;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ring_kernel<H, A, C, V6, G, X>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  if ((lds + 2048) * (size_t)wgs > 160 * 1024) return ring_bad("LDS per workgroup x workgroups per CU exceeds the CU's 160 KB");
  hipLaunchKernelGGL((ring_kernel<H, A, C, V6, G, X>), dim3((uint32_t)(num_cus * wgs)), dim3(kRingBlock), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_ring(const RingLaunch& r, const LaunchCfg& cfg, int wgs_per_cu, bool coop, hipStream_t s) {
  RingArgs a;
  a.t = r.f.t;
  a.pkts = reinterpret_cast<const uint4*>(r.pkts);
  a.inmeta = r.inmeta;
  a.out = reinterpret_cast<uint4*>(r.out);
  a.out_meta = r.out_meta;
  a.ring_mask = r.ring_mask;
  a.ctl = r.ctl; a.flags = r.flags; a.st = r.st; a.svc = r.svc;
  a.flow_ctr = r.f.flow_ctr; a.port_ctr = r.f.port_ctr; a.drop_ctr = r.f.drop_ctr;
  a.acl_wfrag = reinterpret_cast<const v4i*>(r.f.acl_wfrag);
  a.acl_cinit = reinterpret_cast<const v4i*>(r.f.acl_cinit);
  a.acl_tiles = r.f.acl_tiles;
  a.toep_frag = reinterpret_cast<const v4i*>(r.f.toep_frag);
  a.toep_tab = r.f.toep_tab;
  a.deadline = r.deadline_ticks;
  a.side = r.f.side;
  a.flows2[0] = r.f.t.flows;
  a.flows2[1] = r.flows_alt ? r.flows_alt : r.f.t.flows;
  a.flags_bits = r.f.flags;
  a.sets = r.sets;
  a.lds_tiles = r.lds_tiles;
  a.epoch0 = r.epoch0;
  a.ctrl = r.ctrl;
  a.faddr = reinterpret_cast<const unsigned long long*>(r.faddr);
  a.gde = r.gde;
  a.xpeers = r.xpeers;
  if (r.xpeers && r.xpeers_h)
    for (uint32_t i = 0; i < r.nplanes && i < kMaxXferPlanes; ++i) a.xpv[i] = r.xpeers_h[i];
  a.xplane = r.xplane;
  a.nplanes = r.nplanes;
  a.xfer_wgs = r.xpeers ? r.xfer_wgs : 0u;
  a.xpend = r.xpend;
  a.nq = r.queues ? r.queues : 1u;
  // every queue needs a workgroup; the side list indexes slots of one ring only
  if ((uint64_t)cfg.num_cus * (uint64_t)wgs_per_cu < a.nq || (a.nq > 1 && a.side.cnt)) return ring_bad("fewer workgroups than queues, or a side list with several queues");
  if (coop && (!a.sets || a.lds_tiles < a.acl_tiles)) return ring_bad("coop ring without table sets or with fewer LDS tiles than ACL tiles");
  if (!a.port_ctr || !a.drop_ctr || !a.ctl || !a.flags || !a.st) return ring_bad("missing counters / control words");
  if (((r.ring_mask + 1) & r.ring_mask) != 0 || r.ring_mask < 63) return ring_bad("ring size not a power of two >= 64");
  if (cfg.acl_mode == kAclMfma && (a.acl_tiles == 0 || a.acl_tiles > kAclMaxRules / 16 || !a.acl_wfrag || !a.acl_cinit))
    return ring_bad("ACL tiles out of range or missing fragments");
  if (cfg.hash_mode == kHashMfma && !a.toep_frag) return ring_bad("MFMA hash without its fragments");
  if (cfg.hash_mode == kHashLds && !a.toep_tab) return ring_bad("LDS hash without its table");
  if (wgs_per_cu < 1 || wgs_per_cu > 8 || cfg.num_cus < 1) return ring_bad("workgroups per CU not in [1, 8]");
  const int h = cfg.hash_mode, ac = cfg.acl_mode;
  if (a.xpeers) {   // split chains across planes: the XF instances (IPv4 tables, MFMA ACL, no GDE)
    if (ac != kAclMfma || h == kHashScalar || a.gde || v6_keys(a.t)) return hipErrorNotSupported;
    if (!a.xpend || a.xfer_wgs == 0 || a.nplanes == 0 || a.nplanes > kMaxXferPlanes || a.xplane >= a.nplanes ||
        (uint64_t)cfg.num_cus * (uint64_t)wgs_per_cu < (uint64_t)a.nq + a.xfer_wgs)
      return ring_bad("cross-plane hops: bad peers / pending words / too few workgroups for queues + inbox service");
#define NFDP_XCASE(HH, CC) \
    if (h == HH && coop == CC) return launch_ring_t<HH, kAclMfma, CC, false, false, true>(a, cfg.num_cus, wgs_per_cu, s);
    NFDP_XCASE(kHashLds, true) NFDP_XCASE(kHashLds, false) NFDP_XCASE(kHashMfma, true) NFDP_XCASE(kHashMfma, false)
#undef NFDP_XCASE
    return ring_bad("no ring instance for this configuration");
  }
  if (a.gde) {   // GPU-direct egress: its instances (LDS or MFMA hash, MFMA ACL, IPv4 or IPv6 tables)
    if (ac != kAclMfma || h == kHashScalar) return hipErrorNotSupported;
    const bool v6 = v6_keys(a.t);
#define NFDP_GCASE(HH, CC, VV) \
    if (h == HH && coop == CC && v6 == VV) return launch_ring_t<HH, kAclMfma, CC, VV, true>(a, cfg.num_cus, wgs_per_cu, s);
    NFDP_GCASE(kHashLds, true, false) NFDP_GCASE(kHashLds, false, false) NFDP_GCASE(kHashLds, true, true)
    NFDP_GCASE(kHashLds, false, true) NFDP_GCASE(kHashMfma, true, false) NFDP_GCASE(kHashMfma, false, false)
    NFDP_GCASE(kHashMfma, true, true) NFDP_GCASE(kHashMfma, false, true)
#undef NFDP_GCASE
    return ring_bad("no ring instance for this configuration");
  }
  if (v6_keys(a.t)) {   // IPv6 flows / rules: the V6 instances (LDS or MFMA hash, MFMA ACL)
    if (ac != kAclMfma || h == kHashScalar) return hipErrorNotSupported;
    if (h == kHashLds) return coop ? launch_ring_t<kHashLds, kAclMfma, true, true>(a, cfg.num_cus, wgs_per_cu, s)
                                   : launch_ring_t<kHashLds, kAclMfma, false, true>(a, cfg.num_cus, wgs_per_cu, s);
    return coop ? launch_ring_t<kHashMfma, kAclMfma, true, true>(a, cfg.num_cus, wgs_per_cu, s)
                : launch_ring_t<kHashMfma, kAclMfma, false, true>(a, cfg.num_cus, wgs_per_cu, s);
  }
#define NFDP_RCASE(HH, AA)                                                                   \
  if (h == HH && ac == AA)                                                                   \
    return coop ? launch_ring_t<HH, AA, true>(a, cfg.num_cus, wgs_per_cu, s)                 \
                : launch_ring_t<HH, AA, false>(a, cfg.num_cus, wgs_per_cu, s);
  NFDP_RCASE(0, 0) NFDP_RCASE(0, 1) NFDP_RCASE(0, 2)
  NFDP_RCASE(1, 0) NFDP_RCASE(1, 1) NFDP_RCASE(1, 2)
  NFDP_RCASE(2, 0) NFDP_RCASE(2, 1) NFDP_RCASE(2, 2)
#undef NFDP_RCASE
  return ring_bad("no ring instance for this configuration");
}

// ------------------------------------------------------------------------------------------
// Host engine
// ------------------------------------------------------------------------------------------
namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("ring: ") + what + ": " + hipGetErrorString(e));
}
using Clock = std::chrono::steady_clock;
inline double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }
}  // namespace

RingEngine::RingEngine(uint32_t capacity, int num_cus, int wgs_per_cu, bool coop, bool host_slots, uint32_t queues)
    : cap_(capacity), nch_(capacity / 64), nq_(queues), num_cus_(num_cus), wgs_(wgs_per_cu), coop_(coop),
      host_slots_(host_slots) {
  if (capacity < 64 || (capacity & (capacity - 1)) || capacity > (1u << 24))
    throw std::invalid_argument("ring: capacity must be a power of two in [64, 2^24]");
  if (num_cus < 1 || wgs_per_cu < 1 || wgs_per_cu > 8) throw std::invalid_argument("ring: bad grid");
  if (queues < 1 || queues > 64 || (uint64_t)queues > (uint64_t)num_cus * wgs_per_cu)
    throw std::invalid_argument("ring: queues in [1, 64] and at most one per workgroup");
  if ((uint64_t)capacity * queues > (1u << 26)) throw std::invalid_argument("ring: capacity x queues too large");
  qs_.reset(new Queue[nq_]);
  ck(hipGetDevice(&device_), "get device");
  // control lines + completion flags: pinned, coherent (the GPU polls / writes them over PCIe)
  ck(hipHostMalloc(reinterpret_cast<void**>(&ctl_), sizeof(RingCtl) * nq_, hipHostMallocCoherent | hipHostMallocMapped),
     "host alloc ctl");
  ck(hipHostMalloc(reinterpret_cast<void**>(&flags_), (size_t)nq_ * nch_ * 4, hipHostMallocCoherent | hipHostMallocMapped),
     "host alloc flags");
  std::memset(ctl_, 0, sizeof(RingCtl) * nq_);
  std::memset(flags_, 0, (size_t)nq_ * nch_ * 4);
  ck(hipHostMalloc(reinterpret_cast<void**>(&ctrl_), sizeof(RingCtrlRing), hipHostMallocCoherent | hipHostMallocMapped),
     "host alloc ctrl");
  std::memset(ctrl_, 0, sizeof(RingCtrlRing));
  ck(hipMalloc(reinterpret_cast<void**>(&st_), sizeof(RingDevState) * nq_), "dev alloc state");
  // Slots: HBM (the wire side is the GPU: NIC DMA into device memory), or pinned coherent host
  // memory (host-resident rings — pod vhost / AF_XDP style): the kernel's system-coherent buffer
  // ops then read and write the frames over PCIe directly, with no separate copy step.
  auto slot_alloc = [&](void** p, size_t bytes, const char* what) {
    if (host_slots_) {
      void* h = nullptr;
      ck(hipHostMalloc(&h, bytes, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable), what);
      std::memset(h, 0, bytes);
      ck(hipHostGetDevicePointer(p, h, 0), what);
      host_ptrs_.push_back(h);
    } else {
      ck(hipMalloc(p, bytes), what);
      ck(hipMemset(*p, 0, bytes), what);
    }
  };
  const size_t slots = (size_t)capacity * nq_;
  slot_alloc(reinterpret_cast<void**>(&d_in_), slots * 64, "alloc in");
  slot_alloc(reinterpret_cast<void**>(&d_im_), slots * 4, "alloc inmeta");
  slot_alloc(reinterpret_cast<void**>(&d_out_), slots * 64, "alloc out");
  slot_alloc(reinterpret_cast<void**>(&d_meta_), slots * 4, "alloc meta");
  if (host_slots_) {   // frame addresses (zero-copy rx; set_frame_addrs)
    slot_alloc(reinterpret_cast<void**>(&d_faddr_), slots * 8, "alloc frame addresses");
    h_faddr_ = static_cast<uint64_t*>(host_ptrs_.back());
    for (size_t i = 0; i < slots; ++i) h_faddr_[i] = reinterpret_cast<uint64_t>(d_in_) + i * 64u;
  }
  ck(hipMalloc(reinterpret_cast<void**>(&d_svc_), (size_t)nq_ * nch_ * 4 * kSvcWords), "dev alloc svc");
  // Table sets: pinned, coherent host memory the grid reads (a few hundred bytes, once per set
  // change).  Staging one is a host store, never a copy on a stream: with resident grids on the
  // device a stream may share a hardware queue with one of them and would never be served.
  ck(hipHostMalloc(reinterpret_cast<void**>(&h_sets_), 2 * sizeof(RingTableSet), hipHostMallocCoherent | hipHostMallocMapped),
     "host alloc table sets");
  std::memset(static_cast<void*>(h_sets_), 0, 2 * sizeof(RingTableSet));
  ck(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_sets_), h_sets_, 0), "device ptr table sets");
  ck(hipMalloc(reinterpret_cast<void**>(&dd_sets_), 2 * sizeof(RingTableSet)), "dev alloc table sets");
  ck(hipMemset(dd_sets_, 0, 2 * sizeof(RingTableSet)), "memset table sets");
  ck(hipMemset(d_svc_, 0, (size_t)nq_ * nch_ * 4 * kSvcWords), "memset");
  // (the launch stream is created by start() and destroyed by stop(): a resident grid holds its
  // stream's hardware queue, and a stopped ring should not keep one that other streams then share)
}

RingEngine::~RingEngine() {
  try {
    if (running_) stop(60.0);
  } catch (...) {
  }
  release_streams();
  for (void* d : {(void*)st_, (void*)d_svc_, (void*)dd_sets_, (void*)d_gde_, (void*)d_xin_, (void*)d_xent_,
                  (void*)d_xpeers_})
    (void)hipFree(d);
  if (h_xpend_) (void)hipHostFree(h_xpend_);
  (void)hipHostFree(h_sets_);
  if (host_slots_) {
    for (void* h : host_ptrs_) (void)hipHostFree(h);
  } else {
    for (void* d : {(void*)d_in_, (void*)d_im_, (void*)d_out_, (void*)d_meta_}) (void)hipFree(d);
  }
  (void)hipHostFree(ctl_);
  (void)hipHostFree(flags_);
  (void)hipHostFree(ctrl_);
}

void RingEngine::start(const FusedLaunch& f, const LaunchCfg& cfg, double deadline_s, const void* flows_alt) {
  if (running_) throw std::runtime_error("ring: already running");
  if (!(deadline_s > 0.0) || deadline_s > 3600.0) throw std::invalid_argument("ring: deadline in (0, 3600] s");
  if ((uint64_t)cfg.num_cus * (uint64_t)wgs_ < nq_) throw std::invalid_argument("ring: fewer workgroups than queues");
  const uint32_t ep = epoch();
  launch_ = f;
  // coop rings: the session's tables are table set (epoch bit 1); the LDS layout holds up to
  // kLdsAclTiles rule tiles, so a later set with more tiles than that needs a relaunch
  lds_tiles_ = coop_ ? std::max<uint32_t>(f.acl_tiles, kLdsAclTiles) : f.acl_tiles;
  if (coop_) stage_tables(f, (int)((ep & kEpochSetBit) >> 1));   // (before the state upload: its serial)
  // resume at the published positions: tickets restart at prod/64, nothing outstanding
  std::vector<RingDevState> s(nq_);
  for (uint32_t q = 0; q < nq_; ++q) {
    if (completed(q) != published(q)) throw std::runtime_error("ring: previous session left chunks unprocessed");
    const uint64_t p = published(q);
    std::memset(&s[q], 0, sizeof(RingDevState));
    s[q].claim = p / 64;
    s[q].dprod = ring_word(p, ep);
    __atomic_store_n(&ctl_[q].prod, ring_word(p, ep), __ATOMIC_RELEASE);
  }
  s[0].set_serial[0] = h_sets_[0].serial;
  s[0].set_serial[1] = h_sets_[1].serial;
  for (uint32_t q = 0; q < nq_; ++q) s[q].gde_turn = s[q].gde_commit = s[q].claim;   // GPU-direct egress: first ticket's turns
  if (!stream_) create_stream();
  ck(hipMemcpyAsync(st_, s.data(), sizeof(RingDevState) * nq_, hipMemcpyHostToDevice, stream_), "state upload");
  // both table sets into the grid's HBM copies (the host's are current: stage_tables wrote them)
  ck(hipMemcpyAsync(dd_sets_, h_sets_, 2 * sizeof(RingTableSet), hipMemcpyHostToDevice, stream_), "table sets upload");
  ck(hipStreamSynchronize(stream_), "state upload");  // `s` lives on this stack frame
  RingLaunch r;
  r.f = f;
  r.sets = dd_sets_;
  r.lds_tiles = lds_tiles_;
  r.epoch0 = ep;
  {
    // entries posted but not applied by a previous session are dropped: the relaunch stages the
    // host's tables, which hold them already
    std::lock_guard<std::mutex> gc(ctrl_mu_);
    __atomic_store_n(&ctrl_->done, ctrl_head_, __ATOMIC_RELEASE);
    void* dc = nullptr;
    ck(hipHostGetDevicePointer(&dc, ctrl_, 0), "device ptr ctrl");
    r.ctrl = reinterpret_cast<RingCtrlRing*>(dc);
  }
  r.pkts = d_in_; r.inmeta = d_im_; r.out = d_out_; r.out_meta = d_meta_;
  r.faddr = faddr_on_ ? d_faddr_ : nullptr;
  r.ring_mask = cap_ - 1;
  r.queues = nq_;
  void* dctl = nullptr;
  void* dflags = nullptr;
  ck(hipHostGetDevicePointer(&dctl, ctl_, 0), "device ptr ctl");
  ck(hipHostGetDevicePointer(&dflags, flags_, 0), "device ptr flags");
  r.ctl = reinterpret_cast<RingCtl*>(dctl);
  r.flags = reinterpret_cast<uint32_t*>(dflags);
  r.st = st_;
  r.svc = d_svc_;
  r.deadline_ticks = (unsigned long long)(deadline_s * 1e8);  // s_memrealtime: 100 MHz
  r.flows_alt = flows_alt;
  r.gde = d_gde_;
  xfer_active_ = false;
  if (d_xin_ && d_xpeers_ && !v6_keys(f.t)) {   // (IPv6 tables: the V6 instances, hand-offs run in place)
    // the inbox as the previous session left it: peers may already be sending again, so nothing is
    // reset - the tickets restart at the first entry not yet consumed (the consumer counts the
    // consumed ones of that chunk as done by their seq)
    XferInbox h{};
    ck(hipMemcpyAsync(&h, d_xin_, sizeof(h), hipMemcpyDeviceToHost, stream_), "xfer inbox");
    ck(hipStreamSynchronize(stream_), "xfer inbox");
    uint64_t first = h.tail;
    if (h.tail) {
      const uint64_t lo = h.tail > xcap_ ? h.tail - xcap_ : 0;
      std::vector<XferEntry> ents(xcap_);
      ck(hipMemcpyAsync(ents.data(), d_xent_, (size_t)xcap_ * sizeof(XferEntry), hipMemcpyDeviceToHost, stream_),
         "xfer entries");
      ck(hipStreamSynchronize(stream_), "xfer entries");
      for (uint64_t i = lo; i < h.tail; ++i)
        if (ents[i & (xcap_ - 1)].seq != ((i + 1) | kXferDone)) { first = i; break; }
    }
    const uint64_t claim = first / 64;
    ck(hipMemcpyAsync(reinterpret_cast<uint8_t*>(d_xin_) + offsetof(XferInbox, claim), &claim, 8, hipMemcpyHostToDevice,
                      stream_), "xfer claim");
    ck(hipStreamSynchronize(stream_), "xfer claim");
    r.xpeers = d_xpeers_;
    r.xpeers_h = h_xpeers_.data();
    r.xplane = xplane_;
    r.nplanes = nplanes_;
    r.xfer_wgs = xwgs_;
    r.xpend = d_xpend_;
    std::memset(h_xpend_, 0, (size_t)nq_ * nch_ * 4);   // (chunk pending counts are added to: a new session starts at 0)
    xfer_active_ = true;
  }
  g_ring_why = "";
  const hipError_t le = launch_ring(r, cfg, wgs_, coop_, stream_);
  if (le != hipSuccess) throw std::runtime_error(std::string("ring: launch: ") + hipGetErrorString(le) +
                                                 (*g_ring_why ? std::string(" (") + g_ring_why + ")" : std::string()));
  set_running(true);
}

// ---- GPU-direct egress table -------------------------------------------------------------------
void RingEngine::gde_enable(bool on) {
  if (running_) throw std::runtime_error("ring: gde_enable while running");
  if (!on) {
    if (d_gde_) (void)hipFree(d_gde_);
    d_gde_ = nullptr;
    return;
  }
  if (d_gde_) return;
  const size_t bytes = sizeof(GdeRing) * (size_t)kMaxPorts * nq_;
  ck(hipMalloc(reinterpret_cast<void**>(&d_gde_), bytes), "alloc gde table");
  ck(hipMemset(d_gde_, 0, bytes), "memset gde table");
  ck(hipDeviceSynchronize(), "gde table");
}

uint64_t RingEngine::gde_write(uint32_t port, uint32_t q, const GdeRing& e) {
  if (!d_gde_) throw std::runtime_error("ring: GPU-direct egress is off");
  if (port >= (uint32_t)kMaxPorts || q >= nq_) throw std::invalid_argument("ring: gde entry out of range");
  GdeRing* dst = d_gde_ + (size_t)port * nq_ + q;
  if (!running_) {
    ck(hipMemcpy(dst, &e, sizeof(GdeRing), hipMemcpyHostToDevice), "gde entry");
    return 0;
  }
  // running: through the control mailbox, the entry's words first and its valid word last (a wave
  // never sees a valid entry with stale addresses); the grid's LDS copies do not hold it
  uint32_t w[16];
  std::memcpy(w, &e, sizeof(w));
  const uint64_t dev = reinterpret_cast<uint64_t>(dst);
  uint64_t seq = 0;
  if (e.valid) seq = post_ctrl(dev, w, 10, 1.0, false);
  return std::max(seq, post_ctrl(dev + 40, &w[10], 1, 1.0, false));
}

uint64_t RingEngine::gde_set(uint32_t port, uint32_t q, uint64_t ctl, uint64_t desc, uint64_t buf, uint32_t ring_size,
                             uint32_t buf_size, uint32_t head, uint32_t tail) {
  if (ring_size < 2 || (ring_size & (ring_size - 1)) || buf_size < 64 || !ctl || !desc || !buf)
    throw std::invalid_argument("ring: bad gde ring");
  GdeRing e{};
  e.ctl = ctl; e.desc = desc; e.buf = buf;
  e.mask = ring_size - 1; e.buf_size = buf_size; e.head = head; e.tail_cache = tail; e.valid = 1;
  return gde_write(port, q, e);
}

std::vector<uint64_t> RingEngine::gde_stats() {
  if (running_) throw std::runtime_error("ring: gde_stats while running");
  std::vector<RingDevState> s(nq_);
  ck(hipMemcpy(s.data(), st_, sizeof(RingDevState) * nq_, hipMemcpyDeviceToHost), "gde stats");
  std::vector<uint64_t> v;
  for (const auto& x : s) {
    v.push_back(x.gde_wait); v.push_back(x.gde_sect); v.push_back(x.gde_chunks); v.push_back(x.gde_frames);
    v.push_back(x.gde_full);
  }
  return v;
}

// ---- SFC hops across GPUs (ring.h XferEntry) -----------------------------------------------------
void RingEngine::xfer_enable(uint32_t entries, uint32_t wgs) {
  if (running_) throw std::runtime_error("ring: xfer_enable while running");
  for (void* d : {(void*)d_xin_, (void*)d_xent_, (void*)d_xpeers_}) (void)hipFree(d);
  if (h_xpend_) (void)hipHostFree(h_xpend_);
  d_xin_ = nullptr; d_xent_ = nullptr; d_xpeers_ = nullptr; h_xpend_ = d_xpend_ = nullptr;
  xcap_ = xwgs_ = nplanes_ = 0;
  if (!entries) return;
  if (entries < 64 || (entries & (entries - 1)) || entries > (1u << 22))
    throw std::invalid_argument("ring: inbox entries must be a power of two in [64, 2^22]");
  if (wgs < 1 || (uint64_t)num_cus_ * wgs_ < (uint64_t)nq_ + wgs)
    throw std::invalid_argument("ring: inbox workgroups leave a queue without a workgroup");
  ck(hipMalloc(reinterpret_cast<void**>(&d_xin_), sizeof(XferInbox)), "alloc inbox");
  ck(hipMalloc(reinterpret_cast<void**>(&d_xent_), (size_t)entries * sizeof(XferEntry)), "alloc inbox entries");
  ck(hipMemset(d_xin_, 0, sizeof(XferInbox)), "memset inbox");
  ck(hipMemset(d_xent_, 0, (size_t)entries * sizeof(XferEntry)), "memset inbox entries");
  ck(hipHostMalloc(reinterpret_cast<void**>(&h_xpend_), (size_t)nq_ * nch_ * 4,
                   hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable), "host alloc xpend");
  std::memset(h_xpend_, 0, (size_t)nq_ * nch_ * 4);
  ck(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_xpend_), h_xpend_, 0), "device ptr xpend");
  xcap_ = entries;
  xwgs_ = wgs;
}

RingEngine::XferDesc RingEngine::xfer_desc() const {
  if (!d_xin_) throw std::runtime_error("ring: cross-GPU hops are off (xfer_enable)");
  XferDesc d;
  d.inbox = reinterpret_cast<uint64_t>(d_xin_);
  d.entries = reinterpret_cast<uint64_t>(d_xent_);
  // the out slots / metas / pending words as any GPU reaches them (pinned host memory: one address
  // for every agent; HBM slots: this device's, reached over xGMI with peer access)
  d.out = reinterpret_cast<uint64_t>(host_slots_ ? host_ptrs_[2] : (void*)d_out_);
  d.out_meta = reinterpret_cast<uint64_t>(host_slots_ ? host_ptrs_[3] : (void*)d_meta_);
  d.xpend = reinterpret_cast<uint64_t>(h_xpend_);
  d.cap = xcap_;
  d.ring_mask = cap_ - 1;
  d.nq = nq_;
  return d;
}

void RingEngine::xfer_set_peers(uint32_t my_plane, const std::vector<XferDesc>& planes) {
  if (running_) throw std::runtime_error("ring: xfer_set_peers while running");
  if (!d_xin_) throw std::runtime_error("ring: cross-GPU hops are off (xfer_enable)");
  if (planes.empty() || planes.size() > kMaxXferPlanes || my_plane >= planes.size())
    throw std::invalid_argument("ring: 1..16 planes, this one among them");
  std::vector<XferPeer> v(planes.size());
  for (size_t k = 0; k < planes.size(); ++k) {
    const XferDesc& d = planes[k];
    if (!d.inbox || !d.entries || !d.out || !d.out_meta || !d.xpend || d.cap < 64 || (d.cap & (d.cap - 1)) ||
        d.ring_mask < 63 || ((d.ring_mask + 1) & d.ring_mask) || d.nq < 1)
      throw std::invalid_argument("ring: bad plane descriptor");
    v[k] = XferPeer{reinterpret_cast<XferInbox*>(d.inbox), reinterpret_cast<XferEntry*>(d.entries), d.cap - 1,
                    d.ring_mask, reinterpret_cast<uint4*>(d.out), reinterpret_cast<uint32_t*>(d.out_meta),
                    reinterpret_cast<uint32_t*>(d.xpend), d.nq, 0u};
  }
  if (planes[my_plane].inbox != reinterpret_cast<uint64_t>(d_xin_))
    throw std::invalid_argument("ring: my_plane's descriptor is not this ring's");
  if (d_xpeers_) (void)hipFree(d_xpeers_);
  d_xpeers_ = nullptr;
  ck(hipMalloc(reinterpret_cast<void**>(&d_xpeers_), sizeof(XferPeer) * v.size()), "alloc peers");
  ck(hipMemcpy(d_xpeers_, v.data(), sizeof(XferPeer) * v.size(), hipMemcpyHostToDevice), "peers");
  h_xpeers_ = v;
  xplane_ = my_plane;
  nplanes_ = (uint32_t)v.size();
}

std::vector<uint64_t> RingEngine::xfer_stats() {
  if (running_) throw std::runtime_error("ring: xfer_stats while running");
  if (!d_xin_) return {};
  XferInbox h{};
  ck(hipMemcpy(&h, d_xin_, sizeof(h), hipMemcpyDeviceToHost), "inbox stats");
  return {h.tail, h.claim, h.t_wait, h.t_work, h.n_timed, h.t_load, h.t_stage, h.t_wb};
}

uint64_t RingEngine::gde_clear(uint32_t port, uint32_t q) {
  GdeRing e{};
  return gde_write(port, q, e);
}

// ---- host memory mapped for the grids (zero-copy rx) --------------------------------------------
// hipHostUnregister waits for the device, which a resident grid never lets go idle: an unmap that
// comes while any ring of this process runs waits here (memory still mapped and pinned) until the
// last ring stops.
namespace {
std::mutex g_grid_mu;
int g_grids = 0;   // (g_grid_mu) rings running in this process
std::vector<std::pair<void*, std::function<void()>>> g_unmaps;   // (g_grid_mu) deferred
void drain_unmaps(std::vector<std::pair<void*, std::function<void()>>>& v) {
  for (auto& u : v) {
    (void)hipHostUnregister(u.first);
    (void)hipGetLastError();
    if (u.second) u.second();
  }
  v.clear();
}
}  // namespace

size_t deferred_host_unmaps() {
  std::lock_guard<std::mutex> g(g_grid_mu);
  return g_unmaps.size();
}

void host_unregister_when_idle(void* p, std::function<void()> after) {
  std::vector<std::pair<void*, std::function<void()>>> now;
  {
    std::lock_guard<std::mutex> g(g_grid_mu);
    g_unmaps.emplace_back(p, std::move(after));
    if (g_grids == 0) now.swap(g_unmaps);
  }
  drain_unmaps(now);
}

void RingEngine::set_running(bool on) {
  if (on == running_) return;
  running_ = on;
  std::vector<std::pair<void*, std::function<void()>>> now;
  {
    std::lock_guard<std::mutex> g(g_grid_mu);
    g_grids += on ? 1 : -1;
    if (g_grids == 0) now.swap(g_unmaps);
  }
  drain_unmaps(now);
}

void RingEngine::stop(double timeout_s) {
  if (!running_) return;
  {
    std::lock_guard<std::mutex> g(mu_);
    const uint32_t ep = epoch();
    for (uint32_t q = 0; q < nq_; ++q) {
      std::lock_guard<std::mutex> gq(qs_[q].mu);
      __atomic_store_n(&ctl_[q].prod, ring_word(qs_[q].prod, ep) | kRingStop, __ATOMIC_RELEASE);
    }
  }
  const auto t0 = Clock::now();
  for (;;) {
    const hipError_t q = hipStreamQuery(stream_);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) { set_running(false); ck(q, "kernel"); }
    if (secs(t0, Clock::now()) > timeout_s) throw std::runtime_error("ring: kernel did not drain before the timeout");
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  release_streams();
  set_running(false);   // (after the stream is gone: a deferred unmap may run now)
  for (uint32_t q = 0; q < nq_; ++q)
    if (completed(q) != published(q)) throw std::runtime_error("ring: stopped with published chunks unprocessed");
}

// The resident grid's stream.  NFDP_RING_STREAM picks how it is made: "prio" (highest priority,
// the default) or "plain" (an ordinary non-blocking stream).  A resident grid holds the hardware
// queue its stream maps to, and HIP maps ordinary streams round-robin onto GPU_MAX_HW_QUEUES (4)
// queues: with enough streams made before it, a ring's stream shares the queue of the default
// stream, and a harvest or copy issued there waits behind the grid forever (r6: the GPU suite hung
// in test_port_placement_hop_pipeline's harvest after the earlier tests' streams; with the ring
// streams at the highest priority - their own queue pool - it passes: profiles/r6_s18).  The
// 1 kHz live-commit p99 is the same either way (profiles/r5_s3_live_commit_hwq_ab.txt); a
// CU-masked stream (hipExtStreamCreateWithCUMask) failed that test and is not offered.
void RingEngine::create_stream() {
  const char* m = std::getenv("NFDP_RING_STREAM");
  if (!(m && std::string(m) == "plain")) {
    int lo = 0, hi = 0;
    ck(hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priorities");
    ck(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi), "stream (priority)");
  } else {
    ck(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "stream");
  }
}

void RingEngine::release_streams() {
  if (stream_) {
    (void)hipStreamSynchronize(stream_);
    (void)hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
}

bool RingEngine::chunk_done(uint64_t chunk, uint32_t q) const {
  const size_t w = (size_t)q * nch_ + (chunk & (nch_ - 1));
  if (__atomic_load_n(&flags_[w], __ATOMIC_ACQUIRE) != (uint32_t)(chunk + 1)) return false;
  // split chains across planes: the chunk's handed-off frames are back (the count was stored
  // before the flag, and each resumer subtracts after its slot stores)
  return !h_xpend_ || __atomic_load_n(&h_xpend_[w], __ATOMIC_ACQUIRE) == 0u;
}

uint64_t RingEngine::completed(uint32_t q) {
  Queue& Q = qs_[q];
  std::lock_guard<std::mutex> g(Q.mu);
  const uint64_t end = Q.prod / 64;
  // A producer reuses a chunk's slots (and its flag word) only once that chunk is done, so every
  // chunk more than a ring behind the newest published one is done, and a flag word holding a
  // LATER chunk's number means its earlier chunk completed.  Producers that track room
  // themselves (the native I/O engine: publish(.., check_room = false)) never advance the floor;
  // without these two rules it would stall more than a ring behind and never catch up.
  if (Q.floor + nch_ < end) Q.floor = end - nch_;
  while (Q.floor < end) {
    const size_t w = (size_t)q * nch_ + (Q.floor & (nch_ - 1));
    const uint32_t v = __atomic_load_n(&flags_[w], __ATOMIC_ACQUIRE);
    if ((int32_t)(v - (uint32_t)(Q.floor + 1)) < 0) break;
    if (v == (uint32_t)(Q.floor + 1) && h_xpend_ && __atomic_load_n(&h_xpend_[w], __ATOMIC_ACQUIRE) != 0u) break;
    ++Q.floor;
  }
  return Q.floor * 64;
}

uint64_t RingEngine::publish(uint32_t n, bool check_room, uint32_t q) {
  if (!running_) throw std::runtime_error("ring: not running");
  if (n == 0 || (n & 63u)) throw std::invalid_argument("ring: publish a positive multiple of 64 packets");
  if (q >= nq_) throw std::invalid_argument("ring: no such queue");
  // check_room = false: the producer tracks slot reuse itself (the native I/O engine frees slots
  // only after it has read their results, a stricter bound than completion)
  const uint64_t done = check_room ? completed(q) : 0;   // (also keeps the in-order floor current)
  Queue& Q = qs_[q];
  std::lock_guard<std::mutex> g(Q.mu);
  if (check_room && Q.prod + n - done > cap_) throw std::runtime_error("ring: no room (wait for completions)");
  Q.prod += n;
  __atomic_store_n(&ctl_[q].prod, ring_word(Q.prod, epoch()), __ATOMIC_RELEASE);
  return Q.prod;
}

bool RingEngine::grace_over() {
  for (uint32_t q = 0; q < nq_; ++q) {
    uint64_t fp;
    {
      std::lock_guard<std::mutex> g(qs_[q].mu);
      fp = qs_[q].flip_prod;
    }
    if (completed(q) < fp) return false;
  }
  return true;
}

void RingEngine::pace_epoch_change() {
  // (mu_ held) at most kEpochGenMask changes within kEpochAliasHostUs: the value a wave saw
  // cannot come round again before its idle-time invalidation (ring_kernel) takes over
  const auto now = Clock::now();
  if (epoch_changes_.size() >= kEpochGenMask) {
    const auto ready = epoch_changes_.front() + std::chrono::microseconds(kEpochAliasHostUs);
    while (Clock::now() < ready) _mm_pause();
    epoch_changes_.pop_front();
  }
  epoch_changes_.push_back(now > Clock::now() ? now : Clock::now());
}

void RingEngine::set_epoch_all(uint32_t e) {
  epoch_.store(e, std::memory_order_release);
  for (uint32_t q = 0; q < nq_; ++q) {
    Queue& Q = qs_[q];
    std::lock_guard<std::mutex> g(Q.mu);
    Q.flip_prod = Q.prod;
    // same count, new epoch: chunks published from here on carry it (the frontier mirrors a word
    // only when its count grows, so this store alone changes nothing for waiting waves)
    if (running_) __atomic_store_n(&ctl_[q].prod, ring_word(Q.prod, e), __ATOMIC_RELEASE);
  }
}

uint32_t RingEngine::change_epoch(bool flow, bool set) {
  if (set && !coop_) throw std::runtime_error("ring: live table sets need a coop ring");
  if (!grace_over()) throw std::runtime_error("ring: flip before the previous flip's grace period ended");
  std::lock_guard<std::mutex> g(mu_);
  pace_epoch_change();
  uint32_t e = epoch_next_gen(epoch());
  if (flow) e ^= kEpochFlowBit;
  if (set) e ^= kEpochSetBit;
  set_epoch_all(e);
  return e;
}

uint32_t RingEngine::bump_epoch() {
  std::lock_guard<std::mutex> g(mu_);
  pace_epoch_change();
  // same copies: only the generation moves, so the flip points (grace periods) stay as they are
  const uint32_t e = epoch_next_gen(epoch());
  epoch_.store(e, std::memory_order_release);
  for (uint32_t q = 0; q < nq_; ++q) {
    std::lock_guard<std::mutex> gq(qs_[q].mu);
    if (running_) __atomic_store_n(&ctl_[q].prod, ring_word(qs_[q].prod, e), __ATOMIC_RELEASE);
  }
  return e;
}

void RingEngine::stage_tables(const FusedLaunch& f, int which) {
  if (which < 0 || which > 1) throw std::invalid_argument("ring: table set 0 or 1");
  // (the LDS layout of a coop grid holds kLdsAclTiles rule tiles: any set fits, tiles beyond them
  // are read from the set's global copy by the kernel as usual)
  RingTableSet ts{};
  ts.t = f.t;
  ts.acl_wfrag = f.acl_wfrag; ts.acl_cinit = f.acl_cinit; ts.acl_tiles = f.acl_tiles;
  ts.toep_frag = f.toep_frag; ts.toep_tab = f.toep_tab;
  std::lock_guard<std::mutex> g(mu_);
  ts.serial = ++set_serial_;
  // the idle set (the grid never reads it until an epoch names it; the epoch word's release store
  // orders this store before it)
  std::memcpy(static_cast<void*>(h_sets_ + which), &ts, sizeof(ts));
  std::atomic_thread_fence(std::memory_order_release);
  if (running_) {
    // the set itself into the grid's HBM copy, then the serial's device mirror, through the
    // running grid's control mailbox (no stream: a stream may share a resident grid's hardware
    // queue), before any flip can name this set.  The grid applies the entries in order and
    // releases them before it reports them done; the flip comes after that.
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&ts);
    const uint32_t nw = sizeof(RingTableSet) / 4;
    const uint64_t dst = reinterpret_cast<uint64_t>(dd_sets_ + which);
    for (uint32_t o = 0; o < nw; o += kCtrlWords)
      (void)post_ctrl(dst + 4ull * o, w + o, std::min<uint32_t>(kCtrlWords, nw - o), 1.0, false);
    const uint64_t seq = post_ctrl(reinterpret_cast<uint64_t>(&st_[0].set_serial[which]), &ts.serial, 1, 1.0, false);
    if (!wait_ctrl(seq, 1.0)) throw std::runtime_error("ring: table set not applied by the grid");
  }
  if (running_) {
    // the side pass (RingPath.side_pass) reads the session's tables from launch()
    launch_.t = f.t;
    launch_.acl_wfrag = f.acl_wfrag; launch_.acl_cinit = f.acl_cinit; launch_.acl_tiles = f.acl_tiles;
    launch_.toep_frag = f.toep_frag; launch_.toep_tab = f.toep_tab;
  }
}

bool RingEngine::wait_grace(double timeout_s) {
  const auto t0 = Clock::now();
  uint32_t spin = 0;
  while (!grace_over()) {
    _mm_pause();
    if ((++spin & 1023u) == 0 && secs(t0, Clock::now()) > timeout_s) return false;
  }
  return true;
}

void RingEngine::set_epoch(uint32_t e) {
  if (running_) throw std::runtime_error("ring: set_epoch while running");
  std::lock_guard<std::mutex> g(mu_);
  set_epoch_all(e & (uint32_t)kRingEpochMask);
}

void RingEngine::set_frame_addrs(bool on) {
  if (running_) throw std::runtime_error("ring: set_frame_addrs while running");
  if (on && !host_slots_) throw std::invalid_argument("ring: frame addresses need host_slots=True");
  if (on && !faddr_on_) {   // every slot starts out naming its own in slot
    const size_t slots = (size_t)cap_ * nq_;
    for (size_t i = 0; i < slots; ++i) h_faddr_[i] = reinterpret_cast<uint64_t>(d_in_) + i * 64u;
  }
  faddr_on_ = on;
}

uint64_t RingEngine::post_write(uint64_t dst, const uint32_t* data, uint32_t n, double timeout_s) {
  if (n == 0 || n > kCtrlWords) throw std::invalid_argument("ring: a control write is 1..12 dwords");
  if (dst == 0 || (dst & 3u)) throw std::invalid_argument("ring: control write to a null / unaligned address");
  bool ok = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (const auto& r : ctrl_regions_)
      ok = ok || (dst >= r.first && dst + 4ull * n <= r.first + r.second);
  }
  if (!ok) throw std::invalid_argument("ring: control write outside the registered table buffers");
  return post_ctrl(dst, data, n, timeout_s);
}

uint64_t RingEngine::post_ctrl(uint64_t dst, const uint32_t* data, uint32_t n, double timeout_s, bool restage) {
  if (!running_) throw std::runtime_error("ring: control write with no grid running");
  std::lock_guard<std::mutex> g(ctrl_mu_);
  const auto t0 = Clock::now();
  while (ctrl_head_ - __atomic_load_n(&ctrl_->done, __ATOMIC_ACQUIRE) >= kCtrlSlots) {   // mailbox full
    if (secs(t0, Clock::now()) > timeout_s || !alive()) throw std::runtime_error("ring: control mailbox not drained");
    _mm_pause();
  }
  RingCtrlEntry& e = ctrl_->e[ctrl_head_ % kCtrlSlots];
  e.dst = dst;
  e.nwords = n | (restage ? 0u : kCtrlNoRestage);
  std::memcpy(e.data, data, 4ull * n);
  __atomic_store_n(&e.seq, (uint32_t)(ctrl_head_ + 1), __ATOMIC_RELEASE);
  ++ctrl_head_;
  __atomic_store_n(&ctrl_->head, ctrl_head_, __ATOMIC_RELEASE);
  return ctrl_head_;
}

uint64_t RingEngine::ctrl_done() const { return __atomic_load_n(&ctrl_->done, __ATOMIC_ACQUIRE); }

bool RingEngine::wait_ctrl(uint64_t seq, double timeout_s) {
  const auto t0 = Clock::now();
  uint32_t spin = 0;
  while (ctrl_done() < seq) {
    _mm_pause();
    if ((++spin & 1023u) == 0 && (secs(t0, Clock::now()) > timeout_s || !alive())) return ctrl_done() >= seq;
  }
  return true;
}

void RingEngine::set_ctrl_regions(const std::vector<std::pair<uint64_t, uint64_t>>& regions) {
  std::lock_guard<std::mutex> g(mu_);
  ctrl_regions_ = regions;
}

bool RingEngine::wait(uint64_t end, double timeout_s, uint32_t q) {
  if (end > published(q)) throw std::invalid_argument("ring: waiting for unpublished packets");
  const auto t0 = Clock::now();
  uint32_t spin = 0;
  while (completed(q) < end) {
    _mm_pause();
    if ((++spin & 1023u) == 0 && secs(t0, Clock::now()) > timeout_s) return false;
  }
  return true;
}

std::vector<double> RingEngine::probe(uint32_t batches, uint32_t batch, uint32_t inflight, double* elapsed_s) {
  if (!running_) throw std::runtime_error("ring: not running");
  if (batch == 0 || (batch & 63u) || inflight == 0 || (uint64_t)batch * inflight > cap_)
    throw std::invalid_argument("ring: probe needs batch % 64 == 0 and batch * inflight <= capacity");
  std::vector<double> lat;
  lat.reserve(batches);
  std::vector<Clock::time_point> t_pub(inflight);
  std::vector<uint64_t> end(inflight);
  uint32_t issued = 0, done = 0;
  const auto t_start = Clock::now();
  while (done < batches) {
    while (issued < batches && issued - done < inflight) {
      const uint32_t k = issued % inflight;
      t_pub[k] = Clock::now();
      end[k] = publish(batch);
      ++issued;
    }
    const uint32_t k = done % inflight;  // batches complete in publication order (floor scan)
    uint32_t spin = 0;
    while (completed() < end[k]) {
      _mm_pause();
      if ((++spin & 0xFFFFu) == 0 && secs(t_start, Clock::now()) > 60.0)
        throw std::runtime_error("ring: probe timed out waiting for completions");
    }
    lat.push_back(std::chrono::duration<double, std::micro>(Clock::now() - t_pub[k]).count());
    ++done;
  }
  if (elapsed_s) *elapsed_s = secs(t_start, Clock::now());
  return lat;
}

}  // namespace nfdp
