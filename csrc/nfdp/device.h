// device.h — device-side building blocks shared by the fused (1-GPU) and sharded (N-GPU)
// kernels: MFMA classification over the bit-expanded FlowKey, vectorized flow-table probe.
#pragma once
#include "host.h"

namespace nfdp {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kBlock = 512;
constexpr int kWaves = kBlock / 64;
constexpr int kLdsPorts = 256;

enum HashMode { kHashScalar = 0, kHashLds = 1, kHashMfma = 2 };
enum AclMode { kAclScalar = 0, kAclMfma = 1, kAclOff = 2 };

// 16 bits -> 16 bytes of {0,1}: byte j = bit j.  (nibble * 0x00204081) spreads 4 bits to 4
// bytes without carries.
__device__ __forceinline__ v4i expand16(uint32_t x) {
  v4i r;
  r[0] = (int)((((x) & 0xFu) * 0x00204081u) & 0x01010101u);
  r[1] = (int)((((x >> 4) & 0xFu) * 0x00204081u) & 0x01010101u);
  r[2] = (int)((((x >> 8) & 0xFu) * 0x00204081u) & 0x01010101u);
  r[3] = (int)((((x >> 12) & 0xFu) * 0x00204081u) & 0x01010101u);
  return r;
}

__device__ __forceinline__ uint32_t pick4(uint32_t g, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return g == 0 ? a : g == 1 ? b : g == 2 ? c : d;
}

// Wave-level classification over the wave's 64 packets (one per lane).  EXEC must be full.
template <int HASH, int ACL>
__device__ __forceinline__ void classify_wave(const FlowKey& key, uint4* kx, const v4i* lw,
                                              const v4i* lc, uint32_t acl_tiles, const v4i* lt,
                                              const uint32_t* ltab, const TablesView& t,
                                              uint32_t& hash, int& acl_rule) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 4, col = lane & 15u;
  v4i bf[4][2];
  if constexpr (HASH == kHashMfma || ACL == kAclMfma) {
    kx[lane] = make_uint4(key.src_ip, key.dst_ip, key.ports, key.meta);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(kx + 16 * tt + col);
      const uint32_t wlo = src[g >> 1], whi = src[2 + (g >> 1)];
      const uint32_t sh = 16u * (g & 1u);
      bf[tt][0] = expand16((wlo >> sh) & 0xFFFFu);
      bf[tt][1] = expand16((whi >> sh) & 0xFFFFu);
    }
  }
  // ---- hash ----
  if constexpr (HASH == kHashMfma) {
    uint32_t hv[4] = {0, 0, 0, 0};
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const v4i a0 = lt[(m * 2 + 0) * 64 + lane], a1 = lt[(m * 2 + 1) * 64 + lane];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        v4i acc = {0, 0, 0, 0};
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf[tt][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf[tt][1], acc, 0, 0, 0);
        uint32_t bits = ((uint32_t)acc[0] & 1u) | (((uint32_t)acc[1] & 1u) << 1) |
                        (((uint32_t)acc[2] & 1u) << 2) | (((uint32_t)acc[3] & 1u) << 3);
        hv[tt] |= bits << (4u * g + 16u * m);
      }
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      hv[tt] |= __shfl_xor(hv[tt], 16);
      hv[tt] |= __shfl_xor(hv[tt], 32);
    }
    hash = __builtin_bitreverse32(pick4(g, hv[0], hv[1], hv[2], hv[3]));
  } else if constexpr (HASH == kHashLds) {
    const uint32_t w[4] = {key.src_ip, key.dst_ip, key.ports, key.meta};
    uint32_t h = 0;
#pragma unroll
    for (int b = 0; b < 16; ++b) h ^= ltab[b * 256 + ((w[b >> 2] >> (8 * (b & 3))) & 0xFFu)];
    hash = h;
  } else {
    hash = toeplitz_scalar(key, t.rss_key);
  }
  // ---- ACL (TCAM) ----
  if constexpr (ACL == kAclMfma) {
    uint32_t best[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    for (uint32_t nt = 0; nt < acl_tiles; ++nt) {
      const v4i a0 = lw[(nt * 2 + 0) * 64 + lane], a1 = lw[(nt * 2 + 1) * 64 + lane];
      const v4i c = lc[nt * 4 + g];
      // Pass 1: does ANY packet of the wave match ANY rule of this tile?  (mismatch counts are
      // >= 0, so a zero minimum = a match.)  Most tiles of a deny-list ACL match nothing, and
      // then the priority epilogue below — 10 VALU per 16 packets — is skipped wave-uniformly.
      uint32_t z = 0xFFFFFFFFu;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf[tt][0], c, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf[tt][1], acc, 0, 0, 0);
        z = min(z, min(min((uint32_t)acc[0], (uint32_t)acc[1]), min((uint32_t)acc[2], (uint32_t)acc[3])));
      }
      if (!__any(z == 0u)) continue;
      // Pass 2 (rare): recompute the tile with the (mismatch << 10 | rule) first-match epilogue.
      // The bias goes through an opaque copy so the MFMAs are not CSE'd with pass 1 (keeping
      // pass-1 accumulators alive would cost 16 VGPRs at the kernel's register peak).
      v4i c2 = c;
      asm volatile("" : "+v"(c2));
      const uint32_t rb = nt * 16u + 4u * g;
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        v4i acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a0, bf[tt][0], c2, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a1, bf[tt][1], acc, 0, 0, 0);
        const uint32_t e0 = ((uint32_t)acc[0] << 10) | (rb + 0);
        const uint32_t e1 = ((uint32_t)acc[1] << 10) | (rb + 1);
        const uint32_t e2 = ((uint32_t)acc[2] << 10) | (rb + 2);
        const uint32_t e3 = ((uint32_t)acc[3] << 10) | (rb + 3);
        best[tt] = min(best[tt], min(min(e0, e1), min(e2, e3)));
      }
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      best[tt] = min(best[tt], (uint32_t)__shfl_xor(best[tt], 16));
      best[tt] = min(best[tt], (uint32_t)__shfl_xor(best[tt], 32));
    }
    const uint32_t b = pick4(g, best[0], best[1], best[2], best[3]);
    acl_rule = (b >> 10) == 0 ? (int)(b & 1023u) : -1;
    if (acl_rule >= (int)t.n_acl) acl_rule = -1;
  } else if constexpr (ACL == kAclScalar) {
    acl_rule = acl_first_match(t, key);
  } else {
    acl_rule = -1;
  }
}

// 2-choice bucket probe.  A bucket is one 128-B line holding 4 x {key, action}; it is loaded
// whole (8 x dwordx4, one line, one trip) and the action comes with the key, so a hit in the
// first bucket costs a single dependent fetch.  The second bucket is touched only on a miss.
__device__ __forceinline__ int64_t flow_probe(const TablesView& t, const FlowKey& k, uint32_t h, uint4& act) {
  const TableHash th = table_hash(h, t.bucket_mask);
  const uint4* fl = reinterpret_cast<const uint4*>(t.flows);
  const uint32_t used = k.meta | kSlotUsed;
  static_assert(kBucketSlots == 4, "probe is written for 4-slot buckets");
  // Named registers, no private array: an indexed local array lands in scratch.
  auto eq = [&](const uint4& e) {
    return e.x == k.src_ip && e.y == k.dst_ip && e.z == k.ports && e.w == used;
  };
  uint32_t b = th.b1;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint4* row = fl + (size_t)b * (kBucketSlots * 2);
    const uint4 k0 = row[0], a0 = row[1], k1 = row[2], a1 = row[3];
    const uint4 k2 = row[4], a2 = row[5], k3 = row[6], a3 = row[7];
    const bool m0 = eq(k0), m1 = eq(k1), m2 = eq(k2), m3 = eq(k3);
    if (m0 | m1 | m2 | m3) {
      act = m0 ? a0 : m1 ? a1 : m2 ? a2 : a3;
      return (int64_t)b * kBucketSlots + (m0 ? 0 : m1 ? 1 : m2 ? 2 : 3);
    }
    b = th.b2;
  }
  return -1;
}

// ---- multi-GPU output segments (shared by the fused REMOTE variant and the sharded stages) ----
constexpr uint32_t kMaxRanks = 64;

// Block-aggregated slot reservation: waves claim offsets in LDS counters (one LDS atomic per
// wave and destination), then ONE global atomic per (workgroup iteration, destination) turns
// them into segment positions.  (A per-wave global atomic on one counter serialised 16K waves
// per 1M packets: 200 us of a 1M-packet ingress pass.)  Called by every thread of the block.
__device__ __forceinline__ uint32_t reserve_block(uint32_t* gcnt, uint32_t dest, bool active, uint32_t nranks,
                                                  uint32_t* lcnt, uint32_t* lbase) {
  const uint32_t lane = threadIdx.x & 63u;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  if (threadIdx.x < nranks) lcnt[threadIdx.x] = 0;
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t o = 0; o < nranks; ++o) {
    const unsigned long long m = __ballot(active && dest == o);
    if (m == 0) continue;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&lcnt[o], (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (active && dest == o) off = base + (uint32_t)__popcll(m & lt);
  }
  __syncthreads();
  if (threadIdx.x < nranks) {
    const uint32_t c = lcnt[threadIdx.x];
    lbase[threadIdx.x] = c ? atomicAdd(&gcnt[threadIdx.x], c) : 0u;
  }
  __syncthreads();
  return active ? lbase[dest] + off : 0xFFFFFFFFu;
}

}  // namespace nfdp
