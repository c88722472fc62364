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

// 8 bits -> 8 FP4 (e2m1) nibbles: bit i -> nibble i = 1.0 (0x2) or 0.0.  Shift-and-mask spread
// (a multiply spread would carry between overlapping copies at nibble pitch).
__device__ __forceinline__ uint32_t spread8_fp4(uint32_t n) {
  uint32_t x = (n | (n << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  return ((x << 1) | (x << 4)) & 0x22222222u;
}
typedef int v8i_t __attribute__((ext_vector_type(8)));
typedef float v4f_t __attribute__((ext_vector_type(4)));
constexpr int kE8M0One = 0x7F7F7F7F;  // block scales 2^0 (every byte)

// ACL (TCAM) rule tiles: 16 rules x 128 key bits per tile.  Up to kLdsAclTiles tiles are staged
// in LDS (A fragments + C init); tiles beyond that are read from the global copy (L2-resident)
// when their prefilter lets a wave through.  The global C-init buffer is followed by the
// per-tile prefilters [tiles][8] and the per-group (8 tiles) prefilters [groups][8] (host.cpp
// build_acl_frags).
constexpr uint32_t kLdsAclTiles = 64;
constexpr uint32_t kAclGroup = kAclGroupTiles;   // (host.h NFDP_ACL_GROUP)
constexpr uint32_t kAclIdxBits = 12;                      // rule index bits: up to 4096 rules
constexpr uint32_t kAclMaxRules = 1u << kAclIdxBits;
constexpr int kE8M0Idx = 0x8B8B8B8B;                      // block scales 2^12 = 2^kAclIdxBits
struct AclView {
  const v4i* lw; const v4i* lc;   // LDS: A fragments of the first ltiles tiles, C init of the first ctiles
  const v4i* gw; const v4i* gc;   // global: all tiles (+ prefilters after gc's tiles * 4 entries)
  uint32_t tiles;
  // tiles staged in LDS (A fragments: a multiple of kAclGroup or all of them; C init: ctiles >=
  // ltiles).  The fused kernel's one-block-per-CU instances stage more than kLdsAclTiles.
  uint32_t ltiles = tiles < kLdsAclTiles ? tiles : kLdsAclTiles;
  uint32_t ctiles = ltiles;
  // prefilter tiles in LDS (one-block-per-CU fused instances): tile t's prefilter is row t % 16 of
  // prefilter tile t / 16 (host.cpp build_acl_frags); ptiles 0: the scalar prefilter cursor
  const v4i* pw = nullptr; const v4i* pc = nullptr;
  uint32_t ptiles = 0;
};
NFDP_HD uint32_t acl_groups(uint32_t tiles) { return (tiles + kAclGroup - 1) / kAclGroup; }
// Raw first-match value (mismatch << 12 | rule) -> rule index or -1.
NFDP_HD int acl_rule_of(uint32_t b, uint32_t n_acl) {
  const int r = (b >> kAclIdxBits) == 0 ? (int)(b & (kAclMaxRules - 1)) : -1;
  return r >= (int)n_acl ? -1 : r;
}

// Wave-level classification over the wave's 64 packets (one per lane).  EXEC must be full.
// ACL (TCAM) on the gfx950 block-scaled FP4 MFMA: v_mfma_scale_f32_16x16x128_f8f6f4 with e2m1
// operands covers the whole 128-bit key in ONE instruction per 16 rules x 16 packets.  Rule
// weights {-1, 0, +1} and key bits {0, 1} are exact in e2m1; the A block scale 2^12 turns them
// into {-4096, 0, +4096} and the C init of rule r is bias_r * 4096 + r, so every accumulator IS
// (mismatch << 12) | r, exactly (|x| < 2^20 in f32).  First match = an integer min over the f32
// bit patterns (all values are >= 0): no second pass, and rules may sit in any tile in any
// order (the host groups similar rules).  Lane l holds K = 32 (l >> 4) + j, j < 32, i.e. bit j
// of key word l >> 4, as nibble j (tools/fp4_probe.hip pins the operand and C/D maps).
// Prefilter: a tile (and a group of 8 tiles) carries the bits ALL its rules care about and agree
// on; a wave skips it - no LDS reads, no MFMAs - unless one of its packets has those bits.
// The MFMA Toeplitz hash keeps the i8 form (it needs the parity of integer sums).
#ifndef NFDP_PIPE_PF
#define NFDP_PIPE_PF 1   // r3 s15 A/B: tile prefilters cost the ClassBench set 41 % (1.95 vs 1.38 ms)
#endif
#ifndef NFDP_ACL_LOOKAHEAD
#define NFDP_ACL_LOOKAHEAD 1   // r4 s25 A/B: ClassBench-style set +5.5 % (7.17 -> 7.56 Gpps) over no lookahead
// (r5: tile MFMAs ping-ponged between two accumulator sets, tile k's minima under tile k+1's
// MFMAs: ClassBench set 7.84 vs 7.92 Gpps without, profiles/r5_s6_ab_acl_pingpong.jsonl - not kept)
#endif
#ifndef NFDP_ACL_PTILES
// prefilter tiles: 16 tiles' prefilters tested by one MFMA per 16 packets, only admitted tiles run.
// r5 s11 A/B on the ClassBench-style set: 7.16 vs 7.71 Gpps without (profiles/r5_s11_ab_ptiles.jsonl):
// half the tile MFMAs, but the per-tile loop loses the straight-line 8-tile groups' overlap, and
// the 2-wave instance is bound by latency, not by its MFMA count.  Off.
// r6 (profiles/r6_s20_acl_ab_wild.jsonl, r6_s21_acl_ab_wild.jsonl): with the rules placed
// source-first (host.cpp NFDP_ACL_ORDER=1) 29 tiles per wave pass their prefilter instead of 37,
// and the prefilter tiles reach 8,060 Mpps against 8,002 for this default; 2 = one cursor over every
// prefilter tile's admitted tiles run in batches of 4 (7,217).  Still off.
#define NFDP_ACL_PTILES 0
#endif
#ifndef NFDP_TILE_PF
#define NFDP_TILE_PF 1   // 4-wave instances: per-tile prefilters inside a passing group (0: group only, A/B)
#endif
#ifndef NFDP_PIPE_UNROLL
#define NFDP_PIPE_UNROLL 1   // r3 s16 A/B: ACL1024 0.3145 vs 0.3211 ms, ClassBench unchanged
#endif
// Toeplitz LDS tables (HASH == kHashLds).  Byte tables: 16 x 256 words (16 KiB), one lookup per
// key byte at a random entry (bank conflicts: ~4-way for 64 random entries over 64 banks).
// NFDP_HASH_NIBBLE=1: 32 x 16 words (2 KiB), two lookups per byte, each table 16 consecutive
// words = 16 distinct banks, so a wave's 64 reads are conflict-free (equal addresses broadcast);
// derived from the byte tables at staging (Toeplitz is XOR-linear: T[v] = T[v & 0xF0] ^ T[v & 0xF]).
#ifndef NFDP_HASH_NIBBLE
#define NFDP_HASH_NIBBLE 0
#endif
constexpr uint32_t kToepLdsWords = NFDP_HASH_NIBBLE ? 32 * 16 : 16 * 256;
__device__ __forceinline__ void stage_toep(uint32_t* dst, const uint32_t* bytes, uint32_t tid, uint32_t nthr) {
  for (uint32_t i = tid; i < kToepLdsWords; i += nthr) {
    if (NFDP_HASH_NIBBLE) {
      const uint32_t pos = i >> 4, x = i & 15u, b = pos >> 1;
      dst[i] = bytes[b * 256 + ((pos & 1u) ? x : (x << 4))];
    } else {
      dst[i] = bytes[i];
    }
  }
}

struct NoHashHook {
  __device__ void operator()(uint32_t) const {}
};

template <int HASH, int ACL, class OnHash = NoHashHook, bool PIPE = false>
__device__ __forceinline__ void classify_wave(const FlowKey& key, uint4* kx, const AclView& av, const v4i* lt,
                                              const uint32_t* ltab, const TablesView& t,
                                              uint32_t& hash, int& acl_rule, uint32_t tile0 = 0,
                                              uint32_t tstep = 1, uint32_t* best_out = nullptr,
                                              OnHash on_hash = OnHash{}) {
  // on_hash(hash) runs between the hash and the ACL (e.g. to issue the flow-bucket fetch early)
  // tile0 / tstep: this wave scans rule tiles tile0, tile0 + tstep, ... (cooperating waves split
  // one chunk's ACL); best_out: the raw (mismatch << 12 | rule) minimum, for combining partials.
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane >> 4, col = lane & 15u;
  v4i bf[4][2];   // i8 B operands (MFMA hash)
  v4i bq[4];      // FP4 B operands (MFMA ACL)
  if constexpr (HASH == kHashMfma || ACL == kAclMfma) {
    // the ACL key's meta word (nfdp.h acl_key_meta) goes to the exchange directly unless the MFMA
    // hash reads the flow key from it too
    kx[lane] = make_uint4(key.src_ip, key.dst_ip, key.ports,
                          (ACL == kAclMfma && HASH != kHashMfma) ? acl_key_meta(key.ports, key.meta) : key.meta);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(kx + 16 * tt + col);
      if constexpr (HASH == kHashMfma) {
        const uint32_t wlo = src[g >> 1], whi = src[2 + (g >> 1)];
        const uint32_t sh = 16u * (g & 1u);
        bf[tt][0] = expand16((wlo >> sh) & 0xFFFFu);
        bf[tt][1] = expand16((whi >> sh) & 0xFFFFu);
      }
      if constexpr (ACL == kAclMfma) {
        uint32_t w = src[g];
        if constexpr (HASH == kHashMfma)
          if (g == 3) w = acl_key_meta(src[2], w);   // (the exchange holds the flow key's meta)
        bq[tt][0] = (int)spread8_fp4(w & 0xFFu);
        bq[tt][1] = (int)spread8_fp4((w >> 8) & 0xFFu);
        bq[tt][2] = (int)spread8_fp4((w >> 16) & 0xFFu);
        bq[tt][3] = (int)spread8_fp4(w >> 24);
      }
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
#if NFDP_HASH_NIBBLE
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const uint32_t v = w[b >> 2] >> (8 * (b & 3));
      h ^= ltab[(2 * b) * 16 + ((v >> 4) & 15u)] ^ ltab[(2 * b + 1) * 16 + (v & 15u)];
    }
#else
#pragma unroll
    for (int b = 0; b < 16; ++b) h ^= ltab[b * 256 + ((w[b >> 2] >> (8 * (b & 3))) & 0xFFu)];
#endif
    hash = h;
#ifdef NFDP_ABL_NO_HASH  // cost attribution only (wrong results): a two-instruction stand-in hash
    hash = (key.src_ip ^ key.ports) * 0x9E3779B1u;
#endif
  } else {
    hash = toeplitz_scalar(key, t.rss_key);
  }
  on_hash(hash);
  // ---- ACL (TCAM) ----
  if constexpr (ACL == kAclMfma) {
    uint32_t best[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
    // prefilters through the constant address space: wave-uniform s_load (lgkmcnt), so testing
    // one never waits for the frame prefetch in flight (vmcnt)
    typedef const __attribute__((address_space(4))) uint32_t* cu32;
    const cu32 pf = (cu32)(reinterpret_cast<const uint32_t*>(av.gc) + (size_t)av.tiles * 16);  // [tiles][8]
    const cu32 gpf = pf + (size_t)av.tiles * 8;                                                // [groups][8]
    auto pass = [&](cu32 f) {
      const uint32_t x = ((key.src_ip & f[0]) ^ f[4]) | ((key.dst_ip & f[1]) ^ f[5]) |
                         ((key.ports & f[2]) ^ f[6]) | ((key.meta & f[3]) ^ f[7]);   // (no port-class bits: host.cpp)
      return __any(x == 0u);
    };
    // tiles past the LDS copy: buffer loads (a distinct path the compiler cannot merge with the
    // ds_reads into FLAT loads)
    const __amdgpu_buffer_rsrc_t r_gw = __builtin_amdgcn_make_buffer_rsrc((void*)av.gw, (short)0,
                                                                         (int)(av.tiles * 1024u), 0x00020000);
    const __amdgpu_buffer_rsrc_t r_gc = __builtin_amdgcn_make_buffer_rsrc((void*)av.gc, (short)0,
                                                                         (int)(av.tiles * 64u), 0x00020000);
    auto run_tile = [&](const v4i& a4, const v4i& ci) {
      const v8i_t a = {a4[0], a4[1], a4[2], a4[3], 0, 0, 0, 0};
      const v4f_t c = {__int_as_float(ci[0]), __int_as_float(ci[1]), __int_as_float(ci[2]), __int_as_float(ci[3])};
      // four independent accumulators (one per 16-packet group) issue back to back
      v4f_t acc[4];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const v8i_t b = {bq[tt][0], bq[tt][1], bq[tt][2], bq[tt][3], 0, 0, 0, 0};
        acc[tt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, kE8M0Idx, 0, kE8M0One);
      }
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        if constexpr (PIPE) {   // (2-wave instances) two 3-input minima, the running minimum first
          const uint32_t m = min(min(best[tt], __float_as_uint(acc[tt][0])), __float_as_uint(acc[tt][1]));
          best[tt] = min(min(m, __float_as_uint(acc[tt][2])), __float_as_uint(acc[tt][3]));
        } else {   // (4-wave instances at the register cap: the form their allocation was tuned with)
          best[tt] = min(best[tt], min(min(__float_as_uint(acc[tt][0]), __float_as_uint(acc[tt][1])),
                                       min(__float_as_uint(acc[tt][2]), __float_as_uint(acc[tt][3]))));
        }
      }
    };
    // Straight-line form for batches (PIPE): the MFMAs always issue; `dead` (wave-uniform, all
    // ones for an empty batch slot) turns the tile's result into "no match".
    auto run_tile_m = [&](const v4i& a4, const v4i& ci, uint32_t dead) {
      const v8i_t a = {a4[0], a4[1], a4[2], a4[3], 0, 0, 0, 0};
      const v4f_t c = {__int_as_float(ci[0]), __int_as_float(ci[1]), __int_as_float(ci[2]), __int_as_float(ci[3])};
      v4f_t acc[4];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        const v8i_t b = {bq[tt][0], bq[tt][1], bq[tt][2], bq[tt][3], 0, 0, 0, 0};
        acc[tt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 4, 4, 0, kE8M0Idx, 0, kE8M0One);
      }
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) {
        best[tt] = min(best[tt], dead | min(min(__float_as_uint(acc[tt][0]), __float_as_uint(acc[tt][1])),
                                            min(__float_as_uint(acc[tt][2]), __float_as_uint(acc[tt][3]))));
      }
    };
    // Two phases so that the LDS-resident tiles never share a join point with global loads (the
    // wait there would be vmcnt(0): the frame prefetch in flight).  Groups of 8 tiles never
    // straddle ltiles (a multiple of 8 unless it covers every tile).
    const uint32_t ngroups = acl_groups(av.tiles);
    const uint32_t lds_groups = min(ngroups, (PIPE ? av.ltiles : kLdsAclTiles) / kAclGroup);
    // Prefilter tiles (PIPE instances, LDS): row j of prefilter tile p is tile 16 p + j's prefilter as
    // a ternary rule, so 4 MFMAs decide 16 tiles for the wave's 64 packets (accumulator < 4096: no
    // cared bit differs, the tile can match).  Only the admitted tiles run, straight from their
    // mask, one fragment ahead.  The scalar cursor below admits whole groups of 8 (per-tile scalar
    // tests cost more than they saved, r3 s15): on the ClassBench-style set 72 tiles per wave ran
    // where 37 can match (r5 s10 simulation).
    bool ptiles_done = false;
    if constexpr (PIPE && NFDP_ACL_PTILES) {
      if (av.ptiles && tstep == 1) {
        ptiles_done = true;
        auto ld_a = [&](uint32_t t) -> v4i {
          if (t < av.ltiles) return av.lw[t * 64 + lane];
          return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r_gw, (t * 64u + lane) * 16u, 0, 0));
        };
        auto ld_c = [&](uint32_t t) -> v4i {
          if (t < av.ctiles) return av.lc[t * 4 + g];
          return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r_gc, (t * 4u + g) * 16u, 0, 0));
        };
#if NFDP_ACL_PTILES == 2
        // one cursor over the admitted tiles of every prefilter tile (tested when the cursor reaches
        // it), run in batches of 4 with the next batch's fragments loading under the current
        // batch's MFMAs (two batches with fixed roles, as the global-tile path below)
        uint32_t pt_next = 0, mcur = 0, mbase = 0;
        constexpr uint32_t kDeadTile = 0xFFFFFFFFu;
        auto ptest = [&](uint32_t pt) -> uint32_t {
          const v4i pa4 = av.pw[pt * 64 + lane], pci = av.pc[pt * 4 + g];
          const v8i_t pa = {pa4[0], pa4[1], pa4[2], pa4[3], 0, 0, 0, 0};
          const v4f_t pc = {__int_as_float(pci[0]), __int_as_float(pci[1]), __int_as_float(pci[2]), __int_as_float(pci[3])};
          v4f_t pacc[4];
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const v8i_t b = {bq[tt][0], bq[tt][1], bq[tt][2], bq[tt][3], 0, 0, 0, 0};
            pacc[tt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(pa, b, pc, 4, 4, 0, kE8M0Idx, 0, kE8M0One);
          }
          uint32_t m = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float mn = fminf(fminf(pacc[0][i], pacc[1][i]), fminf(pacc[2][i], pacc[3][i]));
            const unsigned long long bl = __ballot(mn < 4096.0f);
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
              m |= (((bl >> (16 * gg)) & 0xFFFFull) != 0ull ? 1u : 0u) << (4 * gg + i);
          }
          if (pt * 16u + 16u > av.tiles) m &= (1u << (av.tiles - pt * 16u)) - 1u;
          return __builtin_amdgcn_readfirstlane(m);
        };
        auto next_tile = [&]() -> uint32_t {
          while (!mcur) {
            if (pt_next >= av.ptiles) return kDeadTile;
            mbase = pt_next * 16u;
            mcur = ptest(pt_next++);
          }
          const uint32_t t = mbase + (uint32_t)__builtin_ctz(mcur);
          mcur &= mcur - 1u;
          return t;
        };
        uint32_t b0[4], b1[4];
        v4i a0[4], a1[4], k0[4], k1[4];
        auto fill = [&](uint32_t (&c)[4], v4i (&aa)[4], v4i (&kk)[4]) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            c[k] = next_tile();
            const uint32_t t = c[k] == kDeadTile ? 0u : c[k];
            aa[k] = ld_a(t);
            kk[k] = ld_c(t);
          }
        };
        auto run4 = [&](const uint32_t (&c)[4], const v4i (&aa)[4], const v4i (&kk)[4]) {
#pragma unroll
          for (int k = 0; k < 4; ++k) run_tile_m(aa[k], kk[k], c[k] == kDeadTile ? 0xFFFFFFFFu : 0u);
        };
        fill(b0, a0, k0);
        while (b0[0] != kDeadTile) {
          fill(b1, a1, k1);
          run4(b0, a0, k0);
          if (b1[0] == kDeadTile) break;
          fill(b0, a0, k0);
          run4(b1, a1, k1);
        }
#else
        for (uint32_t pt = 0; pt < av.ptiles; ++pt) {
          const v4i pa4 = av.pw[pt * 64 + lane], pci = av.pc[pt * 4 + g];
          const v8i_t pa = {pa4[0], pa4[1], pa4[2], pa4[3], 0, 0, 0, 0};
          const v4f_t pc = {__int_as_float(pci[0]), __int_as_float(pci[1]), __int_as_float(pci[2]), __int_as_float(pci[3])};
          v4f_t pacc[4];
#pragma unroll
          for (int tt = 0; tt < 4; ++tt) {
            const v8i_t b = {bq[tt][0], bq[tt][1], bq[tt][2], bq[tt][3], 0, 0, 0, 0};
            pacc[tt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(pa, b, pc, 4, 4, 0, kE8M0Idx, 0, kE8M0One);
          }
          // lane l holds rows 4 (l >> 4) + i for packet column l & 15 of each 16-packet group tt
          uint32_t m16 = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float mn = fminf(fminf(pacc[0][i], pacc[1][i]), fminf(pacc[2][i], pacc[3][i]));
            const unsigned long long bl = __ballot(mn < 4096.0f);
#pragma unroll
            for (int gg = 0; gg < 4; ++gg)
              m16 |= (((bl >> (16 * gg)) & 0xFFFFull) != 0ull ? 1u : 0u) << (4 * gg + i);
          }
          const uint32_t base = pt * 16u;
          if (base + 16u > av.tiles) m16 &= (1u << (av.tiles - base)) - 1u;
          m16 = __builtin_amdgcn_readfirstlane(m16);
          if (!m16) continue;
          uint32_t t = base + (uint32_t)__builtin_ctz(m16);
          m16 &= m16 - 1u;
          v4i a = ld_a(t), ci = ld_c(t);
          for (;;) {
            const bool more = m16 != 0u;
            v4i a2 = a, c2 = ci;
            if (more) {
              t = base + (uint32_t)__builtin_ctz(m16);
              m16 &= m16 - 1u;
              a2 = ld_a(t);
              c2 = ld_c(t);
            }
            run_tile(a, ci);
            if (!more) break;
            a = a2;
            ci = c2;
          }
        }
#endif
      }
    }
    // PIPE cursor: this wave's next tile >= t and < lim that passes its group and tile prefilters
    // (scalar; the group verdict is cached).  NFDP_PIPE_PF: 2 = group + tile prefilters, 1 = group
    // prefilters only, 0 = none (prefilters only ever skip work: results are the same).
    uint32_t gcur = 0xFFFFFFFFu;
    bool gok = false;
    auto next = [&](uint32_t t, uint32_t lim) -> uint32_t {
      t += (tile0 + tstep - t % tstep) % tstep;
      while (t < lim) {
        const uint32_t gi = t / kAclGroup;
        if (gi != gcur) { gcur = gi; gok = NFDP_PIPE_PF >= 1 ? pass(gpf + 8 * gi) : true; }
        if (gok && (NFDP_PIPE_PF < 2 || pass(pf + 8 * t))) return t;
        if (!gok) {
          const uint32_t nb = (gi + 1) * kAclGroup;
          t = nb + (tile0 + tstep - nb % tstep) % tstep;
        } else {
          t += tstep;
        }
      }
      return lim;
    };
    if (!ptiles_done) {
      // (batches of 4 LDS tiles with their 8 fragment reads in flight together: slower, r3 s15 A/B)
      for (uint32_t gi = 0; gi < lds_groups; ++gi) {
        if ((!PIPE || NFDP_PIPE_PF >= 1) && !pass(gpf + 8 * gi)) continue;
        const uint32_t t_beg = gi * kAclGroup, t_end = min(av.tiles, t_beg + kAclGroup);
#if NFDP_PIPE_UNROLL
        if (PIPE && NFDP_PIPE_PF < 2 && tstep == 1 && t_end - t_beg == kAclGroup) {
          // a whole group with no tile prefilter: straight-line, so the fragment reads of later
          // tiles issue under the MFMAs of earlier ones
          // (NFDP_ACL_LOOKAHEAD tiles' fragments are read ahead of the tile whose MFMAs issue, so
          // the LDS latency runs under them instead of in front of every tile)
          constexpr uint32_t LA = NFDP_ACL_LOOKAHEAD;
          v4i ab[LA + 1], cb[LA + 1];
#pragma unroll
          for (uint32_t k = 0; k < LA; ++k) {
            ab[k] = av.lw[(t_beg + k) * 64 + lane];
            cb[k] = av.lc[(t_beg + k) * 4 + g];
          }
#pragma unroll
          for (uint32_t k = 0; k < kAclGroup; ++k) {
            if (k + LA < kAclGroup) {
              ab[(k + LA) % (LA + 1)] = av.lw[(t_beg + k + LA) * 64 + lane];
              cb[(k + LA) % (LA + 1)] = av.lc[(t_beg + k + LA) * 4 + g];
            }
            run_tile(ab[k % (LA + 1)], cb[k % (LA + 1)]);
          }
          continue;
        }
#endif
        // this wave's first tile of the group (tiles == tile0 mod tstep)
        for (uint32_t nt = t_beg + (tile0 + tstep - t_beg % tstep) % tstep; nt < t_end; nt += tstep) {
          if (((!PIPE && NFDP_TILE_PF) || (PIPE && NFDP_PIPE_PF >= 2)) && !pass(pf + 8 * nt)) continue;
          run_tile(av.lw[nt * 64 + lane], av.lc[nt * 4 + g]);
        }
      }
    }
    if (!PIPE) {
      // tiles past the LDS copy, one at a time (instances at the 4-wave register budget; their
      // layouts stage C init for exactly the LDS tiles: ctiles == ltiles)
      for (uint32_t gi = lds_groups; gi < ngroups; ++gi) {
        if (!pass(gpf + 8 * gi)) continue;
        const uint32_t t_beg = gi * kAclGroup, t_end = min(av.tiles, t_beg + kAclGroup);
        for (uint32_t nt = t_beg + (tile0 + tstep - t_beg % tstep) % tstep; nt < t_end; nt += tstep) {
          if (!pass(pf + 8 * nt)) continue;
          run_tile(__builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r_gw, (nt * 64u + lane) * 16u, 0, 0)),
                   __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r_gc, (nt * 4u + g) * 16u, 0, 0)));
        }
      }
    } else if (lds_groups < ngroups && !ptiles_done) {
      // (PIPE: the 2-wave instances, which have the registers for 8 tiles in flight)
      // Tiles past the LDS copy: a scalar cursor yields this wave's next tile that passes its group
      // and tile prefilters; A fragments come in batches of 4 buffer loads, the next batch issued
      // before the current one runs (a fixed 4 loads per batch, out-of-range offsets past the last
      // tile read 0, so every wait is a counted vmcnt: one L2 trip per 4 tiles, overlapped with
      // the previous 4 tiles' MFMAs, instead of one exposed trip per tile).  C init from LDS when
      // staged (ctiles), else a buffer load next to its A fragment.
      auto ld_a = [&](uint32_t t) {
        return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r_gw, t < av.tiles ? (t * 64u + lane) * 16u : 0x80000000u, 0, 0));
      };
      auto ld_c = [&](uint32_t t) {
        if (t < av.ctiles) return av.lc[t * 4 + g];
        return __builtin_bit_cast(v4i, __builtin_amdgcn_raw_buffer_load_b128(r_gc, (t * 4u + g) * 16u, 0, 0));
      };
      // two batches with fixed roles (a register copy of a batch still in flight would wait for it)
      uint32_t c0[4], c1[4], t = next(lds_groups * kAclGroup, av.tiles);
      v4i a0[4], a1[4];
      auto fill = [&](uint32_t (&c)[4], v4i (&av4)[4]) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          c[k] = t; av4[k] = ld_a(t);
          if (t < av.tiles) t = next(t + tstep, av.tiles);
        }
      };
      auto run4 = [&](const uint32_t (&c)[4], const v4i (&av4)[4]) {
#pragma unroll
        for (int k = 0; k < 4; ++k) run_tile_m(av4[k], ld_c(c[k] < av.tiles ? c[k] : 0u), c[k] < av.tiles ? 0u : 0xFFFFFFFFu);
      };
      fill(c0, a0);
      while (c0[0] < av.tiles) {
        fill(c1, a1);
        run4(c0, a0);
        if (c1[0] >= av.tiles) break;
        fill(c0, a0);
        run4(c1, a1);
      }
    }
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      best[tt] = min(best[tt], (uint32_t)__shfl_xor(best[tt], 16));
      best[tt] = min(best[tt], (uint32_t)__shfl_xor(best[tt], 32));
    }
    const uint32_t bb = pick4(g, best[0], best[1], best[2], best[3]);
    // f32 bits -> the exact integer (mismatch << 12 | rule); "no tile ran" stays all-ones
    const uint32_t b = bb == 0xFFFFFFFFu ? bb : (uint32_t)__uint_as_float(bb);
    if (best_out) *best_out = b;
    acl_rule = acl_rule_of(b, t.n_acl);
  } else if constexpr (ACL == kAclScalar) {
    acl_rule = acl_first_match(t, key);
  } else {
    acl_rule = -1;
  }
}

// Small tables staged in LDS by the fused and ring kernels (ports < kLdsPorts, chain words,
// ACL verdicts).
constexpr uint32_t kLdsChains = 256;
constexpr size_t kLdsTabBytes = kLdsPorts * sizeof(PortEntry) + kLdsChains * 8 + 1024;

// Table-access policy of the fused kernel (pipeline.h DirectTables contract): LDS copies for
// ports < kLdsPorts, the first kLdsChains chain words and every ACL verdict; global memory for
// the rest (or for everything when the layout has no room: L.tabs false -> nport = nchain = 0).
struct LdsTables {
  const TablesView& t;
  const PortEntry* lport;
  const uint64_t* lchain;
  const uint8_t* lperm;
  uint32_t nport, nchain;
  bool lds_perm;
  // Each accessor reads LDS with ds_read and takes the global fallback behind a wave-uniform
  // branch.  A per-lane `lds ? lptr[i] : gptr[i]` select makes the compiler merge the two
  // pointers into one generic pointer and issue FLAT loads, which count against vmcnt AND
  // lgkmcnt: every table read then waited for the in-flight frame prefetch and stores.
  __device__ __forceinline__ PortEntry port(uint32_t i) const {
    if (nport == 0) return t.ports[i];
    PortEntry pe = lport[i < nport ? i : 0u];
    if (__builtin_expect(__any(i >= nport), 0)) {
      if (i >= nport) pe = t.ports[i];
    }
    return pe;
  }
  __device__ __forceinline__ uint64_t chain_word(uint32_t c) const {
    uint64_t w = nchain ? lchain[c < nchain ? c : 0u] : 0ull;
    if (__builtin_expect(__any(c >= nchain), 0)) {
      if (c >= nchain) w = c < t.n_chains ? *reinterpret_cast<const uint64_t*>(&t.chains[c]) : 0ull;
    }
    return w;
  }
  __device__ __forceinline__ bool permit(int r) const {
    if (r < 0) return t.acl_default_permit != 0;
    if (lds_perm) return lperm[r] != 0;
    return t.acl_permit[r] != 0;
  }
};

// Stage the small tables into LDS (caller provides the three regions; all threads of the block
// call it, a __syncthreads() must follow).  Returns the table-access policy over the copies.
__device__ __forceinline__ LdsTables stage_lds_tables(const TablesView& t, PortEntry* lport, uint64_t* lchain,
                                                      uint8_t* lperm, bool enabled, uint32_t nthreads) {
  const uint32_t nchain = enabled ? min(t.n_chains, kLdsChains) : 0u;
  const uint32_t nperm = t.n_acl + t.n_acl6;           // IPv4 then IPv6 rule verdicts
  const bool lds_perm = enabled && nperm <= 1024;      // verdict bytes staged for up to 1024 rules
  if (enabled) {
    const uint4* gp = reinterpret_cast<const uint4*>(t.ports);
    uint4* lp = reinterpret_cast<uint4*>(lport);
    for (uint32_t i = threadIdx.x; i < kLdsPorts * 2; i += nthreads) lp[i] = gp[i];
    for (uint32_t i = threadIdx.x; i < nchain; i += nthreads) lchain[i] = *reinterpret_cast<const uint64_t*>(&t.chains[i]);
    if (lds_perm)
      for (uint32_t i = threadIdx.x; i < nperm; i += nthreads) lperm[i] = t.acl_permit[i];
  }
  return LdsTables{t, lport, lchain, lperm, enabled ? (uint32_t)kLdsPorts : 0u, nchain, lds_perm};
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

// Wave-cooperative first-bucket probe.  Instead of every lane fetching its own 128-B bucket as
// 8 x 16 B (each dwordx4 instruction touching 64 different lines), 8 lanes fetch one bucket:
// instruction j brings the first-choice buckets of packets 8j..8j+7, 8 whole lines.  Lane L of
// instruction j holds chunk L & 7 (even = slot key, odd = slot action) of packet 8j + (L >> 3)'s
// bucket, compares key chunks against that packet's key (read from the wave's LDS scratch), and
// the matching slot's action lane hands its chunk over through the same scratch.  Packets with
// no match in the first bucket probe the second one per lane (flow_probe's tail; rare at the
// table's <= 50 % load).  Same results as flow_probe.  `probe` false -> slot -1.  EXEC full.
// The probe in two halves, so the bucket fetch can be issued as soon as the hash is known and
// its latency overlap the ACL classification (fused kernel, NFDP_PROBE_EARLY): issue = the eight
// wave-cooperative line loads, finish = key compare, action hand-over and the second choice.
#ifndef NFDP_PROBE_AUX
// >= 0: bucket loads as raw buffer loads with these cache-policy bits; -1: flat loads.  r6 A/B
// (profiles/r6_s26_ab_probe_aux.jsonl, r6_s27_*): buffer loads 15,686 vs 15,437 Mpps and 16,081
// vs 15,964 on another box (policy 0; sc0 / sc1 within noise of it, nt 15,243), ClassBench set
// unchanged - the descriptor's range check replaces the flat loads' 64-bit address arithmetic
#define NFDP_PROBE_AUX 0
#endif
__device__ __forceinline__ void flow_probe_issue(const TablesView& t, uint32_t h, uint4 (&v)[8]) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t c = lane & 7u, q = lane >> 3;
  const uint32_t b1 = h & t.bucket_mask;
#if NFDP_PROBE_AUX >= 0
  const __amdgpu_buffer_rsrc_t r_fl = __builtin_amdgcn_make_buffer_rsrc(
      (void*)t.flows, (short)0, (int)((t.bucket_mask + 1u) * (uint32_t)(kBucketSlots * 32)), 0x00020000);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t bj = (uint32_t)__shfl((int)b1, 8 * j + (int)q);
    v[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r_fl, bj * (uint32_t)(kBucketSlots * 32) + c * 16u,
                                                                          0, NFDP_PROBE_AUX));
  }
#else
  const uint4* fl = reinterpret_cast<const uint4*>(t.flows);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t bj = (uint32_t)__shfl((int)b1, 8 * j + (int)q);
    v[j] = fl[(size_t)bj * (kBucketSlots * 2) + c];
  }
#endif
}

// 16-B equality as one OR of XORs (v_bitop3 chains, one compare).  Written as four field compares
// joined with &&, the compiler packs the v_cmp results into a bit vector (v_cndmask + shifts +
// s_nop per field: 15 VALU per bucket line compare in the probe, r5 s18 ISA histogram).
// The XORs pass through empty asm: without it InstCombine turns or(xor...) == 0 back into the
// <4 x i32> compare.
#ifndef NFDP_EQ16_ASM
#define NFDP_EQ16_ASM 1   // 0: the field compares (A/B)
#endif
__device__ __forceinline__ bool eq16(const uint4& a, const uint4& b) {
#if !NFDP_EQ16_ASM
  return a.x == b.x && a.y == b.y && a.z == b.z && a.w == b.w;
#endif
  uint32_t x = a.x ^ b.x, y = a.y ^ b.y, z = a.z ^ b.z, w = a.w ^ b.w;
  asm("" : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
  return (x | y | z | w) == 0u;
}

__device__ __forceinline__ int64_t flow_probe_finish(const TablesView& t, const FlowKey& k, uint32_t h, bool probe,
                                                     uint4* kx, const uint4 (&v)[8], uint4& act) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t c = lane & 7u, q = lane >> 3;
  const uint32_t b1 = h & t.bucket_mask;
  const uint4* fl = reinterpret_cast<const uint4*>(t.flows);
  // key as stored (meta | used); a non-probing packet gets a w no slot can hold
  kx[lane] = make_uint4(k.src_ip, k.dst_ip, k.ports, probe ? (k.meta | kSlotUsed) : 0xFFFFFFFFu);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // Per instruction j: compare, then the action lane of a matching slot overwrites packet
  // 8j + q's scratch entry (its key is no longer needed: only instruction j reads it).  The
  // packet lanes 8j..8j+7 take their match byte from this j's ballot (one mask live at a time).
  uint32_t sel = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint4 kk = kx[8 * j + q];
    const bool hit = ((c & 1u) == 0u) & eq16(v[j], kk);
    const unsigned long long m = __ballot(hit);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if ((c & 1u) && ((m >> (lane - 1)) & 1ull)) kx[8 * j + q] = v[j];
    if (q == (uint32_t)j) sel = (uint32_t)(m >> (8u * c)) & 0x55u;
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  int64_t slot = -1;
  if (sel) {
    act = kx[lane];
    slot = (int64_t)b1 * kBucketSlots + (__builtin_ctz(sel) >> 1);
  } else if (probe) {
    // second choice, per lane (the first bucket missed)
    const TableHash th = table_hash(h, t.bucket_mask);
    const uint4* row = fl + (size_t)th.b2 * (kBucketSlots * 2);
    const uint32_t used = k.meta | kSlotUsed;
    const uint4 key = make_uint4(k.src_ip, k.dst_ip, k.ports, used);
    auto eq = [&](const uint4& e) { return eq16(e, key); };
    const uint4 k0 = row[0], a0 = row[1], k1 = row[2], a1 = row[3];
    const uint4 k2 = row[4], a2 = row[5], k3 = row[6], a3 = row[7];
    const bool n0 = eq(k0), n1 = eq(k1), n2 = eq(k2), n3 = eq(k3);
    if (n0 | n1 | n2 | n3) {
      act = n0 ? a0 : n1 ? a1 : n2 ? a2 : a3;
      slot = (int64_t)th.b2 * kBucketSlots + (n0 ? 0 : n1 ? 1 : n2 ? 2 : 3);
    }
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  return slot;
}

__device__ __forceinline__ int64_t flow_probe_wave(const TablesView& t, const FlowKey& k, uint32_t h, bool probe,
                                                   uint4* kx, uint4& act) {
  uint4 v[8];
  flow_probe_issue(t, h, v);
  return flow_probe_finish(t, k, h, probe, kx, v, act);
}

// Sum of a u32 over the 64 lanes (EXEC must be full): two quad permutes and two row rotates
// leave every lane of a 16-lane row holding the row sum (DPP: no LDS crossbar round trips), then
// four readlanes add the rows.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false);  // row_ror:8
  return __builtin_amdgcn_readlane(v, 15) + __builtin_amdgcn_readlane(v, 31) +
         __builtin_amdgcn_readlane(v, 47) + __builtin_amdgcn_readlane(v, 63);
}

// Wave-aggregated counter update: lanes whose `idx` is equal are summed and ONE atomic per
// distinct index is issued.  Same-address atomics serialise at the memory side; a chunk of 64
// packets from a handful of ports otherwise costs 64 back-to-back RMWs on a few counter words.
// `inc` = bytes (< 2^16) when `packed` (the word is pkts << 40 | bytes), else a plain count.
// EXEC must be full.
__device__ __forceinline__ void wave_counter_add(unsigned long long* ctr, uint32_t idx, uint32_t inc, bool packed,
                                                 bool active) {
  unsigned long long pending = __ballot(active);
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const uint32_t k = __builtin_amdgcn_readlane(idx, leader);
    const bool mine = active && idx == k;
    const unsigned long long m = __ballot(mine);
    const uint32_t sum = wave_sum_u32(mine ? inc : 0u);  // bytes (or count) of the group
    const unsigned long long v = packed ? (((unsigned long long)__popcll(m) << 40) | sum) : (unsigned long long)sum;
    if ((int)(threadIdx.x & 63u) == leader) atomicAdd(ctr + k, v);
    pending &= ~m;
  }
}

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// Per-workgroup-region form (SideOut::blk_cnt): the wave's claim is an LDS atomic on the
// workgroup's count, so no global atomic at all (a per-wave atomic on one global counter still
// serialised 64K waves at the memory side when every packet is flagged: an overlay egress).
__device__ __forceinline__ void side_list_append_blk(const SideOut& so, uint32_t* lds_n, bool sn, uint32_t i) {
  const unsigned long long m = __ballot(sn);
  const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const int leader = __builtin_ctzll(m);
  uint32_t base = 0;
  if (sn && pre == 0) base = atomicAdd(lds_n, (uint32_t)__builtin_popcountll(m));
  base = __builtin_amdgcn_readlane(base, leader);
  if (sn && base + pre < so.blk_cap) so.list[blockIdx.x * so.blk_cap + base + pre] = i;
}

// Wave-aggregated append to the side list (flagged lanes): ONE atomic on the list counter per wave
// instead of one per lane (every lane of a wave adding to one counter word serialises at the
// memory side; an overlay egress flags every packet for its outer header).  EXEC must be full.
__device__ __forceinline__ void side_list_append(const SideOut& so, bool sn, uint32_t i) {
  const unsigned long long m = __ballot(sn);
  const uint32_t pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  const int leader = __builtin_ctzll(m);
  uint32_t base = 0;
  if (sn && pre == 0) base = atomicAdd(so.cnt + 5, (uint32_t)__builtin_popcountll(m));
  base = __builtin_amdgcn_readlane(base, leader);
  if (sn) {
    const uint32_t q = base + pre;
    if (q < so.cap_list) so.list[q] = i;
    else atomicAdd(so.cnt + 6, 1u);
  }
}


// GPU sink of pipeline.h side_stage: one global atomic per replica / learn event (rare paths:
// flooding, mirroring, ARP-trap and learning ports only).  Replica tx and ARP-trap counts go
// straight to the global counters.
struct GpuSideSink {
  const SideOut& so;
  unsigned long long* port_ctr;
  unsigned long long* drop_ctr;
  __device__ __forceinline__ void rep(const uint32_t* hdr, uint32_t meta, uint32_t src) {
    const uint32_t pos = atomicAdd(so.cnt + 0, 1u);
    if (pos >= so.cap_rep) { atomicAdd(so.cnt + 2, 1u); return; }
    uint4* dst = reinterpret_cast<uint4*>(so.rep_hdr) + (size_t)pos * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q] = make_uint4(hdr[4 * q], hdr[4 * q + 1], hdr[4 * q + 2], hdr[4 * q + 3]);
    so.rep_meta[pos] = meta;
    so.rep_src[pos] = src;
    const uint32_t r = meta_reason(meta), port = meta_port(meta);
    if (r) atomicAdd(drop_ctr + r, 1ull);
    else if (port < (uint32_t)kMaxPorts) atomicAdd(port_ctr + 2 * port + 1, ctr_inc(meta_len(meta)));
  }
  // `nq`: the 16-B chunks the outer header occupies (consumers take its length from its EtherType,
  // iox.cpp / packets.py xhdr_len); the rest of the 128-B record is not written
  __device__ __forceinline__ void xhdr(const uint32_t* hdr, uint32_t src, uint32_t nq) {
    if (!so.xhdr) return;
    uint4* dst = reinterpret_cast<uint4*>(so.xhdr) + (size_t)src * (kXhdrBytes / 16);
#pragma unroll
    for (int q = 0; q < kXhdrBytes / 16; ++q)
      if ((uint32_t)q < nq) dst[q] = make_uint4(hdr[4 * q], hdr[4 * q + 1], hdr[4 * q + 2], hdr[4 * q + 3]);
  }
  __device__ __forceinline__ void learn(uint32_t bridge, uint32_t lo, uint32_t hi, uint32_t port) {
    const uint32_t pos = atomicAdd(so.cnt + 1, 1u);
    if (pos >= so.cap_learn) { atomicAdd(so.cnt + 3, 1u); return; }
    reinterpret_cast<uint4*>(so.learn)[pos] = make_uint4(lo, (hi & 0xFFFFu) | (bridge << 16), port, 0u);
  }
};

// gfx950 store-data hazard: a dwordx4 buffer store whose soffset is an SGPR reads its data VGPRs
// after issue, and a VALU that overwrote them in the very next instruction stored the NEW value
// for some lanes (r5 s8: 4 frames of 64K corrupted, dword 1 of the last chunk pass, the meta
// offset i*4 in their place; tools/store_hazard_scan.py finds the sequence in the assembly).
// LLVM inserts the wait state only when the soffset is not a register.  Every 16-B buffer store
// here goes through store_b128: the asm after it claims to rewrite the stored vector, so its VGPRs
// stay allocated - nothing else can be written into them - until the s_nop has issued.
template <int AUX>
__device__ __forceinline__ void store_b128(v4u w, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b128(w, r, voff, soff, AUX);
  asm volatile("s_nop 1" : "+v"(w));
}

// ---- coalesced frame I/O (tools/copy_bench.hip: 6.4 TB/s vs 1.4 TB/s for per-lane slots) ----
// A wave's 64 slots are one contiguous 4-KiB run.  Each dwordx4 instruction covers 1 KiB of it
// lane-contiguously (16 full 64-B lines) instead of 16 B of 64 different lines, and the wave's
// 1-KiB LDS scratch (the classify key exchange, `kx`) transposes 16 packets per pass between
// "chunk per lane" and "packet per lane".  Chunk c = 64 q + lane of the run is part c & 3 of
// packet c >> 2.  EXEC must be full.  Offsets at or beyond the buffer's num_records (slots
// past n, or `run` = kNoRun) read 0 / drop the store.  `run` is wave-uniform: it rides in the
// instruction's SGPR offset, the lane part is one loop-invariant VGPR plus the immediate.
constexpr uint32_t kNoRun = 0x80000000u;

// LDS layout of one 16-slot pass of the frame transposes (wave_frames_to_lanes / wave_frames_store,
// the ring's write-backs): chunk k of slot f at kx[16k + (f ^ 5k)].  Both sides of a transpose are
// then free of bank conflicts - the 16 lanes that each hold a whole slot and touch chunk k of it,
// and the 64 lanes that each hold one chunk (lane L: chunk L & 3 of slot L >> 2) - where the plain
// [slot][chunk] layout costs the 16-lane side 4-way conflicts (SQ_LDS_BANK_CONFLICT, r6 PMC pass:
// 24M conflict cycles per headline dispatch against 19M active LDS cycles).  Off: the per-chunk
// addresses raise the headline instance's spills from 15 to 19 VGPRs at its 128-VGPR budget, and
// that costs more than the conflicts (r6 s10 A/B, profiles/r6_s10_ab_256.jsonl: 13,961 vs 15,428
// Mpps; ClassBench-style set 7,926 vs 7,972).
#ifndef NFDP_KX_SWZ
#define NFDP_KX_SWZ 0
#endif
__device__ __forceinline__ uint32_t kx_at(uint32_t f, uint32_t k) {
  return NFDP_KX_SWZ ? 16u * k + (f ^ ((5u * k) & 15u)) : 4u * f + k;
}

template <int AUX>
__device__ __forceinline__ void wave_frames_load(__amdgpu_buffer_rsrc_t r, uint32_t run, v4u c[4]) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16u + q * 1024u, run, AUX);
}

// SW: the 16 slots of a pass sit in kx with their 16-B chunks XOR-swizzled per group of 4 slots
// (chunk k of slot s at 4s + (k ^ (s >> 2 & 3))): 16 lanes reading their own 64-B slot otherwise
// hit the banks of lanes 4, 8 and 12 (4-way conflicts).  Off in the fused kernel, whose register
// allocation the extra addressing pushes from 17 to 35 spilled VGPRs.
template <bool SW = false>
__device__ __forceinline__ void wave_frames_to_lanes(uint4* kx, const v4u c[4], uint32_t* d) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t lw = NFDP_KX_SWZ ? kx_at(lane >> 2, lane & 3u) : SW ? lane ^ ((lane >> 4) & 3u) : lane;
  const uint32_t sw = SW && !NFDP_KX_SWZ ? (lane >> 2) & 3u : 0u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    kx[lw] = make_uint4(c[q].x, c[q].y, c[q].z, c[q].w);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if ((lane >> 4) == (uint32_t)q) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 v = kx[NFDP_KX_SWZ ? kx_at(lane & 15u, (uint32_t)k) : 4u * (lane & 15u) + ((uint32_t)k ^ sw)];
        d[4 * k] = v.x; d[4 * k + 1] = v.y; d[4 * k + 2] = v.z; d[4 * k + 3] = v.w;
      }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
}

// `skip`: bit p set -> packet p of the run is not stored (its frame went elsewhere).
template <int AUX>
__device__ __forceinline__ void wave_frames_store(uint4* kx, const uint32_t* o, __amdgpu_buffer_rsrc_t r, uint32_t run,
                                                  unsigned long long skip = 0ull) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if ((lane >> 4) == (uint32_t)q) {
#pragma unroll
      for (int k = 0; k < 4; ++k) kx[kx_at(lane & 15u, k)] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const uint4 v = kx[kx_at(lane >> 2, lane & 3u)];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const v4u w = {v.x, v.y, v.z, v.w};
    const bool drop = (skip >> (16u * q + (lane >> 2))) & 1ull;
    store_b128<AUX>(w, r, drop ? kNoRun : lane * 16u + q * 1024u, run);
  }
}

// Coalesced store of the frames a wave sends to peers.  The lanes bound for one peer hold one
// contiguous run of slots in that peer's segment (reserve_block hands out wave-contiguous
// positions), so each run is written lane-contiguously, 16 packets per pass through the wave's
// 1-KiB LDS scratch, instead of 4 x 16 B per lane at a 64-B stride.  `send` lanes only (their
// `pos` < `cap`); segment d starts at byte d * seg_bytes, its slot 0 at +64.  EXEC must be full.
template <int AUX>
__device__ __forceinline__ void wave_segment_store(uint4* kx, const uint32_t* o, __amdgpu_buffer_rsrc_t r, bool send,
                                                   uint32_t dest, uint32_t pos, uint32_t seg_bytes, uint32_t cap) {
  const uint32_t lane = threadIdx.x & 63u;
  const unsigned long long lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  unsigned long long pending = __ballot(send);
  while (pending) {
    const int leader = __ffsll((long long)pending) - 1;
    const uint32_t d = __builtin_amdgcn_readlane(dest, leader);
    const bool mine = send && dest == d;
    const unsigned long long m = __ballot(mine);
    pending &= ~m;
    const uint32_t cnt = (uint32_t)__popcll(m);
    const uint32_t p0 = __builtin_amdgcn_readlane(pos, leader);  // the leader has rank 0 in the run
    const uint32_t rk = (uint32_t)__popcll(m & lt);
    for (uint32_t sub = 0; sub < cnt; sub += 16) {
      if (mine && rk >= sub && rk < sub + 16) {
#pragma unroll
        for (int k = 0; k < 4; ++k) kx[4u * (rk - sub) + k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const uint4 v = kx[lane];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      const uint32_t n4 = min(16u, cnt - sub) * 4u;
      const bool ok = lane < n4 && p0 + sub + (lane >> 2) < cap;
      const v4u w = {v.x, v.y, v.z, v.w};
      store_b128<AUX>(w, r, ok ? lane * 16u : kNoRun, d * seg_bytes + 64u + (p0 + sub) * 64u);
    }
  }
}

// ---- multi-GPU output segments (shared by the fused REMOTE variant and the sharded stages) ----
constexpr uint32_t kMaxRanks = 64;

// Block-aggregated slot reservation: waves claim offsets in LDS counters (one LDS atomic per
// wave and destination), then ONE global atomic per (workgroup iteration, destination) turns
// them into segment positions.  (A per-wave global atomic on one counter serialised 16K waves
// per 1M packets: 200 us of a 1M-packet ingress pass.)  Called by every thread of the block.
// Double-buffered use in a loop (`lnext` != nullptr): `lcnt` arrives zeroed (the previous call
// zeroed it as its `lnext`; zero both before the loop), and this call zeroes `lnext` while it
// publishes the bases, which saves the leading barrier: two per call instead of three.
__device__ __forceinline__ uint32_t reserve_block(uint32_t* gcnt, uint32_t dest, bool active, uint32_t nranks,
                                                  uint32_t* lcnt, uint32_t* lbase, uint32_t* lnext = nullptr) {
  const uint32_t lane = threadIdx.x & 63u;
  const unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  if (!lnext) {
    if (threadIdx.x < nranks) lcnt[threadIdx.x] = 0;
    __syncthreads();
  }
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
    if (lnext) lnext[threadIdx.x] = 0;
  }
  __syncthreads();
  return active ? lbase[dest] + off : 0xFFFFFFFFu;
}

}  // namespace nfdp
