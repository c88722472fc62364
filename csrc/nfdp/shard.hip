// shard.hip — stage kernels of the flow-sharded multi-GPU pipeline (see shard.h).
#include "device.h"
#include "shard.h"

namespace nfdp {

struct ShardLds {
  size_t acl_w, acl_c, toep_f, toep_t, kx, pc, total;
};
__host__ __device__ inline ShardLds shard_lds(int hash_mode, int acl_mode, uint32_t acl_tiles, bool ports) {
  ShardLds L;
  size_t o = 0;
  const uint32_t lt = acl_tiles < kLdsAclTiles ? acl_tiles : kLdsAclTiles;
  L.acl_w = o; if (acl_mode == kAclMfma) o += (size_t)lt * 64 * 16;
  L.acl_c = o; if (acl_mode == kAclMfma) o += (size_t)lt * 4 * 16;
  L.toep_f = o; if (hash_mode == kHashMfma) o += 2 * 2 * 64 * 16;
  L.toep_t = o; if (hash_mode == kHashLds) o += kToepLdsWords * 4;
  L.kx = o; o += kWaves * 64 * 16;
  L.pc = o; if (ports) o += kLdsPorts * 4 * 4 + kNumReasons * 4;
  L.total = (o + 15) & ~(size_t)15;
  return L;
}

// ------------------------------------------------------------------------------------------
// 1. ingress
// ------------------------------------------------------------------------------------------
template <int HASH, int ACL>
__global__ __launch_bounds__(kBlock) void ingress_kernel(IngressArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const ShardLds L = shard_lds(HASH, ACL, a.acl_tiles, false);
  v4i* lw = reinterpret_cast<v4i*>(smem + L.acl_w);
  v4i* lc = reinterpret_cast<v4i*>(smem + L.acl_c);
  v4i* lt = reinterpret_cast<v4i*>(smem + L.toep_f);
  uint32_t* ltab = reinterpret_cast<uint32_t*>(smem + L.toep_t);
  uint4* kx = reinterpret_cast<uint4*>(smem + L.kx) + (threadIdx.x >> 6) * 64;
  __shared__ uint32_t rcnt[kMaxRanks], rbase[kMaxRanks];
  if constexpr (ACL == kAclMfma) {
    const v4i* gw = reinterpret_cast<const v4i*>(a.acl_wfrag);
    const v4i* gc = reinterpret_cast<const v4i*>(a.acl_cinit);
    const uint32_t lt_ = min(a.acl_tiles, kLdsAclTiles);
    for (uint32_t i = threadIdx.x; i < lt_ * 64; i += kBlock) lw[i] = gw[i];
    for (uint32_t i = threadIdx.x; i < lt_ * 4; i += kBlock) lc[i] = gc[i];
  }
  const AclView av{lw, lc, reinterpret_cast<const v4i*>(a.acl_wfrag), reinterpret_cast<const v4i*>(a.acl_cinit), a.acl_tiles};
  if constexpr (HASH == kHashMfma) {
    const v4i* gt = reinterpret_cast<const v4i*>(a.toep_frag);
    for (uint32_t i = threadIdx.x; i < 256; i += kBlock) lt[i] = gt[i];
  }
  if constexpr (HASH == kHashLds)
    stage_toep(ltab, a.toep_tab, threadIdx.x, kBlock);
  __syncthreads();
  const size_t seg = desc_seg_bytes(a.g.cap_desc);
  for (uint32_t base = blockIdx.x * kBlock; base < a.n; base += gridDim.x * kBlock) {
    const uint32_t i = base + threadIdx.x;
    const bool valid = i < a.n;
    uint32_t d[kSlotDwords];
    uint32_t im = 0;
    if (valid) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = a.pkts[(size_t)i * 4 + q];
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
      }
      im = a.inmeta[i];
    } else {
#pragma unroll
      for (int q = 0; q < kSlotDwords; ++q) d[q] = 0;
    }
    Parsed p;
    IngressState st;
    ingress_stage(a.t, d, im, p, st);
    uint32_t hash = 0;
    int acl = -1;
    classify_wave<HASH, ACL>(st.key, kx, av, lt, ltab, a.t, hash, acl);
    if (__builtin_expect(__any(p.ipv6 && v6_keys(a.t)), 0)) {
      if (p.ipv6) acl = acl_rule_v6(a.t, p, st);
    }
    // (IPv6 flows need the packet's addresses at the probe (flow6_verify): the owner here sees
    // only the 16-B key, so the sharded path keeps IPv6 on L2 / L3 - its launcher clears flow6_on)
    const bool need = valid && !st.reason && p.ipv4;
    const uint32_t owner = owner_of(hash, a.g.nranks);
    const uint32_t pos = reserve_block(a.cnt, owner, need, a.g.nranks, rcnt, rbase);
    if (valid) {
      uint32_t ref = kRefNone;
      if (need) {
        if (pos < a.g.cap_desc) {
          uint4* dst = reinterpret_cast<uint4*>(a.send_desc + owner * seg) + 2 * (1 + pos);
          dst[0] = make_uint4(st.key.src_ip, st.key.dst_ip, st.key.ports, st.key.meta);
          dst[1] = make_uint4(st.wire_len, 0u, 0u, 0u);
          ref = (owner << 24) | pos;
        } else {
          ref = kRefOverflow;
        }
      }
      a.ref[i] = ref;
      a.aux[i] = (uint32_t)(acl + 1) | ((hash & 7u) << 16);  // ACL rule + 1, LAG hash bits
    }
  }
}

__global__ void seg_header_kernel(const uint32_t* cnt, uint8_t* buf, uint32_t nranks, size_t seg_bytes, uint32_t cap) {
  const uint32_t o = threadIdx.x;
  if (o < nranks) {
    const uint32_t c = cnt[o] < cap ? cnt[o] : cap;
    *reinterpret_cast<uint4*>(buf + o * seg_bytes) = make_uint4(c, cap, 0, 0);
  }
}

// ------------------------------------------------------------------------------------------
// 3. owner: lookups for descriptors received from every rank
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void owner_kernel(OwnerArgs a) {
  __shared__ uint32_t ltab[16 * 256];
  for (uint32_t i = threadIdx.x; i < 4096; i += 256) ltab[i] = a.toep_tab[i];
  __syncthreads();
  const size_t seg = desc_seg_bytes(a.g.cap_desc), vseg = verdict_seg_bytes(a.g.cap_desc);
  const uint32_t total = a.g.nranks * a.g.cap_desc;
  for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
    const uint32_t s = idx / a.g.cap_desc, j = idx % a.g.cap_desc;
    const uint4* src = reinterpret_cast<const uint4*>(a.recv_desc + s * seg);
    const uint32_t count = src[0].x;
    if (j >= count) continue;
    const uint4 dv = src[2 * (1 + j)];
    const uint32_t wlen = src[2 * (1 + j) + 1].x;
    const FlowKey k{dv.x, dv.y, dv.z, dv.w};
    const uint32_t w[4] = {k.src_ip, k.dst_ip, k.ports, k.meta};
    uint32_t h = 0;
#pragma unroll
    for (int b = 0; b < 16; ++b) h ^= ltab[b * 256 + ((w[b >> 2] >> (8 * (b & 3))) & 0xFFu)];
    uint4 v;
    const int64_t slot = flow_probe(a.t, k, h, v);
    uint4 out = make_uint4(0, 0, 0, 0);
    if (slot >= 0) {
      out = make_uint4(v.x, v.y, v.z, 1u);  // same packing as FlowAction, status=1
      if (a.flow_ctr) atomicAdd(a.flow_ctr + slot, ctr_inc(wlen));
    }
    reinterpret_cast<uint4*>(a.send_verdict + s * vseg)[1 + j] = out;
  }
}

// ------------------------------------------------------------------------------------------
// 5. apply: NF chain on the local packet, local egress or hand-off to the egress GPU
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void apply_kernel(ApplyArgs a) {
  __shared__ uint32_t pc[kLdsPorts * 4];
  __shared__ uint32_t drops[kNumReasons];
  __shared__ uint32_t rcnt[kMaxRanks], rbase[kMaxRanks];
  for (uint32_t i = threadIdx.x; i < kLdsPorts * 4; i += kBlock) pc[i] = 0;
  if (threadIdx.x < kNumReasons) drops[threadIdx.x] = 0;
  __syncthreads();
  const size_t dseg = verdict_seg_bytes(a.g.cap_desc);
  const size_t pseg = pkt_seg_bytes(a.g.cap_pkt);
  const unsigned long long t0 = a.t0 ? *a.t0 : 0ull;
  for (uint32_t base = blockIdx.x * kBlock; base < a.n; base += gridDim.x * kBlock) {
    const uint32_t i = base + threadIdx.x;
    const bool valid = i < a.n;
    uint32_t d[kSlotDwords];
    uint32_t im = 0, ref = kRefNone, aux = 0;
    if (valid) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = a.pkts[(size_t)i * 4 + q];
        d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
      }
      im = a.inmeta[i]; ref = a.ref[i]; aux = a.aux[i];
    } else {
#pragma unroll
      for (int q = 0; q < kSlotDwords; ++q) d[q] = 0;
    }
    Parsed p;
    IngressState st;
    ingress_stage(a.t, d, im, p, st);
    bool hit = false;
    FlowAction act = {};
    if (ref == kRefOverflow) {
      st.reason = st.reason ? st.reason : kOverflow;
    } else if (ref != kRefNone) {
      const uint32_t o = ref >> 24, pos = ref & 0xFFFFFFu;
      const uint4 v = reinterpret_cast<const uint4*>(a.recv_verdict + o * dseg)[1 + pos];
      hit = v.w == 1u;
      act.chain_id = v.x & 0xFFFFu; act.out_port = v.x >> 16; act.nat_ip = v.y;
      act.nat_port = v.z & 0xFFFFu; act.vlan = v.z >> 16;
    }
    EgressDecision e = chain_stage(a.t, p, st, hit, act, (int)(aux & 0xFFFFu) - 1, aux >> 16);
    uint32_t eg = a.g.rank;
    if (!e.reason) eg = a.t.ports[e.out_port].gpu;
    const bool remote = valid && !e.reason && eg != a.g.rank && eg < a.g.nranks;
    const uint32_t pos = reserve_block(a.pcnt, eg, remote, a.g.nranks, rcnt, rbase);
    if (valid) {
      uint32_t o[kSlotDwords];
      emit(p, e.tci, e.push != 0, o);
      const uint32_t olen = egress_len(p, e);
      uint32_t reason = e.reason;
      if (remote && pos >= a.g.cap_pkt) reason = kOverflow;
      uint4* dst;
      if (remote && reason == kOk) {
        uint8_t* segp = a.send_pkt + eg * pseg;
        dst = reinterpret_cast<uint4*>(segp + 64 + (size_t)pos * 64);
        reinterpret_cast<uint32_t*>(segp + pkt_meta_off(a.g.cap_pkt))[pos] = make_meta(e.out_port, olen, kOk, e.xhdr != 0);
        a.out_meta[i] = make_meta(e.out_port, olen, kRemote);
      } else {
        dst = a.out + (size_t)i * 4;
        a.out_meta[i] = make_meta(reason == kOverflow ? kPortNone : e.out_port, reason == e.reason ? olen : 0u, reason, !reason && e.xhdr, !reason && e.flood);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) dst[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
      if (st.in_port < kLdsPorts) {
        atomicAdd(&pc[st.in_port], 1u); atomicAdd(&pc[kLdsPorts + st.in_port], st.wire_len);
      } else if (st.in_port < (uint32_t)kMaxPorts) {
        atomicAdd(a.port_ctr + 2 * st.in_port, ctr_inc(st.wire_len));
      }
      if (reason) {
        atomicAdd(&drops[reason & (kNumReasons - 1)], 1u);
      } else if (!remote) {
        if (e.out_port < kLdsPorts) {
          atomicAdd(&pc[2 * kLdsPorts + e.out_port], 1u); atomicAdd(&pc[3 * kLdsPorts + e.out_port], olen);
        } else {
          atomicAdd(a.port_ctr + 2 * e.out_port + 1, ctr_inc(olen));
        }
        if (a.lat && (i & 15u) == 0) a.lat[i >> 4] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
      }
    }
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < kLdsPorts; q += kBlock) {
    if (pc[q]) atomicAdd(a.port_ctr + 2 * q, ((unsigned long long)pc[q] << 40) | pc[kLdsPorts + q]);
    if (pc[2 * kLdsPorts + q])
      atomicAdd(a.port_ctr + 2 * q + 1, ((unsigned long long)pc[2 * kLdsPorts + q] << 40) | pc[3 * kLdsPorts + q]);
  }
  if (threadIdx.x < kNumReasons && drops[threadIdx.x])
    atomicAdd(a.drop_ctr + threadIdx.x, (unsigned long long)drops[threadIdx.x]);
}

// ------------------------------------------------------------------------------------------
// 7. egress of packets received from peers: tx counters + latency
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void egress_kernel(EgressArgs a) {
  __shared__ uint32_t pc[kLdsPorts * 2];
  for (uint32_t i = threadIdx.x; i < kLdsPorts * 2; i += 256) pc[i] = 0;
  __syncthreads();
  const size_t pseg = pkt_seg_bytes(a.g.cap_pkt);
  const uint32_t total = a.g.nranks * a.g.cap_pkt;
  const unsigned long long t0 = a.t0 ? *a.t0 : 0ull;
  for (uint32_t idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
    const uint32_t s = idx / a.g.cap_pkt, j = idx % a.g.cap_pkt;
    if (s == a.g.rank) continue;
    const uint8_t* segp = a.recv_pkt + s * pseg;
    const uint32_t count = reinterpret_cast<const uint32_t*>(segp)[0];
    if (j >= count) continue;
    const uint32_t m = reinterpret_cast<const uint32_t*>(segp + pkt_meta_off(a.g.cap_pkt))[j];
    const uint32_t port = meta_port(m), len = meta_len(m);
    if (port < kLdsPorts) {
      atomicAdd(&pc[port], 1u); atomicAdd(&pc[kLdsPorts + port], len);
    } else if (port < (uint32_t)kMaxPorts) {
      atomicAdd(a.port_ctr + 2 * port + 1, ctr_inc(len));
    }
    if (a.lat && (j & 15u) == 0) a.lat[idx >> 4] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0);
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < kLdsPorts; q += 256)
    if (pc[q]) atomicAdd(a.port_ctr + 2 * q + 1, ((unsigned long long)pc[q] << 40) | pc[kLdsPorts + q]);
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
template <int H, int A>
static hipError_t launch_ingress_t(const IngressArgs& a, int num_cus, hipStream_t s) {
  // static LDS of the kernel (reservation counters) + dynamic tables must fit 160 KiB
  constexpr size_t kStatic = 2 * kMaxRanks * sizeof(uint32_t);
  constexpr size_t kMaxDyn = 160 * 1024 - kStatic;
  const size_t lds = shard_lds(H, A, a.acl_tiles, false).total;
  if (lds > kMaxDyn) return hipErrorInvalidValue;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&ingress_kernel<H, A>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxDyn);
    if (e != hipSuccess) return e;
    attr = true;
  }
  int per_cu = (int)((160 * 1024) / (lds + kStatic));
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  uint32_t grid = (uint32_t)(per_cu * num_cus);
  const uint32_t need = (a.n + kBlock - 1) / kBlock;
  if (need < grid) grid = need;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL((ingress_kernel<H, A>), dim3(grid), dim3(kBlock), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_ingress(const IngressArgs& a, int hash_mode, int acl_mode, int num_cus, hipStream_t s) {
  if (a.g.nranks == 0 || a.g.nranks > kMaxRanks || a.g.cap_desc >= (1u << 24)) return hipErrorInvalidValue;
  if (acl_mode == kAclMfma && (a.acl_tiles == 0 || a.acl_tiles > kAclMaxRules / 16)) return hipErrorInvalidValue;
#define NFDP_CASE(HH, AA) if (hash_mode == HH && acl_mode == AA) return launch_ingress_t<HH, AA>(a, num_cus, s);
  NFDP_CASE(1, 0) NFDP_CASE(1, 1) NFDP_CASE(1, 2)
  NFDP_CASE(2, 0) NFDP_CASE(2, 1) NFDP_CASE(2, 2)
#undef NFDP_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_seg_headers(const uint32_t* cnt, uint8_t* buf, uint32_t nranks, size_t seg_bytes, uint32_t cap,
                              hipStream_t s) {
  if (nranks > 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(seg_header_kernel, dim3(1), dim3(nranks <= 64 ? 64 : 1024), 0, s, cnt, buf, nranks, seg_bytes, cap);
  return hipGetLastError();
}

hipError_t launch_owner(const OwnerArgs& a, int num_cus, hipStream_t s) {
  const uint32_t total = a.g.nranks * a.g.cap_desc;
  uint32_t grid = (total + 255) / 256;
  const uint32_t cap = (uint32_t)num_cus * 4;
  if (grid > cap) grid = cap;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(owner_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_apply(const ApplyArgs& a, int num_cus, hipStream_t s) {
  if (a.g.nranks == 0 || a.g.nranks > kMaxRanks) return hipErrorInvalidValue;
  uint32_t grid = (uint32_t)num_cus * 4;
  const uint32_t need = (a.n + kBlock - 1) / kBlock;
  if (need < grid) grid = need;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(apply_kernel, dim3(grid), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_egress(const EgressArgs& a, int num_cus, hipStream_t s) {
  const uint32_t total = a.g.nranks * a.g.cap_pkt;
  uint32_t grid = (total + 255) / 256;
  const uint32_t cap = (uint32_t)num_cus * 4;
  if (grid > cap) grid = cap;
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(egress_kernel, dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace nfdp
