// copy_bench.hip — price the frame I/O pattern of the fused kernel on MI355X.
//   lane  : current design, lane i loads / stores its own 64-B slot as 4 x dwordx4 (stride 64 B
//           across lanes: every instruction touches 64 different lines, 16 B each)
//   xpose : each dwordx4 instruction covers 1 KiB contiguous (lane-contiguous), a 4-KiB LDS
//           tile per wave transposes to one-packet-per-lane and back (optionally XOR-swizzled)
//   coal  : lane-contiguous copy without the transpose (lower bound)
// 4M slots of 64 B + 4-B meta in, same out; grid = 512 x 512 grid-striding (the fused shape).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
constexpr int kBufCfg = 0x00020000;
constexpr int kNt = 2;

template <int MODE>
__global__ __launch_bounds__(512) void copy(const uint4* in, const uint32_t* im, uint4* out, uint32_t* om, uint32_t n) {
  __shared__ v4u tile[8][256];
  const __amdgpu_buffer_rsrc_t r_in = __builtin_amdgcn_make_buffer_rsrc((void*)in, (short)0, (int)(n * 64u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_out = __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)(n * 64u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_im = __builtin_amdgcn_make_buffer_rsrc((void*)im, (short)0, (int)(n * 4u), kBufCfg);
  const __amdgpu_buffer_rsrc_t r_om = __builtin_amdgcn_make_buffer_rsrc((void*)om, (short)0, (int)(n * 4u), kBufCfg);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  v4u* t = tile[w];
  for (uint32_t base = blockIdx.x * 512u; base < n; base += gridDim.x * 512u) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t wbase = (base + w * 64u) * 64u;  // byte offset of this wave's 64 slots
    v4u d[4];
    if (MODE == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_raw_buffer_load_b128(r_in, i * 64u + 16u * q, 0, kNt);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = __builtin_amdgcn_raw_buffer_load_b128(r_in, wbase + (q * 64u + lane) * 16u, 0, kNt);
    }
    uint32_t m = __builtin_amdgcn_raw_buffer_load_b32(r_im, i * 4u, 0, kNt);
    if (MODE == 1 || MODE == 2) {
      // chunk c = q*64 + lane belongs to packet c >> 2, part c & 3; swizzle part ^ (packet & 3)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t c = q * 64u + lane, pk = c >> 2, pt = c & 3u;
        t[pk * 4u + (MODE == 2 ? (pt ^ (pk & 3u)) : pt)] = d[q];
      }
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = t[lane * 4u + (MODE == 2 ? (q ^ (lane & 3u)) : q)];
      // ---- (per-packet work would go here: lane owns packet base + w*64 + lane) ----
      d[0].x ^= m;
#pragma unroll
      for (int q = 0; q < 4; ++q) t[lane * 4u + (MODE == 2 ? (q ^ (lane & 3u)) : q)] = d[q];
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t c = q * 64u + lane, pk = c >> 2, pt = c & 3u;
        d[q] = t[pk * 4u + (MODE == 2 ? (pt ^ (pk & 3u)) : pt)];
      }
      __builtin_amdgcn_wave_barrier();
    } else {
      d[0].x ^= m;
    }
    if (MODE == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) __builtin_amdgcn_raw_buffer_store_b128(d[q], r_out, i * 64u + 16u * q, 0, kNt);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) __builtin_amdgcn_raw_buffer_store_b128(d[q], r_out, wbase + (q * 64u + lane) * 16u, 0, kNt);
    }
    __builtin_amdgcn_raw_buffer_store_b32(m + 1u, r_om, i * 4u, 0, kNt);
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

template <int MODE>
static float run(const uint4* in, const uint32_t* im, uint4* out, uint32_t* om, uint32_t n, int iters, int grid) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  copy<MODE><<<grid, 512>>>(in, im, out, om, n);
  CK(hipEventRecord(a));
  for (int k = 0; k < iters; ++k) copy<MODE><<<grid, 512>>>(in, im, out, om, n);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main() {
  const uint32_t n = 1u << 22;
  uint4 *in, *out;
  uint32_t *im, *om;
  CK(hipMalloc(&in, (size_t)n * 64));
  CK(hipMalloc(&out, (size_t)n * 64));
  CK(hipMalloc(&im, (size_t)n * 4));
  CK(hipMalloc(&om, (size_t)n * 4));
  CK(hipMemset(in, 1, (size_t)n * 64));
  CK(hipMemset(im, 2, (size_t)n * 4));
  for (int grid : {512, 1024, 8192}) {
    const float t0 = run<0>(in, im, out, om, n, 20, grid);
    const float t1 = run<3>(in, im, out, om, n, 20, grid);
    const float t2 = run<1>(in, im, out, om, n, 20, grid);
    const float t3 = run<2>(in, im, out, om, n, 20, grid);
    const double gb = (double)n * 136 / 1e9;
    std::printf("{\"grid\": %d, \"slots\": %u, \"lane_us\": %.1f, \"coal_us\": %.1f, \"xpose_us\": %.1f, "
                "\"xpose_swz_us\": %.1f, \"lane_TBps\": %.2f, \"xpose_swz_TBps\": %.2f}\n",
                grid, n, t0, t1, t2, t3, gb / t0 * 1e3, gb / t3 * 1e3);
  }
  return 0;
}
