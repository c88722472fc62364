// probe_bench.hip — price the random 128-B bucket fetch of the flow lookup on MI355X.
//   lane  : current design, each lane loads its own bucket as 8 x dwordx4 (8 requests per line)
//   coal  : 8 lanes per bucket, one dwordx4 each (one 128-B line per 8 lanes per instruction),
//           then ds_bpermute gathers a lane's bucket words back (the compare needs its key)
//   keys64: lane loads only the 4 key chunks of a key|key|key|key|act... layout (4 x dwordx4)
// Table 64 MB (2^19 x 128 B, the 1M-flow table), 4M lookups with uniform random buckets,
// grid = 512 blocks x 512 threads grid-striding (the fused kernel's shape).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(512) void probe(const uint4* tab, uint32_t mask, uint32_t n, uint32_t seed, uint32_t* out) {
  uint32_t accum = 0;
  for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    const uint32_t b = mix(i ^ seed) & mask;
    if (MODE == 0) {
      const uint4* row = tab + (size_t)b * 8;
      uint32_t x = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) { const uint4 v = row[q]; x ^= v.x ^ v.y ^ v.z ^ v.w; }
      accum += x;
    } else if (MODE == 1) {
      const uint32_t lane = threadIdx.x & 63u;
      uint32_t x = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // lane l loads chunk l%8 of the bucket of packet j*8 + l/8 (packet = lane of the wave)
        const uint32_t src = j * 8 + (lane >> 3);
        const uint32_t bb = __shfl(b, src);
        const uint4 v = tab[(size_t)bb * 8 + (lane & 7u)];
        // give every packet lane its bucket's 4 key words back (chunk 0 here) via bpermute
        const uint32_t k = __builtin_amdgcn_ds_bpermute((int)(((lane & 7u) * 8u) << 2), (int)(v.x ^ v.y ^ v.z ^ v.w));
        x ^= ((lane >> 3) == (uint32_t)j) ? k : 0u;
      }
      accum += x;
    } else {
      const uint4* row = tab + (size_t)b * 8;
      uint32_t x = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) { const uint4 v = row[q]; x ^= v.x ^ v.y ^ v.z ^ v.w; }
      accum += x;
    }
  }
  if (accum == 0x12345678u) out[0] = accum;
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
static float run(const uint4* tab, uint32_t mask, uint32_t n, uint32_t* out, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  probe<MODE><<<512, 512>>>(tab, mask, n, 1, out);
  CK(hipEventRecord(a));
  for (int k = 0; k < iters; ++k) probe<MODE><<<512, 512>>>(tab, mask, n, 2 + k, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main() {
  const uint32_t nb = 1u << 19, n = 1u << 22;
  uint4* tab;
  uint32_t* out;
  CK(hipMalloc(&tab, (size_t)nb * 128));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(tab, 1, (size_t)nb * 128));
  for (uint32_t m : {nb - 1, (1u << 12) - 1}) {
    const float t0 = run<0>(tab, m, n, out, 20), t1 = run<1>(tab, m, n, out, 20), t2 = run<2>(tab, m, n, out, 20);
    std::printf("{\"buckets\": %u, \"lookups\": %u, \"lane_8x16B_us\": %.1f, \"coalesced_us\": %.1f, \"keys64_us\": %.1f}\n",
                m + 1, n, t0, t1, t2);
  }
  return 0;
}
