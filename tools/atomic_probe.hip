// atomic_probe.hip — price random 8-byte counter updates (the per-flow counter of the fused
// kernel) on MI355X:
//   dev   : device-scope atomicAdd into one 16 MB table (current design)
//   xcd   : per-XCD replica (HW_REG_XCC_ID), workgroup-scope atomic -> executes in the local L2
//   xcdag : per-XCD replica, agent-scope atomic
// then checks that the replicas sum to the device-scope table.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  return x & 7u;
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(512) void upd(unsigned long long* ctr, uint32_t mask, uint32_t n, uint32_t seed) {
  const size_t stride = (size_t)mask + 1;
  unsigned long long* base = ctr;
  if (MODE != 0) base += (size_t)xcc_id() * stride;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = mix(i ^ seed) & mask;
    const unsigned long long v = (1ull << 40) | 64u;
    if (MODE == 0) atomicAdd(base + s, v);
    if (MODE == 1) __hip_atomic_fetch_add(base + s, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (MODE == 2) __hip_atomic_fetch_add(base + s, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void fold(const unsigned long long* rep, unsigned long long* out, uint32_t n) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  unsigned long long s = 0;
  for (int r = 0; r < 8; ++r) s += rep[(size_t)r * n + j];
  out[j] = s;
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
static float run(unsigned long long* p, uint32_t mask, uint32_t n, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int grid = 256 * 8;
  upd<MODE><<<grid, 512>>>(p, mask, n, 1);
  CK(hipEventRecord(a));
  for (int k = 0; k < iters; ++k) upd<MODE><<<grid, 512>>>(p, mask, n, 2 + k);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main() {
  const uint32_t slots = 1u << 21, mask = slots - 1, n = 1u << 22;
  const int iters = 20;
  unsigned long long *dev, *rep, *folded;
  CK(hipMalloc(&dev, slots * 8ull));
  CK(hipMalloc(&rep, slots * 8ull * 8));
  CK(hipMalloc(&folded, slots * 8ull));
  for (int pass = 0; pass < 2; ++pass) {
    CK(hipMemset(dev, 0, slots * 8ull));
    CK(hipMemset(rep, 0, slots * 64ull));
    const float t0 = run<0>(dev, mask, n, iters);
    const float t1 = run<1>(rep, mask, n, iters);
    CK(hipMemset(rep, 0, slots * 64ull));
    CK(hipMemset(dev, 0, slots * 8ull));
    run<0>(dev, mask, n, iters);
    run<1>(rep, mask, n, iters);
    fold<<<(slots + 255) / 256, 256>>>(rep, folded, slots);
    CK(hipDeviceSynchronize());
    std::vector<unsigned long long> h0(slots), h1(slots);
    CK(hipMemcpy(h0.data(), dev, slots * 8ull, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h1.data(), folded, slots * 8ull, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (uint32_t j = 0; j < slots; ++j) bad += h0[j] != h1[j];
    CK(hipMemset(rep, 0, slots * 64ull));
    const float t2 = run<2>(rep, mask, n, iters);
    std::printf("{\"pass\": %d, \"updates\": %u, \"dev_us\": %.1f, \"xcd_wg_us\": %.1f, \"xcd_agent_us\": %.1f, "
                "\"mismatch\": %zu}\n", pass, n, t0 * 1e3, t1 * 1e3, t2 * 1e3, bad);
  }
  return 0;
}
