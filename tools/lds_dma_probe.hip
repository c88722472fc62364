// lds_dma_probe: is data a gfx950 direct-to-LDS buffer load (buffer_load_dword[x4] ... lds) wrote
// complete when the compiler's s_waitcnt vmcnt(N > 0) says so, while later stores / atomics of the
// same wave are still outstanding?
//
// The round-2 experiment that prefetched the fused kernel's next frame straight into LDS
// corrupted a few output dwords ("lanes = 3 mod 4, first dword of each 16-B chunk") although the
// wait the compiler put before the LDS read looked right (docs/DATAPLANE.md, batch kernel notes).
// This probe reduces that loop to its memory pattern: per iteration each wave
//   1. reads the frame the previous iteration's LDS DMA brought (the compiler waits for it),
//   2. issues the next frame's LDS DMA (64 lanes x 16 B = one 1-KiB run),
//   3. issues a per-lane random 8-B atomic (the flow counter) and a 16-B store per lane (the output),
// and checks every dword it read from LDS against the source.  Mismatches are counted per lane % 4
// and per dword of the 16-B chunk.  A second kernel waits with vmcnt(0) before the LDS read
// (`drain`): the control.  `single_buffer`: one LDS buffer per wave (the round-2 layout), so the
// next DMA overwrites what this iteration's ds_read is reading (a write-after-read hazard between
// the LDS read and the DMA's LDS write, which s_waitcnt vmcnt does not cover).
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_dma_probe.hip -o tools/bin/lds_dma_probe
// Run:   tools/bin/lds_dma_probe [iterations per wave] [size: 4 | 16]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      std::exit(2);                                                                               \
    }                                                                                             \
  } while (0)

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

template <int SIZE, bool DRAIN, bool SINGLE = false, int PRESSURE = 0>
__global__ __launch_bounds__(kBlock) void probe(const uint32_t* src, uint32_t n_runs, uint32_t iters,
                                                unsigned long long* ctr, uint32_t ctr_mask, uint4* out,
                                                unsigned long long* bad) {
  __shared__ __attribute__((aligned(16))) uint32_t buf[kWaves][2][256];   // per wave: 2 x 1 KiB
  __shared__ uint32_t tab[4096];                                          // PRESSURE: random LDS lookups
  for (uint32_t i = threadIdx.x; i < 4096; i += kBlock) tab[i] = i * 2654435761u;
  __syncthreads();
  uint32_t sink = 0;
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * kWaves + wave, nw = gridDim.x * kWaves;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)(n_runs * 1024u), 0x00020000);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)(n_runs * 1024u), 0x00020000);
  unsigned long long nbad[4] = {0, 0, 0, 0};
  uint32_t run = gw % n_runs;
  // the first run's DMA
  if constexpr (SIZE == 16)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)&buf[wave][0][0], 16, lane * 16u, run * 1024u, 0, 0);
  else
    for (int k = 0; k < 4; ++k)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)&buf[wave][0][k * 64], 4, lane * 4u + k * 256u, run * 1024u, 0, 0);
  for (uint32_t it = 0; it < iters; ++it) {
    // SINGLE: one LDS buffer per wave, as the round-2 prefetch had: the next frame's DMA targets
    // the bytes this iteration's ds_read is reading
    const uint32_t cur = SINGLE ? 0u : (it & 1u);
    const uint32_t nxt = (run + nw) % n_runs;
    if constexpr (DRAIN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // PRESSURE: this wave's LDS queue holds that many random lookups (the fused kernel's hash /
    // table reads) in front of the frame read, so the read completes late
    uint32_t h = run ^ lane;
#pragma unroll
    for (int k = 0; k < PRESSURE; ++k) h ^= tab[(h * 0x9E3779B1u + k) & 4095u];
    // 1. read this iteration's frame from LDS (lane-contiguous 16 B, the layout the DMA wrote)
    const uint4 v = *reinterpret_cast<const uint4*>(&buf[wave][cur][lane * 4]);
    // 2. the next frame's DMA into the other buffer
    if constexpr (SIZE == 16)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)&buf[wave][SINGLE ? 0u : (cur ^ 1u)][0], 16, lane * 16u, nxt * 1024u, 0, 0);
    else
      for (int k = 0; k < 4; ++k)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)&buf[wave][SINGLE ? 0u : (cur ^ 1u)][k * 64], 4, lane * 4u + k * 256u, nxt * 1024u, 0, 0);
    sink ^= h;
    // check against the source (frame word = run * 256 + dword index, written by the host)
    const uint32_t w0 = run * 256u + lane * 4u;
    const uint32_t got[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) nbad[k] += got[k] != w0 + (uint32_t)k;
    // 3. the flow-counter atomic and the output store of this frame
    atomicAdd(ctr + ((v.x * 2654435761u) & ctr_mask), 1ull);
    typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
    const v4u_t vv = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(vv, ro, lane * 16u, run * 1024u, 0);
    run = nxt;
  }
  if (sink == 0x12345678u) bad[16] = sink;   // (keeps the pressure reads)
  // per lane % 4 and dword: bad[(lane & 3) * 4 + k]
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (nbad[k]) atomicAdd(bad + (lane & 3u) * 4u + k, nbad[k]);
}

template <int SIZE, bool DRAIN, bool SINGLE = false, int PRESSURE = 0>
static void run(const uint32_t* d_src, uint32_t n_runs, uint32_t iters, unsigned long long* d_ctr, uint32_t mask,
                uint4* d_out, unsigned long long* d_bad, int cus) {
  CK(hipMemset(d_bad, 0, 16 * 8));
  hipLaunchKernelGGL((probe<SIZE, DRAIN, SINGLE, PRESSURE>), dim3(cus * 8), dim3(kBlock), 0, 0, d_src, n_runs, iters, d_ctr, mask, d_out, d_bad);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  unsigned long long h[16];
  CK(hipMemcpy(h, d_bad, sizeof(h), hipMemcpyDeviceToHost));
  unsigned long long tot = 0;
  for (auto x : h) tot += x;
  std::printf("{\"size\": %d, \"lds_pressure\": %d, \"single_buffer\": %s, \"drain\": %s, \"waves\": %d, \"iters\": %u, \"reads\": %llu, \"bad\": %llu, \"bad_by_lane_mod4_dword\": [",
              SIZE, PRESSURE, SINGLE ? "true" : "false", DRAIN ? "true" : "false", cus * 8 * kWaves, iters, (unsigned long long)cus * 8 * kBlock * iters * 4ull, tot);
  for (int i = 0; i < 16; ++i) std::printf("%s%llu", i ? ", " : "", h[i]);
  std::printf("]}\n");
}

int main(int argc, char** argv) {
  const uint32_t iters = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 2000;
  const int size = argc > 2 ? std::atoi(argv[2]) : 16;
  hipDeviceProp_t prop{};
  CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t n_runs = 1u << 16;   // 64 MiB of frames
  std::vector<uint32_t> h((size_t)n_runs * 256);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint32_t)i;
  uint32_t* d_src = nullptr;
  uint4* d_out = nullptr;
  unsigned long long *d_ctr = nullptr, *d_bad = nullptr;
  const uint32_t mask = (1u << 21) - 1;   // 16 MiB of counters
  CK(hipMalloc(reinterpret_cast<void**>(&d_src), h.size() * 4));
  CK(hipMalloc(reinterpret_cast<void**>(&d_out), h.size() * 4));
  CK(hipMalloc(reinterpret_cast<void**>(&d_ctr), (mask + 1ull) * 8));
  CK(hipMalloc(reinterpret_cast<void**>(&d_bad), 17 * 8));
  CK(hipMemcpy(d_src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(d_ctr, 0, (mask + 1ull) * 8));
  if (size == 16) {
    run<16, false>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
    run<16, true>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
    run<16, false, true>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
    run<16, true, true>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
    run<16, false, false, 32>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
    run<16, false, true, 32>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
    run<16, true, true, 32>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
  } else {
    run<4, false>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
    run<4, true>(d_src, n_runs, iters, d_ctr, mask, d_out, d_bad, prop.multiProcessorCount);
  }
  return 0;
}
