// hwq_probe: do streams share a hardware queue with a resident (never-returning) grid?
//
// HIP maps ordinary streams round-robin onto GPU_MAX_HW_QUEUES hardware queues per device; a kernel
// that never returns holds its queue, so any stream mapped to the same queue waits behind it.  This
// probe launches a spinner grid (a few workgroups that poll a pinned host flag, with a device-side
// deadline every wave reaches) on a stream created one of three ways:
//   plain   hipStreamCreateWithFlags
//   cumask  hipExtStreamCreateWithCUMask (all CUs): a CU mask is a queue property, so the runtime
//           is expected to give such a stream a queue of its own
//   prio    hipStreamCreateWithPriority (highest)
// then creates `n` further ordinary streams, launches a tiny kernel on each (and one on the null
// stream) and reports which of them completed while the spinner still ran.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/hwq_probe.hip -o tools/bin/hwq_probe
// Run:   GPU_MAX_HW_QUEUES=4 tools/bin/hwq_probe cumask 12 [warm] [pre]
//   warm: launch `tiny` once (and wait) before the spinner: lazy code-object loading out of the way
//   pre:  create the other streams before the spinner's
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                                     \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      std::exit(2);                                                                               \
    }                                                                                             \
  } while (0)

__global__ void spinner(volatile uint32_t* stop, uint32_t* started, unsigned long long deadline_ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) atomicAdd(started, 1u);
  // every wave leaves at the deadline (100 MHz clock) even if the host never sets `stop`
  while (__atomic_load_n(stop, __ATOMIC_ACQUIRE) == 0u) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > deadline_ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
}

// a spinner that never reads host memory: the same wait as a plain clock loop (1 s)
__global__ void spinner_clock(uint32_t* started, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) atomicAdd(started, 1u);
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void tiny(uint32_t* out, uint32_t v) {
  if (threadIdx.x == 0) out[0] = v;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "plain";
  const int n = argc > 2 ? std::atoi(argv[2]) : 8;
  bool warm = false, pre = false, clock = false;
  for (int i = 3; i < argc; ++i) {
    warm = warm || std::string(argv[i]) == "warm";
    pre = pre || std::string(argv[i]) == "pre";
    clock = clock || std::string(argv[i]) == "clock";
  }
  hipDeviceProp_t prop{};
  CK(hipGetDeviceProperties(&prop, 0));
  const char* hwq = std::getenv("GPU_MAX_HW_QUEUES");
  uint32_t *h_stop = nullptr, *h_started = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&h_stop), 4, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(reinterpret_cast<void**>(&h_started), 4, hipHostMallocCoherent | hipHostMallocMapped));
  *h_stop = 0;
  *h_started = 0;
  uint32_t *d_stop = nullptr, *d_started = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_stop), h_stop, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_started), h_started, 0));
  uint32_t* d_out = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&d_out), 4 * (n + 1)));
  if (warm) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, (hipStream_t)0, d_out, 0u);
    CK(hipDeviceSynchronize());
  }
  std::vector<hipStream_t> ss(n);
  if (pre)
    for (int i = 0; i < n; ++i) CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
  hipStream_t ring{};
  if (mode == "cumask") {
    const uint32_t words = (uint32_t)((prop.multiProcessorCount + 31) / 32);
    std::vector<uint32_t> mask(words, 0xFFFFFFFFu);
    if (prop.multiProcessorCount % 32) mask.back() = (1u << (prop.multiProcessorCount % 32)) - 1u;
    CK(hipExtStreamCreateWithCUMask(&ring, words, mask.data()));
  } else if (mode == "prio") {
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    CK(hipStreamCreateWithPriority(&ring, hipStreamNonBlocking, hi));
  } else {
    CK(hipStreamCreateWithFlags(&ring, hipStreamNonBlocking));
  }
  const unsigned long long deadline = 300000000ull;   // 3 s
  const auto t_launch = std::chrono::steady_clock::now();
  if (clock) hipLaunchKernelGGL(spinner_clock, dim3(8), dim3(64), 0, ring, d_started, 100000000ull);   // 1 s
  else hipLaunchKernelGGL(spinner, dim3(8), dim3(64), 0, ring, d_stop, d_started, deadline);
  CK(hipGetLastError());
  const auto t0 = std::chrono::steady_clock::now();
  while (__atomic_load_n(h_started, __ATOMIC_ACQUIRE) < 8u &&
         std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  for (int i = 0; i < n; ++i) {
    if (!pre) CK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
    hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, ss[i], d_out + i, (uint32_t)i);
  }
  hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, (hipStream_t)0, d_out + n, (uint32_t)n);
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  int blocked = 0;
  std::string which;
  for (int i = 0; i <= n; ++i) {
    const hipError_t q = hipStreamQuery(i < n ? ss[i] : (hipStream_t)0);
    const bool done = q == hipSuccess;
    if (!done) {
      ++blocked;
      which += (i < n ? std::to_string(i) : std::string("null")) + " ";
    }
  }
  const bool spinning = hipStreamQuery(ring) == hipErrorNotReady;
  // when did the other streams finish?  (ms after the spinner's launch; the host stops the
  // host-polling spinner at ~600 ms, the clock spinner ends at 1000 ms by itself)
  std::this_thread::sleep_for(std::chrono::milliseconds(300));
  const double t_stop = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_launch).count();
  __atomic_store_n(h_stop, 1u, __ATOMIC_RELEASE);
  std::string fin;
  for (int i = 0; i < n; ++i) {
    CK(hipStreamSynchronize(ss[i]));
    const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_launch).count();
    if (i < 3) fin += std::to_string((int)t) + " ";
  }
  CK(hipStreamSynchronize(ring));
  const double t_ring = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_launch).count();
  CK(hipDeviceSynchronize());
  std::fprintf(stdout, "{\"clock\": %s, \"host_stop_ms\": %d, \"first_streams_done_ms\": \"%s\", \"spinner_done_ms\": %d}\n",
               clock ? "true" : "false", (int)t_stop, fin.c_str(), (int)t_ring);
  std::printf("{\"mode\": \"%s\", \"warm\": %s, \"pre\": %s, \"GPU_MAX_HW_QUEUES\": \"%s\", \"streams\": %d, "
              "\"spinner_started\": %u, \"spinner_running_at_check\": %s, \"blocked\": %d, \"blocked_streams\": \"%s\"}\n",
              mode.c_str(), warm ? "true" : "false", pre ? "true" : "false", hwq ? hwq : "(unset)", n,
              __atomic_load_n(h_started, __ATOMIC_ACQUIRE), spinning ? "true" : "false", blocked, which.c_str());
  for (int i = 0; i < n; ++i) CK(hipStreamDestroy(ss[i]));
  CK(hipStreamDestroy(ring));
  return 0;
}
