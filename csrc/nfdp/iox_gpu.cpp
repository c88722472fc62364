// iox_gpu.cpp — the I/O engine's GPU backend (iox.h GpuBackend): ring queues in pinned host
// slots of the persistent ring kernel (ring.h) and MAC learning into the device table.
#include <algorithm>
#include <stdexcept>
#include <string>

#include "iox.h"

namespace nfdp {
namespace iox {

namespace {
void hck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("iox: ") + what + ": " + hipGetErrorString(e));
}
inline uint32_t pow2_at_least(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
}  // namespace

// ---------------------------------------------------------------------------------- GpuBackend
GpuBackend::GpuBackend(RingEngine* ring) : ring_(ring), cap_(ring->capacity()) {
  if (!ring->host_slots()) throw std::invalid_argument("iox: the ring needs host_slots=True");
  in_ = static_cast<uint8_t*>(ring->host_ptr(0));
  im_ = static_cast<uint32_t*>(ring->host_ptr(1));
  out_ = static_cast<uint8_t*>(ring->host_ptr(2));
  om_ = static_cast<uint32_t*>(ring->host_ptr(3));
}

GpuBackend::~GpuBackend() {
  if (d_learn_) (void)hipFree(d_learn_);
  if (learn_stream_) (void)hipStreamDestroy(learn_stream_);
}

void GpuBackend::thread_init() { hck(hipSetDevice(ring_->device()), "set device"); }

// Host memory pinned and mapped for every device (portable): a second backend finds it
// registered already and only looks up its address.
uint64_t GpuBackend::map_host(const void* p, size_t n, std::function<void(std::function<void()>)>* release) {
  thread_init();
  void* h = const_cast<void*>(p);
  const hipError_t e = hipHostRegister(h, n, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e == hipSuccess) {
    // (unregistering waits for the device: deferred while any ring grid is resident)
    *release = [h](std::function<void()> after) { host_unregister_when_idle(h, std::move(after)); };
  } else {
    (void)hipGetLastError();
    if (e != hipErrorHostMemoryAlreadyRegistered) return 0;
  }
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    if (*release) { (*release)(nullptr); *release = nullptr; }
    return 0;
  }
  return reinterpret_cast<uint64_t>(d);
}

void GpuBackend::apply_learn(const uint32_t* ev, uint32_t n, uint32_t stamp) {
  if (!n) return;
  thread_init();
  if (!learn_stream_) hck(hipStreamCreateWithFlags(&learn_stream_, hipStreamNonBlocking), "learn stream");
  const auto mt = ring_->mac_table();
  if (!mt.first) return;
  if (n > learn_cap_) {
    if (d_learn_) hck(hipFree(d_learn_), "free");
    learn_cap_ = pow2_at_least(std::max<uint32_t>(n, 1024));
    hck(hipMalloc(reinterpret_cast<void**>(&d_learn_), ((size_t)learn_cap_ * 4 + 4) * 4), "learn buffer");
  }
  uint32_t* cnt = d_learn_ + (size_t)learn_cap_ * 4;
  const uint32_t hdr[4] = {n, 0, 0, 0};
  hck(hipMemcpyAsync(d_learn_, ev, (size_t)n * 16, hipMemcpyHostToDevice, learn_stream_), "learn events");
  hck(hipMemcpyAsync(cnt, hdr, 16, hipMemcpyHostToDevice, learn_stream_), "learn count");
  hck(launch_mac_learn(mt.first, mt.second, d_learn_, cnt, n, stamp, cnt + 1, learn_stream_), "learn kernel");
  hck(hipStreamSynchronize(learn_stream_), "learn sync");
  ring_->bump_epoch();   // chunks published from now on drop cached MAC-table lines first
}

}  // namespace iox
}  // namespace nfdp
