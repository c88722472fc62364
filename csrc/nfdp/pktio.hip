// pktio.hip — host <-> HBM packet I/O engine (see pktio.h).
#include "pktio.h"

#include <stdexcept>
#include <string>

namespace nfdp {

namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("pktio: ") + what + ": " + hipGetErrorString(e));
}
}  // namespace

PacketIo::PacketIo(uint32_t capacity, uint32_t depth) : cap_(capacity), depth_(depth), slots_(depth) {
  if (capacity == 0 || depth == 0 || depth > 16 || capacity >= (1u << 25))
    throw std::invalid_argument("pktio: capacity in [1, 2^25), depth in [1, 16]");
  // three non-blocking streams: copy engines for each direction + the compute stream
  ck(hipStreamCreateWithFlags(&up_, hipStreamNonBlocking), "stream");
  ck(hipStreamCreateWithFlags(&comp_, hipStreamNonBlocking), "stream");
  ck(hipStreamCreateWithFlags(&down_, hipStreamNonBlocking), "stream");
  const size_t fb = (size_t)capacity * 64, mb = (size_t)capacity * 4;
  for (Slot& s : slots_) {
    // pinned (page-locked) host memory: the SDMA engines read/write it directly
    ck(hipHostMalloc(reinterpret_cast<void**>(&s.h_in), fb, hipHostMallocDefault), "host alloc");
    ck(hipHostMalloc(reinterpret_cast<void**>(&s.h_im), mb, hipHostMallocDefault), "host alloc");
    ck(hipHostMalloc(reinterpret_cast<void**>(&s.h_out), fb, hipHostMallocDefault), "host alloc");
    ck(hipHostMalloc(reinterpret_cast<void**>(&s.h_meta), mb, hipHostMallocDefault), "host alloc");
    ck(hipMalloc(reinterpret_cast<void**>(&s.d_in), fb), "dev alloc");
    ck(hipMalloc(reinterpret_cast<void**>(&s.d_im), mb), "dev alloc");
    ck(hipMalloc(reinterpret_cast<void**>(&s.d_out), fb), "dev alloc");
    ck(hipMalloc(reinterpret_cast<void**>(&s.d_meta), mb), "dev alloc");
    ck(hipMalloc(reinterpret_cast<void**>(&s.d_lat), ((size_t)capacity / 16 + 1) * 4), "dev alloc");
    ck(hipEventCreate(&s.e0), "event");
    ck(hipEventCreate(&s.e_up), "event");
    ck(hipEventCreate(&s.e_kern), "event");
    ck(hipEventCreate(&s.e_down), "event");
  }
}

PacketIo::~PacketIo() {
  // drain everything in flight before freeing (a freed pinned buffer under an SDMA copy faults)
  (void)hipStreamSynchronize(up_);
  (void)hipStreamSynchronize(comp_);
  (void)hipStreamSynchronize(down_);
  for (Slot& s : slots_) {
    for (void* h : {(void*)s.h_in, (void*)s.h_im, (void*)s.h_out, (void*)s.h_meta}) (void)hipHostFree(h);
    for (void* d : {(void*)s.d_in, (void*)s.d_im, (void*)s.d_out, (void*)s.d_meta, (void*)s.d_lat}) (void)hipFree(d);
    for (hipEvent_t e : {s.e0, s.e_up, s.e_kern, s.e_down}) (void)hipEventDestroy(e);
  }
  (void)hipStreamDestroy(up_);
  (void)hipStreamDestroy(comp_);
  (void)hipStreamDestroy(down_);
}

void PacketIo::submit(uint32_t si, uint32_t n, FusedLaunch f, const LaunchCfg& cfg) {
  if (si >= depth_) throw std::out_of_range("pktio: slot");
  if (n > cap_) throw std::invalid_argument("pktio: batch larger than the slot capacity");
  Slot& s = slots_[si];
  if (s.busy && hipEventQuery(s.e_down) != hipSuccess) throw std::runtime_error("pktio: slot still in flight");
  s.n = n;
  s.busy = true;
  if (n == 0) {
    ck(hipEventRecord(s.e0, up_), "record");
    ck(hipEventRecord(s.e_up, up_), "record");
    ck(hipEventRecord(s.e_kern, up_), "record");
    ck(hipEventRecord(s.e_down, up_), "record");
    return;
  }
  ck(hipEventRecord(s.e0, up_), "record");
  // batch-release stamp at upload start: latency samples then cover host -> HBM -> kernel
  if (f.t0) ck(launch_stamp(const_cast<unsigned long long*>(f.t0), up_), "stamp");
  ck(hipMemcpyAsync(s.d_in, s.h_in, (size_t)n * 64, hipMemcpyHostToDevice, up_), "H2D frames");
  ck(hipMemcpyAsync(s.d_im, s.h_im, (size_t)n * 4, hipMemcpyHostToDevice, up_), "H2D meta");
  ck(hipEventRecord(s.e_up, up_), "record");
  ck(hipStreamWaitEvent(comp_, s.e_up, 0), "wait");
  f.pkts = s.d_in; f.inmeta = s.d_im; f.out = s.d_out; f.out_meta = s.d_meta; f.n = n; f.lat = s.d_lat;
  ck(launch_fused(f, cfg, comp_), "fused kernel");
  ck(hipEventRecord(s.e_kern, comp_), "record");
  ck(hipStreamWaitEvent(down_, s.e_kern, 0), "wait");
  ck(hipMemcpyAsync(s.h_out, s.d_out, (size_t)n * 64, hipMemcpyDeviceToHost, down_), "D2H frames");
  ck(hipMemcpyAsync(s.h_meta, s.d_meta, (size_t)n * 4, hipMemcpyDeviceToHost, down_), "D2H meta");
  ck(hipEventRecord(s.e_down, down_), "record");
}

void PacketIo::wait(uint32_t si) {
  if (si >= depth_) throw std::out_of_range("pktio: slot");
  if (slots_[si].busy) ck(hipEventSynchronize(slots_[si].e_down), "sync");
}

bool PacketIo::ready(uint32_t si) {
  if (si >= depth_) throw std::out_of_range("pktio: slot");
  return !slots_[si].busy || hipEventQuery(slots_[si].e_down) == hipSuccess;
}

void PacketIo::timings(uint32_t si, float* h2d, float* kern, float* d2h, float* total) {
  Slot& s = slots_[si];
  wait(si);
  ck(hipEventElapsedTime(h2d, s.e0, s.e_up), "elapsed");
  ck(hipEventElapsedTime(kern, s.e_up, s.e_kern), "elapsed");
  ck(hipEventElapsedTime(d2h, s.e_kern, s.e_down), "elapsed");
  ck(hipEventElapsedTime(total, s.e0, s.e_down), "elapsed");
}

}  // namespace nfdp
