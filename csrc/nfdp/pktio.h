// pktio.h — host <-> HBM packet I/O engine.
//
// Role of the reference's VFIO PEM/DPI layer (octep_cp_lib soc/vfio.c: hugepage-backed host
// memory, DPI DMA engine moving packets between host and the DPU): on an MI355X node the wire
// side of the data plane is host memory (NIC rings, AF_XDP umem, pod vhost rings), so the engine
// owns DEPTH pinned host slots and DEPTH device slots and moves each batch
//   host_in[s] --SDMA(H2D stream)--> dev_in[s] --fused kernel (compute stream)--> dev_out[s]
//   dev_out[s] --SDMA(D2H stream)--> host_out[s]
// with events chaining the three streams, so batch s+1's upload and batch s-1's download overlap
// batch s's kernel (copy engines and CUs run concurrently).  A slot is reusable once its D2H
// event has completed (`wait`/`ready`).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "host.h"

namespace nfdp {

class PacketIo {
 public:
  PacketIo(uint32_t capacity, uint32_t depth);
  ~PacketIo();
  PacketIo(const PacketIo&) = delete;
  PacketIo& operator=(const PacketIo&) = delete;

  uint32_t capacity() const { return cap_; }
  uint32_t depth() const { return depth_; }
  uint8_t* host_in(uint32_t s) const { return slots_[s].h_in; }        // cap * 64 B frames
  uint32_t* host_inmeta(uint32_t s) const { return slots_[s].h_im; }   // cap in_port | len << 16
  uint8_t* host_out(uint32_t s) const { return slots_[s].h_out; }
  uint32_t* host_meta(uint32_t s) const { return slots_[s].h_meta; }
  uint32_t* dev_lat(uint32_t s) const { return slots_[s].d_lat; }

  // Enqueue slot s with n packets: upload, run `f` (pkts/inmeta/out/out_meta/lat/n filled in
  // here), download.  Non-blocking; the previous use of the slot must have completed.
  void submit(uint32_t s, uint32_t n, FusedLaunch f, const LaunchCfg& cfg);
  void wait(uint32_t s);
  bool ready(uint32_t s);
  // timings of the last completed use of slot s (ms): upload, kernel, download, end-to-end
  void timings(uint32_t s, float* h2d, float* kern, float* d2h, float* total);

 private:
  struct Slot {
    uint8_t *h_in = nullptr, *h_out = nullptr;
    uint32_t *h_im = nullptr, *h_meta = nullptr;
    uint8_t *d_in = nullptr, *d_out = nullptr;
    uint32_t *d_im = nullptr, *d_meta = nullptr, *d_lat = nullptr;
    hipEvent_t e0{}, e_up{}, e_kern{}, e_down{};
    uint32_t n = 0;
    bool busy = false;
  };
  uint32_t cap_, depth_;
  std::vector<Slot> slots_;
  hipStream_t up_{}, comp_{}, down_{};
};

}  // namespace nfdp
