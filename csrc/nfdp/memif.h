// memif.h — shared-memory packet interface between a pod (or NF) and the data plane.
//
// The reference's DPU data ports are kernel-bypass: OvS-DPDK ports bound with
// `type=dpdk options:dpdk-devargs=<pci>` on a netdev-datapath bridge
// (internal/daemon/vendor-specific-plugins/marvell/ovs-dp/ovsdp.go:39-55), or FXP silicon queues.
// The MI355X data plane's equivalent for container endpoints is a shared-memory vport: one
// region (a /dev/shm file, or any fd that can be mmap'ed) per vport holding two single-producer
// single-consumer descriptor rings and their frame buffers.  No syscall on the fast path: the
// pod's application writes a frame and bumps `head` (release); the I/O engine (iox.h) reads it,
// copies its 64-B header slot into the GPU ring and later bumps `tail` once the egress copy no
// longer needs the payload (the frame stays in place while the GPU works on its header).
//
//   region  = [Hdr 64 B][Ctl ring 0 .. R, 128 B each][Desc ring 0 .. R][buffers ring 0 .. R]
//   ring 0     = pod -> data plane (the pod produces)
//   ring 1..R  = data plane -> pod (the engine produces; one ring per engine queue, as a NIC
//                gives every queue its own tx ring: the queues' tx threads never share a ring,
//                a lock or a cache line; the pod drains all R)
//   slot i of a ring always uses buffer i (the consumer returns slots in order).
//
// Header-only, no HIP: the I/O engine, the pod-side endpoint and the standalone traffic tool
// (csrc/pktgen) share it.
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace nfdp {
namespace memif {

constexpr uint64_t kMagic = 0x4d49463335355846ull;   // "FX553FIM"
constexpr uint32_t kVersion = 2;
constexpr uint32_t kMaxRxRings = 64;   // data plane -> pod rings (R)

struct alignas(64) Hdr {
  uint64_t magic;
  uint32_t version;
  uint32_t ring_size;      // slots per ring (power of two)
  uint32_t buf_size;       // bytes per frame buffer (>= the largest frame)
  uint32_t flags;
  uint8_t mac[8];          // the vport's MAC (informational, set by the data plane)
  std::atomic<uint32_t> peer_up;   // pod side attached (informational)
  uint32_t rx_rings;       // R: data plane -> pod rings
  uint32_t pad[4];
};
static_assert(sizeof(Hdr) == 64, "memif Hdr");

struct alignas(64) Ctl {
  std::atomic<uint32_t> head;   // written by the producer
  uint32_t pad0[15];
  std::atomic<uint32_t> tail;   // written by the consumer
  uint32_t pad1[15];
};
static_assert(sizeof(Ctl) == 128, "memif Ctl");

struct Desc {
  uint32_t len;
  uint32_t flags;
};

inline size_t region_bytes(uint32_t ring_size, uint32_t buf_size, uint32_t rx_rings = 1) {
  const size_t n = 1 + (size_t)rx_rings;
  return sizeof(Hdr) + n * sizeof(Ctl) + n * (size_t)ring_size * sizeof(Desc) + n * (size_t)ring_size * buf_size;
}

// A mapped region (either side).  `create` sizes and initialises it; otherwise it attaches.
class Region {
 public:
  Region() = default;
  Region(const std::string& path, bool create, uint32_t ring_size = 1024, uint32_t buf_size = 2048, uint32_t rx_rings = 1) {
    open(path, create, ring_size, buf_size, rx_rings);
  }
  ~Region() { close(); }
  Region(const Region&) = delete;
  Region& operator=(const Region&) = delete;

  void open(const std::string& path, bool create, uint32_t ring_size, uint32_t buf_size, uint32_t rx_rings = 1) {
    if (create) {
      if (rx_rings < 1 || rx_rings > kMaxRxRings) throw std::invalid_argument("memif: rx_rings must be in [1, 64]");
      if (ring_size < 2 || (ring_size & (ring_size - 1)) || ring_size > (1u << 20))
        throw std::invalid_argument("memif: ring_size must be a power of two in [2, 2^20]");
      if (buf_size < 64 || buf_size > (1u << 16) || (buf_size & 63))
        throw std::invalid_argument("memif: buf_size must be a multiple of 64 in [64, 65536]");
      // a fresh file, never the old one truncated: a previous region at this path may still be
      // mapped (a removed port the engine keeps for its frames in flight, a pod not yet detached)
      ::unlink(path.c_str());
      fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_EXCL, 0600);
      if (fd_ < 0) throw std::runtime_error("memif: cannot create " + path);
      bytes_ = region_bytes(ring_size, buf_size, rx_rings);
      if (ftruncate(fd_, (off_t)bytes_) != 0) { close(); throw std::runtime_error("memif: ftruncate " + path); }
    } else {
      fd_ = ::open(path.c_str(), O_RDWR);
      if (fd_ < 0) throw std::runtime_error("memif: cannot open " + path);
      struct stat st {};
      if (fstat(fd_, &st) != 0 || (size_t)st.st_size < sizeof(Hdr)) { close(); throw std::runtime_error("memif: bad region " + path); }
      bytes_ = (size_t)st.st_size;
    }
    // MAP_POPULATE: the page tables are filled now, not on the fast path (a first-touch fault
    // costs ~1-2 us in a VM, i.e. more than the whole per-frame budget)
    base_ = static_cast<uint8_t*>(mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd_, 0));
    if (base_ == MAP_FAILED) { base_ = nullptr; close(); throw std::runtime_error("memif: mmap " + path); }
    {
      struct stat st {};
      if (fstat(fd_, &st) == 0) { dev_ = (uint64_t)st.st_dev; ino_ = (uint64_t)st.st_ino; }
    }
    if (create) {
      std::memset(base_, 0, bytes_);   // allocates every page of the region up front
      hdr()->version = kVersion;
      hdr()->ring_size = ring_size;
      hdr()->buf_size = buf_size;
      hdr()->rx_rings = rx_rings;
      __atomic_store_n(&hdr()->magic, kMagic, __ATOMIC_RELEASE);   // publishes the geometry above
    } else {
      // the creator publishes the geometry with a release store of the magic: acquire the magic
      // FIRST, then read the geometry (once: the peer can rewrite the shared header at any time),
      // validate it against the mapping, and never look at the shared copy again
      const uint64_t magic = __atomic_load_n(&hdr()->magic, __ATOMIC_ACQUIRE);
      const uint32_t version = hdr()->version;
      ring_size = hdr()->ring_size;
      buf_size = hdr()->buf_size;
      rx_rings = hdr()->rx_rings;
      if (magic != kMagic || version != kVersion || ring_size < 2 || (ring_size & (ring_size - 1)) ||
          ring_size > (1u << 20) || buf_size < 64 || buf_size > (1u << 16) || rx_rings < 1 || rx_rings > kMaxRxRings ||
          bytes_ < region_bytes(ring_size, buf_size, rx_rings)) {
        close();
        throw std::runtime_error("memif: " + path + " is not a memif region");
      }
    }
    // private geometry: every index below is masked with these, so a peer that corrupts the
    // shared header or descriptors can at worst garble its own frames, never reach outside the map
    ring_size_ = ring_size;
    mask_ = ring_size - 1;
    buf_size_ = buf_size;
    nrings_ = 1 + rx_rings;
    desc_base_ = base_ + sizeof(Hdr) + (size_t)nrings_ * sizeof(Ctl);
    buf_base_ = desc_base_ + (size_t)nrings_ * ring_size * sizeof(Desc);
    path_ = path;
  }
  // The mapping and descriptor, handed over: this object no longer owns them (a region whose
  // memory must outlive it - still mapped for a GPU - is freed later through free()).
  struct Detached {
    uint8_t* base = nullptr;
    size_t bytes = 0;
    int fd = -1;
    void free() {
      if (base) munmap(base, bytes);
      base = nullptr;
      if (fd >= 0) ::close(fd);
      fd = -1;
    }
  };
  Detached detach() {
    Detached d{base_, bytes_, fd_};
    base_ = nullptr;
    fd_ = -1;
    return d;
  }
  void close() {
    if (base_) munmap(base_, bytes_);
    base_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }
  bool is_open() const { return base_ != nullptr; }
  const std::string& path() const { return path_; }
  // The path still names this region's file (not a newer region created at the same path).
  bool path_is_mine() const {
    struct stat st {};
    return !path_.empty() && ::stat(path_.c_str(), &st) == 0 && (uint64_t)st.st_dev == dev_ && (uint64_t)st.st_ino == ino_;
  }
  Hdr* hdr() const { return reinterpret_cast<Hdr*>(base_); }
  size_t bytes() const { return bytes_; }
  uint8_t* base() const { return base_; }
  // geometry: private snapshots taken at open (never re-read from the shared header)
  uint32_t ring_size() const { return ring_size_; }
  uint32_t mask() const { return mask_; }
  uint32_t buf_size() const { return buf_size_; }
  uint32_t rx_rings() const { return nrings_ - 1; }   // R
  // ring r (0: pod -> data plane, 1..R: data plane -> pod); out-of-range indices wrap
  Ctl* ctl(uint32_t r) const { return reinterpret_cast<Ctl*>(base_ + sizeof(Hdr)) + r % nrings_; }
  Desc* desc(uint32_t r) const { return reinterpret_cast<Desc*>(desc_base_) + (size_t)(r % nrings_) * ring_size_; }
  uint8_t* buf(uint32_t r, uint32_t slot) const {
    return buf_base_ + ((size_t)(r % nrings_) * ring_size_ + (slot & mask_)) * buf_size_;
  }

 private:
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  size_t bytes_ = 0;
  uint32_t ring_size_ = 0, mask_ = 0, buf_size_ = 0, nrings_ = 2;
  uint8_t* desc_base_ = nullptr;
  uint8_t* buf_base_ = nullptr;
  std::string path_;
  uint64_t dev_ = 0, ino_ = 0;   // the mapped file's identity
};

// Producer side of one ring: reserve -> fill buffer -> commit (batched head publication).
struct Producer {
  const Region* r = nullptr;
  uint32_t ring = 0;
  uint32_t head = 0;         // private copy (published with commit())
  uint32_t tail_cache = 0;   // last tail seen
  void init(const Region* reg, uint32_t rg) {
    r = reg; ring = rg;
    head = r->ctl(rg)->head.load(std::memory_order_relaxed);
    tail_cache = r->ctl(rg)->tail.load(std::memory_order_acquire);
  }
  uint32_t room() {
    if (head - tail_cache >= r->ring_size()) tail_cache = r->ctl(ring)->tail.load(std::memory_order_acquire);
    return r->ring_size() - (head - tail_cache);
  }
  // Write one frame assembled from up to three pieces; false when the ring is full or the frame
  // does not fit a buffer.
  bool put(const uint8_t* a, uint32_t na, const uint8_t* b = nullptr, uint32_t nb = 0, const uint8_t* c = nullptr,
           uint32_t nc = 0) {
    const uint32_t n = na + nb + nc;
    if (n > r->buf_size() || room() == 0) return false;
    uint8_t* dst = r->buf(ring, head);
    __builtin_prefetch(r->buf(ring, head + 8), 1, 3);   // the buffers of later puts: ownership requested early
    if (na) std::memcpy(dst, a, na);
    if (nb) std::memcpy(dst + na, b, nb);
    if (nc) std::memcpy(dst + na + nb, c, nc);
    Desc& d = r->desc(ring)[head & r->mask()];
    d.len = n;
    d.flags = 0;
    ++head;
    return true;
  }
  // A frame whose bytes are all in one 64-B slot (`src` holds 64 readable bytes, n <= 64): one
  // fixed-size 64-B copy into the buffer (>= 64 B) instead of a variable-length memcpy call.
  bool put_slot(const uint8_t* src, uint32_t n) {
    if (n > 64 || r->buf_size() < 64 || room() == 0) return false;
    uint8_t* dst = r->buf(ring, head);
    __builtin_prefetch(r->buf(ring, head + 8), 1, 3);
    std::memcpy(dst, src, 64);
    Desc& d = r->desc(ring)[head & r->mask()];
    d.len = n;
    d.flags = 0;
    ++head;
    return true;
  }
  void commit() { r->ctl(ring)->head.store(head, std::memory_order_release); }
};

// Consumer side of one ring.  `next` walks received frames; `release` hands slots back in order.
struct Consumer {
  const Region* r = nullptr;
  uint32_t ring = 0;
  uint32_t next = 0;         // next slot to read
  uint32_t head_cache = 0;
  uint32_t released = 0;     // slots below this went back to the producer
  void init(const Region* reg, uint32_t rg) {
    r = reg; ring = rg;
    next = released = r->ctl(rg)->tail.load(std::memory_order_relaxed);
    head_cache = r->ctl(rg)->head.load(std::memory_order_acquire);
  }
  // Frames ready to read.  Bounded by the ring: a producer that publishes a bogus head never
  // makes the consumer hold more than ring_size slots at once.
  uint32_t available() {
    if (head_cache == next) head_cache = r->ctl(ring)->head.load(std::memory_order_acquire);
    const uint32_t a = head_cache - next, room = r->ring_size() - (next - released);
    return a < room ? a : room;
  }
  // Frame at the read cursor (valid until released); advances the cursor.
  const uint8_t* get(uint32_t& len) {
    const Desc& d = r->desc(ring)[next & r->mask()];
    len = d.len < r->buf_size() ? d.len : r->buf_size();
    const uint8_t* p = r->buf(ring, next);
    __builtin_prefetch(r->buf(ring, next + 8), 0, 3);   // later frames' first line, fetched ahead
    ++next;
    return p;
  }
  // Return every slot below `upto` to the producer.
  void release_to(uint32_t upto) {
    released = upto;
    r->ctl(ring)->tail.store(upto, std::memory_order_release);
  }
};

}  // namespace memif
}  // namespace nfdp
