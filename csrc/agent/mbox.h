// mbox.h — host <-> device control mailbox in shared memory.
//
// Role of the reference's BAR4 control mailbox (octep_ctrl_mbox.{h,c}, SURVEY NAT5/K15): a small
// info block plus two byte rings (host->fw "H2F", fw->host "F2H") carrying 16-byte-header
// messages.  On an MI355X node there is no PCIe endpoint between the host driver and the data
// plane's control agent — both are host processes — so the region is a MAP_SHARED file (tmpfs
// under /var/run/dpu-daemon) and every shared index is a lock-free std::atomic with
// acquire/release ordering instead of MMIO reads/writes through a BAR.
//
// Layout (all little-endian, offsets in bytes):
//   [0,256)    Info: magic, region size, host version/status/heartbeat, fw version/status/heartbeat
//   [256,272)  H2F ring control: prod, cons, size
//   [272,288)  F2H ring control
//   [288, 288+Q)       H2F ring bytes
//   [288+Q, 288+2Q)    F2H ring bytes,  Q = (size - 288) / 2 rounded down to 8
// A record = MsgHdr (16 B) + payload rounded up to 8 B; records wrap around the ring end byte by
// byte (the ring copy of K15).  One slot of 8 bytes is always kept free so prod == cons means
// empty unambiguously (the reference's |pi-ci| % sz arithmetic cannot tell full from empty).
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace agent {

constexpr uint64_t kMboxMagic = 0xdeaddeadbeefbeefull;
constexpr uint32_t kInfoBytes = 256;
constexpr uint32_t kQCtlBytes = 16;
constexpr uint32_t kHeaderBytes = kInfoBytes + 2 * kQCtlBytes;  // 288
constexpr uint32_t kMinQueueBytes = 64;

constexpr uint32_t version(uint32_t maj, uint32_t min, uint32_t pat) { return (maj << 16) | (min << 8) | pat; }
constexpr uint32_t kCpVersionMin = version(1, 0, 0);
constexpr uint32_t kCpVersionMax = version(1, 0, 1);

enum class Status : uint64_t { Invalid = 0, Init = 1, Ready = 2, Uninit = 3 };

enum MsgFlags : uint32_t { kFlagReq = 1u << 0, kFlagResp = 1u << 1, kFlagNotify = 1u << 2, kFlagCustom = 1u << 3 };

// 16-byte message header: function address (pem 4b | pf 9b | rsvd 2b | is_vf 1b), vf index,
// payload size, flags, id for matching responses.
struct MsgHdr {
  uint16_t fn;       // pem | pf << 4 | is_vf << 15
  uint16_t vf_idx;
  uint32_t sz;       // payload bytes (excluding header)
  uint32_t flags;
  uint16_t msg_id;
  uint16_t rsvd;

  static uint16_t make_fn(uint32_t pem, uint32_t pf, bool is_vf) {
    return (uint16_t)((pem & 0xF) | ((pf & 0x1FF) << 4) | (is_vf ? 0x8000 : 0));
  }
  uint32_t pem() const { return fn & 0xF; }
  uint32_t pf() const { return (fn >> 4) & 0x1FF; }
  bool is_vf() const { return (fn & 0x8000) != 0; }
};
static_assert(sizeof(MsgHdr) == 16, "message header is 16 bytes");

struct Msg {
  MsgHdr hdr{};
  std::vector<uint8_t> data;
};

// Info block as seen through atomics (the struct is placement-mapped onto the region).
struct alignas(8) Info {
  std::atomic<uint64_t> magic;          // 0
  std::atomic<uint64_t> region_sz;      // 8
  std::atomic<uint64_t> host_version;   // 16
  std::atomic<uint64_t> host_status;    // 24
  std::atomic<uint64_t> host_heartbeat; // 32
  std::atomic<uint64_t> host_resets;    // 40   host-requested resets ("PERST") so far
  std::atomic<uint32_t> h2f_waiters;    // 48   fw-side threads sleeping on the H2F doorbell
  std::atomic<uint32_t> f2h_waiters;    // 52   host-side threads sleeping on the F2H doorbell
  uint8_t pad0[136 - 56];
  std::atomic<uint64_t> fw_version;     // 136  min << 32 | max
  std::atomic<uint64_t> fw_status;      // 144
  std::atomic<uint64_t> fw_heartbeat;   // 152
  std::atomic<uint64_t> fw_resets;      // 160  resets the fw side has acknowledged
  std::atomic<uint64_t> fw_hb_interval; // 168  ms between heartbeat increments
  std::atomic<uint64_t> fw_hb_miss;     // 176  missed intervals after which the host declares fw dead
  uint8_t pad1[256 - 184];
};
static_assert(sizeof(Info) == kInfoBytes, "info block is 256 bytes");

struct alignas(8) QCtl {
  std::atomic<uint32_t> prod;
  std::atomic<uint32_t> cons;
  uint32_t sz;
  std::atomic<uint32_t> bell;  // doorbell: bumped on every push, futex word for sleeping consumers
};
static_assert(sizeof(QCtl) == kQCtlBytes, "queue control is 16 bytes");

// One direction of the mailbox.
//
// Doorbells (the role of the reference's OEI interrupt triggers, cnxk.c:177-230): the producer
// bumps `bell` after publishing a record and FUTEX_WAKEs only when the consumer side announced a
// sleeper in `waiters`; a consumer sleeps with FUTEX_WAIT on `bell` (a shared-mapping futex works
// across processes) instead of polling.  waiters++ / re-check / wait on the consumer and
// bell++ / check waiters on the producer, both seq_cst, cannot lose a wakeup.
class Ring {
 public:
  Ring() = default;
  // `sz` is the queue size validated by Mailbox::open/create; it is cached here so a peer that
  // rewrites the shared `sz` field cannot steer copies outside the region.
  Ring(QCtl* ctl, uint8_t* base, uint32_t sz, std::atomic<uint32_t>* waiters = nullptr)
      : ctl_(ctl), base_(base), sz_(sz), waiters_(waiters) {}
  uint32_t bell() const { return ctl_->bell.load(std::memory_order_seq_cst); }
  void ring();                                     // bump the doorbell, wake sleepers
  bool wait_bell(uint32_t seen, int timeout_us);   // true once bell != seen (woken or already)
  uint32_t size() const { return sz_; }
  uint32_t used() const;
  uint32_t space() const;  // bytes a producer may still write
  // Returns false (nothing written) when the record does not fit.
  bool push(const MsgHdr& h, const void* payload);
  // Returns false when empty.  `out.data` is resized to the payload size.
  bool pop(Msg& out);
  void reset();

 private:
  void copy_in(uint32_t off, const void* src, uint32_t n);
  void copy_out(uint32_t off, void* dst, uint32_t n) const;
  // Shared cursors are peer-writable: a cursor outside [0, sz) or not 8-aligned means the ring
  // is corrupt.  Resets the ring and throws (same path as an oversized record).
  uint32_t cursor(const std::atomic<uint32_t>& c, std::memory_order mo) const;
  QCtl* ctl_ = nullptr;
  uint8_t* base_ = nullptr;
  uint32_t sz_ = 0;
  std::atomic<uint32_t>* waiters_ = nullptr;
};

// A mapped mailbox region.  `create` formats a new region (fw side owns formatting, as the
// device does for BAR4); `open` maps an existing one.
class Mailbox {
 public:
  static Mailbox create(const std::string& path, uint32_t size);
  static Mailbox open(const std::string& path);
  Mailbox() = default;
  Mailbox(Mailbox&& o) noexcept;
  Mailbox& operator=(Mailbox&& o) noexcept;
  Mailbox(const Mailbox&) = delete;
  ~Mailbox();

  Info& info() const { return *reinterpret_cast<Info*>(mem_); }
  Ring& h2f() { return h2f_; }
  Ring& f2h() { return f2h_; }
  uint32_t size() const { return size_; }
  uint32_t queue_bytes() const { return qsz_; }
  const std::string& path() const { return path_; }
  bool valid() const { return mem_ != nullptr; }
  // Format rings (both empty) without touching host-owned info fields.
  void reset_rings();

 private:
  void bind();
  std::string path_;
  uint8_t* mem_ = nullptr;
  uint32_t size_ = 0;
  uint32_t qsz_ = 0;
  Ring h2f_, f2h_;
};

inline uint32_t align8(uint32_t x) { return (x + 7u) & ~7u; }

}  // namespace agent
