// mbox.cpp — shared-memory control mailbox (see mbox.h for the layout).
#include "mbox.h"

#include <linux/futex.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <climits>
#include <ctime>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstring>
#include <new>
#include <stdexcept>

namespace agent {

uint32_t Ring::cursor(const std::atomic<uint32_t>& c, std::memory_order mo) const {
  const uint32_t v = c.load(mo);
  if (v >= sz_ || (v & 7u)) {
    ctl_->prod.store(0, std::memory_order_relaxed);
    ctl_->cons.store(0, std::memory_order_release);
    throw std::runtime_error("mailbox: ring cursor out of range (ring corrupt)");
  }
  return v;
}

uint32_t Ring::used() const {
  const uint32_t sz = sz_;
  const uint32_t p = cursor(ctl_->prod, std::memory_order_acquire);
  const uint32_t c = cursor(ctl_->cons, std::memory_order_acquire);
  return (p + sz - c) % sz;
}

uint32_t Ring::space() const {
  const uint32_t u = used();
  return sz_ - u - 8;  // one 8-byte slot stays free: prod == cons <=> empty
}

void Ring::copy_in(uint32_t off, const void* src, uint32_t n) {
  const uint32_t sz = sz_;
  const uint32_t first = n < sz - off ? n : sz - off;
  std::memcpy(base_ + off, src, first);
  if (n > first) std::memcpy(base_, static_cast<const uint8_t*>(src) + first, n - first);
}

void Ring::copy_out(uint32_t off, void* dst, uint32_t n) const {
  const uint32_t sz = sz_;
  const uint32_t first = n < sz - off ? n : sz - off;
  std::memcpy(dst, base_ + off, first);
  if (n > first) std::memcpy(static_cast<uint8_t*>(dst) + first, base_, n - first);
}

bool Ring::push(const MsgHdr& h, const void* payload) {
  const uint32_t rec = (uint32_t)sizeof(MsgHdr) + align8(h.sz);
  if (rec > space()) return false;
  const uint32_t sz = sz_;
  const uint32_t p = cursor(ctl_->prod, std::memory_order_relaxed);
  copy_in(p, &h, sizeof(MsgHdr));
  if (h.sz) copy_in((p + (uint32_t)sizeof(MsgHdr)) % sz, payload, h.sz);
  ctl_->prod.store((p + rec) % sz, std::memory_order_release);
  ring();
  return true;
}

bool Ring::pop(Msg& out) {
  const uint32_t sz = sz_;
  const uint32_t c = cursor(ctl_->cons, std::memory_order_relaxed);
  const uint32_t p = cursor(ctl_->prod, std::memory_order_acquire);
  if (p == c) return false;
  copy_out(c, &out.hdr, sizeof(MsgHdr));
  const uint32_t avail = (p + sz - c) % sz;
  const uint32_t rec = (uint32_t)sizeof(MsgHdr) + align8(out.hdr.sz);
  if (rec > avail) {  // corrupt producer: drop everything rather than read garbage
    ctl_->cons.store(p, std::memory_order_release);
    throw std::runtime_error("mailbox: record larger than queued bytes (ring corrupt)");
  }
  out.data.resize(out.hdr.sz);
  if (out.hdr.sz) copy_out((c + (uint32_t)sizeof(MsgHdr)) % sz, out.data.data(), out.hdr.sz);
  ctl_->cons.store((c + rec) % sz, std::memory_order_release);
  return true;
}

static long futex(std::atomic<uint32_t>* w, int op, uint32_t val, const timespec* ts) {
  static_assert(sizeof(std::atomic<uint32_t>) == sizeof(uint32_t), "futex word");
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), op, val, ts, nullptr, 0);
}

void Ring::ring() {
  ctl_->bell.fetch_add(1, std::memory_order_seq_cst);
  if (!waiters_ || waiters_->load(std::memory_order_seq_cst) != 0) futex(&ctl_->bell, FUTEX_WAKE, INT32_MAX, nullptr);
}

bool Ring::wait_bell(uint32_t seen, int timeout_us) {
  if (bell() != seen) return true;
  if (timeout_us <= 0) return false;
  if (waiters_) waiters_->fetch_add(1, std::memory_order_seq_cst);
  if (bell() == seen) {
    timespec ts{timeout_us / 1000000, (long)(timeout_us % 1000000) * 1000};
    futex(&ctl_->bell, FUTEX_WAIT, seen, &ts);  // EAGAIN if it already moved, ETIMEDOUT, or woken
  }
  if (waiters_) waiters_->fetch_sub(1, std::memory_order_seq_cst);
  return bell() != seen;
}

void Ring::reset() {
  ctl_->prod.store(0, std::memory_order_relaxed);
  ctl_->cons.store(0, std::memory_order_release);
}

// ------------------------------------------------------------------------------------------------

static uint8_t* map_file(const std::string& path, uint32_t size, bool create) {
  const int fd = ::open(path.c_str(), create ? (O_RDWR | O_CREAT) : O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("mailbox: cannot open " + path);
  if (create && ::ftruncate(fd, size) != 0) {
    ::close(fd);
    throw std::runtime_error("mailbox: cannot size " + path);
  }
  void* m = ::mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) throw std::runtime_error("mailbox: mmap failed for " + path);
  return static_cast<uint8_t*>(m);
}

void Mailbox::bind() {
  auto* q = reinterpret_cast<QCtl*>(mem_ + kInfoBytes);
  Info& in = info();
  h2f_ = Ring(&q[0], mem_ + kHeaderBytes, qsz_, &in.h2f_waiters);
  f2h_ = Ring(&q[1], mem_ + kHeaderBytes + qsz_, qsz_, &in.f2h_waiters);
}

Mailbox Mailbox::create(const std::string& path, uint32_t size) {
  if (size <= kHeaderBytes) throw std::invalid_argument("mailbox: size must exceed the 288-byte header");
  const uint32_t qsz = ((size - kHeaderBytes) / 2) & ~7u;
  if (qsz < kMinQueueBytes) throw std::invalid_argument("mailbox: each queue needs at least 64 bytes");
  Mailbox mb;
  mb.path_ = path;
  mb.size_ = size;
  mb.qsz_ = qsz;
  mb.mem_ = map_file(path, size, true);
  std::memset(mb.mem_, 0, size);
  new (mb.mem_) Info();
  auto* q = reinterpret_cast<QCtl*>(mb.mem_ + kInfoBytes);
  new (&q[0]) QCtl();
  new (&q[1]) QCtl();
  q[0].sz = qsz;
  q[1].sz = qsz;
  mb.bind();
  Info& in = mb.info();
  in.region_sz.store(size, std::memory_order_relaxed);
  in.fw_version.store(((uint64_t)kCpVersionMin << 32) | kCpVersionMax, std::memory_order_relaxed);
  in.fw_status.store((uint64_t)Status::Init, std::memory_order_relaxed);
  in.magic.store(kMboxMagic, std::memory_order_release);
  return mb;
}

Mailbox Mailbox::open(const std::string& path) {
  struct stat st {};
  if (::stat(path.c_str(), &st) != 0) throw std::runtime_error("mailbox: no region at " + path);
  if ((uint64_t)st.st_size <= kHeaderBytes) throw std::runtime_error("mailbox: region too small");
  Mailbox mb;
  mb.path_ = path;
  mb.size_ = (uint32_t)st.st_size;
  mb.mem_ = map_file(path, mb.size_, false);
  if (mb.info().magic.load(std::memory_order_acquire) != kMboxMagic) {
    throw std::runtime_error("mailbox: bad magic (region not formatted by a control agent)");
  }
  // Both queue sizes come from the peer-writable region: they must agree, be 8-aligned, at least
  // kMinQueueBytes, and both rings must fit inside the mapping, or every later copy could run
  // past the region.
  const QCtl* q = reinterpret_cast<const QCtl*>(mb.mem_ + kInfoBytes);
  const uint32_t qsz = q[0].sz;
  if (qsz != q[1].sz || (qsz & 7u) || qsz < kMinQueueBytes ||
      (uint64_t)kHeaderBytes + 2ull * qsz > (uint64_t)mb.size_)
    throw std::runtime_error("mailbox: queue geometry does not fit the region (corrupt header)");
  mb.qsz_ = qsz;
  mb.bind();
  return mb;
}

void Mailbox::reset_rings() {
  h2f_.reset();
  f2h_.reset();
}

Mailbox::Mailbox(Mailbox&& o) noexcept { *this = std::move(o); }

Mailbox& Mailbox::operator=(Mailbox&& o) noexcept {
  if (this != &o) {
    if (mem_) ::munmap(mem_, size_);
    path_ = std::move(o.path_);
    mem_ = o.mem_;
    size_ = o.size_;
    qsz_ = o.qsz_;
    o.mem_ = nullptr;
    if (mem_) bind();
  }
  return *this;
}

Mailbox::~Mailbox() {
  if (mem_) ::munmap(mem_, size_);
}

}  // namespace agent
