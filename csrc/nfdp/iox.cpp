// iox.cpp — native packet I/O engine (see iox.h).  Host code only: the GPU backend (the one part
// that calls HIP) is iox_gpu.cpp, so the engine, its ports and the oracle backend also build as
// plain C++ under ThreadSanitizer / AddressSanitizer (iox_stress.cpp, native/build.py).
#include "iox.h"

#include <arpa/inet.h>
#include <errno.h>
#include <immintrin.h>
#include <linux/if_ether.h>
#include <linux/if_packet.h>
#include <net/if.h>
#include <pthread.h>
#include <sched.h>
#include <sys/socket.h>

#include <algorithm>
#include <chrono>
#include <stdexcept>

namespace nfdp {
namespace iox {

namespace {
using Clock = std::chrono::steady_clock;
inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}
inline uint32_t pow2_at_least(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
// A frame's first h <= 64 bytes into a 64-B slot, the rest of the slot zeroed: four 16-B loads,
// masked, four stores (no libc memcpy / memset calls on the per-frame path).  Reads 64 bytes at
// src: every port's rx buffer holds at least that much (memif / AF_PACKET / AF_XDP frames 2048 B,
// TAP 9728 B) except the recirculation port's, which takes the plain copy.
inline void slot_copy(uint8_t* dst, const uint8_t* src, uint32_t h) {
  alignas(16) static const int8_t kIdx[64] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                                              16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,
                                              32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47,
                                              48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63};
  const __m128i lim = _mm_set1_epi8((char)h);
  for (int k = 0; k < 4; ++k) {
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 16 * k));
    const __m128i m = _mm_cmpgt_epi8(lim, _mm_load_si128(reinterpret_cast<const __m128i*>(kIdx + 16 * k)));
    _mm_storeu_si128(reinterpret_cast<__m128i*>(dst + 16 * k), _mm_and_si128(v, m));
  }
}

// outer-header bytes of a side-pass record (IPv6 underlay: 70, IPv4: 50; ethertype at 12..13)
inline uint32_t xhdr_len(const uint8_t* rec) { return (rec[12] == 0x86 && rec[13] == 0xDD) ? kEncap6Bytes : kEncapBytes; }
}  // namespace

// ---------------------------------------------------------------------------------- Port
Port::Port(uint32_t window) {
  const uint32_t w = pow2_at_least(std::max<uint32_t>(window, 2));
  done_.reset(new std::atomic<uint8_t>[w]);
  for (uint32_t i = 0; i < w; ++i) done_[i].store(0, std::memory_order_relaxed);
  mask_ = w - 1;
}

uint32_t Port::tx_batch(const TxItem* it, uint32_t n, uint32_t txq) {
  const uint32_t nq = std::min<uint32_t>(std::max<uint32_t>(tx_queues(), 1), kMaxTxQueues);
  const uint32_t q = txq % nq;
  uint32_t ok = 0;
  uint64_t bytes = 0;
  {
    std::lock_guard<std::mutex> g(tx_mu_[q].mu);
    for (uint32_t i = 0; i < n; ++i) {
      const TxItem& x = it[i];
      if (!tx_locked(q, x.a, x.na, x.b, x.nb, x.c, x.nc)) break;   // full: the rest of the batch finds no room either
      ++ok;
      bytes += x.na + x.nb + x.nc;
    }
    if (ok) flush_locked(q);
  }
  // one add per batch (several tx queues may count at once)
  auto add = [](std::atomic<uint64_t>& c, uint64_t v) {
    if (v) c.fetch_add(v, std::memory_order_relaxed);
  };
  add(tx_pkts, ok);
  add(tx_bytes, bytes);
  add(tx_full, n - ok);
  return ok;
}

void Port::reclaim() {
  uint32_t r = rel_;
  while (r != seen_ && done_[r & mask_].load(std::memory_order_acquire)) {
    done_[r & mask_].store(0, std::memory_order_relaxed);
    ++r;
  }
  if (r != rel_) {
    rel_ = r;
    release_to(r);
  }
}

// ---------------------------------------------------------------------------------- MemifPort
MemifPort::MemifPort(const std::string& path, uint32_t ring_size, uint32_t buf_size, uint32_t tx_rings)
    : Port(ring_size), reg_(path, true, ring_size, buf_size, std::min<uint32_t>(std::max<uint32_t>(tx_rings, 1), kMaxTxQueues)),
      unlink_(true) {
  nprod_ = reg_.rx_rings();
  prod_.reset(new Prod[nprod_]);
  cons_.init(&reg_, 0);
  for (uint32_t q = 0; q < nprod_; ++q) prod_[q].init(&reg_, 1 + q);
  set_first_seq(cons_.next);
}

MemifPort::~MemifPort() {
  if (unlink_ && reg_.path_is_mine()) ::unlink(reg_.path().c_str());   // (not a successor's file)
  if (rx_mapped()) {
    // mapped for the GPUs: the region's memory stays until that mapping is gone (deferred while
    // rings run), so it goes with the unmapping, not with this object
    auto mem = std::make_shared<memif::Region::Detached>(reg_.detach());
    unmap_rx([mem] { mem->free(); });
  }
}

uint32_t MemifPort::rx(RxRef* out, uint32_t max) {
  const uint32_t n = std::min(cons_.available(), max);
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t seq = cons_.next;
    uint32_t len = 0;
    const uint8_t* p = cons_.get(len);
    out[i] = RxRef{p, len, seq, ~0u};
  }
  return n;
}

// ---------------------------------------------------------------------------------- PacketPort
PacketPort::PacketPort(const std::string& ifname, uint32_t frames, uint32_t frame_size)
    : Port(frames), nframes_(pow2_at_least(frames)), fsize_(pow2_at_least(std::max<uint32_t>(frame_size, 2048))) {
  fd_ = ::socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
  if (fd_ < 0) throw std::runtime_error("iox: AF_PACKET socket (needs CAP_NET_RAW)");
  auto fail = [&](const char* what) {
    const int e = errno;
    if (map_) munmap(map_, map_bytes_);
    ::close(fd_);
    fd_ = -1;
    throw std::runtime_error(std::string("iox: ") + what + " on " + ifname + ": " + std::strerror(e));
  };
  int ver = TPACKET_V2;
  if (setsockopt(fd_, SOL_PACKET, PACKET_VERSION, &ver, sizeof(ver)) != 0) fail("PACKET_VERSION");
  int one = 1;
#ifdef PACKET_IGNORE_OUTGOING
  (void)setsockopt(fd_, SOL_PACKET, PACKET_IGNORE_OUTGOING, &one, sizeof(one));   // our own tx, older kernels filter below
#endif
  (void)setsockopt(fd_, SOL_PACKET, PACKET_QDISC_BYPASS, &one, sizeof(one));
  tpacket_req req{};
  req.tp_frame_size = fsize_;
  req.tp_block_size = std::max<uint32_t>(fsize_, 4096);
  req.tp_frame_nr = nframes_;
  req.tp_block_nr = nframes_ * fsize_ / req.tp_block_size;
  if (setsockopt(fd_, SOL_PACKET, PACKET_RX_RING, &req, sizeof(req)) != 0) fail("PACKET_RX_RING");
  if (setsockopt(fd_, SOL_PACKET, PACKET_TX_RING, &req, sizeof(req)) != 0) fail("PACKET_TX_RING");
  map_bytes_ = 2 * (size_t)nframes_ * fsize_;
  void* m = mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (m == MAP_FAILED) fail("mmap");
  map_ = static_cast<uint8_t*>(m);
  sockaddr_ll sll{};
  sll.sll_family = AF_PACKET;
  sll.sll_protocol = htons(ETH_P_ALL);
  sll.sll_ifindex = (int)if_nametoindex(ifname.c_str());
  if (sll.sll_ifindex == 0) fail("if_nametoindex");
  if (bind(fd_, reinterpret_cast<sockaddr*>(&sll), sizeof(sll)) != 0) fail("bind");
  // A bridge port sees every frame on its link, not only those for its own MAC: a NIC used as the
  // uplink filters unicast in hardware otherwise.  Membership-based (reference counted by the
  // kernel, dropped with the socket), so the netdev's own promiscuity setting is left alone.
  packet_mreq mr{};
  mr.mr_ifindex = sll.sll_ifindex;
  mr.mr_type = PACKET_MR_PROMISC;
  (void)setsockopt(fd_, SOL_PACKET, PACKET_ADD_MEMBERSHIP, &mr, sizeof(mr));
  vlan_copy_.resize((size_t)nframes_ * (fsize_ + 4));
}

PacketPort::~PacketPort() {
  if (map_) munmap(map_, map_bytes_);
  if (fd_ >= 0) ::close(fd_);
}

uint8_t* PacketPort::frame(int ring, uint32_t i) const {
  return map_ + ((size_t)ring * nframes_ + (i & (nframes_ - 1))) * fsize_;
}

uint32_t PacketPort::rx(RxRef* out, uint32_t max) {
  uint32_t n = 0;
  while (n < max) {
    auto* h = reinterpret_cast<tpacket2_hdr*>(frame(0, rx_next_));
    const uint32_t st = __atomic_load_n(&h->tp_status, __ATOMIC_ACQUIRE);
    if (!(st & TP_STATUS_USER)) break;
    const uint32_t seq = rx_next_++;
    const auto* sll = reinterpret_cast<const sockaddr_ll*>(reinterpret_cast<uint8_t*>(h) + TPACKET_ALIGN(sizeof(tpacket2_hdr)));
    const uint8_t* data = reinterpret_cast<uint8_t*>(h) + h->tp_mac;
    uint32_t len = h->tp_snaplen;
    if (sll->sll_pkttype == PACKET_OUTGOING || len < 14) {   // our own transmissions / runts: len 0 = skip
      out[n++] = RxRef{data, 0, seq, ~0u};
      continue;
    }
    if ((st & TP_STATUS_VLAN_VALID) && h->tp_vlan_tci && len + 4 <= fsize_) {
      // the kernel moved the 802.1Q tag into the aux data: put it back in front of the ethertype
      uint8_t* c = vlan_copy_.data() + (size_t)(seq & (nframes_ - 1)) * (fsize_ + 4);
      std::memcpy(c, data, 12);
      const uint16_t tpid = (st & TP_STATUS_VLAN_TPID_VALID) && h->tp_vlan_tpid ? h->tp_vlan_tpid : 0x8100;
      c[12] = tpid >> 8; c[13] = tpid & 0xFF;
      c[14] = h->tp_vlan_tci >> 8; c[15] = h->tp_vlan_tci & 0xFF;
      std::memcpy(c + 16, data + 12, len - 12);
      data = c;
      len += 4;
    }
    out[n++] = RxRef{data, len, seq, ~0u};
  }
  return n;
}

void PacketPort::release_to(uint32_t seq_end) {
  // frames [released .. seq_end) go back to the kernel
  for (uint32_t s = rel_done_; s != seq_end; ++s) {
    auto* h = reinterpret_cast<tpacket2_hdr*>(frame(0, s));
    __atomic_store_n(&h->tp_status, (uint32_t)TP_STATUS_KERNEL, __ATOMIC_RELEASE);
  }
  rel_done_ = seq_end;
}

bool PacketPort::tx_locked(uint32_t, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
  auto* h = reinterpret_cast<tpacket2_hdr*>(frame(1, tx_next_));
  uint32_t st = __atomic_load_n(&h->tp_status, __ATOMIC_ACQUIRE);
  if (st == TP_STATUS_WRONG_FORMAT) st = TP_STATUS_AVAILABLE;
  const uint32_t n = na + nb + nc;
  const size_t off = TPACKET2_HDRLEN - sizeof(sockaddr_ll);
  if (st != TP_STATUS_AVAILABLE || off + n > fsize_) return false;
  uint8_t* d = reinterpret_cast<uint8_t*>(h) + off;
  if (na) std::memcpy(d, a, na);
  if (nb) std::memcpy(d + na, b, nb);
  if (nc) std::memcpy(d + na + nb, c, nc);
  h->tp_len = n;
  __atomic_store_n(&h->tp_status, (uint32_t)TP_STATUS_SEND_REQUEST, __ATOMIC_RELEASE);
  ++tx_next_;
  return true;
}

void PacketPort::flush_locked(uint32_t) { (void)::sendto(fd_, nullptr, 0, MSG_DONTWAIT, nullptr, 0); }

// ---------------------------------------------------------------------------------- FdPort
FdPort::FdPort(int fd, uint32_t nbufs, uint32_t buf_size)
    : Port(nbufs), fd_(fd), nbufs_(pow2_at_least(nbufs)), bsize_(buf_size) {
  bufs_.resize((size_t)nbufs_ * bsize_);
  txbuf_.resize(bsize_ + 256);
}

uint32_t FdPort::rx(RxRef* out, uint32_t max) {
  uint32_t n = 0;
  while (n < max && next_ - freed_.load(std::memory_order_acquire) < nbufs_) {
    uint8_t* b = bufs_.data() + (size_t)(next_ & (nbufs_ - 1)) * bsize_;
    const ssize_t r = ::read(fd_, b, bsize_);
    if (r <= 0) break;   // EAGAIN (nothing pending) or EIO (netdev down)
    out[n++] = RxRef{b, (uint32_t)r, next_, ~0u};
    ++next_;
  }
  return n;
}

bool FdPort::tx_locked(uint32_t, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
  const uint32_t n = na + nb + nc;
  if (n > txbuf_.size()) return false;
  uint8_t* d = txbuf_.data();
  if (na) std::memcpy(d, a, na);
  if (nb) std::memcpy(d + na, b, nb);
  if (nc) std::memcpy(d + na + nb, c, nc);
  return ::write(fd_, d, n) == (ssize_t)n;
}

// ---------------------------------------------------------------------------------- RecircPort
void RecircPort::push(uint32_t in_port, const uint8_t* f, uint32_t n) {
  std::lock_guard<std::mutex> g(mu_);
  q_.emplace_back(in_port, std::vector<uint8_t>(f, f + n));
}

uint32_t RecircPort::rx(RxRef* out, uint32_t max) {
  std::lock_guard<std::mutex> g(mu_);
  uint32_t n = 0;
  while (n < max && !q_.empty() && live_.size() < window()) {
    live_.push_back(std::move(q_.front()));
    q_.pop_front();
    auto& e = live_.back();
    out[n++] = RxRef{e.second.data(), (uint32_t)e.second.size(), next_++, e.first};
  }
  return n;
}

void RecircPort::release_to(uint32_t seq_end) {
  std::lock_guard<std::mutex> g(mu_);
  while (base_ != seq_end && !live_.empty()) {
    live_.pop_front();
    ++base_;
  }
}

// ---------------------------------------------------------------------------------- Toeplitz tables
ToeplitzTab::ToeplitzTab(const uint8_t* rss_key) : tab((size_t)16 * 256) {
  // XOR-linear in the key bits: the hash of a key is the XOR of the hashes of its bytes alone
  for (int b = 0; b < 16; ++b)
    for (uint32_t v = 0; v < 256; ++v) {
      uint8_t raw[16] = {};
      raw[b] = (uint8_t)v;
      FlowKey k;
      std::memcpy(&k, raw, sizeof(k));
      tab[(size_t)b * 256 + v] = toeplitz_scalar(k, rss_key);
    }
}

namespace {
struct TabHash {   // side_stage's hasher: by pointer (the tables are 16 KiB)
  const ToeplitzTab* t;
  uint32_t operator()(const FlowKey& k) const { return (*t)(k); }
};

uint32_t owner_tab(const uint8_t* hdr, uint32_t len, uint32_t in_port, const PortEntry* ports, const ToeplitzTab& h,
                   uint32_t n, bool v6) {
  if (n <= 1) return 0;
  uint32_t d[kSlotDwords] = {};
  std::memcpy(d, hdr, std::min<uint32_t>(len, kSlotBytes));
  TablesView tv{};
  tv.ports = ports;
  tv.flow6_on = v6 ? 1u : 0u;   // IPv6 keys folded as the owners' tables hold them
  Parsed p;
  IngressState st;
  ingress_stage(tv, DirectTables{tv}, d, (in_port & 0xFFFFu) | (std::min<uint32_t>(len, kMaxFrame) << 16), p, st);
  if (!st.reason && (p.ipv4 || (v6 && p.ipv6))) return owner_of(h(st.key), n);
  return in_port % n;
}
}  // namespace

uint32_t frame_owner(const uint8_t* hdr, uint32_t len, uint32_t in_port, const PortEntry* ports, const uint8_t* rss_key,
                     uint32_t n, bool v6) {
  if (n <= 1) return 0;
  if (!ports || !rss_key) return in_port % n;
  uint32_t d[kSlotDwords] = {};
  std::memcpy(d, hdr, std::min<uint32_t>(len, kSlotBytes));
  TablesView tv{};
  tv.ports = ports;
  tv.flow6_on = v6 ? 1u : 0u;
  Parsed p;
  IngressState st;
  ingress_stage(tv, DirectTables{tv}, d, (in_port & 0xFFFFu) | (std::min<uint32_t>(len, kMaxFrame) << 16), p, st);
  if (!st.reason && (p.ipv4 || (v6 && p.ipv6))) return owner_of(toeplitz_scalar(st.key, rss_key), n);
  return in_port % n;
}

// ---------------------------------------------------------------------------------- SideTables
SideTables::SideTables(const Src& s) {
  ports_.assign((size_t)kMaxPorts + 2, PortEntry{});
  if (s.ports) std::memcpy(ports_.data(), s.ports, std::min<size_t>(s.n_ports, kMaxPorts) * sizeof(PortEntry));
  if (s.macs && s.mac_mask != ~0u && ((s.mac_mask + 1) & s.mac_mask) == 0)
    macs_.assign(s.macs, s.macs + (size_t)s.mac_mask + 1);
  if (s.lag && s.n_lag_groups) lag_.assign(s.lag, s.lag + (size_t)s.n_lag_groups * kLagWays);
  if (s.flood && s.n_flood) {
    // every row a link can name (< kFloodMaxRows) exists in the copy: side_stage follows links
    // without knowing how many rows the control plane allocated
    flood_.assign((size_t)std::max<size_t>(s.flood_rows, kFloodMaxRows) * kFloodWays, (uint16_t)kPortNone);
    std::memcpy(flood_.data(), s.flood, s.flood_rows * kFloodWays * sizeof(uint16_t));
  }
  if (s.tunnels && s.n_tunnels) tun_.assign(s.tunnels, s.tunnels + s.n_tunnels);
  if (s.tunnels6 && s.n_tunnels6) tun6_.assign(s.tunnels6, s.tunnels6 + s.n_tunnels6);
  rss_.assign(64, 0);
  if (s.rss_key) std::memcpy(rss_.data(), s.rss_key, 52);
  hash_ = ToeplitzTab(rss_.data());
  t_.ports = ports_.data();
  t_.macs = macs_.empty() ? nullptr : macs_.data();
  t_.mac_mask = macs_.empty() ? 0 : s.mac_mask;
  t_.rss_key = rss_.data();
  t_.lag_members = lag_.empty() ? nullptr : lag_.data();
  t_.n_lag_groups = lag_.empty() ? 0 : s.n_lag_groups;
  t_.flood = flood_.empty() ? nullptr : flood_.data();
  t_.n_flood = flood_.empty() ? 0 : s.n_flood;
  t_.tunnels = tun_.empty() ? nullptr : tun_.data();
  t_.n_tunnels = (uint32_t)tun_.size();
  t_.tunnels6 = tun6_.empty() ? nullptr : tun6_.data();
  t_.n_tunnels6 = (uint32_t)tun6_.size();
  t_.flow6_on = s.v6 ? 1u : 0u;   // the key fold only (make_key): the side pass never probes flows
}

// ---------------------------------------------------------------------------------- OracleBackend
OracleBackend::OracleBackend(uint32_t capacity, uint32_t queues) : cap_(capacity), nq_(queues) {
  if (capacity < 64 || (capacity & (capacity - 1))) throw std::invalid_argument("iox: oracle capacity: power of two >= 64");
  if (queues < 1 || queues > 64) throw std::invalid_argument("iox: oracle queues in [1, 64]");
  in_.assign((size_t)cap_ * nq_ * kSlotBytes, 0);
  out_.assign((size_t)cap_ * nq_ * kSlotBytes, 0);
  im_.assign((size_t)cap_ * nq_, 0);
  om_.assign((size_t)cap_ * nq_, 0);
  prod_.reset(new std::atomic<uint64_t>[nq_]);
  for (uint32_t q = 0; q < nq_; ++q) prod_[q].store(0);
}

void OracleBackend::configure(const TablesView& t, uint64_t* flow_ctr, uint64_t* port_ctr, uint64_t* drop_ctr,
                              MacEntry* macs, uint32_t mac_mask) {
  std::lock_guard<std::mutex> g(run_mu_);
  t_ = t; flow_ctr_ = flow_ctr; port_ctr_ = port_ctr; drop_ctr_ = drop_ctr;
  macs_ = macs; mac_mask_ = mac_mask;
  configured_ = true;
}

void OracleBackend::run_segment(uint32_t q, uint32_t pos, uint32_t n) {
  const size_t p = (size_t)q * cap_ + (pos & (cap_ - 1));
  oracle_run(t_, reinterpret_cast<const uint32_t*>(in_.data() + p * kSlotBytes), im_.data() + p, n,
             reinterpret_cast<uint32_t*>(out_.data() + p * kSlotBytes), om_.data() + p, flow_ctr_, port_ctr_,
             drop_ctr_, nullptr, nullptr, nullptr);
}

void OracleBackend::set_frame_addrs(bool on) {
  if (!on) { fa_.clear(); return; }
  fa_.resize((size_t)cap_ * nq_);
  for (size_t i = 0; i < fa_.size(); ++i) fa_[i] = reinterpret_cast<uint64_t>(in_.data() + i * kSlotBytes);
}

uint64_t OracleBackend::publish(uint32_t q, uint32_t n) {
  if (!configured_) throw std::runtime_error("iox: oracle backend not configured");
  if (q >= nq_) throw std::invalid_argument("iox: no such queue");
  if (n == 0 || (n & 63u) || n > cap_) throw std::invalid_argument("iox: publish a multiple of 64 packets");
  const uint64_t prod = prod_[q].load(std::memory_order_relaxed);
  uint32_t* im = in_meta(q);
  uint32_t* om = om_.data() + (size_t)q * cap_;
  // real packets first, filler slots (kRingPadMeta) at the end of the publish: run the prefix
  uint32_t real = 0;
  while (real < n && im[(prod + real) & (cap_ - 1)] != kRingPadMeta) ++real;
  for (uint32_t i = real; i < n; ++i) om[(prod + i) & (cap_ - 1)] = make_meta(kPortNone, 0, kMalformed);
  if (!fa_.empty()) {
    // what the GPU ring does in frame-address mode: each frame from where its address points,
    // the bytes past its length zero
    for (uint32_t i = 0; i < n; ++i) {
      const size_t pos = (size_t)q * cap_ + ((prod + i) & (cap_ - 1));
      uint8_t* slot = in_.data() + pos * kSlotBytes;
      const uint8_t* src = reinterpret_cast<const uint8_t*>(fa_[pos]);
      if (src == slot) continue;
      const uint32_t len = i < real ? std::min<uint32_t>(im_[pos] >> 16, kSlotBytes) : 0u;
      std::memcpy(slot, src, len);
      std::memset(slot + len, 0, kSlotBytes - len);
    }
  }
  {
    std::unique_lock<std::mutex> g(run_mu_, std::defer_lock);
    if (serial_) g.lock();
    uint32_t done = 0;
    while (done < real) {
      const uint32_t p = (uint32_t)((prod + done) & (cap_ - 1));
      const uint32_t k = std::min(real - done, cap_ - p);   // contiguous piece (a wrap splits it)
      run_segment(q, p, k);
      done += k;
    }
  }
  prod_[q].store(prod + n, std::memory_order_release);
  return prod + n;
}

void OracleBackend::apply_learn(const uint32_t* ev, uint32_t n, uint32_t stamp) {
  std::lock_guard<std::mutex> g(run_mu_);
  if (macs_ && n) mac_learn_cpu(macs_, mac_mask_, ev, n, stamp);
}

// ---------------------------------------------------------------------------------- WireBackend
namespace {
inline uint32_t mac_slot(uint64_t k, uint32_t mask) { return (uint32_t)((k * 0x9E3779B97F4A7C15ull) >> 40) & mask; }
}  // namespace

WireBackend::WireBackend(uint32_t capacity, uint32_t queues, const std::vector<std::pair<uint64_t, uint32_t>>& m)
    : OracleBackend(capacity, queues) {
  tmask_ = pow2_at_least(std::max<uint32_t>(16, (uint32_t)m.size() * 4)) - 1;
  tab_.assign((size_t)tmask_ + 1, {0, 0});
  for (const auto& e : m) {
    const uint64_t k = (e.first & 0xFFFFFFFFFFFFull) + 1;
    uint32_t i = mac_slot(k, tmask_);
    while (tab_[i].first && tab_[i].first != k) i = (i + 1) & tmask_;
    tab_[i] = {k, e.second};
  }
  serial_ = false;   // no shared state: queues run in parallel
  configure(TablesView{}, nullptr, nullptr, nullptr, nullptr, 0);
}

void WireBackend::run_segment(uint32_t q, uint32_t pos, uint32_t n) {
  const size_t p = (size_t)q * cap_ + (pos & (cap_ - 1));
  std::memcpy(out_.data() + p * kSlotBytes, in_.data() + p * kSlotBytes, (size_t)n * kSlotBytes);
  for (uint32_t i = 0; i < n; ++i) {
    const uint8_t* f = in_.data() + (p + i) * kSlotBytes;
    uint64_t k = 0;
    std::memcpy(&k, f, 6);
    k += 1;
    const uint32_t len = im_[p + i] >> 16;
    uint32_t j = mac_slot(k, tmask_), port = kPortNone;
    while (tab_[j].first) {
      if (tab_[j].first == k) { port = tab_[j].second; break; }
      j = (j + 1) & tmask_;
    }
    om_[p + i] = port == kPortNone ? make_meta(kPortNone, 0, kMalformed) : make_meta(port, len, kOk);
  }
}

// ---------------------------------------------------------------------------------- Engine
Engine::Engine(uint32_t burst, uint32_t inflight, uint32_t tx_workers, uint32_t queues, uint32_t max_inflight_frames)
    : burst_(burst), inflight_(std::max<uint32_t>(inflight, 1)), workers_(std::max<uint32_t>(tx_workers, 1)),
      nq_(queues), max_frames_(max_inflight_frames), inline_tx_(tx_workers == 0) {
  if (burst_ < 1 || burst_ > (1u << 16)) throw std::invalid_argument("iox: burst in [1, 65536]");
  if (workers_ > 16) throw std::invalid_argument("iox: at most 16 tx workers per queue");
  if (nq_ < 1 || nq_ > 64) throw std::invalid_argument("iox: queues in [1, 64]");
  if (max_frames_ && max_frames_ < 64) throw std::invalid_argument("iox: max_inflight_frames >= 64 (or 0: ring capacity)");
  ports_ = std::make_shared<PortTab>((size_t)kMaxPorts + 2);
  auto c = std::make_shared<Cfg>();
  c->redirect.assign((size_t)kMaxPorts + 2, 0xFFFFFFFFu);
  c->side_ports.assign((size_t)kMaxPorts + 2, 0);
  cfg_ = c;
  recirc_ = std::make_shared<RecircPort>(4096);
  for (uint32_t q = 0; q < nq_; ++q) {
    auto Q = std::make_unique<Queue>();
    Q->id = q;
    Q->wst.reset(new QStats[workers_]);
    Q->side_ctr.reset(new std::atomic<uint64_t>[(size_t)2 * kMaxPorts]);
    for (size_t i = 0; i < (size_t)2 * kMaxPorts; ++i) Q->side_ctr[i].store(0);
    Q->side_drop.reset(new std::atomic<uint64_t>[kNumReasons]);
    for (int i = 0; i < kNumReasons; ++i) Q->side_drop[i].store(0);
    queues_.push_back(std::move(Q));
  }
}

Engine::~Engine() {
  try {
    stop();
  } catch (...) {
  }
}

template <class F>
void Engine::update_cfg(F f) {
  std::lock_guard<std::mutex> g(cfg_mu_);
  auto c = std::make_shared<Cfg>(*std::atomic_load(&cfg_));
  f(*c);
  std::atomic_store(&cfg_, std::shared_ptr<const Cfg>(c));
  cfg_ver_.fetch_add(1, std::memory_order_release);
}

void Engine::add_backend(std::shared_ptr<Backend> b) {
  if (run_) throw std::runtime_error("iox: add backends before start()");
  if (b->queues() < nq_) throw std::invalid_argument("iox: the backend has fewer ring queues than the engine");
  const uint32_t g = (uint32_t)backends_.size();
  backends_.push_back(b);
  for (uint32_t q = 0; q < nq_; ++q) {
    auto L = std::make_unique<Lane>();
    L->be = b;
    L->q = q;
    L->g = g;
    L->slots.reset(new Burst[inflight_]);
    queues_[q]->lanes.push_back(L.get());
    lanes_.push_back(std::move(L));
  }
  update_cfg([&](Cfg& c) { c.side.resize(backends_.size()); });
}

void Engine::add_port(uint32_t id, std::shared_ptr<Port> p, int queue) {
  if (id >= (uint32_t)kMaxPorts) throw std::invalid_argument("iox: port id out of range");
  std::lock_guard<std::mutex> g(ports_mu_);
  auto t = std::make_shared<PortTab>(*ports_);
  if ((*t)[id].p) queues_[(*t)[id].q]->nports.fetch_sub(1);
  uint32_t q = 0;
  if (queue >= 0) {
    q = (uint32_t)queue % nq_;
  } else {   // least loaded queue
    for (uint32_t k = 1; k < nq_; ++k)
      if (queues_[k]->nports.load() < queues_[q]->nports.load()) q = k;
  }
  if (gde_.load() && (*t)[id].p) {
    // a port replaced at this id: its GPU egress entry off (applied by every grid), then every
    // chunk published before the clear must be through - one that read the old entry could still
    // be reserving in it and would advance the new entry's head over slots it never wrote
    gde_unregister(id);
    if (run_.load()) {
      std::vector<uint64_t> heads(lanes_.size());
      for (size_t k = 0; k < lanes_.size(); ++k) heads[k] = lanes_[k]->head.load(std::memory_order_acquire);
      const auto t0 = Clock::now();
      for (;;) {
        bool done = true;
        for (size_t k = 0; k < lanes_.size() && done; ++k) done = lanes_[k]->done.load(std::memory_order_acquire) >= heads[k];
        if (done || !run_.load()) break;
        if (Clock::now() - t0 > std::chrono::seconds(5)) throw std::runtime_error("iox: bursts before a port replacement did not finish");
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    }
  }
  if (zero_copy_.load()) map_port(*p);   // before any packet thread can see the port
  if (gde_.load()) gde_register(id, *p);
  reap_retired(false);
  (*t)[id] = PortRef{std::move(p), q};
  queues_[q]->nports.fetch_add(1);
  std::atomic_store(&ports_, std::shared_ptr<const PortTab>(t));
  ports_ver_.fetch_add(1, std::memory_order_release);
}

std::shared_ptr<Port> Engine::remove_port(uint32_t id) {
  if (id >= (uint32_t)kMaxPorts) return nullptr;
  std::lock_guard<std::mutex> g(ports_mu_);
  auto t = std::make_shared<PortTab>(*ports_);
  auto old = (*t)[id].p;
  if (old) queues_[(*t)[id].q]->nports.fetch_sub(1);
  // GPU-direct egress off for it first, applied by every grid: chunks published from here on
  // leave its frames to the host path (which finds no port); earlier ones are waited for below
  if (old && gde_.load()) gde_unregister(id);
  (*t)[id] = PortRef{};
  std::atomic_store(&ports_, std::shared_ptr<const PortTab>(t));
  ports_ver_.fetch_add(1, std::memory_order_release);
  // Frames of it may still be in a pipeline (an rx thread's snapshot still lists it until its
  // next loop, bursts in flight point into its rx memory — mapped for the GPU with zero-copy rx):
  // the engine keeps the port alive until no burst can refer to it (reap_retired), or until stop().
  if (old) retired_.push_back(Retired{ports_ver_.load(), {}, old});
  reap_retired(false);
  return old;
}

void Engine::reap_retired(bool all) {
  if (all || !run_.load()) {   // (stopped: every burst was delivered or handed back)
    retired_.clear();
    return;
  }
  for (auto& r : retired_) {
    if (!r.heads.empty()) continue;
    bool seen = true;
    for (auto& Q : queues_) seen = seen && Q->ports_seen.load(std::memory_order_acquire) >= r.ver;
    if (!seen) break;          // (versions only grow: later entries are not seen either)
    r.heads.resize(lanes_.size());
    for (size_t k = 0; k < lanes_.size(); ++k) r.heads[k] = lanes_[k]->head.load(std::memory_order_acquire);
  }
  while (!retired_.empty() && !retired_.front().heads.empty()) {
    const auto& h = retired_.front().heads;
    bool done = true;
    for (size_t k = 0; k < lanes_.size() && done; ++k) done = lanes_[k]->done.load(std::memory_order_acquire) >= h[k];
    if (!done) break;
    retired_.pop_front();
  }
}

size_t Engine::retired_ports() {
  std::lock_guard<std::mutex> g(ports_mu_);
  reap_retired(false);
  return retired_.size();
}

void Engine::map_port(Port& p) {
  const auto mem = p.rx_memory();
  if (!mem.first || !mem.second || p.zc_.lo) return;
  if (p.zc_.release && p.zc_.off.size() == backends_.size()) {   // still mapped from before
    p.zc_.lo = mem.first;
    p.zc_.hi = mem.first + mem.second;
    return;
  }
  Port::Mapped m;
  m.off.assign(backends_.size(), 0);
  for (size_t g = 0; g < backends_.size(); ++g) {
    std::function<void(std::function<void()>)> rel;
    const uint64_t a = backends_[g]->map_host(mem.first, mem.second, &rel);
    if (rel) m.release = std::move(rel);   // (at most one backend registers: the first)
    if (!a) {   // a backend cannot read it: the port's frames are copied, as without the mode
      if (m.release) m.release(nullptr);
      return;
    }
    m.off[g] = (int64_t)(a - reinterpret_cast<uint64_t>(mem.first));
  }
  m.lo = mem.first;
  m.hi = mem.first + mem.second;
  p.zc_ = std::move(m);
}

void Engine::gde_register(uint32_t id, Port& p) {
  auto* mp = dynamic_cast<MemifPort*>(&p);
  if (!mp) return;
  const memif::Region& reg = mp->region();
  // the region mapped for every backend (the zero-copy rx mapping: it covers the whole region);
  // without zero-copy rx the rx path keeps copying (lo / hi cleared)
  const bool had = p.zc_.lo != nullptr;
  map_port(p);
  if (p.zc_.off.size() != backends_.size()) return;   // some backend cannot reach it
  if (!zero_copy_.load() && !had) p.zc_.lo = p.zc_.hi = nullptr;
  for (size_t k = 0; k < lanes_.size(); ++k) {
    Lane* L = lanes_[k].get();
    const uint32_t r = 1u + nq_ + (uint32_t)k;
    if (!L->be->gde_ok() || r > reg.rx_rings()) continue;
    const int64_t off = p.zc_.off[L->g];
    auto dev = [&](const void* h) { return (uint64_t)((int64_t)reinterpret_cast<uint64_t>(h) + off); };
    memif::Ctl* c = reg.ctl(r);
    L->be->gde_set(id, L->q, dev(c), dev(reg.desc(r)), dev(reg.buf(r, 0)), reg.ring_size(), reg.buf_size(),
                   c->head.load(std::memory_order_acquire), c->tail.load(std::memory_order_acquire));
  }
}

void Engine::gde_unregister(uint32_t id) {
  for (size_t k = 0; k < lanes_.size(); ++k) {
    Lane* L = lanes_[k].get();
    if (!L->be->gde_ok()) continue;
    const uint64_t seq = L->be->gde_clear(id, L->q);
    if (seq && !L->be->gde_wait(seq, 2.0)) throw std::runtime_error("iox: a grid did not apply the egress removal");
  }
}

void Engine::set_gpu_egress(bool on) {
  if (run_) throw std::runtime_error("iox: set_gpu_egress while running");
  std::lock_guard<std::mutex> g(ports_mu_);
  gde_ = on;
  for (uint32_t id = 0; id < ports_->size(); ++id) {
    const PortRef& r = (*ports_)[id];
    if (!r.p) continue;
    if (on) gde_register(id, *r.p);
    else gde_unregister(id);
  }
}

void Engine::set_zero_copy(bool on) {
  if (run_) throw std::runtime_error("iox: set_zero_copy while running");
  std::lock_guard<std::mutex> g(ports_mu_);
  zero_copy_ = on;
  for (const PortRef& r : *ports_) {
    if (!r.p) continue;
    if (on) map_port(*r.p);
    else r.p->zc_.lo = r.p->zc_.hi = nullptr;   // copied from now on (the mapping stays with the port)
  }
}

std::shared_ptr<Port> Engine::port(uint32_t id) {
  auto t = std::atomic_load(&ports_);
  return id < t->size() ? (*t)[id].p : nullptr;
}

int Engine::port_queue(uint32_t id) {
  auto t = std::atomic_load(&ports_);
  return id < t->size() && (*t)[id].p ? (int)(*t)[id].q : -1;
}

void Engine::set_steering(const std::vector<PortEntry>& ports, const std::vector<uint8_t>& rss_key, bool v6,
                          const std::vector<uint32_t>& port_owner) {
  if (rss_key.size() < 20) throw std::invalid_argument("iox: rss key too short");
  auto s = std::make_shared<Steer>();
  s->port_owner = port_owner;
  s->ports = ports;
  s->ports.resize((size_t)kMaxPorts + 2);
  s->rss_key = rss_key;
  s->rss_key.resize(std::max<size_t>(rss_key.size(), 64), 0);
  s->v6 = v6;
  s->hash = ToeplitzTab(s->rss_key.data());
  update_cfg([&](Cfg& c) { c.steer = s; });
}

void Engine::set_redirects(const std::vector<std::pair<uint32_t, uint32_t>>& m) {
  update_cfg([&](Cfg& c) {
    c.redirect.assign((size_t)kMaxPorts + 2, 0xFFFFFFFFu);
    for (const auto& e : m)
      if (e.first < c.redirect.size()) c.redirect[e.first] = e.second;
  });
}

void Engine::set_redirect(uint32_t port, uint32_t underlay) {
  update_cfg([&](Cfg& c) {
    if (port < c.redirect.size()) c.redirect[port] = underlay;
  });
}

void Engine::set_side_ports(const std::vector<uint32_t>& ports) {
  update_cfg([&](Cfg& c) {
    c.side_ports.assign((size_t)kMaxPorts + 2, 0);
    for (uint32_t p : ports)
      if (p < c.side_ports.size()) c.side_ports[p] = 1;
  });
}

void Engine::set_side_always(bool on) {
  update_cfg([&](Cfg& c) { c.side_always = on; });
}

void Engine::set_side_tables(uint32_t backend, std::shared_ptr<SideTables> t) {
  update_cfg([&](Cfg& c) {
    if (backend >= c.side.size()) c.side.resize(backend + 1);
    c.side[backend] = std::move(t);
  });
}

uint32_t Engine::owner(const Steer* s, uint32_t n, const uint8_t* f, uint32_t len, uint32_t in_port) {
  if (n <= 1) return 0;
  if (!s) return in_port % n;
  if (!s->port_owner.empty())   // port placement: the ingress port's GPU (hop-affine chains)
    return in_port < s->port_owner.size() ? s->port_owner[in_port] % n : in_port % n;
  return owner_tab(f, len, in_port, s->ports.data(), s->hash, n, s->v6);
}

uint32_t Engine::owner_of_frame(const uint8_t* f, uint32_t len, uint32_t in_port) const {
  return owner(cfg()->steer.get(), (uint32_t)backends_.size(), f, len, in_port);
}

void Engine::start() {
  if (run_) return;
  if (backends_.empty()) throw std::runtime_error("iox: no backend");
  {
    std::lock_guard<std::mutex> g(err_mu_);
    err_.clear();
  }
  abandon_ = false;
  run_ = true;
  learner_run_ = true;
  for (auto& L : lanes_) {
    const uint64_t p = L->be->published(L->q);
    L->freed_pos.store(p);
  }
  learner_ = std::thread(&Engine::learner_loop, this);
  for (auto& Q : queues_) {
    for (uint32_t w = 0; w < (inline_tx_ ? 0u : workers_); ++w) {
      Q->tx.emplace_back(&Engine::tx_loop, this, Q.get(), w);
      pin(Q->tx.back(), Q->cpus);
    }
    Q->rx = std::thread(&Engine::rx_loop, this, Q.get());
    pin(Q->rx, Q->cpus);
  }
}

void Engine::pin(std::thread& t, const std::vector<int>& cpus) {
  if (cpus.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus)
    if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
  (void)pthread_setaffinity_np(t.native_handle(), sizeof(set), &set);   // best effort (a cpuset may refuse)
}

void Engine::set_queue_cpus(uint32_t q, const std::vector<int>& cpus) {
  if (q >= nq_) throw std::invalid_argument("iox: no such queue");
  if (run_) throw std::runtime_error("iox: queue CPUs are set before start()");
  queues_[q]->cpus = cpus;
}

bool Engine::lanes_idle() const {
  for (auto& L : lanes_)
    if (L->done.load(std::memory_order_acquire) != L->head.load(std::memory_order_acquire)) return false;
  return true;
}

void Engine::stop() {
  run_ = false;
  for (auto& Q : queues_)
    if (Q->rx.joinable()) Q->rx.join();
  // the tx workers deliver what was published; a pipeline that stopped completing is abandoned
  const auto t0 = Clock::now();
  while (!lanes_idle() && !abandon_.load() && Clock::now() - t0 < std::chrono::seconds(10))
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  abandon_ = true;
  for (auto& Q : queues_) {
    for (auto& t : Q->tx)
      if (t.joinable()) t.join();
    Q->tx.clear();
  }
  {
    std::lock_guard<std::mutex> g(learn_mu_);
    learner_run_ = false;
  }
  learn_cv_.notify_all();
  if (learner_.joinable()) learner_.join();
  // frames of abandoned bursts go back to their ports (a rebuilt engine reuses the ports)
  for (auto& L : lanes_) {
    for (uint32_t k = 0; k < inflight_; ++k) {
      Burst& b = L->slots[k];
      if (b.state.load() != 0) {
        for (const Pkt& q : b.pkts) q.holder->complete(q.seq);
        b.pkts.clear();
        b.reps.clear();
        b.cfg.reset();
        b.state.store(0);
      }
    }
    L->done.store(L->head.load());
    for (const Pkt& q : L->stage) q.holder->complete(q.seq);   // read but never published
    L->stage.clear();
  }
  std::lock_guard<std::mutex> g(ports_mu_);
  reap_retired(true);
}

void Engine::pause() {
  ctl_epoch_.fetch_add(1);
  pause_n_.fetch_add(1);
  if (!run_) return;
  const uint64_t want = ctl_epoch_.load();
  const auto t0 = Clock::now();
  for (;;) {
    bool idle = true;
    for (auto& Q : queues_) idle = idle && Q->held_epoch.load(std::memory_order_acquire) >= want;
    idle = idle && lanes_idle();
    if (idle || !run_) return;
    if (Clock::now() - t0 > std::chrono::seconds(10)) throw std::runtime_error("iox: pause timed out");
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void Engine::resume() {
  if (pause_n_.load() > 0) pause_n_.fetch_sub(1);
}

void Engine::hold() {
  ctl_epoch_.fetch_add(1);
  hold_n_.fetch_add(1);
  if (!run_) return;
  const uint64_t want = ctl_epoch_.load();
  const auto t0 = Clock::now();
  for (;;) {
    bool held = true;
    for (auto& Q : queues_) held = held && Q->held_epoch.load(std::memory_order_acquire) >= want;
    if (held || !run_) return;
    if (Clock::now() - t0 > std::chrono::seconds(10)) throw std::runtime_error("iox: hold timed out");
    _mm_pause();
  }
}

void Engine::release() {
  if (hold_n_.load() > 0) hold_n_.fetch_sub(1);
}

std::string Engine::error() const {
  std::lock_guard<std::mutex> g(err_mu_);
  return err_;
}

void Engine::fail(const std::string& what) {
  {
    std::lock_guard<std::mutex> g(err_mu_);
    if (err_.empty()) err_ = what;
  }
  run_ = false;
  abandon_ = true;
}

std::vector<Punt> Engine::take_punts(size_t max) {
  std::lock_guard<std::mutex> g(punt_mu_);
  std::vector<Punt> v;
  while (!punts_.empty() && v.size() < max) {
    v.push_back(std::move(punts_.front()));
    punts_.pop_front();
  }
  return v;
}

std::vector<double> Engine::take_latency_us() {
  std::vector<double> v;
  for (auto& Q : queues_) {
    std::lock_guard<std::mutex> g(Q->lat_mu);
    v.insert(v.end(), Q->lat_us.begin(), Q->lat_us.end());
    Q->lat_us.clear();
  }
  return v;
}

std::unordered_map<std::string, uint64_t> Engine::stats() const {
  std::unordered_map<std::string, uint64_t> m;
  auto fold = [&](const QStats& s) {
    m["rx"] += s.rx.load(); m["tx"] += s.tx.load(); m["drop"] += s.drop.load(); m["punt"] += s.punt.load();
    m["recirc"] += s.recirc.load(); m["replicas"] += s.reps.load(); m["bursts"] += s.bursts.load();
    m["side_passes"] += s.side.load(); m["no_netdev"] += s.no_port.load(); m["tx_full"] += s.tx_full.load();
    m["publish_ns"] += s.pub_ns.load(); m["deliver_ns"] += s.deliver_ns.load(); m["rx_idle_polls"] += s.idle.load();
    m["rx_wait_tx"] += s.wait_tx.load(); m["learn_events"] += s.learn.load(); m["rx_held"] += s.held.load();
    m["zero_copy_frames"] += s.zc.load(); m["gpu_tx"] += s.gde.load();
  };
  for (auto& Q : queues_) {
    fold(Q->st);
    for (uint32_t w = 0; w < workers_; ++w) fold(Q->wst[w]);
  }
  m["punt_dropped"] = punt_drop_.load();
  m["queues"] = nq_;
  {
    std::lock_guard<std::mutex> g(learn_mu_);
    m["learn_applied"] = learn_applied_n_;
    m["learn_dropped"] = learn_dropped_;
  }
  return m;
}

std::vector<uint64_t> Engine::side_port_counters() const {
  std::vector<uint64_t> v((size_t)2 * kMaxPorts, 0);
  for (auto& Q : queues_)
    for (size_t i = 0; i < v.size(); ++i) v[i] += Q->side_ctr[i].load(std::memory_order_relaxed);
  return v;
}

std::vector<uint64_t> Engine::side_drop_counters() const {
  std::vector<uint64_t> v(kNumReasons, 0);
  for (auto& Q : queues_)
    for (int i = 0; i < kNumReasons; ++i) v[i] += Q->side_drop[i].load(std::memory_order_relaxed);
  return v;
}

void Engine::punt(QStats& st, uint32_t in_port, uint32_t reason, const uint8_t* a, uint32_t na, const uint8_t* b,
                  uint32_t nb) {
  std::lock_guard<std::mutex> g(punt_mu_);
  if (punts_.size() >= 4096) { punt_drop_.fetch_add(1); return; }
  Punt p;
  p.in_port = (uint16_t)in_port;
  p.reason = (uint8_t)reason;
  p.frame.reserve(na + nb);
  p.frame.insert(p.frame.end(), a, a + na);
  if (nb) p.frame.insert(p.frame.end(), b, b + nb);
  punts_.push_back(std::move(p));
  st.add(st.punt, 1);
}

void Engine::flush_learning() {
  std::unique_lock<std::mutex> lk(learn_mu_);
  const uint64_t want = learn_seq_;
  learn_cv_.wait_for(lk, std::chrono::seconds(10), [&] { return learn_applied_ >= want || !learner_run_; });
}

void Engine::learner_loop() {
  std::vector<uint32_t> ev;
  try {
    for (;;) {
      uint64_t seq;
      {
        std::unique_lock<std::mutex> lk(learn_mu_);
        learn_cv_.wait(lk, [&] { return !learn_q_.empty() || !learner_run_; });
        if (learn_q_.empty()) return;   // stopping with nothing left
        ev.swap(learn_q_);
        learn_q_.clear();
        seq = learn_seq_;
      }
      const uint32_t n = (uint32_t)(ev.size() / 4);
      const uint32_t stamp = ++learn_stamp_;
      // every GPU learns what any of them saw (one MAC table model for the node); then the side
      // passes' snapshots, so they stop reporting the MAC
      for (auto& b : backends_) b->apply_learn(ev.data(), n, stamp);
      auto c = cfg();
      for (auto& st : c->side)
        if (st && st->has_macs()) {
          std::unique_lock<std::shared_mutex> g(st->mac_mu);
          mac_learn_cpu(st->macs(), st->mac_mask(), ev.data(), n, stamp);
        }
      {
        std::lock_guard<std::mutex> lk(learn_mu_);
        learn_applied_ = seq;
        learn_applied_n_ += n;
      }
      learn_cv_.notify_all();
      ev.clear();
    }
  } catch (const std::exception& e) {
    {
      std::lock_guard<std::mutex> lk(learn_mu_);
      learner_run_ = false;
    }
    learn_cv_.notify_all();
    fail(std::string("learner: ") + e.what());
  }
}

#ifndef NFDP_IOX_YIELD_MASK
#define NFDP_IOX_YIELD_MASK 0xFFFFu
#endif
constexpr uint32_t kYieldMask = NFDP_IOX_YIELD_MASK;   // idle polls between yields of a spinning thread

struct Engine::TxCtx {
  TxScratch sc;
  std::vector<uint64_t> cur;                   // per lane: the next burst id to handle
  std::vector<Clock::time_point> wait_since;   // per lane: since when its next burst is incomplete
  std::vector<uint8_t> waiting;
  uint32_t idle = 0;
  Snap<Cfg> csnap;
  Snap<PortTab> psnap;
  explicit TxCtx(size_t lanes) : cur(lanes, 0), wait_since(lanes), waiting(lanes, 0) {
    sc.by_port.resize((size_t)kMaxPorts + 2);
  }
};

void Engine::rx_loop(Queue* Q) {
  std::vector<RxRef> buf(burst_);
  std::unique_ptr<TxCtx> tx;   // run to completion: this thread delivers its lanes' bursts too
  if (inline_tx_) tx.reset(new TxCtx(Q->lanes.size()));
  uint32_t idle_polls = 0;
  uint32_t rr = 0;
  std::shared_ptr<const PortTab> cached;
  uint64_t cached_ver = ~0ull;
  Snap<Cfg> csnap;
  std::vector<std::pair<uint32_t, Port*>> active;    // ports of this queue this thread owns and polls
  std::vector<std::pair<uint32_t, Port*>> pending;   // ports of this queue another rx thread still holds
  const uint32_t nb = (uint32_t)backends_.size();
  const uint32_t q = Q->id;
  QStats& st = Q->st;
  auto release_all = [&]() {
    for (auto& a : active) a.second->rx_owner_.store(-1, std::memory_order_release);
    active.clear();
  };
  try {
    while (run_) {
      if (pause_n_.load(std::memory_order_acquire) || hold_n_.load(std::memory_order_acquire)) {
        // nothing is being published by this thread from here until it sees the flags clear
        Q->held_epoch.store(ctl_epoch_.load(std::memory_order_acquire), std::memory_order_release);
        st.add(st.held, 1);
        if (tx) (void)tx_poll(Q, 0, *tx);   // bursts in flight still complete (pause waits for them)
        for (int k = 0; k < 64 && (pause_n_.load() || hold_n_.load()); ++k) _mm_pause();
        if (pause_n_.load()) std::this_thread::sleep_for(std::chrono::microseconds(10));
        continue;
      }
      const uint64_t pv = ports_ver_.load(std::memory_order_acquire);
      if (pv != cached_ver) {
        auto tab = std::atomic_load(&ports_);
        cached_ver = pv;
        std::vector<std::pair<uint32_t, Port*>> want;
        for (uint32_t i = 0; i < (uint32_t)tab->size(); ++i)
          if ((*tab)[i].p && (*tab)[i].q == q) want.emplace_back(i, (*tab)[i].p.get());
        std::vector<std::pair<uint32_t, Port*>> keep;
        for (auto& a : active) {
          const bool still = std::any_of(want.begin(), want.end(), [&](const auto& w) { return w.second == a.second; });
          if (still) keep.push_back(a);
          else a.second->rx_owner_.store(-1, std::memory_order_release);   // moved away or removed: let go
        }
        active.swap(keep);
        pending.clear();
        for (auto& w : want)
          if (std::none_of(active.begin(), active.end(), [&](const auto& a) { return a.second == w.second; }))
            pending.push_back(w);
        // frames staged from a port no longer in the table are dropped (handed back, never
        // published): from here on no burst of this thread can refer to a removed port
        for (Lane* L : Q->lanes) {
          if (L->stage.empty()) continue;
          size_t k = 0;
          for (const Pkt& pk : L->stage) {
            bool live = pk.holder == recirc_.get();
            for (uint32_t i = 0; i < (uint32_t)tab->size() && !live; ++i) live = (*tab)[i].p.get() == pk.holder;
            if (live) L->stage[k++] = pk;
            else pk.holder->complete(pk.seq);
          }
          L->stage.resize(k);
        }
        Q->ports_seen.store(pv, std::memory_order_release);
        cached = tab;   // (after letting go: the old snapshot may hold the last reference to a removed port)
      }
      // take over ports whose previous rx thread has let go (acquire: its reads of the port happened before)
      for (size_t k = 0; k < pending.size();) {
        int exp = -1;
        if (pending[k].second->rx_owner_.compare_exchange_strong(exp, (int)q, std::memory_order_acquire)) {
          active.push_back(pending[k]);
          pending[k] = pending.back();
          pending.pop_back();
        } else {
          ++k;
        }
      }
      for (auto& a : active) a.second->reclaim();
      if (q == 0) recirc_->reclaim();
      const Cfg* c = &cfg_of(csnap);
      const Steer* steer = c->steer.get();
      // room: a burst of k frames takes ceil(k / 64) chunks on its lane; bound the take by the
      // fullest lane (frames are steered after they are read), counting what is staged already
      uint32_t take = burst_;
      for (Lane* L : Q->lanes) {
        if (!L->be->ready() ||
            L->head.load(std::memory_order_relaxed) - L->done.load(std::memory_order_acquire) >= inflight_) {
          take = 0;
          break;
        }
        // slots are reusable once DELIVERED (their out slot / meta read), not merely completed
        const uint64_t used = L->be->published(q) - L->freed_pos.load(std::memory_order_acquire);
        uint64_t room = L->be->capacity() > used ? L->be->capacity() - used : 0;
        if (max_frames_) room = std::min<uint64_t>(room, max_frames_ > used ? max_frames_ - used : 0);
        room &= ~63ull;
        const uint64_t staged = L->stage.size();
        L->room = room;
        take = (uint32_t)std::min<uint64_t>(take, room > staged ? room - staged : 0);
        take = (uint32_t)std::min<uint64_t>(take, burst_ > staged ? burst_ - staged : 0);
      }
      const uint64_t t_rx = now_ns();
      uint32_t got = 0;
      if (take) {
        auto read_port = [&](uint32_t pid, Port* p, uint32_t max) {
          const uint32_t n = p->rx(buf.data(), max);
          uint64_t pk = 0, by = 0;
          for (uint32_t i = 0; i < n; ++i) {
            const RxRef& r = buf[i];
            p->handed_out(r.seq);
            if (r.len < 14 || r.len > kMaxFrame) { p->complete(r.seq); continue; }   // runt / oversize / own tx
            const uint32_t in_port = r.in_port != ~0u ? r.in_port : pid;
            const uint32_t o = nb > 1 ? owner(steer, nb, r.data, r.len, in_port) : 0u;
            Lane* L = Q->lanes[o];
            if (L->stage.empty()) L->stage_t0 = t_rx;
            L->stage.push_back(Pkt{in_port, r.seq, r.data, r.len, p});
            ++pk;
            by += r.len;
          }
          p->count_rx(pk, by);
          got += (uint32_t)pk;
          return n;
        };
        if (q == 0) (void)read_port(0, recirc_.get(), take);
        // every port gets an equal share of the burst first (round-robin start), then leftovers
        const uint32_t np = (uint32_t)active.size();
        if (np) {
          const uint32_t share = std::max<uint32_t>(1, take / np);
          uint32_t taken = got;
          for (int pass = 0; pass < 2 && taken < take; ++pass) {
            for (uint32_t k = 0; k < np && taken < take; ++k) {
              const auto& a = active[(rr + k) % np];
              taken += read_port(a.first, a.second, std::min(take - taken, pass ? take : share));
            }
          }
          rr = (rr + 1) % np;
        }
        st.add(st.rx, got);
      }
      // publication: a lane's staged frames go out at once when nothing of the lane is in
      // flight (the unloaded case: no added latency); under load they gather into whole 64-slot
      // chunks (no padding, fewer bursts for the GPU and the tx threads), bounded in time by
      // the coalescing window and in size by the burst / the lane's room
      const std::vector<uint8_t>& side_ports = c->side_ports;
      const bool side_always = c->side_always;
      const uint64_t win = coalesce_ns_.load(std::memory_order_relaxed);
      const uint32_t cmin = coalesce_frames_.load(std::memory_order_relaxed);
      uint32_t pubs = 0;
      for (Lane* L : Q->lanes) {
        if (L->stage.empty()) continue;
        const uint64_t head = L->head.load(std::memory_order_relaxed);
        const uint64_t inflight = head - L->done.load(std::memory_order_acquire);
        if (inflight >= inflight_ || !L->be->ready()) continue;
        const uint32_t k = (uint32_t)L->stage.size();
        const bool go = inflight == 0 || k >= cmin || k >= burst_ || k + 64 > L->room || t_rx - L->stage_t0 >= win;
        if (!go) continue;
        Backend& be = *L->be;
        const uint32_t npad = (k + 63u) & ~63u;
        const uint64_t start = be.published(q);
        uint32_t* im = be.in_meta(q);
        const uint32_t cmask = be.capacity() - 1;
        Burst& b = L->slots[head % inflight_];   // free: head - done < inflight
        b.start = start;
        b.end = start + npad;
        b.t_rx_ns = L->stage_t0;
        bool side = side_always;
        uint64_t* fa = be.frame_addrs(q);
        if (fa) {
          // zero-copy: the pipeline reads a mapped port's frame in place (16-B aligned, its first
          // 64 bytes inside the mapping); any other frame is copied and read from its in slot
          uint32_t zc = 0;
          for (uint32_t i = 0; i < k; ++i) {
            const Pkt& pk = L->stage[i];
            const uint32_t pos = (uint32_t)((start + i) & cmask);
            const Port::Mapped& m = pk.holder->zc_;
            if (pk.data >= m.lo && pk.data + kSlotBytes <= m.hi && L->g < m.off.size() &&
                !(reinterpret_cast<uintptr_t>(pk.data) & 15u)) {
              fa[pos] = (uint64_t)((int64_t)reinterpret_cast<uint64_t>(pk.data) + m.off[L->g]);
              ++zc;
            } else {
              uint8_t* slot = be.in_slot(q, pos);
              const uint32_t h = std::min<uint32_t>(pk.len, kSlotBytes);
              std::memcpy(slot, pk.data, h);
              if (h < kSlotBytes) std::memset(slot + h, 0, kSlotBytes - h);
              fa[pos] = be.in_slot_addr(q, pos);
            }
            im[pos] = (pk.port & 0xFFFFu) | (pk.len << 16);
            side = side || (pk.port < side_ports.size() && side_ports[pk.port]);
          }
          for (uint32_t i = k; i < npad; ++i) fa[(start + i) & cmask] = be.in_slot_addr(q, (uint32_t)(start + i));
          st.add(st.zc, zc);
        } else {
          for (uint32_t i = 0; i < k; ++i) {
            const Pkt& pk = L->stage[i];
            uint8_t* slot = be.in_slot(q, (uint32_t)(start + i));
            if (i + 4 < k) {   // later slots' lines (last written by the GPU) and frames, requested early
              __builtin_prefetch(be.in_slot(q, (uint32_t)(start + i + 4)), 1, 3);
              __builtin_prefetch(L->stage[i + 4].data, 0, 3);
            }
            const uint32_t h = std::min<uint32_t>(pk.len, kSlotBytes);
            if (pk.holder != recirc_.get()) {
              slot_copy(slot, pk.data, h);
            } else {
              std::memcpy(slot, pk.data, h);
              if (h < kSlotBytes) std::memset(slot + h, 0, kSlotBytes - h);
            }
            im[(start + i) & cmask] = (pk.port & 0xFFFFu) | (pk.len << 16);
            side = side || (pk.port < side_ports.size() && side_ports[pk.port]);
          }
        }
        for (uint32_t i = k; i < npad; ++i) im[(start + i) & cmask] = kRingPadMeta;
        b.side = side;
        b.cfg = csnap.p;   // (one refcount per burst: the snapshot this burst's tables belong to)
        b.pkts.swap(L->stage);
        L->stage.clear();
        b.id = head;
        b.left.store(workers_, std::memory_order_relaxed);
        b.state.store(1, std::memory_order_release);
        L->head.store(head + 1, std::memory_order_release);
        const uint64_t tp0 = now_ns();
        be.publish(q, npad);
        st.add(st.pub_ns, now_ns() - tp0);
        st.add(st.bursts, 1);
        ++pubs;
      }
      const uint32_t dlv = tx ? tx_poll(Q, 0, *tx) : 0u;
      if (got == 0 && pubs == 0 && dlv == 0) {
        st.add(take ? st.idle : st.wait_tx, 1);
        _mm_pause();
        if ((++idle_polls & kYieldMask) == 0) std::this_thread::yield();
      }
    }
    if (tx) {   // stopping: deliver what was published (a pipeline that stopped completing throws)
      const auto t0 = Clock::now();
      while (!tx_drained(Q, *tx) && !abandon_.load() && Clock::now() - t0 < std::chrono::seconds(10))
        if (!tx_poll(Q, 0, *tx)) _mm_pause();
    }
    release_all();
  } catch (const std::exception& e) {
    release_all();
    fail(std::string("rx: ") + e.what());
  }
}

namespace {
// side_stage's sink for one burst: replicas and outer headers stay with the burst, learn events
// go to the learner (consecutive duplicates of one burst folded)
struct BurstSink {
  std::vector<Replica>& reps;
  std::vector<uint8_t>& xbuf;
  std::vector<uint8_t>& has_x;
  std::vector<uint32_t>& learn_ev;
  uint32_t i = 0;   // packet index in the burst
  void rep(const uint32_t* hdr, uint32_t meta, uint32_t) {
    reps.emplace_back();
    Replica& r = reps.back();
    r.src = i;
    r.meta = meta;
    std::memcpy(r.hdr, hdr, kSlotBytes);
  }
  void xhdr_rec(const uint32_t* x) {
    std::memcpy(xbuf.data() + (size_t)i * kXhdrBytes, x, kXhdrBytes);
    has_x[i] = 1;
  }
  void xhdr(const uint32_t* x, uint32_t, uint32_t) { xhdr_rec(x); }
  void learn(uint32_t bridge, uint32_t lo, uint32_t hi, uint32_t port) {
    const uint32_t e1 = (hi & 0xFFFFu) | (bridge << 16);
    const size_t n = learn_ev.size();
    if (n >= 4 && learn_ev[n - 4] == lo && learn_ev[n - 3] == e1 && learn_ev[n - 2] == port) return;
    learn_ev.insert(learn_ev.end(), {lo, e1, port, 0u});
  }
};
}  // namespace

void Engine::side_work(Queue* Q, Lane* L, Burst& b, const Cfg& c, TxScratch& sc, uint32_t w) {
  Backend& be = *L->be;
  const uint32_t q = Q->id, cmask = be.capacity() - 1;
  const uint32_t* om = be.out_meta(q);
  const uint32_t* im = be.in_meta(q);
  const uint32_t np = (uint32_t)b.pkts.size();
  SideTables* stab = L->g < c.side.size() ? c.side[L->g].get() : nullptr;
  if (!stab) return;   // no snapshot (no side features configured): flagged packets fall to deliver()'s checks
  const TablesView& t = stab->view();
  const TabHash hasher{&stab->hash()};
  const std::vector<uint8_t>& sp = c.side_ports;
  const bool zc = be.frame_addrs(q) != nullptr;
  sc.learn.clear();
  BurstSink sink{b.reps, b.xhdr, b.has_x, sc.learn};
  std::shared_lock<std::shared_mutex> g(stab->mac_mu);   // the learner updates the snapshot's MAC table
  for (uint32_t i = 0; i < np; ++i) {
    const uint32_t pos = (uint32_t)((b.start + i) & cmask);
    const uint32_t m = om[pos];
    const uint32_t port = b.pkts[i].port;
    if (!(m & (kMetaFlood | kMetaXhdr)) && !c.side_always && !(port < sp.size() && sp[port])) continue;
    if ((m & kMetaXhdr) && b.xhdr.empty()) {
      b.xhdr.assign((size_t)np * kXhdrBytes, 0);
      b.has_x.assign(np, 0);
    }
    sink.i = i;
    const uint32_t* fin = reinterpret_cast<const uint32_t*>(be.in_slot(q, pos));
    alignas(16) uint32_t zf[kSlotBytes / 4];
    if (zc) {   // (a zero-copy frame may not be in its in slot: the frame itself, zero-padded)
      const uint32_t h = std::min<uint32_t>(b.pkts[i].len, kSlotBytes);
      std::memset(zf, 0, sizeof(zf));
      std::memcpy(zf, b.pkts[i].data, h);
      fin = zf;
    }
    side_stage(t, DirectTables{t}, fin, im[pos],
               reinterpret_cast<const uint32_t*>(be.out_slot(q, pos)), m, i, sink, hasher);
  }
  g.unlock();
  // replicas count where the batch path's side pass counts them (port tx / drop by reason)
  for (const Replica& r : b.reps) {
    const uint32_t rr = meta_reason(r.meta), p = meta_port(r.meta);
    if (rr) {
      auto& d = Q->side_drop[rr & (kNumReasons - 1)];
      d.store(d.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
    } else if (p < (uint32_t)kMaxPorts) {
      auto& cp = Q->side_ctr[2 * (size_t)p];
      auto& cb = Q->side_ctr[2 * (size_t)p + 1];
      cp.store(cp.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
      cb.store(cb.load(std::memory_order_relaxed) + meta_len(r.meta), std::memory_order_relaxed);
    }
  }
  QStats& st = Q->wst[w];
  st.add(st.side, 1);
  if (!sc.learn.empty()) {
    st.add(st.learn, sc.learn.size() / 4);
    {
      std::lock_guard<std::mutex> lk(learn_mu_);
      if (learn_q_.size() < (1u << 20)) {
        learn_q_.insert(learn_q_.end(), sc.learn.begin(), sc.learn.end());
        ++learn_seq_;
      } else {
        learn_dropped_ += sc.learn.size() / 4;
      }
    }
    learn_cv_.notify_one();
  }
}

void Engine::deliver(Queue* Q, Lane* L, Burst& b, uint32_t w, const Cfg& c, const PortTab& tab, TxScratch& sc) {
  Backend& be = *L->be;
  const uint32_t q = Q->id, cmask = be.capacity() - 1;
  const uint32_t* om = be.out_meta(q);
  const std::vector<uint32_t>& red = c.redirect;
  auto route = [&](uint32_t port) {   // tunnel port -> its underlay port
    return port < red.size() && red[port] != 0xFFFFFFFFu ? red[port] : port;
  };
  TxTally tally;
  auto add = [&](uint32_t port, const TxItem& it) {
    if (port >= tab.size() || !tab[port].p) { ++tally.no_port; return; }
    auto& v = sc.by_port[port];
    if (v.empty()) sc.touched.push_back(port);
    v.push_back(it);
  };
  const uint32_t np = (uint32_t)b.pkts.size();
  const uint32_t nw = workers_;
  auto mine = [&](uint32_t port) { return nw == 1 || port % nw == w; };   // no division with one worker
  constexpr uint32_t kAhead = 8;   // out slots of later packets are fetched ahead
  for (uint32_t i = 0; i < np; ++i) {
    if (i + kAhead < np) {
      const uint32_t pa = (uint32_t)((b.start + i + kAhead) & cmask);
      if (mine(route(meta_port(om[pa])))) __builtin_prefetch(be.out_slot(q, pa), 0, 0);
    }
    const Pkt& pk = b.pkts[i];
    const uint32_t pos = (uint32_t)((b.start + i) & cmask);
    const uint32_t meta = om[pos];
    const uint32_t reason = meta_reason(meta), oport = meta_port(meta), olen = meta_len(meta);
    if (meta_is_gde(meta)) {   // the grid wrote it into the pod's ring itself
      if (w == 0) ++tally.gde;
      continue;
    }
    if (reason == 0) {
      const uint32_t dst = route(oport);
      if (!mine(dst)) continue;
      const uint8_t* x = nullptr;
      uint32_t xl = 0;
      if (meta & kMetaXhdr) {
        if (b.has_x.empty() || !b.has_x[i]) { ++tally.drop; continue; }   // never sent bare
        x = b.xhdr.data() + (size_t)i * kXhdrBytes;
        xl = xhdr_len(x);
      }
      uint32_t hl = 0, to = 0;
      out_tail(pk.len, olen, xl, hl, to);
      if (to > pk.len) to = pk.len;
      add(dst, TxItem{x, xl, be.out_slot(q, pos), hl, pk.data + to, pk.len - to});
    } else if (w != 0) {
      continue;
    } else if (reason == kRecirc && olen <= pk.len) {
      recirc_->push(oport, pk.data + (pk.len - olen), olen);   // terminated tunnel: the inner frame re-enters
      QStats& st = Q->wst[w];
      st.add(st.recirc, 1);
    } else if (reason == kRecirc6) {
      punt(Q->wst[w], pk.port, reason, pk.data, pk.len, nullptr, 0);   // the VNI lookup needs the whole frame
    } else {
      ++tally.drop;
    }
  }
  for (const Replica& r : b.reps) {
    const Pkt& pk = b.pkts[r.src];
    uint32_t hl = 0, to = 0;
    const uint32_t rlen = meta_len(r.meta), rr = meta_reason(r.meta);
    out_tail(pk.len, rlen, 0, hl, to);
    if (to > pk.len) to = pk.len;
    if (rr) {
      if (w == 0) punt(Q->wst[w], pk.port, rr, r.hdr, hl, pk.data + to, pk.len - to);   // ARP trap: the slow path's copy
    } else {
      const uint32_t dst = route(meta_port(r.meta));
      if (mine(dst)) {
        add(dst, TxItem{nullptr, 0, r.hdr, hl, pk.data + to, pk.len - to});
        ++tally.reps;
      }
    }
  }
  // one locked batch per egress port
  for (uint32_t port : sc.touched) {
    auto& v = sc.by_port[port];
    const uint32_t ok = tab[port].p->tx_batch(v.data(), (uint32_t)v.size(), q);   // this queue's tx ring
    tally.tx += ok;
    tally.full += v.size() - ok;
    v.clear();
  }
  sc.touched.clear();
  QStats& st = Q->wst[w];
  st.add(st.tx, tally.tx);
  st.add(st.tx_full, tally.full);
  st.add(st.no_port, tally.no_port);
  st.add(st.drop, tally.drop);
  st.add(st.reps, tally.reps);
  st.add(st.gde, tally.gde);
}

void Engine::finish(Queue* Q, Lane* L, Burst& b) {
  for (const Pkt& q : b.pkts) q.holder->complete(q.seq);
  const double us = (double)(now_ns() - b.t_rx_ns) * 1e-3;
  {
    std::lock_guard<std::mutex> g(Q->lat_mu);
    if (Q->lat_us.size() < (1u << 18)) Q->lat_us.push_back(us);
  }
  b.pkts.clear();
  b.reps.clear();
  b.xhdr.clear();
  b.has_x.clear();
  b.cfg.reset();
  L->freed_pos.store(b.end, std::memory_order_release);
  b.state.store(0, std::memory_order_release);
  L->done.fetch_add(1, std::memory_order_release);
}

uint32_t Engine::tx_poll(Queue* Q, uint32_t w, TxCtx& x) {
  const uint32_t nl = (uint32_t)Q->lanes.size();
  const uint32_t want = w == 0 ? 1u : 2u;
  QStats& st = Q->wst[w];
  uint32_t handled = 0;
  for (uint32_t li = 0; li < nl; ++li) {
    Lane* L = Q->lanes[li];
    Burst& b = L->slots[x.cur[li] % inflight_];
    if (!(b.state.load(std::memory_order_acquire) >= want && b.id == x.cur[li])) continue;
    if (w == 0) {
      // leader: completion, side work, then the burst is ready for every worker
      if (!L->be->range_done(Q->id, b.start, b.end)) {
        if (!x.waiting[li]) { x.waiting[li] = 1; x.wait_since[li] = Clock::now(); }
        else if ((++x.idle & 0xFFFu) == 0) {
          const auto waited = Clock::now() - x.wait_since[li];
          if (waited > std::chrono::milliseconds(200) && !L->be->alive())
            throw std::runtime_error("tx: the ring kernel is gone (device deadline or fault)");
          if (waited > std::chrono::seconds(5)) throw std::runtime_error("tx: burst not completed within 5 s");
        }
        continue;
      }
      x.waiting[li] = 0;
      const Cfg* c = b.cfg ? b.cfg.get() : &cfg_of(x.csnap);
      bool side = b.side;
      if (!side) {
        const uint32_t* om = L->be->out_meta(Q->id);
        const uint32_t cm = L->be->capacity() - 1;
        for (uint64_t p = b.start; p < b.start + b.pkts.size() && !side; ++p)
          side = (om[p & cm] & (kMetaFlood | kMetaXhdr)) != 0;
      }
      if (side) side_work(Q, L, b, *c, x.sc, w);
      b.state.store(2, std::memory_order_release);
      const uint64_t td0 = now_ns();
      deliver(Q, L, b, w, *c, ports_of(x.psnap), x.sc);
      st.add(st.deliver_ns, now_ns() - td0);
    } else {
      const Cfg& c = b.cfg ? *b.cfg : cfg_of(x.csnap);
      const uint64_t td0 = now_ns();
      deliver(Q, L, b, w, c, ports_of(x.psnap), x.sc);
      st.add(st.deliver_ns, now_ns() - td0);
    }
    if (b.left.fetch_sub(1, std::memory_order_acq_rel) == 1) finish(Q, L, b);
    ++x.cur[li];
    ++handled;
  }
  return handled;
}

bool Engine::tx_drained(Queue* Q, const TxCtx& x) const {
  for (uint32_t li = 0; li < (uint32_t)Q->lanes.size(); ++li) {
    const Lane* L = Q->lanes[li];
    if (L->done.load() != L->head.load() || x.cur[li] != L->head.load()) return false;
  }
  return true;
}

void Engine::tx_loop(Queue* Q, uint32_t w) {
  try {
    TxCtx x(Q->lanes.size());
    for (;;) {
      if (tx_poll(Q, w, x)) {
        x.idle = 0;
        continue;
      }
      if (abandon_.load(std::memory_order_relaxed)) return;
      if (!run_.load(std::memory_order_relaxed) && tx_drained(Q, x)) return;
      _mm_pause();
      if ((++x.idle & 0x3FFu) == 0) (void)ports_of(x.psnap);   // idle: let go of a replaced port table too
      if ((x.idle & kYieldMask) == 0) std::this_thread::yield();
    }
  } catch (const std::exception& e) {
    fail(std::string("tx: ") + e.what());
  }
}

}  // namespace iox
}  // namespace nfdp
