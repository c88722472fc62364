// iox.cpp — native packet I/O engine (see iox.h).
#include "iox.h"

#include <arpa/inet.h>
#include <errno.h>
#include <immintrin.h>
#include <linux/if_ether.h>
#include <linux/if_packet.h>
#include <net/if.h>
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
void hck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("iox: ") + what + ": " + hipGetErrorString(e));
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

bool Port::tx(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
  std::lock_guard<std::mutex> g(tx_mu_);
  const bool ok = tx_locked(a, na, b, nb, c, nc);
  if (ok) {
    tx_dirty_ = true;
    tx_pkts.fetch_add(1, std::memory_order_relaxed);
    tx_bytes.fetch_add(na + nb + nc, std::memory_order_relaxed);
  } else {
    tx_full.fetch_add(1, std::memory_order_relaxed);
  }
  return ok;
}

void Port::flush() {
  std::lock_guard<std::mutex> g(tx_mu_);
  if (tx_dirty_) flush_locked();
  tx_dirty_ = false;
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
MemifPort::MemifPort(const std::string& path, uint32_t ring_size, uint32_t buf_size)
    : Port(ring_size), reg_(path, true, ring_size, buf_size), unlink_(true) {
  cons_.init(&reg_, 0);
  prod_.init(&reg_, 1);
  set_first_seq(cons_.next);
}

MemifPort::~MemifPort() {
  if (unlink_) ::unlink(reg_.path().c_str());
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

bool MemifPort::tx_locked(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
  return prod_.put(a, na, b, nb, c, nc);
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

bool PacketPort::tx_locked(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
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

void PacketPort::flush_locked() { (void)::sendto(fd_, nullptr, 0, MSG_DONTWAIT, nullptr, 0); }

// ---------------------------------------------------------------------------------- FdPort
FdPort::FdPort(int fd, uint32_t nbufs, uint32_t buf_size)
    : Port(nbufs), fd_(fd), nbufs_(pow2_at_least(nbufs)), bsize_(buf_size) {
  bufs_.resize((size_t)nbufs_ * bsize_);
  lens_.resize(nbufs_);
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

bool FdPort::tx_locked(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
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

// ---------------------------------------------------------------------------------- GpuBackend
GpuBackend::GpuBackend(RingEngine* ring) : ring_(ring) {
  if (!ring->host_slots()) throw std::invalid_argument("iox: the ring needs host_slots=True");
  in_ = static_cast<uint8_t*>(ring->host_ptr(0));
  im_ = static_cast<uint32_t*>(ring->host_ptr(1));
  out_ = static_cast<uint8_t*>(ring->host_ptr(2));
  om_ = static_cast<uint32_t*>(ring->host_ptr(3));
}

GpuBackend::~GpuBackend() {
  if (side_stream_) (void)hipStreamDestroy(side_stream_);
}

void GpuBackend::thread_init() {
  hck(hipSetDevice(ring_->device()), "set device");
  if (!side_stream_) hck(hipStreamCreateWithFlags(&side_stream_, hipStreamNonBlocking), "side stream");
}

void GpuBackend::side_pass(SideBatch& out) {
  const FusedLaunch& f = ring_->launch();
  if (!f.side.cnt) return;
  if (!side_stream_) thread_init();
  hipStream_t s = side_stream_;
  hck(launch_side(f.t, ring_->dev_in(), ring_->dev_inmeta(), ring_->dev_out(), ring_->dev_meta(), f.side, f.port_ctr,
                  f.drop_ctr, s, ring_->capacity(), true), "side kernel");
  if (f.side.cap_learn && f.t.macs)
    hck(launch_mac_learn(const_cast<MacEntry*>(f.t.macs), f.t.mac_mask, f.side.learn, f.side.cnt + 1, f.side.cap_learn,
                         stamp++, f.side.cnt + 4, s), "learn kernel");
  h_cnt_.assign(8, 0);
  hck(hipMemcpyAsync(h_cnt_.data(), f.side.cnt, 32, hipMemcpyDeviceToHost, s), "side counts");
  hck(hipStreamSynchronize(s), "side sync");
  const uint32_t n = std::min(h_cnt_[0], f.side.cap_rep);
  if (n) {
    h_meta_.resize(n); h_src_.resize(n); h_hdr_.resize((size_t)n * kSlotDwords);
    hck(hipMemcpyAsync(h_meta_.data(), f.side.rep_meta, n * 4ull, hipMemcpyDeviceToHost, s), "rep meta");
    hck(hipMemcpyAsync(h_src_.data(), f.side.rep_src, n * 4ull, hipMemcpyDeviceToHost, s), "rep src");
    hck(hipMemcpyAsync(h_hdr_.data(), f.side.rep_hdr, n * 64ull, hipMemcpyDeviceToHost, s), "rep hdr");
  }
  if (f.side.xhdr) {
    out.xall.resize((size_t)capacity() * kXhdrBytes);
    hck(hipMemcpyAsync(out.xall.data(), f.side.xhdr, out.xall.size(), hipMemcpyDeviceToHost, s), "xhdr");
  }
  hck(hipMemsetAsync(f.side.cnt, 0, 32, s), "side reset");
  hck(hipStreamSynchronize(s), "side sync");
  out.reps.resize(n);
  for (uint32_t k = 0; k < n; ++k) {
    out.reps[k].src_pos = h_src_[k];
    out.reps[k].meta = h_meta_[k];
    std::memcpy(out.reps[k].hdr, &h_hdr_[(size_t)k * kSlotDwords], kSlotBytes);
  }
  out.learned = h_cnt_[1];
  if (out.learned) ring_->bump_epoch();   // learned MACs: the next chunks drop cached table lines
}

// ---------------------------------------------------------------------------------- OracleBackend
OracleBackend::OracleBackend(uint32_t capacity) : cap_(capacity) {
  if (capacity < 64 || (capacity & (capacity - 1))) throw std::invalid_argument("iox: oracle capacity: power of two >= 64");
  in_.assign((size_t)cap_ * kSlotBytes, 0);
  out_.assign((size_t)cap_ * kSlotBytes, 0);
  im_.assign(cap_, 0);
  om_.assign(cap_, 0);
}

void OracleBackend::configure(const TablesView& t, uint64_t* flow_ctr, uint64_t* port_ctr, uint64_t* drop_ctr,
                              const SideOut& side, MacEntry* macs, uint32_t mac_mask) {
  t_ = t; flow_ctr_ = flow_ctr; port_ctr_ = port_ctr; drop_ctr_ = drop_ctr; side_ = side;
  macs_ = macs; mac_mask_ = mac_mask;
  configured_ = true;
}

void OracleBackend::run_segment(uint32_t pos, uint32_t n) {
  const uint32_t p = pos & (cap_ - 1);
  if (side_.cnt) std::memset(side_.cnt, 0, 32);
  oracle_run(t_, reinterpret_cast<const uint32_t*>(in_.data() + (size_t)p * kSlotBytes), im_.data() + p, n,
             reinterpret_cast<uint32_t*>(out_.data() + (size_t)p * kSlotBytes), om_.data() + p, flow_ctr_, port_ctr_,
             drop_ctr_, nullptr, nullptr, side_.cnt ? &side_ : nullptr);
  if (!side_.cnt) return;
  const uint32_t nr = std::min(side_.cnt[0], side_.cap_rep);
  for (uint32_t k = 0; k < nr; ++k) {
    Replica r;
    r.src_pos = (p + side_.rep_src[k]) & (cap_ - 1);
    r.meta = side_.rep_meta[k];
    std::memcpy(r.hdr, side_.rep_hdr + (size_t)k * kSlotDwords, kSlotBytes);
    pending_.reps.push_back(r);
  }
  if (side_.xhdr) {
    if (pending_.xall.empty()) pending_.xall.assign((size_t)cap_ * kXhdrBytes, 0);
    for (uint32_t i = 0; i < n; ++i)
      if (om_[p + i] & kMetaXhdr)
        std::memcpy(pending_.xall.data() + (size_t)(p + i) * kXhdrBytes,
                    reinterpret_cast<const uint8_t*>(side_.xhdr) + (size_t)i * kXhdrBytes, kXhdrBytes);
  }
  const uint32_t nl = std::min(side_.cnt[1], side_.cap_learn);
  if (nl && macs_) {
    mac_learn_cpu(macs_, mac_mask_, side_.learn, nl, stamp);
    pending_.learned += nl;
  }
}

uint64_t OracleBackend::publish(uint32_t n) {
  if (!configured_) throw std::runtime_error("iox: oracle backend not configured");
  if (n == 0 || (n & 63u) || n > cap_) throw std::invalid_argument("iox: publish a multiple of 64 packets");
  // real packets first, filler slots (kRingPadMeta) at the end of the publish: run the prefix
  uint32_t real = 0;
  while (real < n && im_[(prod_ + real) & (cap_ - 1)] != kRingPadMeta) ++real;
  for (uint32_t i = real; i < n; ++i) om_[(prod_ + i) & (cap_ - 1)] = make_meta(kPortNone, 0, kMalformed);
  uint32_t done = 0;
  while (done < real) {
    const uint32_t p = (uint32_t)((prod_ + done) & (cap_ - 1));
    const uint32_t k = std::min(real - done, cap_ - p);   // contiguous piece (a wrap splits it)
    run_segment(p, k);
    done += k;
  }
  ++stamp;
  prod_ += n;
  return prod_;
}

void OracleBackend::side_pass(SideBatch& out) {
  out.reps.swap(pending_.reps);
  out.xall.swap(pending_.xall);
  out.learned = pending_.learned;
  pending_ = SideBatch{};
}

// ---------------------------------------------------------------------------------- Engine
Engine::Engine(uint32_t burst, uint32_t inflight, uint32_t tx_workers)
    : burst_(burst), inflight_(std::max<uint32_t>(inflight, 1)), workers_(std::max<uint32_t>(tx_workers, 1)) {
  if (burst_ < 1 || burst_ > (1u << 16)) throw std::invalid_argument("iox: burst in [1, 65536]");
  if (workers_ > 16) throw std::invalid_argument("iox: at most 16 tx workers per backend");
  ports_ = std::make_shared<PortTab>((size_t)kMaxPorts + 2);
  redirect_.assign((size_t)kMaxPorts + 2, 0xFFFFFFFFu);
  side_ports_.assign((size_t)kMaxPorts + 2, 0);
  recirc_ = std::make_shared<RecircPort>(4096);
}

Engine::~Engine() {
  try {
    stop();
  } catch (...) {
  }
}

void Engine::add_backend(std::shared_ptr<Backend> b) {
  if (run_) throw std::runtime_error("iox: add backends before start()");
  auto L = std::make_unique<Lane>();
  L->be = std::move(b);
  L->slots.reset(new Burst[inflight_]);
  lanes_.push_back(std::move(L));
}

void Engine::add_port(uint32_t id, std::shared_ptr<Port> p) {
  if (id >= (uint32_t)kMaxPorts) throw std::invalid_argument("iox: port id out of range");
  std::lock_guard<std::mutex> g(ports_mu_);
  auto t = std::make_shared<PortTab>(*ports_);
  (*t)[id] = std::move(p);
  std::atomic_store(&ports_, std::shared_ptr<const PortTab>(t));
}

std::shared_ptr<Port> Engine::remove_port(uint32_t id) {
  if (id >= (uint32_t)kMaxPorts) return nullptr;
  std::lock_guard<std::mutex> g(ports_mu_);
  auto t = std::make_shared<PortTab>(*ports_);
  auto old = (*t)[id];
  (*t)[id].reset();
  std::atomic_store(&ports_, std::shared_ptr<const PortTab>(t));
  return old;   // frames of it still in flight keep it alive through the snapshot the threads hold
}

std::shared_ptr<Port> Engine::port(uint32_t id) {
  auto t = std::atomic_load(&ports_);
  return id < t->size() ? (*t)[id] : nullptr;
}

void Engine::set_steering(const std::vector<PortEntry>& ports, const std::vector<uint8_t>& rss_key, bool v6) {
  if (run_ && !pause_) throw std::runtime_error("iox: set_steering while running (pause first)");
  if (rss_key.size() < 20) throw std::invalid_argument("iox: rss key too short");
  steer_ports_ = ports;
  steer_ports_.resize((size_t)kMaxPorts + 2);
  rss_key_ = rss_key;
  steer_v6_ = v6;
}

void Engine::set_redirect(uint32_t port, uint32_t underlay) {
  if (port < redirect_.size()) redirect_[port] = underlay;
}

void Engine::set_side_ports(const std::vector<uint32_t>& ports) {
  std::vector<uint8_t> s((size_t)kMaxPorts + 2, 0);
  for (uint32_t p : ports)
    if (p < s.size()) s[p] = 1;
  side_ports_.swap(s);   // read by the rx thread; set while paused (or benignly racy: a flag per port)
}

bool Engine::needs_side(uint32_t in_port) const {
  return side_always_.load(std::memory_order_relaxed) || (in_port < side_ports_.size() && side_ports_[in_port]);
}

uint32_t frame_owner(const uint8_t* hdr, uint32_t len, uint32_t in_port, const PortEntry* ports, const uint8_t* rss_key,
                     uint32_t n, bool v6) {
  if (n <= 1) return 0;
  if (!ports || !rss_key) return in_port % n;
  uint32_t d[kSlotDwords] = {};
  std::memcpy(d, hdr, std::min<uint32_t>(len, kSlotBytes));
  TablesView tv{};
  tv.ports = ports;
  tv.flow6_on = v6 ? 1u : 0u;   // IPv6 keys folded as the owners' tables hold them
  Parsed p;
  IngressState st;
  ingress_stage(tv, DirectTables{tv}, d, (in_port & 0xFFFFu) | (std::min<uint32_t>(len, kMaxFrame) << 16), p, st);
  if (!st.reason && (p.ipv4 || (v6 && p.ipv6))) return owner_of(toeplitz_scalar(st.key, rss_key), n);
  return in_port % n;
}

uint32_t Engine::owner_of_frame(const uint8_t* f, uint32_t len, uint32_t in_port) const {
  const uint32_t n = (uint32_t)lanes_.size();
  if (n <= 1) return 0;
  if (steer_ports_.empty() || rss_key_.empty()) return in_port % n;
  return frame_owner(f, len, in_port, steer_ports_.data(), rss_key_.data(), n, steer_v6_);
}

void Engine::start() {
  if (run_) return;
  if (lanes_.empty()) throw std::runtime_error("iox: no backend");
  {
    std::lock_guard<std::mutex> g(err_mu_);
    err_.clear();
  }
  run_ = true;
  pause_ = false;
  for (auto& L : lanes_) L->freed_pos.store(L->be->published());
  for (auto& L : lanes_)
    for (uint32_t w = 0; w < workers_; ++w) L->th.emplace_back(&Engine::tx_loop, this, L.get(), w);
  rx_th_ = std::thread(&Engine::rx_loop, this);
}

void Engine::stop() {
  const bool was = run_.exchange(false);
  if (rx_th_.joinable()) rx_th_.join();
  for (auto& L : lanes_) {
    for (auto& t : L->th)
      if (t.joinable()) t.join();
    L->th.clear();
  }
  (void)was;
}

void Engine::pause() {
  pause_ = true;
  if (!run_) return;
  const auto t0 = Clock::now();
  for (;;) {
    bool idle = paused_ack_.load();
    for (auto& L : lanes_) idle = idle && L->done.load() == L->head;
    if (idle || !run_) return;
    if (Clock::now() - t0 > std::chrono::seconds(10)) throw std::runtime_error("iox: pause timed out");
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

void Engine::resume() {
  paused_ack_ = false;
  pause_ = false;
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
  std::lock_guard<std::mutex> g(lat_mu_);
  std::vector<double> v;
  v.swap(lat_us_);
  return v;
}

std::unordered_map<std::string, uint64_t> Engine::stats() const {
  return {{"rx", st_rx_.load()},         {"tx", st_tx_.load()},         {"drop", st_drop_.load()},
          {"punt", st_punt_.load()},     {"recirc", st_recirc_.load()}, {"replicas", st_reps_.load()},
          {"bursts", st_bursts_.load()}, {"side_passes", st_side_.load()}, {"no_netdev", st_no_port_.load()},
          {"punt_dropped", st_punt_drop_.load()}, {"tx_full", st_tx_full_.load()},
          {"publish_ns", st_pub_ns_.load()}, {"deliver_ns", st_deliver_ns_.load()},
          {"rx_idle_polls", st_idle_.load()}, {"rx_wait_tx", st_wait_tx_.load()}};
}

void Engine::punt(uint32_t in_port, uint32_t reason, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb) {
  std::lock_guard<std::mutex> g(punt_mu_);
  if (punts_.size() >= 4096) { st_punt_drop_.fetch_add(1); return; }
  Punt p;
  p.in_port = (uint16_t)in_port;
  p.reason = (uint8_t)reason;
  p.frame.reserve(na + nb);
  p.frame.insert(p.frame.end(), a, a + na);
  if (nb) p.frame.insert(p.frame.end(), b, b + nb);
  punts_.push_back(std::move(p));
  st_punt_.fetch_add(1, std::memory_order_relaxed);
}

void Engine::send(const PortTab& tab, uint32_t port, const uint8_t* x, uint32_t nx, const uint8_t* h, uint32_t nh,
                  const uint8_t* t, uint32_t nt, std::vector<Port*>& touched, TxTally& tally) {
  if (port < redirect_.size() && redirect_[port] != 0xFFFFFFFFu) port = redirect_[port];   // tunnel -> underlay
  Port* p = port < tab.size() ? tab[port].get() : nullptr;
  if (!p) { ++tally.no_port; return; }
  if (p->tx(x, nx, h, nh, t, nt)) {
    ++tally.tx;
    if (touched.empty() || touched.back() != p)
      if (std::find(touched.begin(), touched.end(), p) == touched.end()) touched.push_back(p);
  } else {
    ++tally.full;
  }
}

void Engine::rx_loop() {
  std::vector<RxRef> buf(burst_);
  uint32_t rr = 0;
  std::shared_ptr<const PortTab> cached;
  std::vector<std::pair<uint32_t, Port*>> active;   // configured ports of the snapshot, in id order
  try {
    while (run_) {
      if (pause_) {
        paused_ack_ = true;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
        continue;
      }
      paused_ack_ = false;
      auto tab = std::atomic_load(&ports_);
      if (tab != cached) {
        cached = tab;
        active.clear();
        for (uint32_t i = 0; i < (uint32_t)tab->size(); ++i)
          if ((*tab)[i]) active.emplace_back(i, (*tab)[i].get());
      }
      for (auto& a : active) a.second->reclaim();
      recirc_->reclaim();
      // room: a burst of k frames takes ceil(k / 64) chunks on its backend; bound the take by
      // the fullest lane (frames are steered after they are read)
      uint32_t take = burst_;
      for (auto& L : lanes_) {
        if (!L->be->ready() || L->head - L->done.load(std::memory_order_acquire) >= inflight_) {
          take = 0;
          st_wait_tx_.fetch_add(1, std::memory_order_relaxed);
          break;
        }
        // slots are reusable once DELIVERED (their out slot / meta read), not merely completed
        const uint64_t used = L->be->published() - L->freed_pos.load(std::memory_order_acquire);
        const uint64_t room = L->be->capacity() > used ? L->be->capacity() - used : 0;
        take = (uint32_t)std::min<uint64_t>(take, room & ~63ull);
      }
      if (take == 0) { _mm_pause(); continue; }
      const uint64_t t_rx = now_ns();
      uint32_t got = 0;
      auto stage = [&](uint32_t pid, Port* p, const RxRef& r) {
        if (r.seq + 1 - p->seen_ <= 0x7FFFFFFFu) p->seen_ = r.seq + 1;
        if (r.len < 14 || r.len > kMaxFrame) { p->complete(r.seq); return; }   // runt / oversize / own tx
        const uint32_t in_port = r.in_port != ~0u ? r.in_port : pid;
        p->rx_pkts.fetch_add(1, std::memory_order_relaxed);
        p->rx_bytes.fetch_add(r.len, std::memory_order_relaxed);
        const uint32_t o = owner_of_frame(r.data, r.len, in_port);
        lanes_[o]->stage.push_back(Pkt{in_port, r.seq, r.data, r.len, p});
        ++got;
      };
      {
        const uint32_t n = recirc_->rx(buf.data(), take);
        for (uint32_t i = 0; i < n; ++i) stage(0, recirc_.get(), buf[i]);
      }
      // every port gets an equal share of the burst first (round-robin start), then leftovers
      const uint32_t np = (uint32_t)active.size();
      if (np) {
        const uint32_t share = std::max<uint32_t>(1, take / np);
        for (int pass = 0; pass < 2 && got < take; ++pass) {
          for (uint32_t k = 0; k < np && got < take; ++k) {
            const auto& a = active[(rr + k) % np];
            const uint32_t n = a.second->rx(buf.data(), std::min(take - got, pass ? take : share));
            for (uint32_t i = 0; i < n; ++i) stage(a.first, a.second, buf[i]);
          }
        }
        rr = (rr + 1) % np;
      }
      if (got == 0) {
        st_idle_.fetch_add(1, std::memory_order_relaxed);
        _mm_pause();
        continue;
      }
      for (auto& Lp : lanes_) {
        Lane* L = Lp.get();
        if (L->stage.empty()) continue;
        std::lock_guard<std::mutex> pg(L->pub_mu);
        Backend& be = *L->be;
        const uint32_t k = (uint32_t)L->stage.size();
        const uint32_t npad = (k + 63u) & ~63u;
        const uint64_t start = be.published();
        uint32_t* im = be.in_meta();
        const uint32_t cmask = be.capacity() - 1;
        Burst& b = L->slots[L->head % inflight_];   // free: head - done < inflight
        b.start = start;
        b.end = start + npad;
        b.t_rx_ns = t_rx;
        b.side = false;
        b.reps.clear();
        b.xhdr.clear();
        for (uint32_t i = 0; i < k; ++i) {
          const Pkt& q = L->stage[i];
          uint8_t* slot = be.in_slot((uint32_t)(start + i));
          const uint32_t h = std::min<uint32_t>(q.len, kSlotBytes);
          std::memcpy(slot, q.data, h);
          if (h < kSlotBytes) std::memset(slot + h, 0, kSlotBytes - h);
          im[(start + i) & cmask] = (q.port & 0xFFFFu) | (q.len << 16);
          b.side = b.side || needs_side(q.port);
        }
        for (uint32_t i = k; i < npad; ++i) im[(start + i) & cmask] = kRingPadMeta;
        b.pkts.swap(L->stage);
        L->stage.clear();
        b.id = L->head;
        b.left.store(workers_, std::memory_order_relaxed);
        b.state.store(1, std::memory_order_release);
        ++L->head;
        const uint64_t tp0 = now_ns();
        be.publish(npad);
        st_pub_ns_.fetch_add(now_ns() - tp0, std::memory_order_relaxed);
        st_bursts_.fetch_add(1, std::memory_order_relaxed);
      }
      st_rx_.fetch_add(got, std::memory_order_relaxed);
    }
  } catch (const std::exception& e) {
    fail(std::string("rx: ") + e.what());
  }
}

void Engine::side_pass(Lane* L, uint64_t from_id) {
  std::lock_guard<std::mutex> pg(L->pub_mu);   // no publish on this lane during the pass
  Backend& be = *L->be;
  const auto t0 = Clock::now();
  while (be.completed() < be.published()) {     // nothing in flight: the side list is final
    _mm_pause();
    if (Clock::now() - t0 > std::chrono::seconds(5)) throw std::runtime_error("side pass: ring did not drain");
  }
  SideBatch sb;
  be.side_pass(sb);
  st_side_.fetch_add(1, std::memory_order_relaxed);
  // Every listed packet belongs to a burst not delivered yet (earlier bursts were covered by
  // earlier passes): hand each replica / outer header to its burst, from_id .. head - 1.
  const uint32_t cap = be.capacity();
  auto burst_of = [&](uint32_t pos) -> Burst* {
    for (uint64_t id = from_id; id < L->head; ++id) {
      Burst& b = L->slots[id % inflight_];
      if (((pos - (uint32_t)b.start) & (cap - 1)) < (uint32_t)b.pkts.size()) return &b;
    }
    return nullptr;
  };
  for (auto& r : sb.reps) {
    Burst* b = burst_of(r.src_pos & (cap - 1));
    if (b) b->reps.push_back(r);
  }
  if (!sb.xall.empty()) {
    for (uint64_t id = from_id; id < L->head; ++id) {
      Burst& b = L->slots[id % inflight_];
      for (uint32_t i = 0; i < (uint32_t)b.pkts.size(); ++i) {
        const uint32_t pos = (uint32_t)((b.start + i) & (cap - 1));
        if (be.out_meta()[pos] & kMetaXhdr)
          b.xhdr.emplace_back(pos, std::vector<uint8_t>(sb.xall.begin() + (size_t)pos * kXhdrBytes,
                                                        sb.xall.begin() + (size_t)(pos + 1) * kXhdrBytes));
      }
    }
  }
  L->side_upto = be.published();
}

void Engine::deliver(Lane* L, Burst& b, uint32_t w, std::vector<Port*>& touched) {
  Backend& be = *L->be;
  const uint32_t cmask = be.capacity() - 1;
  const uint32_t* om = be.out_meta();
  auto tab = std::atomic_load(&ports_);
  auto mine = [&](uint32_t port) {
    if (port < redirect_.size() && redirect_[port] != 0xFFFFFFFFu) port = redirect_[port];
    return port % workers_ == w;
  };
  TxTally tally;
  const uint32_t np = (uint32_t)b.pkts.size();
  constexpr uint32_t kAhead = 8;   // out slots / payloads of later packets are fetched ahead
  for (uint32_t i = 0; i < np; ++i) {
    if (i + kAhead < np) {
      const uint32_t pa = (uint32_t)((b.start + i + kAhead) & cmask);
      if (meta_port(om[pa]) % workers_ == w) __builtin_prefetch(be.out_slot(pa), 0, 0);
    }
    const Pkt& q = b.pkts[i];
    const uint32_t pos = (uint32_t)((b.start + i) & cmask);
    const uint32_t meta = om[pos];
    const uint32_t reason = meta_reason(meta), oport = meta_port(meta), olen = meta_len(meta);
    if (reason == 0) {
      if (!mine(oport)) continue;
      const uint8_t* x = nullptr;
      uint32_t xl = 0;
      if (meta & kMetaXhdr) {
        for (const auto& e : b.xhdr)
          if (e.first == pos) { x = e.second.data(); xl = xhdr_len(x); break; }
        if (!x) { ++tally.drop; continue; }   // never sent bare
      }
      uint32_t hl = 0, to = 0;
      out_tail(q.len, olen, xl, hl, to);
      if (to > q.len) to = q.len;
      send(*tab, oport, x, xl, be.out_slot(pos), hl, q.data + to, q.len - to, touched, tally);
    } else if (w != 0) {
      continue;
    } else if (reason == kRecirc && olen <= q.len) {
      recirc_->push(oport, q.data + (q.len - olen), olen);   // terminated tunnel: the inner frame re-enters
      st_recirc_.fetch_add(1, std::memory_order_relaxed);
    } else if (reason == kRecirc6) {
      punt(q.port, reason, q.data, q.len, nullptr, 0);       // the VNI lookup needs the whole frame
    } else {
      ++tally.drop;
    }
  }
  for (const Replica& r : b.reps) {
    const uint32_t i = (uint32_t)((r.src_pos - (uint32_t)b.start) & cmask);
    const Pkt& q = b.pkts[i];
    uint32_t hl = 0, to = 0;
    const uint32_t rlen = meta_len(r.meta), rr = meta_reason(r.meta);
    out_tail(q.len, rlen, 0, hl, to);
    if (to > q.len) to = q.len;
    if (rr) {
      if (w == 0) punt(q.port, rr, r.hdr, hl, q.data + to, q.len - to);   // ARP trap: the slow path's copy
    } else if (mine(meta_port(r.meta))) {
      send(*tab, meta_port(r.meta), nullptr, 0, r.hdr, hl, q.data + to, q.len - to, touched, tally);
      ++tally.reps;
    }
  }
  // one atomic per counter per burst (per-packet atomics on shared lines cost more than the copy)
  if (tally.tx) st_tx_.fetch_add(tally.tx, std::memory_order_relaxed);
  if (tally.full) st_tx_full_.fetch_add(tally.full, std::memory_order_relaxed);
  if (tally.no_port) st_no_port_.fetch_add(tally.no_port, std::memory_order_relaxed);
  if (tally.drop) st_drop_.fetch_add(tally.drop, std::memory_order_relaxed);
  if (tally.reps) st_reps_.fetch_add(tally.reps, std::memory_order_relaxed);
}

void Engine::finish(Lane* L, Burst& b) {
  for (const Pkt& q : b.pkts) q.holder->complete(q.seq);
  const double us = (double)(now_ns() - b.t_rx_ns) * 1e-3;
  {
    std::lock_guard<std::mutex> g(lat_mu_);
    if (lat_us_.size() < (1u << 20)) lat_us_.push_back(us);
  }
  b.pkts.clear();
  b.reps.clear();
  b.xhdr.clear();
  L->freed_pos.store(b.end, std::memory_order_release);
  b.state.store(0, std::memory_order_release);
  L->done.fetch_add(1, std::memory_order_release);
}

void Engine::tx_loop(Lane* L, uint32_t w) {
  try {
    L->be->thread_init();
    const uint32_t cmask = L->be->capacity() - 1;
    std::vector<Port*> touched;
    for (uint64_t cur = 0;;) {
      Burst& b = L->slots[cur % inflight_];
      const uint32_t want = w == 0 ? 1u : 2u;
      uint32_t spin = 0;
      while (!(b.state.load(std::memory_order_acquire) >= want && b.id == cur)) {
        if (!run_ && L->done.load() == L->head) return;
        _mm_pause();
        if ((++spin & 0xFFFFu) == 0) std::this_thread::yield();
      }
      if (w == 0) {
        // leader: completion, side pass, then the burst is ready for every worker
        const auto t0 = Clock::now();
        spin = 0;
        while (!L->be->range_done(b.start, b.end)) {
          _mm_pause();
          if ((++spin & 0xFFFu) == 0) {
            const auto waited = Clock::now() - t0;
            if (waited > std::chrono::milliseconds(200) && !L->be->alive())
              throw std::runtime_error("tx: the ring kernel is gone (device deadline or fault)");
            if (waited > std::chrono::seconds(5)) throw std::runtime_error("tx: burst not completed within 5 s");
          }
        }
        bool side = b.side;
        const uint32_t* om = L->be->out_meta();
        for (uint64_t p = b.start; p < b.start + b.pkts.size() && !side; ++p)
          side = (om[p & cmask] & (kMetaFlood | kMetaXhdr)) != 0;
        if (side && b.end > L->side_upto) side_pass(L, cur);
        b.state.store(2, std::memory_order_release);
      }
      const uint64_t td0 = now_ns();
      touched.clear();
      deliver(L, b, w, touched);
      for (Port* p : touched) p->flush();
      st_deliver_ns_.fetch_add(now_ns() - td0, std::memory_order_relaxed);
      if (b.left.fetch_sub(1, std::memory_order_acq_rel) == 1) finish(L, b);
      ++cur;
    }
  } catch (const std::exception& e) {
    fail(std::string("tx: ") + e.what());
  }
}

}  // namespace iox
}  // namespace nfdp
