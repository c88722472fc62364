// iox.h — native packet I/O engine: vport netdevs / shared-memory vports <-> the data plane.
//
// The reference's data ports never touch a per-frame interpreter loop: OvS-DPDK polls NIC / vhost
// queues from PMD threads (ovs-dp/ovsdp.go:39-55 binds them `type=dpdk`), the IPU's FXP is
// silicon.  This engine is the MI355X data plane's equivalent, in C++ with Python only
// configuring it.  It is organised like a multi-queue NIC driver:
//
//   queue q (one rx thread + its tx workers) owns a group of ports
//     --rx thread q--> owner GPU g = owner_of(toeplitz(FlowKey), N) (the RSS a NIC would do; 1 GPU: 0)
//       -> 64-B header slot + ingress meta written straight into ring queue q of GPU g (pinned host
//          memory the resident ring kernel reads over PCIe; one kernel per GPU serves every queue,
//          ring.h), bursts padded to whole 64-packet chunks, published at once
//     --tx workers of queue q--> completion flags of each lane (q, g) in order -> egress frames
//          = [outer hdr] ++ out slot[:hl] ++ in_frame[to:len], written to the egress ports in one
//          locked batch per port and burst (the payload never left the rx buffer)
//     -> side work (flood replicas, mirror / ARP copies, MAC learning, tunnel outer headers) is done
//          per burst by the tx leader on the CPU (pipeline.h side_stage over the burst's flagged
//          packets, against a host snapshot of the tables): nothing waits for the ring to drain;
//          learn events go to a learner thread that updates every GPU's MAC table
//     -> rx buffers are handed back to their port in rx order once every frame below is sent.
//
// Queues share nothing on the packet path: no lock, no shared counter line (statistics are per
// queue, port rx counters are per-burst stores of the single rx thread that owns the port).
// Configuration the threads read (steering, redirects, side ports, side tables) is published
// copy-on-write (RCU style): a commit swaps it in without stopping traffic; `hold()` briefly
// stops publication (no drain) so an epoch flip on every GPU plus a configuration swap take
// effect between two bursts of every queue.
//
// Backends: `GpuBackend` (RingEngine with host slots and one ring queue per engine queue: the
// persistent HIP kernel) or `OracleBackend` (the bit-exact C++ pipeline, synchronous: CPU tests /
// no-GPU nodes).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "host.h"
#include "memif.h"
#include "ring.h"

namespace nfdp {
namespace iox {

// Owner GPU of a frame (RSS): owner_of(toeplitz(FlowKey), n) for IPv4 frames the ingress stage
// accepts (the key the flow table is sharded by), in_port % n otherwise.  `hdr` holds the first
// min(len, 64) bytes; `ports` is the port table (kMaxPorts rows).
// `v6`: the data planes keep IPv6 flows / rules, so an IPv6 frame's owner is its folded 5-tuple's
// (the key the owner's table holds); otherwise IPv6 steers by ingress port.
uint32_t frame_owner(const uint8_t* hdr, uint32_t len, uint32_t in_port, const PortEntry* ports, const uint8_t* rss_key,
                     uint32_t n, bool v6 = false);

// Toeplitz hash from byte tables (16 key bytes x 256 values, XOR-linear in the key): the CPU
// twin of the kernels' LDS byte tables, ~20x the bit-serial toeplitz_scalar.  Bit-exact with it.
struct ToeplitzTab {
  std::vector<uint32_t> tab;   // [16][256]
  ToeplitzTab() = default;
  explicit ToeplitzTab(const uint8_t* rss_key);
  uint32_t operator()(const FlowKey& k) const {
    const uint32_t w[4] = {k.src_ip, k.dst_ip, k.ports, k.meta};
    uint32_t h = 0;
    for (int b = 0; b < 16; ++b) h ^= tab[(size_t)b * 256 + ((w[b >> 2] >> (8 * (b & 3))) & 0xFFu)];
    return h;
  }
};

// ---------------------------------------------------------------------------------- ports
struct RxRef {
  const uint8_t* data;
  uint32_t len;
  uint32_t seq;       // port-local rx sequence number (released in order)
  uint32_t in_port;   // ingress port for the pipeline (~0u: the port's own id)
};

// One frame of a tx batch, assembled from up to three pieces (outer header, rewritten header,
// payload tail).
struct TxItem {
  const uint8_t* a; uint32_t na;
  const uint8_t* b; uint32_t nb;
  const uint8_t* c; uint32_t nc;
};

class Port {
 public:
  explicit Port(uint32_t window);
  virtual ~Port() = default;
  // Up to `max` received frames; each stays valid until its sequence number is released.
  virtual uint32_t rx(RxRef* out, uint32_t max) = 0;
  // A batch of frames into tx queue `txq` (mod tx_queues()) under one lock acquisition and one
  // ring commit; returns how many were written (the rest found no room and are dropped, as on a
  // full NIC queue).  Thread safe; writers of different tx queues never share a lock.
  uint32_t tx_batch(const TxItem* items, uint32_t n, uint32_t txq = 0);
  bool tx(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) {
    const TxItem it{a, na, b, nb, c, nc};
    return tx_batch(&it, 1) == 1;
  }
  virtual uint32_t tx_queues() const { return 1; }
  // Memory every frame rx() hands out lies in (zero-copy rx maps it for the pipeline), or null.
  virtual std::pair<const uint8_t*, size_t> rx_memory() const { return {nullptr, 0}; }
  // A frame is done (sent or dropped): any thread.  reclaim(): the owning rx thread only, after
  // marking what rx() handed out (handed_out: sequence numbers up to seq are in use).
  void complete(uint32_t seq) { done_[seq & mask_].store(1, std::memory_order_release); }
  void handed_out(uint32_t seq) {
    if (seq + 1 - seen_ <= 0x7FFFFFFFu) seen_ = seq + 1;
  }
  void reclaim();
  virtual std::string kind() const = 0;
  // rx counters: single writer (the rx thread owning the port) adds a burst at a time
  void count_rx(uint64_t pkts, uint64_t bytes) {
    rx_pkts.store(rx_pkts.load(std::memory_order_relaxed) + pkts, std::memory_order_relaxed);
    rx_bytes.store(rx_bytes.load(std::memory_order_relaxed) + bytes, std::memory_order_relaxed);
  }
  alignas(64) std::atomic<uint64_t> rx_pkts{0}, rx_bytes{0};
  // tx counters: added once per batch
  alignas(64) std::atomic<uint64_t> tx_pkts{0}, tx_full{0}, tx_bytes{0};
  static constexpr uint32_t kMaxTxQueues = 16;

 protected:
  // under tx queue q's lock (q < tx_queues())
  virtual bool tx_locked(uint32_t q, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c,
                         uint32_t nc) = 0;
  virtual void flush_locked(uint32_t) {}
  virtual void release_to(uint32_t seq_end) = 0;   // every frame below seq_end is done
  void set_first_seq(uint32_t s) { rel_ = s; seen_ = s; }
  // Drop the pipeline's mapping of rx_memory(); `after` runs once it is gone (it may be deferred
  // while GPU rings run: a port that frees the memory does so in `after`).  False: nothing was
  // mapped by this port (`after` not called).
  bool rx_mapped() const { return (bool)zc_.release; }
  bool unmap_rx(std::function<void()> after = nullptr) {
    zc_.lo = zc_.hi = nullptr;
    if (!zc_.release) return false;
    auto f = std::move(zc_.release);
    zc_.release = nullptr;
    f(std::move(after));
    return true;
  }
  uint32_t window() const { return mask_ + 1; }
  struct alignas(64) TxLock { std::mutex mu; };
  TxLock tx_mu_[kMaxTxQueues];

 private:
  std::unique_ptr<std::atomic<uint8_t>[]> done_;
  uint32_t mask_;
  uint32_t rel_ = 0;   // next sequence number to release
  uint32_t seen_ = 0;  // rx sequence numbers handed out so far (upper bound of reclaim)
  // The rx queue polling this port (-1: none).  The rx side is single-consumer: a port moved to
  // another queue is polled there only once its previous rx thread has let go of it.
  std::atomic<int> rx_owner_{-1};
  // Zero-copy rx (Engine::set_zero_copy): rx_memory() as the pipelines see it.  Frames in
  // [lo, hi) are read at data + off[g] by backend g; written by the engine before the port is
  // published to the packet threads, read-only afterwards.
  struct Mapped {
    const uint8_t* lo = nullptr;
    const uint8_t* hi = nullptr;
    std::vector<int64_t> off;
    // unregisters the memory (the registering backend's), then runs its argument
    std::function<void(std::function<void()>)> release;
  };
  Mapped zc_;
  friend class Engine;
};

// Shared-memory vport (memif.h): the pod produces ring 0, the engine rings 1..tx_rings (tx
// queue q writes ring 1 + q).
// AF_XDP port on a netdev (the engine's end of a veth pair, or a NIC queue): an XSK socket with its
// UMEM (rx frames handed to the kernel through the fill ring, tx frames from a free pool reclaimed
// through the completion ring) and a 6-instruction XDP program, attached to the netdev through a
// BPF link, that redirects every frame of queue 0 to the socket (bpf_redirect_map on an XSKMAP,
// XDP_PASS when the socket is not there).  Frames reach the engine without an skb or a packet
// socket, the way kernel-netdev pods that are not memif-aware can still be served in bulk.
// Copy mode (veth has no zero-copy AF_XDP); native XDP when the driver has it, else generic.
class XdpPort : public Port {
 public:
  XdpPort(const std::string& ifname, uint32_t frames, uint32_t frame_size = 2048, uint32_t queue = 0);
  ~XdpPort() override;
  uint32_t rx(RxRef* out, uint32_t max) override;
  std::string kind() const override { return "af_xdp"; }
  bool native_mode() const { return native_; }   // XDP in the driver (false: generic / skb mode)

 protected:
  bool tx_locked(uint32_t q, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c,
                 uint32_t nc) override;
  void flush_locked(uint32_t q) override;
  void release_to(uint32_t seq_end) override;

 private:
  struct Ring {                       // one mmapped AF_XDP ring (producer / consumer / descriptors)
    uint32_t* prod = nullptr;
    uint32_t* cons = nullptr;
    uint32_t* flags = nullptr;
    void* desc = nullptr;
    void* map = nullptr;
    size_t map_len = 0;
    uint32_t mask = 0;
  };
  void reclaim_tx();                  // completion ring -> free tx frames
  void kick_tx();                     // publish the tx ring and have the kernel send it all
  void close_all();
  int fd_ = -1, map_fd_ = -1, prog_fd_ = -1, link_fd_ = -1;
  uint8_t* umem_ = nullptr;
  size_t umem_len_ = 0;
  uint32_t nframes_, fsize_;
  Ring rx_, tx_, fill_, comp_;
  std::vector<uint64_t> rx_addr_;     // by rx sequence number: the UMEM frame it holds
  uint32_t rx_next_ = 0, rel_done_ = 0;
  std::vector<uint64_t> tx_free_;     // tx frames the kernel gave back
  uint32_t tx_prod_ = 0;              // private tx producer (published by flush)
  bool native_ = false;
};

class MemifPort : public Port {
 public:
  MemifPort(const std::string& path, uint32_t ring_size, uint32_t buf_size, uint32_t tx_rings = 1);
  ~MemifPort() override;
  uint32_t rx(RxRef* out, uint32_t max) override;
  std::string kind() const override { return "memif"; }
  const std::string& path() const { return reg_.path(); }
  uint32_t tx_queues() const override { return nprod_; }
  std::pair<const uint8_t*, size_t> rx_memory() const override { return {reg_.base(), reg_.bytes()}; }
  const memif::Region& region() const { return reg_; }

 protected:
  bool tx_locked(uint32_t q, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c,
                 uint32_t nc) override {
    // (the engine's header piece `b` is always a 64-B slot: an out slot or a replica's header)
    if (!na && !nc && nb <= 64 && b) return prod_[q].put_slot(b, nb);
    return prod_[q].put(a, na, b, nb, c, nc);
  }
  void flush_locked(uint32_t q) override { prod_[q].commit(); }
  void release_to(uint32_t seq_end) override { cons_.release_to(seq_end); }

 private:
  memif::Region reg_;
  memif::Consumer cons_;
  struct alignas(64) Prod : memif::Producer {};
  std::unique_ptr<Prod[]> prod_;
  uint32_t nprod_;
  bool unlink_;
};

// AF_PACKET TPACKET_V2 rx + tx rings on a netdev (the VSP-side end of a pod's veth pair).
class PacketPort : public Port {
 public:
  PacketPort(const std::string& ifname, uint32_t frames, uint32_t frame_size);
  ~PacketPort() override;
  uint32_t rx(RxRef* out, uint32_t max) override;
  std::string kind() const override { return "af_packet"; }

 protected:
  bool tx_locked(uint32_t q, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c,
                 uint32_t nc) override;
  void flush_locked(uint32_t q) override;
  void release_to(uint32_t seq_end) override;

 private:
  uint8_t* frame(int ring, uint32_t i) const;
  int fd_ = -1;
  uint8_t* map_ = nullptr;
  size_t map_bytes_ = 0;
  uint32_t nframes_, fsize_;
  uint32_t rx_next_ = 0, tx_next_ = 0, rel_done_ = 0;
  std::vector<uint8_t> vlan_copy_;   // frames whose 802.1Q tag the kernel moved to the aux data
};

// A TAP (or any packet) fd: one read() / write() per frame, no copies beyond the syscall's.
class FdPort : public Port {
 public:
  FdPort(int fd, uint32_t nbufs, uint32_t buf_size);
  uint32_t rx(RxRef* out, uint32_t max) override;
  std::string kind() const override { return "fd"; }

 protected:
  bool tx_locked(uint32_t q, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c,
                 uint32_t nc) override;
  void release_to(uint32_t seq_end) override { freed_.store(seq_end, std::memory_order_release); }

 private:
  int fd_;
  uint32_t nbufs_, bsize_;
  std::vector<uint8_t> bufs_;
  uint32_t next_ = 0;
  std::atomic<uint32_t> freed_{0};
  std::vector<uint8_t> txbuf_;
};

// Frames re-entering the pipeline (terminated tunnels, slow-path re-injection): owned copies.
class RecircPort : public Port {
 public:
  explicit RecircPort(uint32_t window) : Port(window) {}
  void push(uint32_t in_port, const uint8_t* f, uint32_t n);
  uint32_t rx(RxRef* out, uint32_t max) override;
  std::string kind() const override { return "recirc"; }

 protected:
  bool tx_locked(uint32_t, const uint8_t*, uint32_t, const uint8_t*, uint32_t, const uint8_t*, uint32_t) override {
    return false;
  }
  void release_to(uint32_t seq_end) override;

 private:
  std::mutex mu_;
  std::deque<std::pair<uint32_t, std::vector<uint8_t>>> q_;       // waiting
  std::deque<std::pair<uint32_t, std::vector<uint8_t>>> live_;    // handed out, not released yet
  uint32_t next_ = 0, base_ = 0;
};

// ---------------------------------------------------------------------------------- side tables
// Host copies of the tables the side pass reads (ports, MAC table, LAG, flood groups, tunnels,
// RSS key), taken at commit time: the control plane may change its own models at any moment,
// the tx leaders read this immutable-but-for-learning snapshot.
class SideTables {
 public:
  struct Src {   // host arrays (copied)
    const PortEntry* ports; size_t n_ports;
    const MacEntry* macs; uint32_t mac_mask;
    const uint16_t* lag; uint32_t n_lag_groups;
    const uint16_t* flood; size_t flood_rows; uint32_t n_flood;
    const TunnelEntry* tunnels; uint32_t n_tunnels;
    const Tunnel6Entry* tunnels6; uint32_t n_tunnels6;
    const uint8_t* rss_key;
    bool v6;   // IPv6 flows / rules in the data plane: IPv6 keys are folded (make_key)
  };
  explicit SideTables(const Src& s);
  const TablesView& view() const { return t_; }
  const ToeplitzTab& hash() const { return hash_; }
  // learning (learner thread) vs the side pass's learn check (tx leaders)
  std::shared_mutex mac_mu;
  MacEntry* macs() { return macs_.data(); }
  uint32_t mac_mask() const { return t_.mac_mask; }
  bool has_macs() const { return !macs_.empty(); }

 private:
  TablesView t_{};
  std::vector<PortEntry> ports_;
  std::vector<MacEntry> macs_;
  std::vector<uint16_t> lag_, flood_;
  std::vector<TunnelEntry> tun_;
  std::vector<Tunnel6Entry> tun6_;
  std::vector<uint8_t> rss_;
  ToeplitzTab hash_;
};

// ---------------------------------------------------------------------------------- backends
class Backend {
 public:
  virtual ~Backend() = default;
  virtual uint32_t queues() const = 0;
  virtual uint32_t capacity() const = 0;                         // slots per queue
  virtual uint8_t* in_slot(uint32_t q, uint32_t pos) = 0;        // pos: ring position (mod capacity)
  virtual uint32_t* in_meta(uint32_t q) = 0;
  virtual const uint8_t* out_slot(uint32_t q, uint32_t pos) = 0;
  virtual const uint32_t* out_meta(uint32_t q) = 0;
  virtual uint64_t published(uint32_t q) = 0;
  virtual uint64_t publish(uint32_t q, uint32_t n) = 0;           // multiple of 64
  virtual bool range_done(uint32_t q, uint64_t start, uint64_t end) = 0;   // positions [start, end) processed
  virtual bool ready() = 0;                                       // can take a publish now (ring running)
  virtual bool alive() { return true; }                           // the pipeline still makes progress (slow check)
  // MAC-learn events ({mac_lo, mac_hi | bridge << 16, port, 0} each) into the MAC table the
  // pipeline reads; learner thread only.
  virtual void apply_learn(const uint32_t* ev, uint32_t n, uint32_t stamp) = 0;
  virtual void thread_init() {}
  // Zero-copy rx.  frame_addrs(q) non-null: the pipeline reads slot i's frame at the address
  // frame_addrs(q)[i] names (the engine writes one for every slot it publishes: a mapped port's
  // frame, or in_slot_addr() for a copied frame or a filler slot).
  virtual uint64_t* frame_addrs(uint32_t) { return nullptr; }
  virtual uint64_t in_slot_addr(uint32_t q, uint32_t pos) { return reinterpret_cast<uint64_t>(in_slot(q, pos)); }
  // Make host memory [p, p + n) readable by the pipeline: its address there (0: cannot).  Sets
  // *release when this call registered it (run it once nothing of the memory is in flight).
  virtual uint64_t map_host(const void*, size_t, std::function<void(std::function<void()>)>*) { return 0; }
  // GPU-direct egress (ring.h GdeRing): the pipeline's grid can deliver memif frames itself;
  // set / clear a (port, queue) ring entry (returns the control-mailbox entry to wait for, 0 when
  // applied at once); wait until the grid applied it.
  virtual bool gde_ok() { return false; }
  virtual uint64_t gde_set(uint32_t, uint32_t, uint64_t, uint64_t, uint64_t, uint32_t, uint32_t, uint32_t, uint32_t) {
    return 0;
  }
  virtual uint64_t gde_clear(uint32_t, uint32_t) { return 0; }
  virtual bool gde_wait(uint64_t, double) { return true; }
};

class GpuBackend : public Backend {
 public:
  explicit GpuBackend(RingEngine* ring);
  ~GpuBackend() override;
  uint32_t queues() const override { return ring_->queues(); }
  uint32_t capacity() const override { return ring_->capacity(); }
  uint8_t* in_slot(uint32_t q, uint32_t pos) override { return in_ + ((size_t)q * cap_ + (pos & (cap_ - 1))) * kSlotBytes; }
  uint32_t* in_meta(uint32_t q) override { return im_ + (size_t)q * cap_; }
  const uint8_t* out_slot(uint32_t q, uint32_t pos) override { return out_ + ((size_t)q * cap_ + (pos & (cap_ - 1))) * kSlotBytes; }
  const uint32_t* out_meta(uint32_t q) override { return om_ + (size_t)q * cap_; }
  uint64_t published(uint32_t q) override { return ring_->published(q); }
  uint64_t publish(uint32_t q, uint32_t n) override { return ring_->publish(n, false, q); }
  bool range_done(uint32_t q, uint64_t start, uint64_t end) override { return ring_->range_done(start, end, q); }
  bool ready() override { return ring_->running(); }
  bool alive() override { return ring_->alive(); }
  void apply_learn(const uint32_t* ev, uint32_t n, uint32_t stamp) override;
  void thread_init() override;
  uint64_t* frame_addrs(uint32_t q) override {
    return ring_->frame_addrs_on() ? ring_->frame_addrs() + (size_t)q * cap_ : nullptr;
  }
  uint64_t in_slot_addr(uint32_t q, uint32_t pos) override { return ring_->in_slot_addr(q, pos); }
  uint64_t map_host(const void* p, size_t n, std::function<void(std::function<void()>)>* release) override;
  bool gde_ok() override { return ring_->gde_on(); }
  uint64_t gde_set(uint32_t port, uint32_t q, uint64_t ctl, uint64_t desc, uint64_t buf, uint32_t ring_size,
                   uint32_t buf_size, uint32_t head, uint32_t tail) override {
    return ring_->gde_set(port, q, ctl, desc, buf, ring_size, buf_size, head, tail);
  }
  uint64_t gde_clear(uint32_t port, uint32_t q) override { return ring_->gde_clear(port, q); }
  bool gde_wait(uint64_t seq, double timeout_s) override { return ring_->wait_ctrl(seq, timeout_s); }

 private:
  RingEngine* ring_;
  uint32_t cap_;
  uint8_t* in_; uint32_t* im_; uint8_t* out_; uint32_t* om_;
  hipStream_t learn_stream_{};
  uint32_t* d_learn_ = nullptr;   // device: [cap] events, then count + dropped words
  uint32_t learn_cap_ = 0;
};

class OracleBackend : public Backend {
 public:
  explicit OracleBackend(uint32_t capacity, uint32_t queues = 1);
  uint32_t queues() const override { return nq_; }
  uint32_t capacity() const override { return cap_; }
  uint8_t* in_slot(uint32_t q, uint32_t pos) override { return in_.data() + ((size_t)q * cap_ + (pos & (cap_ - 1))) * kSlotBytes; }
  uint32_t* in_meta(uint32_t q) override { return im_.data() + (size_t)q * cap_; }
  const uint8_t* out_slot(uint32_t q, uint32_t pos) override { return out_.data() + ((size_t)q * cap_ + (pos & (cap_ - 1))) * kSlotBytes; }
  const uint32_t* out_meta(uint32_t q) override { return om_.data() + (size_t)q * cap_; }
  uint64_t published(uint32_t q) override { return prod_[q].load(std::memory_order_acquire); }
  uint64_t publish(uint32_t q, uint32_t n) override;
  bool range_done(uint32_t q, uint64_t, uint64_t end) override {
    return !gate_.load(std::memory_order_acquire) && end <= published(q);
  }
  bool ready() override { return configured_.load(); }
  // Test hook: while set, published bursts are processed but never reported complete (they stay
  // in flight, as on a busy GPU), so a test can change the configuration under them.
  void set_completion_gate(bool on) { gate_.store(on, std::memory_order_release); }
  void apply_learn(const uint32_t* ev, uint32_t n, uint32_t stamp) override;
  // tables / counters of the CPU DataPlane (replaced after every commit, while the engine is paused)
  void configure(const TablesView& t, uint64_t* flow_ctr, uint64_t* port_ctr, uint64_t* drop_ctr, MacEntry* macs,
                 uint32_t mac_mask);
  // Zero-copy rx on the CPU: frames are gathered from their addresses (host pointers) into the
  // in slots at publish, as the GPU ring reads them (the engine's side of the mode, testable here)
  void set_frame_addrs(bool on);
  uint64_t* frame_addrs(uint32_t q) override { return fa_.empty() ? nullptr : fa_.data() + (size_t)q * cap_; }
  uint64_t map_host(const void* p, size_t, std::function<void(std::function<void()>)>*) override {
    return reinterpret_cast<uint64_t>(p);
  }

 protected:
  virtual void run_segment(uint32_t q, uint32_t pos, uint32_t n);
  uint32_t cap_, nq_;
  std::vector<uint8_t> in_, out_;
  std::vector<uint32_t> im_, om_;
  std::vector<uint64_t> fa_;   // zero-copy: per-slot frame addresses (empty: off)
  std::unique_ptr<std::atomic<uint64_t>[]> prod_;
  std::atomic<bool> configured_{false};
  std::atomic<bool> gate_{false};
  std::mutex run_mu_;   // the pipeline's counters / MAC table are shared by every queue
  bool serial_ = true;  // queues run one at a time (run_mu_)
  TablesView t_{};
  uint64_t *flow_ctr_ = nullptr, *port_ctr_ = nullptr, *drop_ctr_ = nullptr;
  MacEntry* macs_ = nullptr;
  uint32_t mac_mask_ = 0;
};

// A pipeline that costs nothing: every frame leaves unchanged through the port its destination
// MAC is bound to (unknown MACs drop).  It measures the I/O engine alone — ports, steering,
// publication, delivery — the ceiling any pipeline behind it is held to (tools/live_bench.py
// --backend wire).
class WireBackend : public OracleBackend {
 public:
  WireBackend(uint32_t capacity, uint32_t queues, const std::vector<std::pair<uint64_t, uint32_t>>& mac_to_port);

 protected:
  void run_segment(uint32_t q, uint32_t pos, uint32_t n) override;

 private:
  std::vector<std::pair<uint64_t, uint32_t>> tab_;   // open addressing, 48-bit MAC + 1 (0: empty)
  uint32_t tmask_ = 0;
};

// ---------------------------------------------------------------------------------- engine
struct Punt {
  uint16_t in_port;
  uint8_t reason;
  std::vector<uint8_t> frame;
};

struct Replica {
  uint32_t src;         // index of the source packet in its burst
  uint32_t meta;
  uint8_t hdr[kSlotBytes];
};

class Engine {
 public:
  // burst: frames per publish (at most); inflight: bursts in flight per lane; tx_workers:
  // delivery threads per queue (each owns the egress ports with port % tx_workers == its index,
  // so frames of one port from one queue leave in order); queues: rx threads (each with its
  // ring queue on every backend); max_inflight_frames: frames in flight per lane (bounds the
  // engine's own queueing delay: frames beyond it wait in the ports' rings).  tx_workers = 0:
  // run to completion — each queue's rx thread also completes and delivers its own bursts (no
  // delivery threads: one busy thread per queue, the layout that fits a CPU quota best).
  Engine(uint32_t burst, uint32_t inflight_bursts, uint32_t tx_workers = 1, uint32_t queues = 1,
         uint32_t max_inflight_frames = 0);
  ~Engine();
  void add_backend(std::shared_ptr<Backend> b);       // index = GPU (shard) number
  // queue: the rx thread serving the port (-1: the least loaded queue)
  void add_port(uint32_t id, std::shared_ptr<Port> p, int queue = -1);
  void inject(uint32_t in_port, const uint8_t* f, uint32_t n) { recirc_->push(in_port, f, n); }
  std::shared_ptr<Port> remove_port(uint32_t id);
  // removed ports still held because a burst may refer to them (released as lanes deliver)
  size_t retired_ports();
  std::shared_ptr<Port> port(uint32_t id);
  int port_queue(uint32_t id);
  // Configuration (copy-on-write: safe while traffic flows).
  // port_owner non-empty: port placement — every frame goes to the GPU its ingress port is placed
  // on (port_owner[in_port]), not to its flow's owner (MultiDataPlane placement="port").
  void set_steering(const std::vector<PortEntry>& ports, const std::vector<uint8_t>& rss_key, bool v6 = false,
                    const std::vector<uint32_t>& port_owner = {});
  void set_redirects(const std::vector<std::pair<uint32_t, uint32_t>>& tunnel_to_underlay);   // replaces all
  void set_redirect(uint32_t port, uint32_t underlay);   // one entry (0xFFFFFFFF clears it)
  void set_side_ports(const std::vector<uint32_t>& ports); // ingress ports whose packets need side work
  void set_side_always(bool on);
  // Publication coalescing: with bursts of a lane in flight, frames gather until `frames` are
  // staged or the oldest waited `window_us` (an idle lane publishes at once).  (64, 0): every
  // read publishes.
  void set_coalesce(uint32_t frames, double window_us) {
    coalesce_frames_.store(std::max<uint32_t>(frames, 1));
    coalesce_ns_.store((uint64_t)(std::max(window_us, 0.0) * 1e3));
  }
  void set_side_tables(uint32_t backend, std::shared_ptr<SideTables> t);
  // The CPUs queue q's rx thread and tx workers run on (a GPU's NUMA-local CPUs: the lane group
  // serving that GPU); before start().
  void set_queue_cpus(uint32_t q, const std::vector<int>& cpus);
  // Zero-copy rx: map every port's rx memory (rx_memory()) for the backends; a backend reading
  // frames by address (frame_addrs()) then reads mapped frames in place — the engine writes an
  // address per slot instead of copying the frame's first 64 bytes.  Ports added later are
  // mapped as they come.
  void set_zero_copy(bool on);
  bool zero_copy() const { return zero_copy_.load(); }
  // GPU-direct egress: memif ports added from now on (and those present) get a ring per GPU lane
  // (memif ring 1 + queues + lane) that the lane's grid writes itself (ring.h GdeRing); needs the
  // GPU backends' rings gde_enable()d and regions with enough rings (MemifPort tx_rings >= queues +
  // lanes), else the port stays on the host path.  Set while stopped.
  void set_gpu_egress(bool on);
  bool gpu_egress() const { return gde_.load(); }
  void start();
  void stop();
  void pause();    // no publish until resume(); returns once nothing is in flight
  void resume();
  // hold(): no publish until release(), without waiting for the bursts in flight (a commit's
  // epoch flips land between two bursts of every queue); returns once every rx thread holds.
  void hold();
  void release();
  bool running() const { return run_.load(); }
  uint32_t queues() const { return nq_; }
  std::string error() const;
  std::vector<Punt> take_punts(size_t max);
  std::vector<double> take_latency_us();              // rx -> tx time per burst (engine side)
  std::unordered_map<std::string, uint64_t> stats() const;
  // [kMaxPorts][2] replica tx pkts / bytes (side pass output, not in the pipeline's counters)
  std::vector<uint64_t> side_port_counters() const;
  std::vector<uint64_t> side_drop_counters() const;   // [kNumReasons]
  uint32_t owner_of_frame(const uint8_t* f, uint32_t len, uint32_t in_port) const;
  void inject_failure(const std::string& what) { fail(what); }   // fault injection (tests)
  // wait until every learn event found so far is applied (tests / commit ordering)
  void flush_learning();
  // last-seen stamp of learned MAC entries (the control plane's aging clock): never goes back
  uint32_t learn_stamp() const { return learn_stamp_.load(); }
  void set_learn_stamp(uint32_t s) {
    uint32_t c = learn_stamp_.load();
    while (s > c && !learn_stamp_.compare_exchange_weak(c, s)) {
    }
  }

 private:
  struct PortRef { std::shared_ptr<Port> p; uint32_t q = 0; };
  using PortTab = std::vector<PortRef>;
  struct Steer {
    std::vector<PortEntry> ports;
    std::vector<uint8_t> rss_key;
    bool v6 = false;
    ToeplitzTab hash;
    std::vector<uint32_t> port_owner;   // port placement (empty: flow owners)
  };
  struct Cfg {                   // everything the packet threads read from the control plane
    std::vector<uint32_t> redirect;      // tunnel port -> underlay port (0xFFFFFFFF: none)
    std::vector<uint8_t> side_ports;     // ingress ports with side work
    bool side_always = false;
    std::shared_ptr<const Steer> steer;
    std::vector<std::shared_ptr<SideTables>> side;   // per backend
  };
  struct Pkt { uint32_t port; uint32_t seq; const uint8_t* data; uint32_t len; Port* holder; };
  struct Burst {
    uint64_t id = ~0ull;   // burst number on its lane (slot = id % inflight)
    uint64_t start = 0, end = 0;   // ring positions [start, end)
    std::vector<Pkt> pkts;
    bool side = false;     // some ingress port needs side work
    uint64_t t_rx_ns = 0;
    std::vector<Replica> reps;          // side-pass output for this burst
    std::vector<uint8_t> xhdr;          // per packet kXhdrBytes outer-header record (tunnels)
    std::vector<uint8_t> has_x;         // per packet: xhdr record present
    // the configuration (side tables, redirects, side ports) current when the burst was
    // published: its side pass and delivery use the tables its pipeline epoch used, even when a
    // commit swaps the engine's configuration while the burst is in flight
    std::shared_ptr<const Cfg> cfg;
    std::atomic<uint32_t> state{0};   // 0 free, 1 published, 2 ready to deliver (completed + side done)
    std::atomic<uint32_t> left{0};    // delivery workers still working on it
  };
  struct Lane {                 // (queue, backend): one ring queue and its bursts
    std::shared_ptr<Backend> be;
    uint32_t q = 0, g = 0;
    std::unique_ptr<Burst[]> slots;
    std::atomic<uint64_t> head{0};        // rx thread: next burst id
    std::atomic<uint64_t> done{0};        // bursts fully delivered (in order)
    std::atomic<uint64_t> freed_pos{0};   // ring position below which every slot is delivered (reusable)
    std::vector<Pkt> stage;     // rx thread: frames bound for this backend, not published yet
    uint64_t stage_t0 = 0;      // rx time of the first staged frame
    uint64_t room = 0;          // rx thread: free ring slots at the last look (multiple of 64)
  };
  struct alignas(64) QStats {
    std::atomic<uint64_t> rx{0}, tx{0}, drop{0}, punt{0}, recirc{0}, reps{0}, bursts{0}, side{0}, no_port{0},
        tx_full{0}, pub_ns{0}, deliver_ns{0}, idle{0}, wait_tx{0}, learn{0}, held{0}, zc{0}, gde{0};
    void add(std::atomic<uint64_t>& c, uint64_t v) { if (v) c.store(c.load(std::memory_order_relaxed) + v, std::memory_order_relaxed); }
  };
  struct Queue {                // one rx thread + its tx workers
    uint32_t id = 0;
    std::vector<Lane*> lanes;   // one per backend
    std::thread rx;
    std::vector<std::thread> tx;
    std::atomic<uint64_t> held_epoch{0};   // last control epoch (pause / hold) the rx thread acknowledged
    std::atomic<uint64_t> ports_seen{0};   // port-table version the rx thread works from (retiring ports)
    std::vector<int> cpus;      // the queue's threads run on these CPUs (empty: anywhere)
    QStats st;                  // rx-thread counters
    std::unique_ptr<QStats[]> wst;   // per tx worker
    std::unique_ptr<std::atomic<uint64_t>[]> side_ctr;   // per worker x kMaxPorts x 2 (replica tx pkts / bytes)
    std::unique_ptr<std::atomic<uint64_t>[]> side_drop;  // per worker x kNumReasons
    std::atomic<uint32_t> nports{0};
    std::mutex lat_mu;           // rx -> tx time per burst, this queue's samples
    std::vector<double> lat_us;
  };
  struct TxTally { uint64_t tx = 0, full = 0, no_port = 0, drop = 0, reps = 0, gde = 0; };
  struct TxScratch {            // per tx worker
    std::vector<std::vector<TxItem>> by_port;
    std::vector<uint32_t> touched;
    std::vector<uint32_t> learn;   // learn events of the current burst
  };
  struct TxCtx;                 // one delivery loop's state (a tx worker, or an inline rx thread)

  static void pin(std::thread& t, const std::vector<int>& cpus);
  void rx_loop(Queue* Q);
  void tx_loop(Queue* Q, uint32_t w);
  // one pass over the queue's lanes: each lane's next burst, if it is this worker's turn and
  // complete, is side-passed / delivered; returns the bursts handled (never blocks)
  uint32_t tx_poll(Queue* Q, uint32_t w, TxCtx& x);
  bool tx_drained(Queue* Q, const TxCtx& x) const;
  void learner_loop();
  void deliver(Queue* Q, Lane* L, Burst& b, uint32_t w, const Cfg& cfg, const PortTab& tab, TxScratch& sc);
  void side_work(Queue* Q, Lane* L, Burst& b, const Cfg& cfg, TxScratch& sc, uint32_t w);
  void finish(Queue* Q, Lane* L, Burst& b);
  bool lanes_idle() const;
  void punt(QStats& st, uint32_t in_port, uint32_t reason, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb);
  void fail(const std::string& what);
  std::shared_ptr<const Cfg> cfg() const { return std::atomic_load(&cfg_); }
  template <class F> void update_cfg(F f);
  // A packet thread's private reference to a copy-on-write snapshot, re-read only when the
  // snapshot's version moved: the hot loops touch one read-mostly version word, never the
  // shared_ptr's control block (whose atomic load is a global lock in libstdc++) or its refcount.
  template <class T> struct Snap {
    uint64_t ver = ~0ull;
    std::shared_ptr<const T> p;
  };
  const Cfg& cfg_of(Snap<Cfg>& s) const {
    const uint64_t v = cfg_ver_.load(std::memory_order_acquire);
    if (v != s.ver) { s.p = std::atomic_load(&cfg_); s.ver = v; }
    return *s.p;
  }
  const PortTab& ports_of(Snap<PortTab>& s) const {
    const uint64_t v = ports_ver_.load(std::memory_order_acquire);
    if (v != s.ver) { s.p = std::atomic_load(&ports_); s.ver = v; }
    return *s.p;
  }
  static uint32_t owner(const Steer* s, uint32_t n, const uint8_t* f, uint32_t len, uint32_t in_port);

  uint32_t burst_, inflight_, workers_, nq_, max_frames_;
  bool inline_tx_ = false;      // tx_workers == 0: the rx threads deliver (workers_ is then 1)
  std::vector<std::unique_ptr<Lane>> lanes_;     // q * nbackends + g
  std::vector<std::shared_ptr<Backend>> backends_;
  std::vector<std::unique_ptr<Queue>> queues_;
  mutable std::mutex ports_mu_;
  std::atomic<bool> zero_copy_{false};
  std::atomic<bool> gde_{false};
  // removed ports stay referenced a while (frames of theirs may still be in a pipeline: the GPU
  // reads a zero-copy frame where its port holds it)
  // A removed port is released once nothing can refer to it: every rx thread has seen a port
  // table without it (dropping what it had staged from it), and every burst published before
  // that has been delivered (the lanes' done counters passed their heads at that moment).
  struct Retired {
    uint64_t ver;                   // ports_ver_ of the first table without the port
    std::vector<uint64_t> heads;    // per lane: head once every rx thread saw `ver` (empty: not yet)
    std::shared_ptr<Port> p;
  };
  std::deque<Retired> retired_;     // (ports_mu_)
  void map_port(Port& p);            // (ports_mu_)
  void gde_register(uint32_t id, Port& p);   // (ports_mu_) GPU-direct egress rings of a memif port
  void gde_unregister(uint32_t id);          // (ports_mu_) ... off again, applied by every grid
  void reap_retired(bool all);       // (ports_mu_)
  std::shared_ptr<const PortTab> ports_;              // copy-on-write snapshot, by port id
  alignas(64) std::atomic<uint64_t> ports_ver_{0};    // bumped after every ports_ / cfg_ store
  std::atomic<uint64_t> cfg_ver_{0};
  std::shared_ptr<RecircPort> recirc_;
  mutable std::mutex cfg_mu_;                         // writers of cfg_
  std::shared_ptr<const Cfg> cfg_;
  std::atomic<bool> run_{false}, abandon_{false};
  // pause / hold requests (counters: nested commits of several data planes are fine); an rx
  // thread that sees one acknowledges the current control epoch before idling
  std::atomic<uint32_t> pause_n_{0}, hold_n_{0};
  std::atomic<uint64_t> ctl_epoch_{0};
  std::atomic<uint32_t> coalesce_frames_{64};
  std::atomic<uint64_t> coalesce_ns_{0};
  mutable std::mutex err_mu_;
  std::string err_;
  std::mutex punt_mu_;
  std::deque<Punt> punts_;
  std::atomic<uint64_t> punt_drop_{0};
  // learning: tx leaders -> learner thread -> every backend's MAC table + every side snapshot
  mutable std::mutex learn_mu_;
  std::condition_variable learn_cv_;
  std::vector<uint32_t> learn_q_;
  uint64_t learn_seq_ = 0, learn_applied_ = 0, learn_applied_n_ = 0, learn_dropped_ = 0;
  bool learner_run_ = false;
  std::atomic<uint32_t> learn_stamp_{1};
  std::thread learner_;
};

}  // namespace iox
}  // namespace nfdp
