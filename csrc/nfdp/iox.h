// iox.h — native packet I/O engine: vport netdevs / shared-memory vports <-> the data plane.
//
// The reference's data ports never touch a per-frame interpreter loop: OvS-DPDK polls NIC / vhost
// queues from PMD threads (ovs-dp/ovsdp.go:39-55 binds them `type=dpdk`), the IPU's FXP is
// silicon.  This engine is the MI355X data plane's equivalent, in C++ with Python only
// configuring it:
//
//   ports (memif shared-memory vports, AF_PACKET TPACKET_V2 rings on veth/netdevs, TAP fds)
//     --rx thread--> owner GPU = owner_of(toeplitz(FlowKey), N) (the RSS a NIC would do; 1 GPU: 0)
//       -> 64-B header slot + ingress meta written straight into that GPU's ring slots (pinned host
//          memory the resident ring kernel reads over PCIe), bursts padded to whole 64-packet
//          chunks, published at once (no batching delay: a lone packet is its own chunk)
//     --tx thread per GPU--> completion flag -> egress meta -> frame = [outer hdr] ++ out slot[:hl]
//          ++ in_frame[to:len] written to the egress port (the payload never left the rx buffer);
//          side work (flood replicas, mirror / ARP copies, MAC learning, tunnel outer headers)
//          through the side kernel; recirculation (tunnel termination) re-enters on the rx
//          thread; slow-path frames (ARP trap, IPv6 termination) queue up for the control plane
//     -> rx buffers are handed back to their port in rx order once every frame below is sent.
//
// Backends: `GpuBackend` (RingEngine with host slots: the persistent HIP kernel) or
// `OracleBackend` (the bit-exact C++ pipeline, synchronous: CPU tests / no-GPU nodes).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
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

// ---------------------------------------------------------------------------------- ports
struct RxRef {
  const uint8_t* data;
  uint32_t len;
  uint32_t seq;       // port-local rx sequence number (released in order)
  uint32_t in_port;   // ingress port for the pipeline (~0u: the port's own id)
};

class Port {
 public:
  explicit Port(uint32_t window);
  virtual ~Port() = default;
  // Up to `max` received frames; each stays valid until its sequence number is released.
  virtual uint32_t rx(RxRef* out, uint32_t max) = 0;
  // Frame assembled from up to three pieces (outer header, rewritten header, payload tail);
  // false when the port has no room (dropped, as on a full NIC queue).  Thread safe.
  bool tx(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc);
  void flush();
  // A frame is done (sent or dropped): any thread.  reclaim(): rx thread only.
  void complete(uint32_t seq) { done_[seq & mask_].store(1, std::memory_order_release); }
  void reclaim();
  virtual std::string kind() const = 0;
  // rx counters (rx thread) and tx counters (one delivery worker per port) on separate lines
  alignas(64) std::atomic<uint64_t> rx_pkts{0}, rx_bytes{0};
  alignas(64) std::atomic<uint64_t> tx_pkts{0}, tx_full{0}, tx_bytes{0};

 protected:
  virtual bool tx_locked(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) = 0;
  virtual void flush_locked() {}
  virtual void release_to(uint32_t seq_end) = 0;   // every frame below seq_end is done
  void set_first_seq(uint32_t s) { rel_ = s; seen_ = s; }
  uint32_t window() const { return mask_ + 1; }
  std::mutex tx_mu_;
  bool tx_dirty_ = false;

 private:
  std::unique_ptr<std::atomic<uint8_t>[]> done_;
  uint32_t mask_;
  uint32_t rel_ = 0;   // next sequence number to release
  uint32_t seen_ = 0;  // rx sequence numbers handed out so far (upper bound of reclaim)
  friend class Engine;
};

// Shared-memory vport (memif.h): the pod produces ring 0, the engine ring 1.
class MemifPort : public Port {
 public:
  MemifPort(const std::string& path, uint32_t ring_size, uint32_t buf_size);
  ~MemifPort() override;
  uint32_t rx(RxRef* out, uint32_t max) override;
  std::string kind() const override { return "memif"; }
  const std::string& path() const { return reg_.path(); }

 protected:
  bool tx_locked(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) override;
  void flush_locked() override { prod_.commit(); }
  void release_to(uint32_t seq_end) override { cons_.release_to(seq_end); }

 private:
  memif::Region reg_;
  memif::Consumer cons_;
  memif::Producer prod_;
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
  bool tx_locked(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) override;
  void flush_locked() override;
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
  bool tx_locked(const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb, const uint8_t* c, uint32_t nc) override;
  void release_to(uint32_t seq_end) override { freed_.store(seq_end, std::memory_order_release); }

 private:
  int fd_;
  uint32_t nbufs_, bsize_;
  std::vector<uint8_t> bufs_;
  std::vector<uint32_t> lens_;
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
  bool tx_locked(const uint8_t*, uint32_t, const uint8_t*, uint32_t, const uint8_t*, uint32_t) override { return false; }
  void release_to(uint32_t seq_end) override;

 private:
  std::mutex mu_;
  std::deque<std::pair<uint32_t, std::vector<uint8_t>>> q_;       // waiting
  std::deque<std::pair<uint32_t, std::vector<uint8_t>>> live_;    // handed out, not released yet
  uint32_t next_ = 0, base_ = 0;
};

// ---------------------------------------------------------------------------------- backends
struct Replica {
  uint32_t src_pos;     // ring position of the source packet
  uint32_t meta;
  uint8_t hdr[kSlotBytes];
};
struct SideBatch {
  std::vector<Replica> reps;
  std::vector<uint8_t> xall;   // capacity x kXhdrBytes outer-header records by ring slot (tunnels only)
  uint32_t learned = 0;
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual uint32_t capacity() const = 0;
  virtual uint8_t* in_slot(uint32_t pos) = 0;      // pos: ring position (mod capacity)
  virtual uint32_t* in_meta() = 0;
  virtual const uint8_t* out_slot(uint32_t pos) = 0;
  virtual const uint32_t* out_meta() = 0;
  virtual uint64_t published() = 0;
  virtual uint64_t publish(uint32_t n) = 0;        // multiple of 64
  virtual uint64_t completed() = 0;
  virtual bool range_done(uint64_t start, uint64_t end) = 0;   // positions [start, end) processed
  virtual bool ready() = 0;                         // can take a publish now (ring running)
  virtual bool alive() { return true; }             // the pipeline still makes progress (slow check)
  // Side pass over every completed slot the pipeline listed since the last pass (call only when
  // completed() == published(): nothing is in flight).
  virtual void side_pass(SideBatch& out) = 0;
  virtual void thread_init() {}
};

class GpuBackend : public Backend {
 public:
  explicit GpuBackend(RingEngine* ring);
  ~GpuBackend() override;
  uint32_t capacity() const override { return ring_->capacity(); }
  uint8_t* in_slot(uint32_t pos) override { return in_ + (size_t)(pos & (capacity() - 1)) * kSlotBytes; }
  uint32_t* in_meta() override { return im_; }
  const uint8_t* out_slot(uint32_t pos) override { return out_ + (size_t)(pos & (capacity() - 1)) * kSlotBytes; }
  const uint32_t* out_meta() override { return om_; }
  uint64_t published() override { return ring_->published(); }
  uint64_t publish(uint32_t n) override { return ring_->publish(n, false); }
  uint64_t completed() override { return ring_->completed(); }
  bool range_done(uint64_t start, uint64_t end) override { return ring_->range_done(start, end); }
  bool ready() override { return ring_->running(); }
  bool alive() override { return ring_->alive(); }
  void side_pass(SideBatch& out) override;
  void thread_init() override;
  uint32_t stamp = 1;

 private:
  RingEngine* ring_;
  uint8_t* in_; uint32_t* im_; uint8_t* out_; uint32_t* om_;
  hipStream_t side_stream_{};
  std::vector<uint32_t> h_cnt_, h_meta_, h_src_, h_hdr_;
};

class OracleBackend : public Backend {
 public:
  explicit OracleBackend(uint32_t capacity);
  uint32_t capacity() const override { return cap_; }
  uint8_t* in_slot(uint32_t pos) override { return in_.data() + (size_t)(pos & (cap_ - 1)) * kSlotBytes; }
  uint32_t* in_meta() override { return im_.data(); }
  const uint8_t* out_slot(uint32_t pos) override { return out_.data() + (size_t)(pos & (cap_ - 1)) * kSlotBytes; }
  const uint32_t* out_meta() override { return om_.data(); }
  uint64_t published() override { return prod_; }
  uint64_t publish(uint32_t n) override;
  uint64_t completed() override { return prod_; }
  bool range_done(uint64_t, uint64_t end) override { return end <= prod_; }
  bool ready() override { return configured_; }
  void side_pass(SideBatch& out) override;
  // tables / counters / side buffers of the CPU DataPlane (replaced after every commit, while
  // the engine is paused)
  void configure(const TablesView& t, uint64_t* flow_ctr, uint64_t* port_ctr, uint64_t* drop_ctr, const SideOut& side,
                 MacEntry* macs, uint32_t mac_mask);
  uint32_t stamp = 1;

 private:
  void run_segment(uint32_t pos, uint32_t n);
  uint32_t cap_;
  std::vector<uint8_t> in_, out_;
  std::vector<uint32_t> im_, om_;
  uint64_t prod_ = 0;
  bool configured_ = false;
  TablesView t_{};
  uint64_t *flow_ctr_ = nullptr, *port_ctr_ = nullptr, *drop_ctr_ = nullptr;
  SideOut side_{};
  MacEntry* macs_ = nullptr;
  uint32_t mac_mask_ = 0;
  SideBatch pending_;
};

// ---------------------------------------------------------------------------------- engine
struct Punt {
  uint16_t in_port;
  uint8_t reason;
  std::vector<uint8_t> frame;
};

class Engine {
 public:
  // burst: frames per publish (at most); inflight: bursts in flight per backend; tx_workers:
  // delivery threads per backend (each owns the egress ports with port % tx_workers == its index,
  // so frames of one port leave in order)
  Engine(uint32_t burst, uint32_t inflight_bursts, uint32_t tx_workers = 1);
  ~Engine();
  void add_backend(std::shared_ptr<Backend> b);       // index = GPU (shard) number
  void add_port(uint32_t id, std::shared_ptr<Port> p);
  void inject(uint32_t in_port, const uint8_t* f, uint32_t n) { recirc_->push(in_port, f, n); }
  std::shared_ptr<Port> remove_port(uint32_t id);
  std::shared_ptr<Port> port(uint32_t id);
  // Host-side steering inputs (N > 1): a copy of the port table and the RSS key.
  void set_steering(const std::vector<PortEntry>& ports, const std::vector<uint8_t>& rss_key, bool v6 = false);
  void set_redirect(uint32_t port, uint32_t underlay);   // tunnel port -> its underlay port
  void set_side_ports(const std::vector<uint32_t>& ports); // ingress ports whose packets may need side work
  void set_side_always(bool on) { side_always_.store(on); }
  void start();
  void stop();
  void pause();    // no publish until resume(); returns once nothing is in flight
  void resume();
  bool running() const { return run_.load(); }
  std::string error() const;
  std::vector<Punt> take_punts(size_t max);
  std::vector<double> take_latency_us();              // rx -> tx time per burst (engine side)
  std::unordered_map<std::string, uint64_t> stats() const;
  uint32_t owner_of_frame(const uint8_t* f, uint32_t len, uint32_t in_port) const;
  void inject_failure(const std::string& what) { fail(what); }   // fault injection (tests)

 private:
  struct Pkt { uint32_t port; uint32_t seq; const uint8_t* data; uint32_t len; Port* holder; };
  struct Burst {
    uint64_t id = ~0ull;   // burst number on its lane (slot = id % inflight)
    uint64_t start = 0, end = 0;   // ring positions [start, end)
    std::vector<Pkt> pkts;
    bool side = false;
    uint64_t t_rx_ns = 0;
    std::vector<Replica> reps;                                    // side-pass output for this burst
    std::vector<std::pair<uint32_t, std::vector<uint8_t>>> xhdr;  // (position, outer-header record)
    std::atomic<uint32_t> state{0};   // 0 free, 1 published, 2 ready to deliver (completed + side done)
    std::atomic<uint32_t> left{0};    // delivery workers still working on it
  };
  struct Lane {                 // one backend + its delivery workers
    std::shared_ptr<Backend> be;
    std::mutex pub_mu;          // rx thread's staging + publish vs the leader's side pass
    std::unique_ptr<Burst[]> slots;
    uint64_t head = 0;          // rx thread: next burst id
    std::atomic<uint64_t> done{0};   // bursts fully delivered (in order)
    std::atomic<uint64_t> freed_pos{0};   // ring position below which every slot is delivered (reusable)
    std::vector<std::thread> th;
    std::vector<Pkt> stage;     // rx thread: frames bound for this backend
    uint64_t side_upto = 0;     // published count covered by the last side pass (leader only)
  };
  using PortTab = std::vector<std::shared_ptr<Port>>;
  void rx_loop();
  void tx_loop(Lane* L, uint32_t w);
  void deliver(Lane* L, Burst& b, uint32_t w, std::vector<Port*>& touched);
  void finish(Lane* L, Burst& b);
  void side_pass(Lane* L, uint64_t from_id);
  bool needs_side(uint32_t in_port) const;
  struct TxTally { uint64_t tx = 0, full = 0, no_port = 0, drop = 0, reps = 0; };
  void send(const PortTab& tab, uint32_t port, const uint8_t* x, uint32_t nx, const uint8_t* h, uint32_t nh,
            const uint8_t* t, uint32_t nt, std::vector<Port*>& touched, TxTally& tally);
  void punt(uint32_t in_port, uint32_t reason, const uint8_t* a, uint32_t na, const uint8_t* b, uint32_t nb);
  void fail(const std::string& what);

  uint32_t burst_, inflight_, workers_;
  std::vector<std::unique_ptr<Lane>> lanes_;
  mutable std::mutex ports_mu_;
  std::shared_ptr<const PortTab> ports_;              // copy-on-write snapshot, by port id
  std::shared_ptr<RecircPort> recirc_;
  std::vector<uint32_t> redirect_;
  std::vector<uint8_t> side_ports_;
  std::atomic<bool> side_always_{false};
  std::vector<PortEntry> steer_ports_;
  bool steer_v6_ = false;
  std::vector<uint8_t> rss_key_;
  std::atomic<bool> run_{false}, pause_{false}, paused_ack_{false};
  std::thread rx_th_;
  mutable std::mutex err_mu_;
  std::string err_;
  std::mutex punt_mu_;
  std::deque<Punt> punts_;
  std::mutex lat_mu_;
  std::vector<double> lat_us_;
  std::atomic<uint64_t> st_rx_{0}, st_tx_{0}, st_drop_{0}, st_punt_{0}, st_recirc_{0}, st_reps_{0}, st_bursts_{0},
      st_side_{0}, st_no_port_{0}, st_punt_drop_{0}, st_tx_full_{0}, st_pub_ns_{0}, st_deliver_ns_{0},
      st_idle_{0}, st_wait_tx_{0};
};

}  // namespace iox
}  // namespace nfdp
