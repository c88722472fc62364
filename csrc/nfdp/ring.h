// ring.h — low-latency persistent data path: a resident kernel polls an ingress ring.
//
// The batch engine (kernels.hip, pktio.hip) pays a kernel launch and a batch-release barrier per
// batch, which sets the floor of its per-packet latency.  The ring engine removes both: a
// persistent kernel stays resident on the CUs and its waves claim 64-packet chunks of an ingress
// ring as soon as the producer publishes them.  This is the GPU counterpart of the reference's
// always-on DPU datapath (FXP / OvS-DPDK PMD threads polling their rings) and of the Octeon
// control agent's poll loop (octep_cp_agent main.c:307-311), built the CDNA4 way:
//
//   host (or NIC)                          GPU (persistent ring_kernel, 64-wide waves)
//   -------------                          ------------------------------------------
//   frames -> ring slots [R x 64 B]        wave: ticket t = atomicAdd(claim, 1)  (chunk t = slots
//   ctl.prod += n   (release store,                 64t .. 64t+63 mod R, one packet per lane)
//                    pinned coherent       only the FRONTIER wave (64t == dprod) polls ctl.prod over
//                    host memory)            PCIe and mirrors it into device memory (dprod); every
//                                            other wave polls dprod in HBM/L2 -> one PCIe poller
//                                          process the chunk: ingress, MFMA hash/ACL, flow probe,
//                                            chain, emit (same stages as the fused kernel)
//   poll flags[t % (R/64)] == t+1   <----  release fence (system scope), flags[t] = t + 1
//
// Queues: one grid serves Q independent rings ("queues", like a NIC's RSS queues).  Workgroup b
// serves queue b % Q: its own control word, ticket counter, prod mirror, completion flags and
// slot range, so Q host producers (the I/O engine's rx threads) publish without sharing anything
// but the tables.  One resident kernel per GPU whatever Q is: a second persistent grid on the same
// device could wait forever behind the first on a shared hardware queue.
//
// Drain semantics: `stop` makes a wave exit only while it WAITS for an unpublished chunk, and
// tickets are claimed in order, so every chunk published before the stop is processed.  Every
// wave also exits on a device-side deadline (s_memrealtime), so the grid always drains even if
// the host dies.
//
// Table updates under a running ring (epoch flip, no relaunch): the flow table is double
// buffered.  The published word carries a 7-bit epoch next to the packet count
// (stop | count << 7 | epoch); a wave takes the epoch of the word that published its chunk and
// probes copy `epoch & 1`.  The control plane writes its bucket changes into the copy no wave
// reads, flips the epoch (flip(), carried by the next publish), and before it writes that other
// copy again waits for the grace period: every chunk published before the flip has completed
// (wait_grace()), so no wave still reads it.  A lookup therefore never sees a half-written
// bucket, without retries or per-bucket locks on the packet path.  A wave that sees a new epoch
// first drops its cached table lines (agent-scope acquire: CU L1 and XCD L2), so a copy rewritten
// since the wave last read it is never served from a stale line; bump_epoch() (epoch + 2, same
// copy) does only that, for tables changed in place.  The small tables staged in LDS
// (ports, chains, ACL) still take the stop -> drain -> relaunch path.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <functional>
#include <chrono>
#include <cstdint>
#include <memory>
#include <deque>
#include <mutex>
#include <utility>
#include <vector>

#include "host.h"

namespace nfdp {

// Bit 63 of the published-packet counter is the stop flag: one 64-bit word carries both, so a
// wave that sees "stop" also sees the final count (no ordering between two words to get right).
constexpr uint64_t kRingStop = 1ull << 63;
// Ingress meta of a filler slot (a burst that is not a multiple of 64 packets is padded to whole
// chunks): processed like any slot, but it counts nowhere and never reaches the side list.
constexpr uint32_t kRingPadMeta = 0xFFFFFFFFu;
constexpr uint32_t kRingEpochBits = 7;
constexpr uint64_t kRingEpochMask = (1ull << kRingEpochBits) - 1;
// published word = stop | count << 7 | epoch: count-major, so the frontier's atomic max keeps
// the newest count whatever the epoch does (the epoch only changes with a new count or in place)
__host__ __device__ inline uint64_t ring_word(uint64_t count, uint32_t epoch) {
  return (count << kRingEpochBits) | (epoch & kRingEpochMask);
}
// Epoch layout (7 bits): bit 0 = flow-table copy, bit 1 = table set (coop rings: every other
// table, double buffered in device memory and restaged into LDS when it changes), bits 6..2 = a
// generation bumped by every change (a wave seeing any change drops its cached table lines).
constexpr uint32_t kEpochFlowBit = 1u, kEpochSetBit = 2u, kEpochGenShift = 2u, kEpochGenMask = 0x1Fu;
__host__ __device__ inline uint32_t epoch_next_gen(uint32_t e) {
  return (e & (kEpochFlowBit | kEpochSetBit)) | ((((e >> kEpochGenShift) + 1u) & kEpochGenMask) << kEpochGenShift);
}
// Epoch aliasing guard: the host lets at most kEpochGenMask epoch changes happen within
// kEpochAliasHostUs; a wave whose previous chunk is older than kEpochAliasTicks (half of it, in
// s_memrealtime ticks) drops its cached table lines whatever epoch value it sees.
constexpr uint32_t kEpochAliasHostUs = 100;
constexpr unsigned long long kEpochAliasTicks = kEpochAliasHostUs * 100ull / 2;   // 100 MHz
__host__ __device__ inline uint64_t ring_count(uint64_t w) { return (w & ~kRingStop) >> kRingEpochBits; }
__host__ __device__ inline uint32_t ring_epoch(uint64_t w) { return (uint32_t)(w & kRingEpochMask); }

// Everything a coop ring's per-packet stages read besides the flow table: double buffered in
// device memory (table set = epoch bit 1).  A commit writes the idle set and flips; every
// workgroup restages its LDS copies (ports, chains, ACL verdicts and rule tiles, Toeplitz tables)
// from the new set at the first chunk that carries it.  No drain, no relaunch.  `serial` counts
// the host's uploads: a workgroup idle through two flips sees the same set bit again, the serial
// tells it the set was rewritten meanwhile.
struct RingTableSet {
  TablesView t;
  const void* acl_wfrag;
  const void* acl_cinit;
  const void* toep_frag;
  const uint32_t* toep_tab;
  uint32_t acl_tiles;
  uint32_t serial;
  uint32_t pad[2];
};

// Host -> device control block, pinned coherent host memory (one 64-B line).
struct alignas(64) RingCtl {
  uint64_t prod;   // ring_word(packets published, epoch) | kRingStop
  uint32_t pad[14];
};
static_assert(sizeof(RingCtl) == 64, "RingCtl");

// Device-resident ring state (HBM): the ticket counter and the prod mirror on separate 128-B
// lines, so claim atomics and the waiters' polls do not contend for one line.
struct alignas(128) RingDevState {
  uint64_t claim;  // next chunk ticket (64-bit: tickets never wrap)
  uint32_t pad0[30];
  uint64_t dprod;  // device mirror of ctl.prod (advanced by the frontier wave), bit 63 = stop
  uint32_t ctl_gen;   // (queue 0's state only) control-mailbox writes applied so far: a workgroup
                      // seeing it move restages its LDS copies of the small tables
  uint32_t set_serial[2];   // (queue 0's) device mirror of the table sets' serials: written before
                            // the flip that names the set (start(), or the control mailbox), so the
                            // serial check never waits on a host-memory read
  uint32_t gde_pad;
  uint64_t gde_turn;        // GPU-direct egress: the next chunk ticket whose frames may go out (in order)
  uint64_t gde_wait;        // (diagnostics, s_memrealtime ticks) waiting for the turns / in the two
  uint64_t gde_sect;        // serialised sections; chunks, frames delivered, frames left to the host
  uint64_t gde_chunks, gde_frames, gde_full;   // for want of room
  uint64_t gde_commit;      // GPU-direct egress: the next ticket whose ring heads may be published
  uint32_t pad1[12];
};

// Control mailbox: the control plane's small table writes (a port entry on a link / MTU / RX-state
// change, a chain word, a MAC entry), applied by the resident grid itself.  Pinned coherent host
// memory; the host fills an entry, then publishes it (seq, then head, release order); the grid's
// poller wave (workgroup 0, wave 0: when idle, rate-limited, and every 16 chunks when busy) copies
// the words to their device addresses, releases them at agent scope, bumps ctl_gen and reports
// `done`.  No copy engine, no epoch change, no hold: the analogue of the Octeon control agent's
// mailbox that the SoC polls (octep_ctrl_mbox.c / loop.c), with the GPU as the SoC.
constexpr uint32_t kCtrlSlots = 64;
constexpr uint32_t kCtrlWords = 12;
constexpr uint32_t kCtrlNoRestage = 1u << 31;   // RingCtrlEntry.nwords flag: the target is not in any LDS copy
struct alignas(64) RingCtrlEntry {
  uint64_t dst;               // device address of the first dword (4-B aligned)
  uint32_t nwords;            // 1..kCtrlWords
  uint32_t seq;               // entry number + 1 (written after the rest of the entry)
  uint32_t data[kCtrlWords];
};
static_assert(sizeof(RingCtrlEntry) == 64, "RingCtrlEntry");
struct alignas(64) RingCtrlRing {
  uint64_t head;              // host: entries posted
  uint32_t pad0[14];
  uint64_t done;              // device: entries applied (released to every workgroup)
  uint32_t pad1[14];
  RingCtrlEntry e[kCtrlSlots];
};
static_assert(sizeof(RingDevState) == 256, "RingDevState");

// GPU-direct egress (GDE): a frame whose egress port is a memif vport goes from the grid straight
// into that vport's data-plane -> pod ring reserved for this GPU and queue (a ring no host thread
// writes): the frame's 64 B and its descriptor are stored over PCIe, the ring head is published
// with a system-scope store, and the host's tx path never touches the frame (its meta's length
// field says kMetaLenGde).  Chunks of a queue take their turn in ticket order (RingDevState.gde_turn), so a
// pod sees its frames in arrival order; a full ring (the pod's tail, re-read over PCIe when the
// cached one says full) leaves the rest of the chunk's frames to the host path.  Eligible: no drop,
// no side work (flood / tunnel header), the whole frame in the 64-B slot.  One entry per (port,
// queue): the ring's addresses as the GPU sees the mapped memif region, its geometry and the
// producer's private head (device state).
// Out-meta length field of a frame the grid delivered itself (reason kOk, the port field keeps the
// egress port): longer than any frame (kMaxFrame), so no forwarded frame can carry it, whatever its
// port (the marker used to be port 0xFFD, which is the valid vport 4093).
constexpr uint32_t kMetaLenGde = 0x3FFFu;
static_assert(kMetaLenGde > kMaxFrame, "GDE marker must not be a frame length");
NFDP_HD bool meta_is_gde(uint32_t m) { return meta_reason(m) == kOk && meta_len(m) == kMetaLenGde; }
struct alignas(64) GdeRing {
  uint64_t ctl;        // device address of the memif ring's Ctl (head written here, tail read)
  uint64_t desc;       // device address of its Desc[ring_size]
  uint64_t buf;        // device address of its buffer 0
  uint32_t mask;       // ring_size - 1
  uint32_t buf_size;   // bytes per buffer
  uint32_t head;       // producer head (device private copy, published to ctl)
  uint32_t tail_cache; // last pod tail seen
  uint32_t valid;      // 1: in use
  uint32_t pad[5];
};
static_assert(sizeof(GdeRing) == 64, "GdeRing");

// ---- SFC hops across GPUs in the live path (split chains, kHopXfer) --------------------------------
// A chain whose hops sit on different GPU planes runs hop by hop across the planes' resident grids,
// with no host hop and no launch:
//   1. the entry plane's grid (an XF ring instance) runs the hops up to the hand-off, stores the
//      frame's slot / meta as usual, records the chunk's hand-off count in `xpend` (pinned host
//      memory, before any entry is visible), then reserves entries in the next plane's INBOX (its
//      HBM; one system-scope add on the inbox tail per target plane per chunk) and peer-stores the
//      header slot, the HopState record and the way back (entry plane, queue, slot position);
//      each entry's `seq` (idx + 1) is stored after its data;
//   2. the resuming plane's inbox workgroups (the grid's last `xfer_wgs`) claim inbox chunks of 64
//      entries by ticket, run pipeline.h resume_stage on every entry as it becomes ready, and
//      store the final slot and meta straight into the ENTRY ring's out slot (pinned host memory:
//      every GPU reaches it), then subtract the chunk's finished frames from its `xpend` word
//      (system-scope atomic after the stores are done), and mark the entries consumed; a frame its
//      chain hands on again is sent to the next inbox with the same way back;
//   3. the host sees a chunk complete when its flag is written AND its xpend word is back to 0
//      (RingEngine::chunk_done), so a burst is delivered with every frame's final header.
// An entry a ring of the inbox ago must be consumed before a producer overwrites it (its seq says
// so); the inbox is sized for far more frames than the live path keeps in flight.
constexpr uint64_t kXferDone = 1ull << 63;
struct alignas(128) XferEntry {
  uint32_t slot[kSlotDwords];   // header slot as the hops so far left it
  HopState hs;                  // 32 B: what resume_stage needs
  uint32_t origin;              // entry plane | queue << 8
  uint32_t pos;                 // slot position in that queue's ring
  uint32_t t_send;              // producer's s_memrealtime (low word) at the send
  uint32_t pad0;
  uint64_t seq;                 // idx + 1 once written; | kXferDone once consumed
  uint64_t pad1;
};
static_assert(sizeof(XferEntry) == 128, "XferEntry");
struct alignas(128) XferInbox {   // (device memory of the resuming plane)
  uint64_t tail;                  // entries reserved by the producers (system-scope adds)
  uint32_t pad0[30];
  uint64_t claim;                 // inbox chunk tickets claimed by this grid's inbox waves
  // hand-off timing (s_memrealtime ticks, 100 MHz; one sample per resume pass, its first entry):
  // send -> picked up by an inbox wave, picked up -> written back (slot, meta, pending count)
  // (t_work split: entry loaded, chain stages done, write-back complete)
  uint64_t t_wait, t_work, n_timed, t_load, t_stage, t_wb;
  uint32_t pad1[18];
};
static_assert(sizeof(XferInbox) == 256, "XferInbox");
struct XferPeer {                 // one plane, as every grid sees it
  XferInbox* inbox;
  XferEntry* entries;
  uint32_t cap_mask;              // inbox entries - 1
  uint32_t ring_mask;             // its ring's slots per queue - 1
  uint4* out;                     // its ring's out slots / metas (device view; pinned host memory)
  uint32_t* out_meta;
  uint32_t* xpend;                // its ring's [queues][chunks] hand-offs not back yet (pinned)
  uint32_t nq;
  uint32_t pad;
};
constexpr uint32_t kMaxXferPlanes = 16;   // kHopXfer | plane, plane < 16

class RingEngine {
 public:
  // capacity: ring slots per queue (power of two, >= 64).  wgs_per_cu: resident 256-thread
  // workgroups per CU.  coop: the 4 waves of a workgroup share each chunk (ACL tiles split 4 ways:
  // lowest latency); otherwise every wave takes its own chunks (highest throughput).
  // host_slots: ring slots in pinned coherent host memory instead of HBM (zero-copy host I/O).
  // queues: independent rings served by one grid (workgroup b serves queue b % queues).
  RingEngine(uint32_t capacity, int num_cus, int wgs_per_cu = 1, bool coop = true, bool host_slots = false,
             uint32_t queues = 1);
  ~RingEngine();
  RingEngine(const RingEngine&) = delete;
  RingEngine& operator=(const RingEngine&) = delete;

  uint32_t capacity() const { return cap_; }   // per queue
  uint32_t queues() const { return nq_; }
  int device() const { return device_; }                 // HIP device the ring lives on
  const FusedLaunch& launch() const { return launch_; }  // tables / counters / side buffers of the session
  // The MAC table the running grid reads (a live table flip may replace it): learners write here.
  std::pair<MacEntry*, uint32_t> mac_table() const {
    std::lock_guard<std::mutex> g(mu_);
    return {const_cast<MacEntry*>(launch_.t.macs), launch_.t.mac_mask};
  }
  bool running() const { return running_; }
  // The grid is still resident (false once every wave left: stop, or the device deadline passed).
  bool alive() const { return running_ && stream_ && hipStreamQuery(stream_) == hipErrorNotReady; }
  bool host_slots() const { return host_slots_; }
  // device ring buffers (the producer stages frames here before publishing them); queue q's
  // slots follow queue q-1's (q * capacity slots in)
  void* dev_in() const { return d_in_; }
  uint32_t* dev_inmeta() const { return d_im_; }
  void* dev_out() const { return d_out_; }
  uint32_t* dev_meta() const { return d_meta_; }
  uint32_t* dev_svc() const { return d_svc_; }  // per-chunk device service time (ticks, 100 MHz)
  // host_slots rings: host addresses of the pinned in / inmeta / out / meta buffers (all queues)
  void* host_ptr(int i) const { return host_slots_ && i >= 0 && i < (int)host_ptrs_.size() ? host_ptrs_[i] : nullptr; }
  // Frame addresses (host_slots rings): with the mode on, the grid reads slot i's frame from the
  // device address in frame_addrs()[q * capacity + i] (pinned, written by the producer before it
  // publishes) instead of from the in slot — frames are read where the producer's ports hold
  // them (zero-copy rx).  Every published slot needs an address: an in slot's own (in_slot_addr)
  // for frames the producer copied, and for filler slots.  Set while stopped; takes effect at start().
  void set_frame_addrs(bool on);
  bool frame_addrs_on() const { return faddr_on_; }
  uint64_t* frame_addrs() const { return h_faddr_; }
  uint64_t in_slot_addr(uint32_t q, uint32_t pos) const {
    return reinterpret_cast<uint64_t>(d_in_) + ((uint64_t)q * cap_ + (pos & (cap_ - 1))) * 64u;
  }

  // Launch the persistent kernel over the tables/counters in `f` (pkts/out/n are ignored).
  // flows_alt: the second flow-table copy (epoch & 1 == 1); null = single copy (no live flips).
  void start(const FusedLaunch& f, const LaunchCfg& cfg, double deadline_s, const void* flows_alt = nullptr);
  // Drain published chunks, stop every wave, wait for the grid to exit (throws on timeout).
  void stop(double timeout_s = 30.0);

  uint64_t published(uint32_t q = 0) const {
    std::lock_guard<std::mutex> g(qs_[q].mu);
    return qs_[q].prod;
  }
  uint64_t completed(uint32_t q = 0);  // packets of queue q whose chunks all completed (in order)
  // Publish n packets (multiple of 64) on queue q starting at position published(q) % capacity.
  // Throws if the ring lacks room (producer must wait for completions).  Queues publish
  // independently (one lock each): one producer thread per queue never waits for another.
  uint64_t publish(uint32_t n, bool check_room = true, uint32_t q = 0);
  // Every chunk of queue q's positions [start, end) completed (lock-free flag reads; chunks
  // complete out of order across waves, so this looks at each of them).
  bool range_done(uint64_t start, uint64_t end, uint32_t q = 0) const {
    for (uint64_t c = start / 64; c < (end + 63) / 64; ++c)
      if (!chunk_done(c, q)) return false;
    return true;
  }
  // Spin until every chunk of queue q below `end` completed; false on timeout.
  bool wait(uint64_t end, double timeout_s, uint32_t q = 0);

  // Epoch flip (see the header comment): the waves switch to flow-table copy `epoch & 1` for
  // every chunk published from now on.  Throws unless the previous flip's grace period is over.
  uint32_t flip() { return change_epoch(true, false); }
  // One epoch change switching the flow-table copy and / or the table set together (a commit
  // that touched both takes effect for every chunk at once).
  uint32_t change_epoch(bool flow, bool set);
  // Grace period of the last flip: on every queue, every chunk published before it has completed.
  bool grace_over();
  bool wait_grace(double timeout_s);
  // New generation, same copies: chunks published from now on make their waves drop cached
  // table lines first (after the host changed a table in place, e.g. MAC learning).
  uint32_t bump_epoch();
  // Coop rings: write table set `which` (the idle one: 1 - table_set()) ...
  void stage_tables(const FusedLaunch& f, int which);
  // ... and switch to it (same grace rule as flip()).  Returns the new epoch.
  uint32_t flip_tables() { return change_epoch(false, true); }
  int table_set() const { return (int)((epoch() & kEpochSetBit) >> 1); }
  uint32_t lds_acl_tiles() const { return lds_tiles_; }   // ACL tiles the running grid's LDS holds
  uint32_t epoch() const { return epoch_.load(std::memory_order_acquire); }
  void set_epoch(uint32_t e);   // only while stopped

  // Control mailbox (see RingCtrlRing): `n` dwords to device address `dst`, applied by the running
  // grid; coop rings then restage their LDS copies of ports / chain words / ACL verdicts.  Returns
  // the entry's number (ctrl_done() >= it once applied).  Throws if the grid is not running or the
  // mailbox stays full for `timeout_s`.
  uint64_t post_write(uint64_t dst, const uint32_t* data, uint32_t n, double timeout_s = 1.0);
 private:
  // (no region check; restage = false: the grid's LDS copies do not hold the target)
  uint64_t post_ctrl(uint64_t dst, const uint32_t* data, uint32_t n, double timeout_s, bool restage = true);
 public:
  uint64_t ctrl_posted() const { return ctrl_head_; }
  // GPU-direct egress (see GdeRing).  gde_enable while stopped (allocates the [kMaxPorts][queues]
  // table the next start() passes to the grid); gde_set / gde_clear an entry, through the control
  // mailbox while the grid runs (returns the entry's number: once ctrl_done() passes it and every
  // chunk published before it completed, the grid no longer writes that ring) or directly while
  // stopped (returns 0).
  void gde_enable(bool on);
  bool gde_on() const { return d_gde_ != nullptr; }
  uint64_t gde_set(uint32_t port, uint32_t q, uint64_t ctl, uint64_t desc, uint64_t buf, uint32_t ring_size,
                   uint32_t buf_size, uint32_t head, uint32_t tail);
  uint64_t gde_clear(uint32_t port, uint32_t q);
  // (diagnostics, while stopped) per queue: {wait ticks, section ticks, chunks, frames, full}
  std::vector<uint64_t> gde_stats();
  // Cross-GPU hops (see XferEntry).  xfer_enable while stopped: an inbox of `entries` (power of
  // two; 0 = off) served by the grid's last `wgs` workgroups, and the per-chunk pending words.
  // Every plane's descriptor (xfer_desc) then goes to every plane (xfer_set_peers, this one's
  // number among them) before the rings start; rings of one node start and stop together.
  struct XferDesc {
    uint64_t inbox = 0, entries = 0, out = 0, out_meta = 0, xpend = 0;
    uint32_t cap = 0, ring_mask = 0, nq = 0;
  };
  void xfer_enable(uint32_t entries, uint32_t wgs);
  bool xfer_on() const { return d_xin_ != nullptr; }
  bool xfer_active() const { return xfer_active_; }   // the running grid hands frames on (XF instance)
  XferDesc xfer_desc() const;
  void xfer_set_peers(uint32_t my_plane, const std::vector<XferDesc>& planes);
  // (while stopped) {inbox tail, inbox claim}
  std::vector<uint64_t> xfer_stats();
  // Device buffers control writes may target ([base, bytes) each: the running table set's small
  // tables); anything else is refused on the host, so a bad address never reaches the GPU.
  void set_ctrl_regions(const std::vector<std::pair<uint64_t, uint64_t>>& regions);
  uint64_t ctrl_done() const;
  bool wait_ctrl(uint64_t seq, double timeout_s);

  // Closed-loop probe run entirely in C++ (no Python in the timed loop) on queue 0: `batches`
  // batches of `batch` packets, at most `inflight` outstanding.  Returns per-batch
  // publish->completion latencies (µs, host steady clock) and sets *elapsed_s to the wall time.
  std::vector<double> probe(uint32_t batches, uint32_t batch, uint32_t inflight, double* elapsed_s);

 private:
  bool chunk_done(uint64_t chunk, uint32_t q) const;
  void release_streams();
  void create_stream();   // after the grid exited: the launch stream goes
  void set_running(bool on);   // running_, and the process-wide count of running grids
  void pace_epoch_change();
  // (mu_ held) a new epoch for every queue: each queue's flip point is its published count now
  void set_epoch_all(uint32_t e);
  std::deque<std::chrono::steady_clock::time_point> epoch_changes_;   // last kRingEpochMask changes
  // Host-side state of one queue.  Its producer thread and completion scans take `mu`; an epoch
  // change takes the engine lock, then every queue's in turn (publish reads epoch_ under its
  // queue lock, so a queue's word never goes back to an older epoch).
  struct alignas(64) Queue {
    mutable std::mutex mu;
    uint64_t prod = 0;        // host copy of ctl[q].prod's count
    uint64_t floor = 0;       // chunks < floor are complete
    uint64_t flip_prod = 0;   // packets published before the last epoch change
  };
  mutable std::mutex mu_;     // epoch changes / table sets (engine-wide)
  uint32_t cap_, nch_, nq_;
  int num_cus_, wgs_;
  bool coop_;
  bool host_slots_;
  std::vector<void*> host_ptrs_;  // host_slots: pinned allocations to free
  RingCtl* ctl_ = nullptr;        // pinned, coherent: [nq]
  uint32_t* flags_ = nullptr;     // pinned, coherent: [nq][nch] completion sequence numbers
  RingDevState* st_ = nullptr;    // device: [nq]
  uint8_t* d_in_ = nullptr;
  uint32_t* d_im_ = nullptr;
  uint8_t* d_out_ = nullptr;
  uint32_t* d_meta_ = nullptr;
  uint32_t* d_svc_ = nullptr;
  uint64_t* h_faddr_ = nullptr;    // host_slots: [nq][cap] frame addresses (pinned)
  uint64_t* d_faddr_ = nullptr;    // (its device view)
  bool faddr_on_ = false;
  hipStream_t stream_{};
  std::unique_ptr<Queue[]> qs_;
  std::atomic<uint32_t> epoch_{0};   // current flow-table epoch (copy epoch_ & 1)
  bool running_ = false;
  int device_ = 0;
  FusedLaunch launch_{};
  RingTableSet* h_sets_ = nullptr;   // [2] table sets (coop rings): pinned coherent host memory
  RingTableSet* d_sets_ = nullptr;   // (its device view)
  // [2] the grid's copies of the table sets, in HBM: a flip's restage reads them there, not over
  // PCIe.  Filled at start() (a copy before the launch) and, under a running grid, by the grid
  // itself through its control mailbox (stage_tables posts the idle set's words)
  RingTableSet* dd_sets_ = nullptr;
  RingCtrlRing* ctrl_ = nullptr;     // pinned, coherent: the control mailbox
  uint64_t ctrl_head_ = 0;           // (ctrl_mu_) entries posted
  std::mutex ctrl_mu_;
  std::vector<std::pair<uint64_t, uint64_t>> ctrl_regions_;   // (mu_) writable device ranges
  uint32_t lds_tiles_ = 0;
  uint32_t set_serial_ = 0;
  GdeRing* d_gde_ = nullptr;         // [kMaxPorts][nq] (HBM), null: GPU-direct egress off
  uint64_t gde_write(uint32_t port, uint32_t q, const GdeRing& e);
  XferInbox* d_xin_ = nullptr;       // cross-GPU hops: this plane's inbox header (HBM)
  XferEntry* d_xent_ = nullptr;      // ... and entries
  uint32_t xcap_ = 0, xwgs_ = 0;
  uint32_t* h_xpend_ = nullptr;      // [nq][nch] hand-offs per chunk not back yet (pinned)
  uint32_t* d_xpend_ = nullptr;      // (its device view)
  XferPeer* d_xpeers_ = nullptr;     // [nplanes] (HBM), null: peers not set
  std::vector<XferPeer> h_xpeers_;   // the same, host copy (RingArgs::xpv)
  uint32_t xplane_ = 0, nplanes_ = 0;
  bool xfer_active_ = false;
};

// hipHostUnregister(p), then after(), once no ring of this process is running (at once if none
// is): the unregistration waits for the device, which a resident grid never leaves idle.
void host_unregister_when_idle(void* p, std::function<void()> after);
// Host regions whose unregistration waits for every ring grid of the process to stop (zero-copy
// memif vports removed while rings run): the live path restarts its rings when they pile up.
size_t deferred_host_unmaps();

// Launch the persistent kernel (ring.hip).  Exposed for the engine only.
struct RingLaunch {
  FusedLaunch f;
  const void* pkts; const uint32_t* inmeta; void* out; uint32_t* out_meta;
  uint32_t ring_mask;
  uint32_t queues;            // independent rings (per-queue buffers follow each other)
  RingCtl* ctl; uint32_t* flags; RingDevState* st; uint32_t* svc;
  unsigned long long deadline_ticks;
  const void* flows_alt;  // second flow-table copy (epoch & 1 == 1); f.t.flows is copy 0
  const RingTableSet* sets;   // coop: the two table sets
  uint32_t lds_tiles;         // coop: ACL tiles the LDS layout is sized for (>= any set's tiles)
  uint32_t epoch0;            // epoch at launch (its set bit names the set to stage first)
  RingCtrlRing* ctrl;         // device view of the control mailbox
  const uint64_t* faddr;      // frame addresses per slot (null: frames are in the in slots)
  GdeRing* gde = nullptr;     // GPU-direct egress table [kMaxPorts][queues] (null: off)
  const XferPeer* xpeers = nullptr;   // cross-GPU hops: every plane (null: off)
  const XferPeer* xpeers_h = nullptr; // the same records in host memory (copied into the kernargs)
  uint32_t xplane = 0, nplanes = 0, xfer_wgs = 0;
  uint32_t* xpend = nullptr;          // this ring's pending hand-offs per chunk
};
hipError_t launch_ring(const RingLaunch& r, const LaunchCfg& cfg, int wgs_per_cu, bool coop, hipStream_t s);

}  // namespace nfdp
