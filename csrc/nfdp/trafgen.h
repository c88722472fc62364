// trafgen.h — pod-side traffic generator / sink over memif vports (memif.h), for the live-path
// benchmark and tests.  The reference's only traffic benchmark is kubernetes-traffic-flow-tests
// (iperf-udp, pod <-> pod over default-sriov-net: hack/cluster-configs/ocp-tft-config.yaml:1-22);
// this is the packet-rate / latency version of it for the shared-memory vports: every pod replays
// its own frame templates into its vport as fast as allowed (or at a fixed rate) and counts what
// arrives on it, with a send timestamp (steady clock, ns) written after the L4 header of every
// frame, so one-way pod -> pod latency is measured on one clock.
//
// Header-only, no HIP: linked into the _nfdp module and into the standalone `dpu-trafgen` tool.
#pragma once
#include <immintrin.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "memif.h"

namespace nfdp {
namespace trafgen {

struct Pod {
  std::string path;                 // memif region of the pod's vport
  std::vector<uint8_t> frames;      // templates, each `stride` bytes
  std::vector<uint32_t> lens;       // template lengths
  uint32_t stride = 0;
  std::vector<uint32_t> ts_off;     // timestamp offset of each template (filled by run())
};

struct Config {
  double duration_s = 1.0;
  double warmup_s = 0.1;            // received frames older than this are not counted
  double rate_pps = 0.0;            // aggregate offered rate; 0 = as fast as the vports accept
  uint32_t threads = 1;             // generator threads (pods are split between them)
  uint32_t burst = 32;              // frames per ring commit
  uint32_t max_samples = 1u << 20;  // latency samples kept (every received frame until full)
  uint32_t inflight = 0;            // all pods: max frames sent and not yet received (0 = unbounded);
                                    // 1 = closed loop (unloaded latency).  Lost frames time out after 20 ms.
};

struct Result {
  uint64_t sent = 0, received = 0, tx_full = 0, bad = 0;
  double elapsed_s = 0.0;           // measured window
  std::vector<double> lat_us;       // one-way latency samples of the measured window
  std::vector<uint64_t> rx_per_pod, tx_per_pod;
};

inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Byte offset of the timestamp: right after the L4 header (UDP 8 B, TCP 20 B) of an IPv4 frame,
// after a 802.1Q tag if present; 0 when the frame is too short / not IPv4.  A VXLAN frame (outer
// IPv4 / UDP to 4789) carries it in its inner frame: a pod behind a VTEP receives the encapsulated
// copy of what another pod sent.
inline uint32_t ts_offset(const uint8_t* f, uint32_t len, int depth = 0) {
  uint32_t l3 = 14;
  if (len >= 18 && f[12] == 0x81 && f[13] == 0x00) l3 = 18;
  if (len < l3 + 20 || f[l3 - 2] != 0x08 || f[l3 - 1] != 0x00) return 0;
  const uint32_t ihl = (f[l3] & 0xFu) * 4u;
  const uint32_t l4 = l3 + ihl + (f[l3 + 9] == 6 ? 20u : 8u);
  if (depth == 0 && f[l3 + 9] == 17 && l4 + 8 + 14 <= len && f[l3 + ihl + 2] == 0x12 && f[l3 + ihl + 3] == 0xB5) {
    const uint32_t in = l4 + 8;   // past the 8-B VXLAN header
    const uint32_t o = ts_offset(f + in, len - in, 1);
    return o ? in + o : 0;
  }
  return l4 + 8 <= len ? l4 : 0;
}

inline Result run(std::vector<Pod> pods, const Config& cfg) {
  const size_t np = pods.size();
  for (auto& p : pods) {
    p.ts_off.resize(p.lens.size());
    for (size_t c = 0; c < p.lens.size(); ++c) p.ts_off[c] = ts_offset(p.frames.data() + c * p.stride, p.lens[c]);
  }
  std::vector<std::unique_ptr<memif::Region>> regs;
  for (const auto& p : pods) regs.emplace_back(new memif::Region(p.path, false));
  const uint32_t nth = std::max<uint32_t>(1, std::min<uint32_t>(cfg.threads, (uint32_t)np));
  std::atomic<uint32_t> ready{0};
  std::atomic<int64_t> outstanding{0};
  std::atomic<uint64_t> last_rx{now_ns()};
  const uint64_t t_start = now_ns();
  const uint64_t t_meas = t_start + (uint64_t)(cfg.warmup_s * 1e9);
  const uint64_t t_end = t_meas + (uint64_t)(cfg.duration_s * 1e9);
  struct PerThread {
    uint64_t sent = 0, recv = 0, full = 0, bad = 0;
    std::vector<double> lat;
    std::vector<uint64_t> rx_pod, tx_pod;
  };
  std::vector<PerThread> pt(nth);
  std::vector<std::thread> th;
  const double per_thread_rate = cfg.rate_pps > 0 ? cfg.rate_pps / nth : 0.0;
  for (uint32_t t = 0; t < nth; ++t) {
    th.emplace_back([&, t]() {
      PerThread& me = pt[t];
      me.rx_pod.assign(np, 0);
      me.tx_pod.assign(np, 0);
      me.lat.reserve(std::min<uint32_t>(cfg.max_samples / nth + 1, 1u << 20));
      std::vector<size_t> mine;
      for (size_t i = t; i < np; i += nth) mine.push_back(i);
      std::vector<memif::Producer> prod(mine.size());
      std::vector<std::vector<memif::Consumer>> cons(mine.size());   // every data plane -> pod ring
      std::vector<uint32_t> cursor(mine.size(), 0);
      for (size_t k = 0; k < mine.size(); ++k) {
        prod[k].init(regs[mine[k]].get(), 0);
        cons[k].resize(regs[mine[k]]->rx_rings());
        for (uint32_t r = 0; r < (uint32_t)cons[k].size(); ++r) cons[k][r].init(regs[mine[k]].get(), 1 + r);
        regs[mine[k]]->hdr()->peer_up.store(1);
      }
      ready.fetch_add(1);
      uint64_t credit_t = now_ns();
      double credit = 0.0;
      for (;;) {
        const uint64_t now = now_ns();
        if (now >= t_end) break;
        // ---- tx: one burst per pod (rate-limited by a token bucket when rate_pps > 0)
        uint32_t allow = cfg.burst;
        if (per_thread_rate > 0) {
          credit += (double)(now - credit_t) * 1e-9 * per_thread_rate;
          credit_t = now;
          credit = std::min(credit, (double)cfg.burst * mine.size());
        }
        for (size_t k = 0; k < mine.size(); ++k) {
          const Pod& pd = pods[mine[k]];
          if (pd.lens.empty()) continue;
          uint32_t n = allow;
          if (per_thread_rate > 0) n = std::min<uint32_t>(n, (uint32_t)credit);
          if (cfg.inflight) {
            int64_t o = outstanding.load(std::memory_order_acquire);
            if (o > 0 && now - last_rx.load(std::memory_order_relaxed) > 20000000ull) {   // lost: give the credit back
              outstanding.compare_exchange_strong(o, 0);
              last_rx.store(now, std::memory_order_relaxed);
              o = 0;
            }
            n = (uint32_t)std::min<int64_t>(n, std::max<int64_t>(0, (int64_t)cfg.inflight - o));
          }
          uint32_t put = 0;
          const uint64_t ts = now_ns();   // one send time per burst: the burst leaves together
          for (uint32_t i = 0; i < n; ++i) {
            const uint32_t c = cursor[k];
            const uint8_t* f = pd.frames.data() + (size_t)c * pd.stride;
            const uint32_t len = pd.lens[c];
            if (prod[k].room() == 0) { ++me.full; break; }
            uint8_t* dst = prod[k].r->buf(0, prod[k].head);
            __builtin_prefetch(prod[k].r->buf(0, prod[k].head + 8), 1, 3);
            std::memcpy(dst, f, len);
            const uint32_t off = pd.ts_off[c];
            if (off) std::memcpy(dst + off, &ts, 8);
            memif::Desc& d = prod[k].r->desc(0)[prod[k].head & prod[k].r->mask()];
            d.len = len;
            d.flags = 0;
            ++prod[k].head;
            cursor[k] = (c + 1) % (uint32_t)pd.lens.size();
            ++put;
          }
          if (put) {
            prod[k].commit();
            if (now >= t_meas) { me.sent += put; me.tx_pod[mine[k]] += put; }
            if (cfg.inflight) outstanding.fetch_add(put, std::memory_order_acq_rel);
            if (per_thread_rate > 0) credit -= put;
          }
        }
        // ---- rx: everything that arrived on this thread's pods
        for (size_t k = 0; k < mine.size(); ++k) for (memif::Consumer& cn : cons[k]) {
          uint32_t avail = cn.available();
          if (!avail) continue;
          const uint64_t trx = now_ns();
          uint32_t mine_rx = 0;   // frames of this run (a previous run's leftovers do not give credit back)
          for (uint32_t i = 0; i < avail; ++i) {
            uint32_t len = 0;
            const uint8_t* f = cn.get(len);
            const uint32_t off = ts_offset(f, len);
            uint64_t ts = 0;
            if (off) std::memcpy(&ts, f + off, 8);
            if (!off || ts > trx) { ++me.bad; continue; }
            if (ts < t_start) continue;                // queued before this run started
            ++mine_rx;
            if (ts >= t_meas) {
              ++me.recv;
              ++me.rx_pod[mine[k]];
              if (me.lat.size() < cfg.max_samples / nth + 1) me.lat.push_back((double)(trx - ts) * 1e-3);
            }
          }
          cn.release_to(cn.next);
          if (cfg.inflight) {
            outstanding.fetch_sub(mine_rx, std::memory_order_acq_rel);
            last_rx.store(trx, std::memory_order_relaxed);
          }
        }
      }
    });
  }
  for (auto& x : th) x.join();
  Result r;
  r.rx_per_pod.assign(np, 0);
  r.tx_per_pod.assign(np, 0);
  for (auto& p : pt) {
    r.sent += p.sent; r.received += p.recv; r.tx_full += p.full; r.bad += p.bad;
    r.lat_us.insert(r.lat_us.end(), p.lat.begin(), p.lat.end());
    for (size_t i = 0; i < np; ++i) { r.rx_per_pod[i] += p.rx_pod[i]; r.tx_per_pod[i] += p.tx_pod[i]; }
  }
  r.elapsed_s = cfg.duration_s;
  return r;
}

// CPU share probe: `threads` threads busy-loop together for `seconds`; returns the CPU seconds
// they were granted (summed CLOCK_THREAD_CPUTIME_ID).  Divided by the wall time that is the number
// of CPUs the process really gets — under a CFS quota, less than `threads` once the quota is
// reached, whatever `nproc` says.  Threads only (no fork: the caller may hold a GPU context).
inline double cpu_share_probe(uint32_t threads, double seconds) {
  std::vector<std::thread> th;
  std::vector<double> used(threads, 0.0);
  const uint64_t t_end = now_ns() + (uint64_t)(seconds * 1e9);
  for (uint32_t t = 0; t < threads; ++t) {
    th.emplace_back([&, t]() {
      volatile uint64_t x = 0;
      while (now_ns() < t_end) x = x + 1;
      timespec ts{};
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
      used[t] = (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
    });
  }
  for (auto& x : th) x.join();
  double s = 0.0;
  for (double u : used) s += u;
  return s;
}

}  // namespace trafgen
}  // namespace nfdp
