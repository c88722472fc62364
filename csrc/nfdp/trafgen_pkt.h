// trafgen_pkt.h — the pod-side generator / sink of trafgen.h for kernel-netdev pods: every pod is
// one interface inside its own network namespace (the pod end of a veth pair, as the CNI leaves
// it), driven through AF_PACKET TPACKET_V2 rings (iox.h PacketPort) opened inside that namespace,
// or (`xdp`) through an AF_XDP socket with its redirect program on the pod's interface (iox.h
// XdpPort: an AF_XDP-capable pod application, e.g. a DPDK af_xdp PMD, on a plain veth).
// The same generator feeds the native engine's veth vports and the Linux bridge comparator
// (tools/live_bench.py --comparator), so both are measured with identical pods.
//
// Header-only; linked into the _nfdp module.
#pragma once
#include <fcntl.h>
#include <sched.h>
#include <unistd.h>

#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "iox.h"
#include "trafgen.h"

namespace nfdp {
namespace trafgen {

struct NetPod {
  std::string netns;                // /var/run/netns/<name> ("" = this namespace)
  std::string ifname;               // the pod's interface inside it
  std::vector<uint8_t> frames;      // templates, each `stride` bytes
  std::vector<uint32_t> lens;
  uint32_t stride = 0;
};

// A PacketPort (or XdpPort) opened inside `netns` (a helper thread enters the namespace: namespaces
// are per thread, the caller's never changes; the socket stays bound to the pod's interface).
inline std::shared_ptr<iox::Port> open_in_netns(const std::string& netns, const std::string& ifname,
                                                uint32_t frames, bool xdp = false) {
  std::shared_ptr<iox::Port> port;
  std::string err;
  std::thread t([&] {
    try {
      if (!netns.empty()) {
        const int fd = ::open(netns.c_str(), O_RDONLY | O_CLOEXEC);
        if (fd < 0) throw std::runtime_error("trafgen: cannot open " + netns);
        const int r = setns(fd, CLONE_NEWNET);
        ::close(fd);
        if (r != 0) throw std::runtime_error("trafgen: setns " + netns);
      }
      if (xdp) port = std::make_shared<iox::XdpPort>(ifname, frames, 2048);
      else port = std::make_shared<iox::PacketPort>(ifname, frames, 2048);
    } catch (const std::exception& e) {
      err = e.what();
    }
  });
  t.join();
  if (!err.empty()) throw std::runtime_error(err);
  return port;
}

inline Result run_netns(const std::vector<NetPod>& pods, const Config& cfg, bool xdp = false) {
  const size_t np = pods.size();
  std::vector<std::shared_ptr<iox::Port>> ports;
  std::vector<std::vector<uint32_t>> ts_off(np);
  for (size_t k = 0; k < np; ++k) {
    ports.push_back(open_in_netns(pods[k].netns, pods[k].ifname, 4096, xdp));
    for (size_t c = 0; c < pods[k].lens.size(); ++c)
      ts_off[k].push_back(ts_offset(pods[k].frames.data() + c * pods[k].stride, pods[k].lens[c]));
  }
  const uint32_t nth = std::max<uint32_t>(1, std::min<uint32_t>(cfg.threads, (uint32_t)np));
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
      std::vector<uint32_t> cursor(mine.size(), 0);
      std::vector<iox::TxItem> items(cfg.burst);
      std::vector<iox::RxRef> refs(512);
      uint64_t credit_t = now_ns();
      double credit = 0.0;
      for (;;) {
        const uint64_t now = now_ns();
        if (now >= t_end) break;
        if (per_thread_rate > 0) {
          credit += (double)(now - credit_t) * 1e-9 * per_thread_rate;
          credit_t = now;
          credit = std::min(credit, (double)cfg.burst * mine.size());
        }
        for (size_t k = 0; k < mine.size(); ++k) {
          const NetPod& pd = pods[mine[k]];
          if (pd.lens.empty()) continue;
          uint32_t n = cfg.burst;
          if (per_thread_rate > 0) n = std::min<uint32_t>(n, (uint32_t)credit);
          if (!n) continue;
          const uint64_t ts = now_ns();
          for (uint32_t i = 0; i < n; ++i) {
            const uint32_t c = cursor[k];
            const uint8_t* f = pd.frames.data() + (size_t)c * pd.stride;
            const uint32_t len = pd.lens[c], off = ts_off[mine[k]][c];
            items[i] = off ? iox::TxItem{f, off, reinterpret_cast<const uint8_t*>(&ts), 8, f + off + 8, len - off - 8}
                           : iox::TxItem{f, len, nullptr, 0, nullptr, 0};
            cursor[k] = (c + 1) % (uint32_t)pd.lens.size();
          }
          const uint32_t put = ports[mine[k]]->tx_batch(items.data(), n);
          me.full += n - put;
          if (put && now >= t_meas) { me.sent += put; me.tx_pod[mine[k]] += put; }
          if (per_thread_rate > 0) credit -= put;
        }
        for (size_t k = 0; k < mine.size(); ++k) {
          iox::Port& port = *ports[mine[k]];
          const uint32_t got = port.rx(refs.data(), (uint32_t)refs.size());
          if (!got) continue;
          const uint64_t trx = now_ns();
          for (uint32_t i = 0; i < got; ++i) {
            const iox::RxRef& r = refs[i];
            if (r.len >= 14) {
              const uint32_t off = ts_offset(r.data, r.len);
              uint64_t ts = 0;
              if (off) std::memcpy(&ts, r.data + off, 8);
              if (!off || ts > trx) {
                ++me.bad;
              } else if (ts >= t_meas) {
                ++me.recv;
                ++me.rx_pod[mine[k]];
                if (me.lat.size() < cfg.max_samples / nth + 1) me.lat.push_back((double)(trx - ts) * 1e-3);
              }
            }
            port.handed_out(r.seq);
            port.complete(r.seq);
          }
          port.reclaim();
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

}  // namespace trafgen
}  // namespace nfdp
