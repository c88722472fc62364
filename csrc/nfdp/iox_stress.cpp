// iox_stress.cpp — concurrency stress of the native I/O engine (iox.h) for ThreadSanitizer and
// AddressSanitizer + UBSan builds (dpu_operator_amd/native/build.py build_sanitized("iox-*")).
// Host code only: two bit-exact oracle backends stand in for two GPUs, so the whole engine runs —
// queues, owner steering, tx workers, the per-burst side pass, the learner — with none of HIP.
//
//   iox-stress <dir> [seconds]
//
// Six memif pods on one learning L2 bridge (one pod MAC unknown: its frames flood), driven by the
// trafgen generator / sinks, while a control thread keeps changing everything the control plane
// can change under traffic:
//   * pause -> reconfigure the oracle backends -> resume   (a commit on oracle planes)
//   * hold -> new side-table snapshot, redirect map, side ports -> release   (a live GPU commit)
//   * steering key / port table swaps
//   * a port removed and re-added while its pod keeps sending
//   * punts / latency samples / statistics / side counters read concurrently
//   * an injected engine failure, then a rebuilt engine over the same ports and backends.
// Exit 0 when the checks hold; the sanitizer runtime makes any race or memory error fatal.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "iox.h"
#include "trafgen.h"

using namespace nfdp;
using namespace nfdp::iox;
using clk = std::chrono::steady_clock;

static int g_fail = 0;
#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);  \
      ++g_fail;                                                                  \
    }                                                                            \
  } while (0)

namespace {
constexpr uint32_t kPods = 6, kBridge = 1;

void mac_of(uint32_t pod, uint8_t m[6]) {
  const uint8_t b[6] = {0x02, 0x5e, 0x00, 0x00, 0x10, (uint8_t)(pod + 1)};
  std::memcpy(m, b, 6);
}
uint32_t lo_of(const uint8_t m[6]) { return m[0] | (m[1] << 8) | (m[2] << 16) | ((uint32_t)m[3] << 24); }
uint32_t hi_of(const uint8_t m[6]) { return m[4] | (m[5] << 8); }

// The tables of a small learning bridge (host arrays the oracle reads in place).
struct Bridge {
  std::vector<PortEntry> ports = std::vector<PortEntry>((size_t)kMaxPorts + 2);
  std::vector<MacEntry> macs = std::vector<MacEntry>(1024);         // the pipeline's table (learned into)
  std::vector<MacEntry> model;                                       // the control plane's copy (snapshots)
  std::vector<FlowSlot> flows = std::vector<FlowSlot>(16 * kBucketSlots);
  std::vector<uint16_t> flood = std::vector<uint16_t>((size_t)(kBridge + 1) * kFloodWays, (uint16_t)kPortNone);
  std::vector<uint8_t> rss = std::vector<uint8_t>(64);
  // counters per backend (each plane owns its own, as MultiDataPlane planes do)
  std::vector<std::vector<uint64_t>> port_ctr = std::vector<std::vector<uint64_t>>(2, std::vector<uint64_t>((size_t)2 * kMaxPorts)),
                                     drop_ctr = std::vector<std::vector<uint64_t>>(2, std::vector<uint64_t>(16)),
                                     flow_ctr = std::vector<std::vector<uint64_t>>(2, std::vector<uint64_t>(16 * kBucketSlots));
  std::vector<std::vector<MacEntry>> dev_macs;   // each plane's own MAC table (learned into)
  void configure(std::vector<std::shared_ptr<OracleBackend>>& bes) {
    if (dev_macs.size() != bes.size()) dev_macs.assign(bes.size(), macs);
    for (size_t g = 0; g < bes.size(); ++g) {
      TablesView t = view();
      t.macs = dev_macs[g].data();
      bes[g]->configure(t, flow_ctr[g].data(), port_ctr[g].data(), drop_ctr[g].data(), dev_macs[g].data(), 1023);
    }
  }
  Bridge() {
    std::mt19937 rng(7);
    for (auto& b : rss) b = (uint8_t)rng();
    std::memset(macs.data(), 0, macs.size() * sizeof(MacEntry));
    std::memset(flows.data(), 0, flows.size() * sizeof(FlowSlot));
    for (uint32_t p = 0; p < kPods; ++p) {
      PortEntry& e = ports[p];
      std::memset(&e, 0, sizeof(e));
      e.flags = kPortValid | kPortLearn;
      e.bridge_id = kBridge;
      flood[(size_t)kBridge * kFloodWays + p] = (uint16_t)p;
      if (p + 1 < kPods) {   // static MACs for all but the last pod: its traffic floods
        uint8_t m[6];
        mac_of(p, m);
        const uint32_t ev[4] = {lo_of(m), hi_of(m) | (kBridge << 16), p, 0};
        mac_learn_cpu(macs.data(), 1023, ev, 1, 1);
      }
    }
    model = macs;
  }
  TablesView view() {
    TablesView t{};
    t.ports = ports.data();
    t.macs = macs.data();
    t.mac_mask = 1023;
    t.flows = flows.data();
    t.bucket_mask = 15;
    t.rss_key = rss.data();
    t.acl_default_permit = 1;
    t.flood = flood.data();
    t.n_flood = kBridge + 1;
    return t;
  }
  std::shared_ptr<SideTables> side() {
    SideTables::Src s{};
    s.ports = ports.data(); s.n_ports = kMaxPorts;
    s.macs = model.data(); s.mac_mask = 1023;
    s.flood = flood.data(); s.flood_rows = kBridge + 1; s.n_flood = kBridge + 1;
    s.rss_key = rss.data();
    return std::make_shared<SideTables>(s);
  }
};

// 64-B IPv4 / UDP frames from pod `src` to the other pods (and to the unknown one: flooded)
trafgen::Pod pod_frames(const std::string& path, uint32_t src) {
  trafgen::Pod p;
  p.path = path;
  p.stride = 64;
  if (src + 1 == kPods) return p;   // the unknown pod only listens: frames to it keep flooding
  for (uint32_t d = 0; d < kPods; ++d) {
    if (d == src) continue;
    for (uint32_t k = 0; k < 4; ++k) {
      uint8_t f[64] = {};
      uint8_t dm[6], sm[6];
      mac_of(d, dm);
      mac_of(src, sm);
      std::memcpy(f, dm, 6);
      std::memcpy(f + 6, sm, 6);
      f[12] = 0x08; f[13] = 0x00;
      f[14] = 0x45; f[16] = 0; f[17] = 46; f[22] = 64; f[23] = 17;
      f[26] = 10; f[27] = 0; f[28] = 0; f[29] = (uint8_t)(src + 1);
      f[30] = 10; f[31] = 0; f[32] = 0; f[33] = (uint8_t)(d + 1);
      f[34] = 0x10; f[35] = (uint8_t)k; f[36] = 0x00; f[37] = 80; f[38] = 0; f[39] = 26;
      p.frames.insert(p.frames.end(), f, f + 64);
      p.lens.push_back(60);
    }
  }
  return p;
}

std::unique_ptr<Engine> make_engine(Bridge& br, std::vector<std::shared_ptr<OracleBackend>>& bes,
                                    std::vector<std::shared_ptr<Port>>& ports) {
  auto e = std::make_unique<Engine>(128, 16, 2, 2, 1024);
  br.configure(bes);
  for (auto& b : bes) e->add_backend(b);
  e->set_zero_copy(true);   // backend 1 reads frames by address (in the pods' regions): zero-copy rx
  for (uint32_t p = 0; p < kPods; ++p) e->add_port(p, ports[p]);
  e->set_steering(br.ports, br.rss, false);
  std::vector<uint32_t> side;
  for (uint32_t p = 0; p < kPods; ++p) side.push_back(p);
  e->set_side_ports(side);
  for (uint32_t g = 0; g < bes.size(); ++g) e->set_side_tables(g, br.side());
  e->start();
  return e;
}
}  // namespace

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const double secs = argc > 2 ? std::atof(argv[2]) : 1.5;
  Bridge br;
  std::vector<std::shared_ptr<OracleBackend>> bes = {std::make_shared<OracleBackend>(1024, 2),
                                                     std::make_shared<OracleBackend>(1024, 2)};
  bes[1]->set_frame_addrs(true);
  std::vector<std::shared_ptr<Port>> ports;
  std::vector<trafgen::Pod> pods;
  for (uint32_t p = 0; p < kPods; ++p) {
    const std::string path = dir + "/pod" + std::to_string(p);
    ports.push_back(std::make_shared<MemifPort>(path, 512, 2048));
    pods.push_back(pod_frames(path, p));
  }
  auto eng = make_engine(br, bes, ports);

  trafgen::Config cfg;
  cfg.duration_s = secs;
  cfg.warmup_s = 0.05;
  cfg.threads = 2;
  cfg.burst = 16;
  trafgen::Result res;
  std::thread gen([&] { res = trafgen::run(pods, cfg); });

  const auto t_end = clk::now() + std::chrono::duration<double>(secs + 0.05);
  std::mt19937 rng(1);
  uint32_t ops = 0, restarts = 0;
  bool injected = false;
  while (clk::now() < t_end) {
    switch (rng() % 6) {
      case 0:   // a commit on oracle planes: nothing in flight while the tables move
        eng->pause();
        br.configure(bes);
        eng->resume();
        break;
      case 1: {  // a live commit: publication held, configuration swapped
        eng->hold();
        for (uint32_t g = 0; g < bes.size(); ++g) eng->set_side_tables(g, br.side());
        eng->set_redirects({{(uint32_t)kPods + 10, 0u}});
        std::vector<uint32_t> side;
        for (uint32_t p = 0; p < kPods; ++p)
          if (rng() & 1) side.push_back(p);
        eng->set_side_ports(side);
        eng->set_side_always((rng() & 3) == 0);
        eng->release();
        break;
      }
      case 2:
        eng->set_steering(br.ports, br.rss, (rng() & 1) != 0);
        break;
      case 3: {  // a port goes away and comes back while its pod keeps sending
        auto old = eng->remove_port(3);
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        eng->add_port(3, old ? old : ports[3], (int)(rng() % 2));
        break;
      }
      case 4: {
        (void)eng->take_punts(64);
        (void)eng->take_latency_us();
        auto st = eng->stats();
        (void)eng->side_port_counters();
        (void)eng->side_drop_counters();
        CHECK(st["queues"] == 2);
        break;
      }
      case 5:
        if (!injected && clk::now() > t_end - std::chrono::duration<double>(secs / 2)) {
          injected = true;
          eng->inject_failure("stress: injected");
          CHECK(!eng->running());
          CHECK(eng->error() == "stress: injected");
          eng->stop();
          eng = make_engine(br, bes, ports);   // same ports, same backends: a supervisor restart
          ++restarts;
        }
        break;
    }
    ++ops;
    std::this_thread::sleep_for(std::chrono::microseconds(300));
  }
  gen.join();
  eng->flush_learning();
  auto st = eng->stats();
  CHECK(eng->error().empty());
  eng->stop();
  CHECK(res.sent > 0 && res.received > 0);
  CHECK(res.bad == 0);
  CHECK(restarts == 1);
  CHECK(st["replicas"] > 0);   // floods to the never-learned pod went through the side pass
  CHECK(st["zero_copy_frames"] > 0);
  std::printf("ops %u restarts %u sent %llu received %llu engine rx %llu tx %llu replicas %llu learn %llu\n", ops,
              restarts, (unsigned long long)res.sent, (unsigned long long)res.received,
              (unsigned long long)st["rx"], (unsigned long long)st["tx"], (unsigned long long)st["replicas"],
              (unsigned long long)st["learn_events"]);
  if (g_fail) {
    std::printf("FAILED %d\n", g_fail);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
