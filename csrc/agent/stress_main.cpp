// stress_main.cpp — concurrency stress for the control agent, built with ThreadSanitizer or
// AddressSanitizer+UBSan (race detection, SURVEY §5: the reference relies on `go test -race`
// for its Go parts and has none for the C agent).
//
//   agent-stress [seconds]
// Phase 1: SPSC ring torture — one producer, one consumer, variable-size records that wrap the
//          ring end; every record carries a sequence number and a payload pattern the consumer
//          checks (ordering, tearing).
// Phase 2: agent + host client under load — the fw loop thread, host requests from several
//          threads (HostCtrl serialises them), link flaps and stats updates from data-plane side
//          threads, notification draining, heartbeats and host-requested resets (PERST).
// Exit 0 when every check holds; the sanitizer runtime makes any race / memory error fatal.
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "agent.h"

using namespace agent;
using clk = std::chrono::steady_clock;

static int g_fail = 0;
#define CHECK(c)                                                                   \
  do {                                                                             \
    if (!(c)) {                                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);    \
      ++g_fail;                                                                    \
    }                                                                              \
  } while (0)

static std::string tmp_path(const char* tag) {
  return std::string("/tmp/agent-stress-") + tag + "-" + std::to_string(getpid());
}

static void ring_torture(double secs) {
  const std::string p = tmp_path("ring");
  Mailbox mb = Mailbox::create(p, 4096);
  Ring& r = mb.h2f();
  std::atomic<bool> done{false};
  std::atomic<uint64_t> sent{0};
  std::thread prod([&] {
    uint64_t seq = 0;
    std::vector<uint8_t> buf(512);
    const auto end = clk::now() + std::chrono::duration<double>(secs);
    while (clk::now() < end) {
      const uint32_t n = 8 + (uint32_t)((seq * 2654435761u) % 300);
      for (uint32_t i = 0; i < n; ++i) buf[i] = (uint8_t)(seq + i);
      std::memcpy(buf.data(), &seq, 8);
      MsgHdr h{};
      h.sz = n;
      h.msg_id = (uint16_t)seq;
      h.flags = kFlagReq;
      while (!r.push(h, buf.data())) std::this_thread::yield();
      ++seq;
    }
    sent.store(seq);
    done.store(true, std::memory_order_release);
  });
  uint64_t expect = 0;
  Msg m;
  for (;;) {
    if (r.pop(m)) {
      uint64_t seq;
      std::memcpy(&seq, m.data.data(), 8);
      CHECK(seq == expect);
      CHECK(m.hdr.msg_id == (uint16_t)expect);
      for (uint32_t i = 8; i < m.hdr.sz; ++i)
        if (m.data[i] != (uint8_t)(seq + i)) { CHECK(false); break; }
      ++expect;
    } else if (done.load(std::memory_order_acquire) && r.used() == 0) {
      break;
    } else {
      std::this_thread::yield();
    }
  }
  prod.join();
  CHECK(expect == sent.load());
  std::printf("ring: %llu records\n", (unsigned long long)expect);
  unlink(p.c_str());
}

static AgentConfig small_config(int n_vfs) {
  AgentConfig c;
  c.hb_interval_ms = 5;
  c.hb_miss_count = 200;
  PemCfg pem;
  PfCfg pf;
  pf.iface.mac[0] = 0x02;
  pf.iface.link_state = 1;
  pf.info.hb_interval_ms = c.hb_interval_ms;
  pf.info.hb_miss_count = c.hb_miss_count;
  for (int v = 0; v < n_vfs; ++v) {
    VfCfg vf;
    vf.idx = v;
    vf.iface.mac[0] = 0x02;
    vf.iface.mac[5] = (uint8_t)v;
    vf.iface.link_state = 1;
    vf.iface.dp_port = v;
    pf.vfs.push_back(vf);
  }
  pem.pfs.push_back(pf);
  c.pems.push_back(pem);
  return c;
}

static void agent_load(double secs) {
  const std::string p = tmp_path("mbox");
  const int n_vfs = 8;
  Agent ag(p, small_config(n_vfs), 16384, 4);
  ag.start(-1);
  HostCtrl host(p);
  CHECK(host.wait_ready(5000));
  std::atomic<bool> stop{false};
  std::atomic<uint64_t> reqs{0}, notes{0}, resets{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t) {
    th.emplace_back([&, t] {
      uint32_t x = 12345u + t;
      while (!stop.load()) {
        x = x * 1664525u + 1013904223u;
        Request q{};
        const int vf = (int)(x >> 8) % n_vfs;
        q.hdr.cmd = (uint16_t)((x >> 4) & 1 ? H2F::Mtu : H2F::GetIfStats);
        q.op = (uint16_t)(((x >> 5) & 1) ? Cmd::Set : Cmd::Get);
        q.val16 = (uint16_t)(1000 + (x >> 16) % 8000);
        try {
          Response r = host.request(0, 0, vf, q, 2000);
          CHECK(r.hdr.reply == (uint16_t)Reply::Ok);
          reqs.fetch_add(1);
        } catch (const std::exception& e) {
          // a reset in flight may drop a request; anything else is a failure
          if (resets.load() == 0) { std::fprintf(stderr, "request: %s\n", e.what()); CHECK(false); }
        }
      }
    });
  }
  th.emplace_back([&] {  // data-plane side: link flaps + counter updates
    uint64_t i = 0;
    while (!stop.load()) {
      const FnKey k{0u, 0u, (int32_t)(i % n_vfs)};
      ag.set_link(k, (i & 1) != 0);
      RxStats rx{};
      TxStats tx{};
      rx.pkts = i;
      tx.pkts = 2 * i;
      ag.update_stats(k, rx, tx);
      ++i;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  });
  th.emplace_back([&] {  // host housekeeping: notifications, heartbeat, liveness
    while (!stop.load()) {
      notes.fetch_add(host.take_notifications().size());
      host.host_heartbeat();
      CHECK(host.fw_alive());
      (void)ag.counters();
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });
  th.emplace_back([&] {  // periodic PERST
    const auto end = clk::now() + std::chrono::duration<double>(secs);
    while (clk::now() < end) {
      std::this_thread::sleep_for(std::chrono::milliseconds(150));
      CHECK(host.reset(3000));
      resets.fetch_add(1);
    }
    stop.store(true);
  });
  for (auto& t : th) t.join();
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  notes.fetch_add(host.take_notifications().size());
  ag.stop();
  const AgentCounters c = ag.counters();
  std::printf("agent: %llu requests, %llu notifications, %llu resets (fw saw %llu)\n",
              (unsigned long long)reqs.load(), (unsigned long long)notes.load(),
              (unsigned long long)resets.load(), (unsigned long long)c.resets);
  CHECK(reqs.load() > 100);
  CHECK(notes.load() > 0);
  CHECK(c.resets == resets.load());
  unlink(p.c_str());
}

int main(int argc, char** argv) {
  const double secs = argc > 1 ? std::atof(argv[1]) : 2.0;
  ring_torture(secs);
  agent_load(secs);
  if (g_fail) {
    std::fprintf(stderr, "%d checks failed\n", g_fail);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
