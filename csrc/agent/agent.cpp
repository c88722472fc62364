// agent.cpp — fw-side control agent loop and the host-side control client (see agent.h).
#include "agent.h"

#include <algorithm>

#include <cstring>
#include <stdexcept>

#include "plugin_server.h"

namespace agent {

using clock_t_ = std::chrono::steady_clock;

// ------------------------------------------------------------------------------------------ Agent

Agent::Agent(std::string mbox_path, AgentConfig cfg, uint32_t mbox_size, int max_msgs)
    : path_(std::move(mbox_path)), cfg_(std::move(cfg)), mbox_size_(mbox_size), max_msgs_(max_msgs > 0 ? max_msgs : 6) {}

Agent::~Agent() { stop(); }

void Agent::load_interfaces() {
  std::lock_guard<std::mutex> g(net_.mutex());
  for (const PemCfg& pem : cfg_.pems) {
    for (const PfCfg& pf : pem.pfs) {
      auto init = [](IfState& s, const IfCfg& c) {
        s = IfState{};
        std::memcpy(s.mac, c.mac, 6);
        s.link = c.link_state ? State::Up : State::Down;
        s.rx = c.rx_state ? State::Up : State::Down;
        s.link_info.autoneg = (uint8_t)c.autoneg;
        s.link_info.pause = (uint8_t)c.pause_mode;
        s.link_info.speed = (uint32_t)c.speed;
        s.link_info.supported_modes = (uint64_t)c.supported_modes;
        s.link_info.advertised_modes = (uint64_t)c.advertised_modes;
        s.dp_port = (int32_t)c.dp_port;
      };
      init(net_.iface(FnKey{(uint32_t)pem.idx, (uint32_t)pf.idx, -1}), pf.iface);
      for (const VfCfg& vf : pf.vfs) init(net_.iface(FnKey{(uint32_t)pem.idx, (uint32_t)pf.idx, vf.idx}), vf.iface);
      net_.fw_info = pf.info;
    }
  }
  net_.fw_info.hb_interval_ms = cfg_.hb_interval_ms;
  net_.fw_info.hb_miss_count = cfg_.hb_miss_count;
  net_.bump();  // (re)loaded state: the data plane re-applies it
}

void Agent::start(int plugin_port) {
  if (running_.load()) return;
  mbox_ = Mailbox::create(path_, mbox_size_);
  load_interfaces();
  Info& in = mbox_.info();
  in.fw_hb_interval.store(cfg_.hb_interval_ms, std::memory_order_relaxed);
  in.fw_hb_miss.store(cfg_.hb_miss_count, std::memory_order_relaxed);
  resets_seen_ = in.host_resets.load(std::memory_order_acquire);
  in.fw_resets.store(resets_seen_, std::memory_order_relaxed);
  if (plugin_port >= 0) {
    plugin_ = std::make_unique<PluginServer>(
        plugin_port, [this](const MsgHdr& h, const std::vector<uint8_t>& d) { send_custom(h, d); });
    plugin_->start();
  }
  running_.store(true);
  in.fw_status.store((uint64_t)Status::Ready, std::memory_order_release);  // "fw ready"
  thr_ = std::thread([this] { loop(); });
}

void Agent::stop() {
  if (!running_.exchange(false)) return;
  if (thr_.joinable()) thr_.join();
  if (plugin_) plugin_->stop();
  plugin_.reset();
  if (mbox_.valid()) mbox_.info().fw_status.store((uint64_t)Status::Uninit, std::memory_order_release);
}

void Agent::handle_reset() {
  Info& in = mbox_.info();
  const uint64_t req = in.host_resets.load(std::memory_order_acquire);
  if (req == resets_seen_) return;
  in.fw_status.store((uint64_t)Status::Init, std::memory_order_release);
  mbox_.reset_rings();
  {
    std::lock_guard<std::mutex> g(out_mu_);
    out_.clear();
  }
  load_interfaces();
  resets_seen_ = req;
  {
    std::lock_guard<std::mutex> g(cnt_mu_);
    cnt_.resets++;
  }
  if (plugin_) plugin_->broadcast_event(PluginServer::kEvPerst, {});
  in.fw_resets.store(req, std::memory_order_release);
  in.fw_status.store((uint64_t)Status::Ready, std::memory_order_release);
}

void Agent::flush_out() {
  std::lock_guard<std::mutex> g(out_mu_);
  while (!out_.empty()) {
    const Msg& m = out_.front();
    if (!mbox_.f2h().push(m.hdr, m.data.data())) break;  // host is slow: keep order, retry later
    out_.pop_front();
  }
}

void Agent::process_host(int budget) {
  Info& in = mbox_.info();
  if (in.host_status.load(std::memory_order_acquire) != (uint64_t)Status::Ready) return;
  const uint64_t host_ver = in.host_version.load(std::memory_order_acquire);
  Msg m;
  for (int n = 0; n < budget; ++n) {
    {
      // Never take a request whose response could not be queued behind a full F2H backlog.
      std::lock_guard<std::mutex> g(out_mu_);
      if (out_.size() > 1024) break;
    }
    bool got;
    try {
      got = mbox_.h2f().pop(m);
    } catch (const std::exception&) {
      std::lock_guard<std::mutex> g(cnt_mu_);
      cnt_.bad_msgs++;
      break;
    }
    if (!got) break;
    if (m.hdr.flags & kFlagCustom) {
      {
        std::lock_guard<std::mutex> g(cnt_mu_);
        cnt_.custom_in++;
      }
      if (plugin_) plugin_->broadcast_msg(m);
      continue;
    }
    if (!(m.hdr.flags & kFlagReq) || m.hdr.sz < sizeof(ReqHdr)) {
      std::lock_guard<std::mutex> g(cnt_mu_);
      cnt_.bad_msgs++;
      continue;
    }
    Request req;
    std::memset(&req, 0, sizeof(req));
    std::memcpy(&req, m.data.data(), m.hdr.sz < sizeof(req) ? m.hdr.sz : sizeof(req));
    const Response r = net_.handle(key_of(m.hdr), req, host_ver);
    Msg out;
    out.hdr = m.hdr;
    out.hdr.flags = kFlagResp;
    out.hdr.sz = sizeof(Response);
    out.data.resize(sizeof(Response));
    std::memcpy(out.data.data(), &r, sizeof(Response));
    bool deferred;
    {
      std::lock_guard<std::mutex> g(out_mu_);
      out_.push_back(std::move(out));
      deferred = out_.size() > 1;
    }
    std::lock_guard<std::mutex> g(cnt_mu_);
    cnt_.requests++;
    cnt_.responses++;
    if (deferred) cnt_.resp_deferred++;
  }
}

void Agent::loop() {
  Info& in = mbox_.info();
  const auto hb_every = std::chrono::milliseconds(cfg_.hb_interval_ms ? cfg_.hb_interval_ms : 1000);
  auto next_hb = clock_t_::now();
  while (running_.load(std::memory_order_relaxed)) {
    const uint32_t seen = mbox_.h2f().bell();
    handle_reset();
    process_host(max_msgs_);
    flush_out();
    const auto now = clock_t_::now();
    if (now >= next_hb) {
      in.fw_heartbeat.fetch_add(1, std::memory_order_acq_rel);
      next_hb = now + hb_every;
      std::lock_guard<std::mutex> g(cnt_mu_);
      cnt_.heartbeats++;
    }
    // Sleep on the H2F doorbell (host requests, resets, status changes and local link events
    // ring it) until the next heartbeat is due; with requests left over from the per-iteration
    // budget, or F2H records waiting for ring space, only briefly.
    bool backlog;
    {
      std::lock_guard<std::mutex> g(out_mu_);
      backlog = !out_.empty();
    }
    if (mbox_.h2f().used() != 0 && !backlog) continue;
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(next_hb - clock_t_::now()).count();
    const int cap = backlog ? 200 : 20000;
    mbox_.h2f().wait_bell(seen, (int)std::max<int64_t>(0, std::min<int64_t>(us, cap)));
  }
}

void Agent::set_link(const FnKey& k, bool up) {
  net_.set_link(k, up ? State::Up : State::Down);
  Notify n;
  std::memset(&n, 0, sizeof(n));
  n.hdr.cmd = (uint16_t)F2H::LinkStatus;
  n.state = up ? 1 : 0;
  Msg m;
  m.hdr.fn = MsgHdr::make_fn(std::get<0>(k), std::get<1>(k), std::get<2>(k) >= 0);
  m.hdr.vf_idx = (uint16_t)(std::get<2>(k) >= 0 ? std::get<2>(k) : 0);
  m.hdr.flags = kFlagNotify;
  m.hdr.sz = sizeof(Notify);
  m.data.resize(sizeof(Notify));
  std::memcpy(m.data.data(), &n, sizeof(Notify));
  {
    // Coalesce: a link notification still waiting for ring space is overwritten with the newest
    // state instead of queueing another one, so a flapping link cannot grow the queue (or delay
    // responses queued behind it) without bound — the host only needs the current state.
    std::lock_guard<std::mutex> g(out_mu_);
    bool merged = false;
    for (auto it = out_.rbegin(); it != out_.rend(); ++it) {
      if ((it->hdr.flags & kFlagNotify) && it->hdr.fn == m.hdr.fn && it->hdr.vf_idx == m.hdr.vf_idx) {
        std::memcpy(it->data.data(), &n, sizeof(Notify));
        merged = true;
        break;
      }
    }
    if (!merged) out_.push_back(std::move(m));
  }
  mbox_.h2f().ring();  // wake the fw loop to flush it
  if (plugin_) plugin_->broadcast_event(up ? PluginServer::kEvLinkUp : PluginServer::kEvLinkDown, {});
  std::lock_guard<std::mutex> g(cnt_mu_);
  cnt_.notifications++;
}

void Agent::update_stats(const FnKey& k, const RxStats& rx, const TxStats& tx) { net_.set_stats(k, rx, tx); }

IfState Agent::iface(const FnKey& k) {
  auto s = net_.snapshot();
  auto it = s.find(k);
  if (it == s.end()) throw std::out_of_range("no such function");
  return it->second;
}

std::vector<FnKey> Agent::functions() {
  std::vector<FnKey> out;
  for (auto& kv : net_.snapshot()) out.push_back(kv.first);
  return out;
}

AgentCounters Agent::counters() {
  std::lock_guard<std::mutex> g(cnt_mu_);
  return cnt_;
}

int Agent::plugin_port() const { return plugin_ ? plugin_->port() : -1; }

void Agent::send_custom(const MsgHdr& h, const std::vector<uint8_t>& data) {
  Msg m;
  m.hdr = h;
  m.hdr.flags = kFlagCustom;
  m.hdr.sz = (uint32_t)data.size();
  m.data = data;
  {
    std::lock_guard<std::mutex> g(out_mu_);
    out_.push_back(std::move(m));
  }
  mbox_.h2f().ring();
  std::lock_guard<std::mutex> g(cnt_mu_);
  cnt_.custom_out++;
}

// --------------------------------------------------------------------------------------- HostCtrl

HostCtrl::HostCtrl(const std::string& mbox_path, uint32_t host_version)
    : mbox_(Mailbox::open(mbox_path)), host_version_(host_version) {
  Info& in = mbox_.info();
  in.host_version.store(host_version_, std::memory_order_relaxed);
  in.host_status.store((uint64_t)Status::Ready, std::memory_order_release);
  last_hb_ = in.fw_heartbeat.load(std::memory_order_acquire);
  last_hb_change_ = clock_t_::now();
}

namespace {
// Announces a priority waiter on HostCtrl::mu_ until the lock is taken.
struct PriorityLock {
  explicit PriorityLock(std::atomic<int>& c) : c_(c) { c_.fetch_add(1, std::memory_order_acq_rel); }
  void acquired() {
    if (!done_) c_.fetch_sub(1, std::memory_order_acq_rel);
    done_ = true;
  }
  ~PriorityLock() { acquired(); }
  std::atomic<int>& c_;
  bool done_ = false;
};
}  // namespace

bool HostCtrl::wait_ready(int timeout_ms) {
  const auto dl = clock_t_::now() + std::chrono::milliseconds(timeout_ms);
  Info& in = mbox_.info();
  while (clock_t_::now() < dl) {
    if (in.fw_status.load(std::memory_order_acquire) == (uint64_t)Status::Ready) {
      hb_interval_ms_ = in.fw_hb_interval.load(std::memory_order_relaxed);
      hb_miss_ = in.fw_hb_miss.load(std::memory_order_relaxed);
      return true;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return false;
}

void HostCtrl::set_status(Status s) {
  mbox_.info().host_status.store((uint64_t)s, std::memory_order_release);
  mbox_.h2f().ring();
}

void HostCtrl::drain(int timeout_ms, uint16_t want_id, Response* out, bool* got) {
  const auto dl = clock_t_::now() + std::chrono::milliseconds(timeout_ms);
  Msg m;
  *got = false;
  for (;;) {
    const uint32_t seen = mbox_.f2h().bell();  // read before popping: a later push cannot be missed
    while (mbox_.f2h().pop(m)) {
      if (m.hdr.flags & kFlagResp) {
        if (m.hdr.msg_id == want_id && m.hdr.sz >= sizeof(RespHdr)) {
          std::memset(out, 0, sizeof(Response));
          std::memcpy(out, m.data.data(), m.hdr.sz < sizeof(Response) ? m.hdr.sz : sizeof(Response));
          *got = true;
        }
        // responses to requests that already timed out are dropped
      } else if (m.hdr.flags & kFlagNotify) {
        Notify n;
        std::memset(&n, 0, sizeof(n));
        std::memcpy(&n, m.data.data(), m.hdr.sz < sizeof(n) ? m.hdr.sz : sizeof(n));
        if (notes_.size() >= kMaxPendingNotes) notes_.erase(notes_.begin());  // keep the newest
        notes_.push_back(n);
      } else if (m.hdr.flags & kFlagCustom) {
        custom_.push_back(m);
      }
      if (*got) return;
    }
    if (want_id == 0) return;
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(dl - clock_t_::now()).count();
    if (us <= 0) return;
    mbox_.f2h().wait_bell(seen, (int)std::min<int64_t>(us, 20000));  // F2H doorbell (the fw rang it)
  }
}

Response HostCtrl::request(uint32_t pem, uint32_t pf, int32_t vf, Request req, int timeout_ms) {
  // yield to resets / notification drains waiting for the lock (std::mutex is not fair)
  while (prio_.load(std::memory_order_acquire) > 0) std::this_thread::yield();
  std::lock_guard<std::mutex> g(mu_);
  MsgHdr h{};
  h.fn = MsgHdr::make_fn(pem, pf, vf >= 0);
  h.vf_idx = (uint16_t)(vf >= 0 ? vf : 0);
  h.flags = kFlagReq;
  h.sz = sizeof(Request);
  h.msg_id = next_id_++;
  if (next_id_ == 0) next_id_ = 1;
  const auto dl = clock_t_::now() + std::chrono::milliseconds(timeout_ms);
  while (!mbox_.h2f().push(h, &req)) {
    if (clock_t_::now() >= dl) throw std::runtime_error("mailbox: H2F queue full");
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  Response r;
  bool got = false;
  const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(dl - clock_t_::now()).count();
  drain(left > 0 ? left : 0, h.msg_id, &r, &got);
  if (!got) throw std::runtime_error("mailbox: request timed out");
  return r;
}

std::vector<Notify> HostCtrl::take_notifications() {
  PriorityLock pl(prio_);
  std::lock_guard<std::mutex> g(mu_);
  pl.acquired();
  Response r;
  bool got;
  drain(0, 0, &r, &got);
  std::vector<Notify> out;
  out.swap(notes_);
  return out;
}

std::vector<Msg> HostCtrl::take_custom() {
  PriorityLock pl(prio_);
  std::lock_guard<std::mutex> g(mu_);
  pl.acquired();
  Response r;
  bool got;
  drain(0, 0, &r, &got);
  std::vector<Msg> out;
  out.swap(custom_);
  return out;
}

bool HostCtrl::send_custom(uint32_t pem, uint32_t pf, const std::vector<uint8_t>& data) {
  std::lock_guard<std::mutex> g(mu_);
  MsgHdr h{};
  h.fn = MsgHdr::make_fn(pem, pf, false);
  h.flags = kFlagCustom;
  h.sz = (uint32_t)data.size();
  h.msg_id = next_id_++;
  return mbox_.h2f().push(h, data.data());
}

bool HostCtrl::fw_alive() {
  Info& in = mbox_.info();
  const uint64_t hb = in.fw_heartbeat.load(std::memory_order_acquire);
  const auto now = clock_t_::now();
  if (hb != last_hb_) {
    last_hb_ = hb;
    last_hb_change_ = now;
    return true;
  }
  const auto limit = std::chrono::milliseconds(hb_interval_ms_ * (hb_miss_ ? hb_miss_ : 1));
  return now - last_hb_change_ < limit;
}

void HostCtrl::host_heartbeat() { mbox_.info().host_heartbeat.fetch_add(1, std::memory_order_acq_rel); }

uint64_t HostCtrl::fw_heartbeat() const { return mbox_.info().fw_heartbeat.load(std::memory_order_acquire); }

bool HostCtrl::reset(int timeout_ms) {
  PriorityLock pl(prio_);
  std::lock_guard<std::mutex> g(mu_);
  pl.acquired();
  Info& in = mbox_.info();
  const uint64_t want = in.host_resets.fetch_add(1, std::memory_order_acq_rel) + 1;
  mbox_.h2f().ring();  // PERST: wake the fw loop
  const auto dl = clock_t_::now() + std::chrono::milliseconds(timeout_ms);
  while (clock_t_::now() < dl) {
    if (in.fw_resets.load(std::memory_order_acquire) >= want &&
        in.fw_status.load(std::memory_order_acquire) == (uint64_t)Status::Ready) {
      notes_.clear();
      custom_.clear();
      return true;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return false;
}

}  // namespace agent
