// agent.h — the control-plane agent (fw side) and the host-side control client.
//
// Reference: octep_cp_agent main/loop (SURVEY NAT1-NAT3): parse the SoC config, init the library,
// announce fw-ready, heartbeat on a timer, and loop {process host messages; process events}.
// MI355X design: the "firmware" is a thread of the node's data-plane service.  It owns the
// ctrl-net interface table (CtrlNet), answers host requests on the shared-memory mailbox, emits
// link notifications, keeps a heartbeat word the host watches (hb_interval / hb_miss_count from
// the config), and honours host-requested resets (the PERST of the reference: rings are
// re-formatted and interface state is reloaded from the configuration).
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "config.h"
#include "ctrl_net.h"
#include "mbox.h"

namespace agent {

class PluginServer;

struct AgentCounters {
  uint64_t requests = 0, responses = 0, notifications = 0, resp_deferred = 0, bad_msgs = 0;
  uint64_t heartbeats = 0, resets = 0, custom_in = 0, custom_out = 0;
};

class Agent {
 public:
  Agent(std::string mbox_path, AgentConfig cfg, uint32_t mbox_size = 32768, int max_msgs = 6);
  ~Agent();

  void start(int plugin_port = -1);  // plugin_port: -1 none, 0 ephemeral, else fixed
  void stop();
  bool running() const { return running_.load(); }

  void set_link(const FnKey& k, bool up);     // also notifies the host (F2H LINK_STATUS)
  void update_stats(const FnKey& k, const RxStats& rx, const TxStats& tx);
  IfState iface(const FnKey& k);
  std::vector<FnKey> functions();
  AgentCounters counters();
  int plugin_port() const;
  // Custom (plugin) message to the host on the F2H ring.
  void send_custom(const MsgHdr& h, const std::vector<uint8_t>& data);
  CtrlNet& ctrl() { return net_; }

 private:
  void load_interfaces();
  void loop();
  void handle_reset();
  void process_host(int budget);
  void flush_out();

  std::string path_;
  AgentConfig cfg_;
  uint32_t mbox_size_;
  int max_msgs_;
  Mailbox mbox_;
  CtrlNet net_;
  std::thread thr_;
  std::atomic<bool> running_{false};
  std::mutex out_mu_;
  std::deque<Msg> out_;           // F2H records waiting for ring space (responses, notifies, custom)
  std::mutex cnt_mu_;
  AgentCounters cnt_;
  uint64_t resets_seen_ = 0;
  std::unique_ptr<PluginServer> plugin_;
};

// Host-side client: what the host netdev driver does with the mailbox.
class HostCtrl {
 public:
  static constexpr size_t kMaxPendingNotes = 4096;
  explicit HostCtrl(const std::string& mbox_path, uint32_t host_version = kCpVersionMax);
  bool wait_ready(int timeout_ms);
  // Synchronous request for function (pem, pf, vf|-1); throws on timeout.
  Response request(uint32_t pem, uint32_t pf, int32_t vf, Request req, int timeout_ms = 1000);
  std::vector<Notify> take_notifications();
  std::vector<Msg> take_custom();
  bool send_custom(uint32_t pem, uint32_t pf, const std::vector<uint8_t>& data);
  // Failure detection: false once the fw heartbeat has not moved for hb_miss intervals.
  bool fw_alive();
  void host_heartbeat();
  // Host-requested reset (PERST): waits until the fw side acknowledged it.
  bool reset(int timeout_ms);
  void set_status(Status s);
  uint64_t fw_heartbeat() const;
  Mailbox& mbox() { return mbox_; }

 private:
  void drain(int timeout_ms, uint16_t want_id, Response* out, bool* got);
  Mailbox mbox_;
  uint32_t host_version_;
  uint16_t next_id_ = 1;
  std::mutex mu_;
  std::atomic<int> prio_{0};  // resets / drains waiting for mu_: requests back off
  std::vector<Notify> notes_;
  std::vector<Msg> custom_;
  uint64_t last_hb_ = 0;
  std::chrono::steady_clock::time_point last_hb_change_;
  uint64_t hb_interval_ms_ = 1000, hb_miss_ = 20;
};

}  // namespace agent
