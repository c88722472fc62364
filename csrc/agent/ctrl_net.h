// ctrl_net.h — control-net message schema carried by the mailbox, and the fw-side handler.
//
// Same command set and version gating as the reference's ctrl-net protocol (octep_ctrl_net.h,
// SURVEY NAT10): H2F MTU, MAC, GET_IF_STATS, GET_XSTATS, GET_Q_STATS, LINK_STATUS, RX_STATE,
// LINK_INFO, GET_INFO, DEV_REMOVE (all v1.0.0) and OFFLOADS (v1.0.1); F2H LINK_STATUS notify.
// Requests and responses are fixed-size POD records so both sides can be plain C++ (or Python
// struct) without a serializer.  Interface statistics come from the GPU data plane's per-port
// counters (PortStats is filled by the control plane from DataPlane.port_counters()).
#pragma once
#include <atomic>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>

#include "mbox.h"

namespace agent {

enum class Cmd : uint16_t { Get = 0, Set = 1 };
enum class State : uint16_t { Down = 0, Up = 1 };
enum class Reply : uint16_t { Ok = 0, GenericFail = 1, InvalidParam = 2, Unsupported = 3 };

enum class H2F : uint16_t {
  Invalid = 0, Mtu, Mac, GetIfStats, GetXStats, GetQStats, LinkStatus, RxState, LinkInfo, GetInfo,
  DevRemove, Offloads, Max
};
enum class F2H : uint16_t { Invalid = 0, LinkStatus, Max };

// Minimum control-plane version that understands each host->fw command.
uint32_t h2f_min_version(H2F c);

struct ReqHdr {
  uint16_t sender;
  uint16_t receiver;
  uint16_t cmd;      // H2F / F2H
  uint16_t rsvd;
};

struct RespHdr {
  uint16_t sender;
  uint16_t receiver;
  uint16_t cmd;
  uint16_t reply;    // Reply
};

struct LinkInfo {
  uint64_t supported_modes;
  uint64_t advertised_modes;
  uint8_t autoneg;
  uint8_t pause;
  uint8_t rsvd[2];
  uint32_t speed;    // Mb/s
};

struct Offloads {
  uint16_t rx_offloads;
  uint16_t tx_offloads;
  uint32_t rsvd;
  uint64_t ext_offloads;
};

struct FwInfo {
  uint32_t pkind;
  uint32_t fsz;
  uint64_t hb_interval_ms;
  uint64_t hb_miss_count;
  uint64_t rsvd[2];
};

struct RxStats {
  uint64_t pkts, octets, mcast_pkts, bcast_pkts, dropped, errors, fcs_errors, rsvd;
};
struct TxStats {
  uint64_t pkts, octets, mcast_pkts, bcast_pkts, dropped, errors, collisions, rsvd;
};

// One request record (header + union of bodies) — fixed 48 bytes.
struct Request {
  ReqHdr hdr;
  uint16_t op;       // Cmd (get/set) for commands that have one
  uint16_t val16;    // MTU / state
  uint8_t mac[6];
  uint8_t pad[2];
  LinkInfo link;     // LINK_INFO set
  Offloads offloads; // OFFLOADS set  (placed after link to keep natural alignment)
};

// One response record — fixed size, large enough for the IF_STATS body.
struct Response {
  RespHdr hdr;
  uint16_t val16;
  uint8_t mac[6];
  LinkInfo link;
  Offloads offloads;
  FwInfo info;
  RxStats rx;
  TxStats tx;
};

struct Notify {
  ReqHdr hdr;        // cmd = F2H
  uint16_t state;
  uint16_t rsvd[3];
};

// Per-function (PF or VF) interface state owned by the fw side.
struct IfState {
  uint8_t mac[6]{};
  uint16_t mtu = 1500;
  State link = State::Down;
  State rx = State::Down;
  LinkInfo link_info{};
  Offloads offloads{};
  RxStats rx_stats{};
  TxStats tx_stats{};
  int32_t dp_port = -1;  // data-plane port whose counters back this interface
  bool removed = false;
};

using FnKey = std::tuple<uint32_t, uint32_t, int32_t>;  // (pem, pf, vf or -1)

// The fw-side command handler: a thread-safe table of interface state.
class CtrlNet {
 public:
  uint16_t max_mtu = 9216;
  uint16_t min_mtu = 68;
  FwInfo fw_info{};

  IfState& iface(const FnKey& k);
  bool has(const FnKey& k) const;
  // Handle one H2F request for function `k` under host version `host_ver` -> response.
  Response handle(const FnKey& k, const Request& req, uint64_t host_ver);
  void set_link(const FnKey& k, State s);
  void set_stats(const FnKey& k, const RxStats& rx, const TxStats& tx);
  std::map<FnKey, IfState> snapshot() const;
  std::mutex& mutex() const { return mu_; }
  // Bumped by every change of an interface's MTU, MAC, link, RX state or removal: the data-plane
  // side polls it and re-applies the interface table to the GPU port flags when it moved.
  uint64_t state_gen() const { return gen_.load(std::memory_order_acquire); }
  void bump() { gen_.fetch_add(1, std::memory_order_acq_rel); }

 private:
  std::atomic<uint64_t> gen_{0};
  mutable std::mutex mu_;
  std::map<FnKey, IfState> ifs_;
};

inline FnKey key_of(const MsgHdr& h) {
  return FnKey{h.pem(), h.pf(), h.is_vf() ? (int32_t)h.vf_idx : -1};
}

}  // namespace agent
