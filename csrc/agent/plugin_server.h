// plugin_server.h — TCP relay between the control agent and external plugin applications.
//
// Reference: octep_plugin_server.c (SURVEY NAT9): a TCP server (default port 49500, at most two
// clients) on its own thread with a select loop, relaying host custom messages and events to
// plugins and plugin messages back to the host.  Framing here: 16-byte header
//   { u32 magic 'DPUP', u16 type, u16 rsvd, u32 len, u32 seq } + len payload bytes.
// Types: HELLO (client->server, answered with HELLO_ACK carrying the protocol version),
// SEND_MSG (client->server: payload = MsgHdr + data for the host, delivered with the CUSTOM flag),
// HOST_MSG (server->clients: a host custom message), EVENT (server->clients: u32 event id).
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "mbox.h"

namespace agent {

class PluginServer {
 public:
  static constexpr uint32_t kMagic = 0x50555044;  // "DPUP"
  static constexpr int kMaxClients = 2;
  static constexpr int kDefaultPort = 49500;
  enum Type : uint16_t { kHello = 1, kHelloAck = 2, kSendMsg = 3, kHostMsg = 4, kEvent = 5, kBye = 6 };
  enum Event : uint32_t { kEvPerst = 1, kEvLinkUp = 2, kEvLinkDown = 3, kEvFwStop = 4 };

  struct FrameHdr {
    uint32_t magic;
    uint16_t type;
    uint16_t rsvd;
    uint32_t len;
    uint32_t seq;
  };

  using ToHost = std::function<void(const MsgHdr&, const std::vector<uint8_t>&)>;

  PluginServer(int port, ToHost to_host);
  ~PluginServer();
  void start();
  void stop();
  int port() const { return port_; }
  int clients() const { return nclients_.load(); }
  void broadcast_msg(const Msg& m);
  void broadcast_event(Event ev, const std::vector<uint8_t>& extra);

 private:
  void run();
  void send_all(uint16_t type, const std::vector<uint8_t>& payload);
  static bool write_frame(int fd, uint16_t type, uint32_t seq, const uint8_t* p, uint32_t n);
  void handle_frame(int fd, const FrameHdr& h, const std::vector<uint8_t>& body);

  int port_;
  ToHost to_host_;
  int lfd_ = -1;
  int wake_[2] = {-1, -1};
  std::thread thr_;
  std::atomic<bool> running_{false};
  std::atomic<int> nclients_{0};
  std::mutex mu_;
  std::vector<int> fds_;
  uint32_t seq_ = 0;
};

}  // namespace agent
