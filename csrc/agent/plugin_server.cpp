// plugin_server.cpp — poll()-based TCP relay (see plugin_server.h).
#include "plugin_server.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <stdexcept>

namespace agent {

PluginServer::PluginServer(int port, ToHost to_host) : port_(port), to_host_(std::move(to_host)) {}

PluginServer::~PluginServer() { stop(); }

void PluginServer::start() {
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (lfd_ < 0) throw std::runtime_error("plugin server: socket() failed");
  int one = 1;
  ::setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port_);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  if (::bind(lfd_, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(lfd_, kMaxClients) != 0) {
    ::close(lfd_);
    lfd_ = -1;
    throw std::runtime_error("plugin server: cannot listen on port " + std::to_string(port_));
  }
  socklen_t len = sizeof(a);
  ::getsockname(lfd_, (sockaddr*)&a, &len);
  port_ = ntohs(a.sin_port);
  if (::pipe2(wake_, O_CLOEXEC | O_NONBLOCK) != 0) throw std::runtime_error("plugin server: pipe failed");
  running_.store(true);
  thr_ = std::thread([this] { run(); });
}

void PluginServer::stop() {
  if (!running_.exchange(false)) return;
  send_all(kEvent, std::vector<uint8_t>{(uint8_t)kEvFwStop, 0, 0, 0});
  const char c = 'x';
  (void)!::write(wake_[1], &c, 1);
  if (thr_.joinable()) thr_.join();
  std::lock_guard<std::mutex> g(mu_);
  for (int fd : fds_) ::close(fd);
  fds_.clear();
  nclients_.store(0);
  if (lfd_ >= 0) ::close(lfd_);
  lfd_ = -1;
  for (int& w : wake_) {
    if (w >= 0) ::close(w);
    w = -1;
  }
}

bool PluginServer::write_frame(int fd, uint16_t type, uint32_t seq, const uint8_t* p, uint32_t n) {
  FrameHdr h{kMagic, type, 0, n, seq};
  std::vector<uint8_t> buf(sizeof(h) + n);
  std::memcpy(buf.data(), &h, sizeof(h));
  if (n) std::memcpy(buf.data() + sizeof(h), p, n);
  size_t off = 0;
  while (off < buf.size()) {
    const ssize_t w = ::send(fd, buf.data() + off, buf.size() - off, MSG_NOSIGNAL);
    if (w <= 0) return false;
    off += (size_t)w;
  }
  return true;
}

void PluginServer::send_all(uint16_t type, const std::vector<uint8_t>& payload) {
  std::lock_guard<std::mutex> g(mu_);
  const uint32_t seq = ++seq_;
  for (int fd : fds_) write_frame(fd, type, seq, payload.data(), (uint32_t)payload.size());
}

void PluginServer::broadcast_msg(const Msg& m) {
  std::vector<uint8_t> p(sizeof(MsgHdr) + m.data.size());
  std::memcpy(p.data(), &m.hdr, sizeof(MsgHdr));
  if (!m.data.empty()) std::memcpy(p.data() + sizeof(MsgHdr), m.data.data(), m.data.size());
  send_all(kHostMsg, p);
}

void PluginServer::broadcast_event(Event ev, const std::vector<uint8_t>& extra) {
  std::vector<uint8_t> p(4 + extra.size());
  const uint32_t e = ev;
  std::memcpy(p.data(), &e, 4);
  if (!extra.empty()) std::memcpy(p.data() + 4, extra.data(), extra.size());
  send_all(kEvent, p);
}

void PluginServer::handle_frame(int fd, const FrameHdr& h, const std::vector<uint8_t>& body) {
  if (h.type == kHello) {
    const uint32_t v = kCpVersionMax;
    std::lock_guard<std::mutex> g(mu_);
    write_frame(fd, kHelloAck, h.seq, reinterpret_cast<const uint8_t*>(&v), 4);
  } else if (h.type == kSendMsg && body.size() >= sizeof(MsgHdr)) {
    MsgHdr mh;
    std::memcpy(&mh, body.data(), sizeof(MsgHdr));
    std::vector<uint8_t> data(body.begin() + sizeof(MsgHdr), body.end());
    if (to_host_) to_host_(mh, data);
  }
}

void PluginServer::run() {
  struct Conn {
    std::vector<uint8_t> buf;
  };
  std::map<int, Conn> conns;
  while (running_.load()) {
    std::vector<pollfd> pfds;
    pfds.push_back({lfd_, POLLIN, 0});
    pfds.push_back({wake_[0], POLLIN, 0});
    for (auto& kv : conns) pfds.push_back({kv.first, POLLIN, 0});
    const int r = ::poll(pfds.data(), pfds.size(), 200);
    if (r <= 0) continue;
    if (pfds[1].revents) break;
    if (pfds[0].revents & POLLIN) {
      const int c = ::accept4(lfd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (c >= 0) {
        if ((int)conns.size() >= kMaxClients) {
          ::close(c);  // the reference caps plugin clients at two
        } else {
          int one = 1;
          ::setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          conns[c] = Conn{};
          std::lock_guard<std::mutex> g(mu_);
          fds_.push_back(c);
          nclients_.store((int)fds_.size());
        }
      }
    }
    for (size_t i = 2; i < pfds.size(); ++i) {
      if (!pfds[i].revents) continue;
      const int fd = pfds[i].fd;
      uint8_t tmp[4096];
      const ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
      bool drop = n <= 0;
      if (!drop) {
        Conn& c = conns[fd];
        c.buf.insert(c.buf.end(), tmp, tmp + n);
        while (c.buf.size() >= sizeof(FrameHdr)) {
          FrameHdr h;
          std::memcpy(&h, c.buf.data(), sizeof(h));
          if (h.magic != kMagic || h.len > (1u << 20)) { drop = true; break; }
          if (c.buf.size() < sizeof(h) + h.len) break;
          std::vector<uint8_t> body(c.buf.begin() + sizeof(h), c.buf.begin() + sizeof(h) + h.len);
          c.buf.erase(c.buf.begin(), c.buf.begin() + sizeof(h) + h.len);
          if (h.type == kBye) { drop = true; break; }
          handle_frame(fd, h, body);
        }
      }
      if (drop) {
        conns.erase(fd);
        std::lock_guard<std::mutex> g(mu_);
        fds_.erase(std::remove(fds_.begin(), fds_.end(), fd), fds_.end());
        nclients_.store((int)fds_.size());
        ::close(fd);
      }
    }
  }
}

}  // namespace agent
