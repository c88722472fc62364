// ctrl_net.cpp — fw-side control-net command handling (see ctrl_net.h).
#include "ctrl_net.h"

namespace agent {

uint32_t h2f_min_version(H2F c) {
  switch (c) {
    case H2F::Offloads: return version(1, 0, 1);
    default: return version(1, 0, 0);
  }
}

IfState& CtrlNet::iface(const FnKey& k) { return ifs_[k]; }

bool CtrlNet::has(const FnKey& k) const {
  std::lock_guard<std::mutex> g(mu_);
  return ifs_.count(k) != 0;
}

void CtrlNet::set_link(const FnKey& k, State s) {
  std::lock_guard<std::mutex> g(mu_);
  ifs_[k].link = s;
  bump();
}

void CtrlNet::set_stats(const FnKey& k, const RxStats& rx, const TxStats& tx) {
  std::lock_guard<std::mutex> g(mu_);
  IfState& s = ifs_[k];
  s.rx_stats = rx;
  s.tx_stats = tx;
}

std::map<FnKey, IfState> CtrlNet::snapshot() const {
  std::lock_guard<std::mutex> g(mu_);
  return ifs_;
}

Response CtrlNet::handle(const FnKey& k, const Request& req, uint64_t host_ver) {
  Response r;
  std::memset(&r, 0, sizeof(r));
  r.hdr.sender = req.hdr.receiver;
  r.hdr.receiver = req.hdr.sender;
  r.hdr.cmd = req.hdr.cmd;
  r.hdr.reply = (uint16_t)Reply::Ok;
  const H2F cmd = (H2F)req.hdr.cmd;
  if (req.hdr.cmd == 0 || req.hdr.cmd >= (uint16_t)H2F::Max) {
    r.hdr.reply = (uint16_t)Reply::InvalidParam;
    return r;
  }
  // A host that negotiated an older protocol must not get answers it cannot parse.
  if (host_ver < h2f_min_version(cmd)) {
    r.hdr.reply = (uint16_t)Reply::Unsupported;
    return r;
  }
  std::lock_guard<std::mutex> g(mu_);
  auto it = ifs_.find(k);
  if (it == ifs_.end() || it->second.removed) {
    r.hdr.reply = (uint16_t)Reply::InvalidParam;
    return r;
  }
  IfState& s = it->second;
  const bool set = req.op == (uint16_t)Cmd::Set;
  switch (cmd) {
    case H2F::Mtu:
      if (set) {
        if (req.val16 < min_mtu || req.val16 > max_mtu) { r.hdr.reply = (uint16_t)Reply::InvalidParam; break; }
        s.mtu = req.val16;
        bump();
      }
      r.val16 = s.mtu;
      break;
    case H2F::Mac:
      if (set) {
        if (req.mac[0] & 1) { r.hdr.reply = (uint16_t)Reply::InvalidParam; break; }  // multicast
        std::memcpy(s.mac, req.mac, 6);
        bump();
      }
      std::memcpy(r.mac, s.mac, 6);
      break;
    case H2F::GetIfStats:
    case H2F::GetXStats:
    case H2F::GetQStats:
      r.rx = s.rx_stats;
      r.tx = s.tx_stats;
      break;
    case H2F::LinkStatus:
      if (set) {
        if (req.val16 > 1) { r.hdr.reply = (uint16_t)Reply::InvalidParam; break; }
        s.link = (State)req.val16;
        bump();
      }
      r.val16 = (uint16_t)s.link;
      break;
    case H2F::RxState:
      if (set) {
        if (req.val16 > 1) { r.hdr.reply = (uint16_t)Reply::InvalidParam; break; }
        s.rx = (State)req.val16;
        bump();
      }
      r.val16 = (uint16_t)s.rx;
      break;
    case H2F::LinkInfo:
      if (set) {
        // only modes the interface supports may be advertised
        if (req.link.advertised_modes & ~s.link_info.supported_modes) { r.hdr.reply = (uint16_t)Reply::InvalidParam; break; }
        s.link_info.advertised_modes = req.link.advertised_modes;
        s.link_info.autoneg = req.link.autoneg;
        s.link_info.pause = req.link.pause;
        if (req.link.speed) s.link_info.speed = req.link.speed;
      }
      r.link = s.link_info;
      break;
    case H2F::GetInfo:
      r.info = fw_info;
      break;
    case H2F::DevRemove:
      s.removed = true;
      s.link = State::Down;
      s.rx = State::Down;
      bump();
      break;
    case H2F::Offloads:
      if (set) s.offloads = req.offloads;
      r.offloads = s.offloads;
      break;
    default:
      r.hdr.reply = (uint16_t)Reply::Unsupported;
  }
  return r;
}

}  // namespace agent
