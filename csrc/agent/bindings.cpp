// bindings.cpp — pybind11 module `_agent`: mailbox, control agent, host control client, config.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "agent.h"
#include "config.h"
#include "plugin_server.h"
#include "soc.h"

namespace py = pybind11;
using namespace agent;

namespace {

py::object cfg_to_py(const CfgValue& v) {
  switch (v.kind) {
    case CfgValue::Kind::Int: return py::int_(v.i);
    case CfgValue::Kind::Bool: return py::bool_(v.i != 0);
    case CfgValue::Kind::Float: return py::float_(v.f);
    case CfgValue::Kind::String: return py::str(v.s);
    case CfgValue::Kind::Array:
    case CfgValue::Kind::List: {
      py::list l;
      for (const auto& x : v.items) l.append(cfg_to_py(x));
      return std::move(l);
    }
    case CfgValue::Kind::Group: {
      py::dict d;
      for (const auto& m : v.members) d[py::str(m.first)] = cfg_to_py(m.second);
      return std::move(d);
    }
  }
  return py::none();
}

FnKey fk(uint32_t pem, uint32_t pf, int32_t vf) { return FnKey{pem, pf, vf}; }

py::dict link_dict(const LinkInfo& l) {
  py::dict d;
  d["supported_modes"] = l.supported_modes;
  d["advertised_modes"] = l.advertised_modes;
  d["autoneg"] = l.autoneg;
  d["pause"] = l.pause;
  d["speed"] = l.speed;
  return d;
}

py::bytes mac_bytes(const uint8_t* m) { return py::bytes(reinterpret_cast<const char*>(m), 6); }

py::dict iface_dict(const IfState& s) {
  py::dict d;
  d["mac"] = mac_bytes(s.mac);
  d["mtu"] = s.mtu;
  d["link"] = (int)s.link;
  d["rx"] = (int)s.rx;
  d["link_info"] = link_dict(s.link_info);
  d["rx_offloads"] = s.offloads.rx_offloads;
  d["tx_offloads"] = s.offloads.tx_offloads;
  d["dp_port"] = s.dp_port;
  d["removed"] = s.removed;
  d["rx_pkts"] = s.rx_stats.pkts;
  d["rx_bytes"] = s.rx_stats.octets;
  d["tx_pkts"] = s.tx_stats.pkts;
  d["tx_bytes"] = s.tx_stats.octets;
  return d;
}

py::dict resp_dict(const Response& r) {
  py::dict d;
  d["reply"] = r.hdr.reply;
  d["cmd"] = r.hdr.cmd;
  d["val"] = r.val16;
  d["mac"] = mac_bytes(r.mac);
  d["link_info"] = link_dict(r.link);
  d["rx_offloads"] = r.offloads.rx_offloads;
  d["tx_offloads"] = r.offloads.tx_offloads;
  d["ext_offloads"] = r.offloads.ext_offloads;
  py::dict info;
  info["pkind"] = r.info.pkind;
  info["hb_interval_ms"] = r.info.hb_interval_ms;
  info["hb_miss_count"] = r.info.hb_miss_count;
  d["info"] = info;
  py::dict rx, tx;
  rx["pkts"] = r.rx.pkts; rx["octets"] = r.rx.octets; rx["dropped"] = r.rx.dropped; rx["errors"] = r.rx.errors;
  tx["pkts"] = r.tx.pkts; tx["octets"] = r.tx.octets; tx["dropped"] = r.tx.dropped; tx["errors"] = r.tx.errors;
  d["rx"] = rx;
  d["tx"] = tx;
  return d;
}

Request make_req(uint16_t cmd, int op) {
  Request q;
  std::memset(&q, 0, sizeof(q));
  q.hdr.cmd = cmd;
  q.op = (uint16_t)(op < 0 ? 0 : op);
  return q;
}

py::tuple msg_tuple(const Msg& m) {
  return py::make_tuple(m.hdr.pem(), m.hdr.pf(), m.hdr.is_vf(), m.hdr.vf_idx, m.hdr.flags, m.hdr.msg_id,
                        py::bytes(reinterpret_cast<const char*>(m.data.data()), m.data.size()));
}

MsgHdr mkhdr(uint32_t pem, uint32_t pf, int32_t vf, uint32_t flags, uint16_t msg_id, size_t n) {
  MsgHdr h{};
  h.fn = MsgHdr::make_fn(pem, pf, vf >= 0);
  h.vf_idx = (uint16_t)(vf >= 0 ? vf : 0);
  h.flags = flags;
  h.msg_id = msg_id;
  h.sz = (uint32_t)n;
  return h;
}

}  // namespace

PYBIND11_MODULE(_agent, m) {
  m.def("detect_gpus", [](const std::string& root) {
    py::list out;
    for (const GpuInfo& g : detect_gpus(root)) {
      py::dict d;
      d["node"] = g.node; d["gfx_target_version"] = g.gfx_target_version; d["gfx_arch"] = g.gfx_arch;
      d["vendor_id"] = g.vendor_id; d["device_id"] = g.device_id; d["model"] = g.model_name;
      d["model_bit"] = g.model; d["simd_count"] = g.simd_count; d["cu_count"] = g.cu_count;
      d["num_xcc"] = g.num_xcc; d["simd_per_cu"] = g.simd_per_cu; d["wave_front_size"] = g.wave_front_size;
      d["lds_size_kb"] = g.lds_size_kb; d["vram_bytes"] = g.vram_bytes; d["numa_node"] = g.numa_node;
      d["pci"] = g.pci;
      out.append(d);
    }
    return out;
  }, py::arg("sys_root") = "/", "AMD Instinct GPUs from the KFD topology (soc.h)");
  m.attr("GPU_CDNA3") = (uint32_t)kGpuCdna3;
  m.attr("GPU_CDNA4") = (uint32_t)kGpuCdna4;

  m.doc() = "MI355X node control agent: shared-memory control mailbox, ctrl-net handler, plugin relay";
  m.attr("CP_VERSION_MIN") = kCpVersionMin;
  m.attr("CP_VERSION_MAX") = kCpVersionMax;
  m.attr("HEADER_BYTES") = kHeaderBytes;
  m.attr("REQUEST_BYTES") = (uint32_t)sizeof(Request);
  m.attr("RESPONSE_BYTES") = (uint32_t)sizeof(Response);
  m.attr("PLUGIN_DEFAULT_PORT") = PluginServer::kDefaultPort;
  m.def("version", &version);
  m.def("parse_config", [](const std::string& text) { return cfg_to_py(parse_config(text)); });
  m.def("config_summary", [](const std::string& text) {
    AgentConfig c = build_agent_config(parse_config(text));
    py::list pems;
    for (const auto& pem : c.pems) {
      py::list pfs;
      for (const auto& pf : pem.pfs) {
        py::list vfs;
        for (const auto& vf : pf.vfs) vfs.append(py::make_tuple(vf.idx, mac_bytes(vf.iface.mac)));
        py::dict d;
        d["idx"] = pf.idx;
        d["mac"] = mac_bytes(pf.iface.mac);
        d["speed"] = pf.iface.speed;
        d["hb_interval"] = pf.info.hb_interval_ms;
        d["hb_miss_count"] = pf.info.hb_miss_count;
        d["vfs"] = vfs;
        pfs.append(d);
      }
      pems.append(py::make_tuple(pem.idx, pfs));
    }
    return pems;
  });

  py::class_<Mailbox>(m, "Mailbox")
      .def_static("create", &Mailbox::create, py::arg("path"), py::arg("size"))
      .def_static("open", &Mailbox::open, py::arg("path"))
      .def_property_readonly("size", &Mailbox::size)
      .def_property_readonly("queue_bytes", &Mailbox::queue_bytes)
      .def("h2f_push", [](Mailbox& mb, uint32_t pem, uint32_t pf, int32_t vf, uint32_t flags, uint16_t id, py::bytes data) {
        std::string s = data;
        return mb.h2f().push(mkhdr(pem, pf, vf, flags, id, s.size()), s.data());
      }, py::arg("pem"), py::arg("pf"), py::arg("vf"), py::arg("flags"), py::arg("msg_id"), py::arg("data"))
      .def("f2h_push", [](Mailbox& mb, uint32_t pem, uint32_t pf, int32_t vf, uint32_t flags, uint16_t id, py::bytes data) {
        std::string s = data;
        return mb.f2h().push(mkhdr(pem, pf, vf, flags, id, s.size()), s.data());
      }, py::arg("pem"), py::arg("pf"), py::arg("vf"), py::arg("flags"), py::arg("msg_id"), py::arg("data"))
      .def("h2f_pop", [](Mailbox& mb) -> py::object {
        Msg msg;
        if (!mb.h2f().pop(msg)) return py::none();
        return msg_tuple(msg);
      })
      .def("f2h_pop", [](Mailbox& mb) -> py::object {
        Msg msg;
        if (!mb.f2h().pop(msg)) return py::none();
        return msg_tuple(msg);
      })
      .def("h2f_used", [](Mailbox& mb) { return mb.h2f().used(); })
      .def("h2f_space", [](Mailbox& mb) { return mb.h2f().space(); })
      .def("info", [](Mailbox& mb) {
        Info& in = mb.info();
        py::dict d;
        d["magic"] = in.magic.load();
        d["host_version"] = in.host_version.load();
        d["host_status"] = in.host_status.load();
        d["fw_status"] = in.fw_status.load();
        d["fw_heartbeat"] = in.fw_heartbeat.load();
        d["fw_version"] = in.fw_version.load();
        d["host_resets"] = in.host_resets.load();
        d["fw_resets"] = in.fw_resets.load();
        return d;
      });

  py::class_<Agent>(m, "Agent")
      .def(py::init([](const std::string& path, const std::string& cfg_text, uint32_t size, int max_msgs) {
             return new Agent(path, build_agent_config(parse_config(cfg_text)), size, max_msgs);
           }),
           py::arg("mbox_path"), py::arg("config"), py::arg("mbox_size") = 32768, py::arg("max_msgs") = 6)
      .def("start", &Agent::start, py::arg("plugin_port") = -1, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Agent::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &Agent::running)
      .def_property_readonly("plugin_port", &Agent::plugin_port)
      .def_property_readonly("state_gen", [](Agent& a) { return a.ctrl().state_gen(); })
      .def("set_link", [](Agent& a, uint32_t pem, uint32_t pf, int32_t vf, bool up) { a.set_link(fk(pem, pf, vf), up); },
           py::arg("pem"), py::arg("pf"), py::arg("vf"), py::arg("up"))
      .def("update_stats", [](Agent& a, uint32_t pem, uint32_t pf, int32_t vf, uint64_t rx_pkts, uint64_t rx_bytes,
                              uint64_t tx_pkts, uint64_t tx_bytes, uint64_t rx_dropped, uint64_t tx_dropped) {
             RxStats rx{};
             TxStats tx{};
             rx.pkts = rx_pkts; rx.octets = rx_bytes; rx.dropped = rx_dropped;
             tx.pkts = tx_pkts; tx.octets = tx_bytes; tx.dropped = tx_dropped;
             a.update_stats(fk(pem, pf, vf), rx, tx);
           },
           py::arg("pem"), py::arg("pf"), py::arg("vf"), py::arg("rx_pkts"), py::arg("rx_bytes"), py::arg("tx_pkts"),
           py::arg("tx_bytes"), py::arg("rx_dropped") = 0, py::arg("tx_dropped") = 0)
      .def("iface", [](Agent& a, uint32_t pem, uint32_t pf, int32_t vf) { return iface_dict(a.iface(fk(pem, pf, vf))); })
      .def("functions", [](Agent& a) {
        py::list l;
        for (auto& k : a.functions()) l.append(py::make_tuple(std::get<0>(k), std::get<1>(k), std::get<2>(k)));
        return l;
      })
      .def("counters", [](Agent& a) {
        AgentCounters c = a.counters();
        py::dict d;
        d["requests"] = c.requests; d["responses"] = c.responses; d["notifications"] = c.notifications;
        d["resp_deferred"] = c.resp_deferred; d["bad_msgs"] = c.bad_msgs; d["heartbeats"] = c.heartbeats;
        d["resets"] = c.resets; d["custom_in"] = c.custom_in; d["custom_out"] = c.custom_out;
        return d;
      });

  py::class_<HostCtrl>(m, "HostCtrl")
      .def(py::init<const std::string&, uint32_t>(), py::arg("mbox_path"), py::arg("host_version") = kCpVersionMax)
      .def("wait_ready", &HostCtrl::wait_ready, py::arg("timeout_ms") = 2000, py::call_guard<py::gil_scoped_release>())
      .def("request", [](HostCtrl& h, uint32_t pem, uint32_t pf, int32_t vf, uint16_t cmd, int op, int val,
                         py::object mac, py::object link, py::object offloads, int timeout_ms) {
             Request q = make_req(cmd, op);
             q.val16 = (uint16_t)(val < 0 ? 0 : val);
             if (!mac.is_none()) {
               std::string s = mac.cast<py::bytes>();
               if (s.size() != 6) throw std::invalid_argument("mac must be 6 bytes");
               std::memcpy(q.mac, s.data(), 6);
             }
             if (!link.is_none()) {
               py::dict l = link.cast<py::dict>();
               q.link.advertised_modes = l.contains("advertised_modes") ? l["advertised_modes"].cast<uint64_t>() : 0;
               q.link.autoneg = l.contains("autoneg") ? l["autoneg"].cast<uint8_t>() : 0;
               q.link.pause = l.contains("pause") ? l["pause"].cast<uint8_t>() : 0;
               q.link.speed = l.contains("speed") ? l["speed"].cast<uint32_t>() : 0;
             }
             if (!offloads.is_none()) {
               py::tuple t = offloads.cast<py::tuple>();
               q.offloads.rx_offloads = t[0].cast<uint16_t>();
               q.offloads.tx_offloads = t[1].cast<uint16_t>();
               q.offloads.ext_offloads = t.size() > 2 ? t[2].cast<uint64_t>() : 0;
             }
             Response r;
             {
               py::gil_scoped_release rel;
               r = h.request(pem, pf, vf, q, timeout_ms);
             }
             return resp_dict(r);
           },
           py::arg("pem"), py::arg("pf"), py::arg("vf"), py::arg("cmd"), py::arg("op") = 0, py::arg("val") = 0,
           py::arg("mac") = py::none(), py::arg("link") = py::none(), py::arg("offloads") = py::none(),
           py::arg("timeout_ms") = 1000)
      .def("notifications", [](HostCtrl& h) {
        py::list l;
        for (const Notify& n : h.take_notifications()) l.append(py::make_tuple(n.hdr.cmd, n.state));
        return l;
      })
      .def("custom", [](HostCtrl& h) {
        py::list l;
        for (const Msg& msg : h.take_custom()) l.append(msg_tuple(msg));
        return l;
      })
      .def("send_custom", [](HostCtrl& h, uint32_t pem, uint32_t pf, py::bytes data) {
        std::string s = data;
        return h.send_custom(pem, pf, std::vector<uint8_t>(s.begin(), s.end()));
      })
      .def("fw_alive", &HostCtrl::fw_alive)
      .def("fw_heartbeat", &HostCtrl::fw_heartbeat)
      .def("host_heartbeat", &HostCtrl::host_heartbeat)
      .def("reset", &HostCtrl::reset, py::arg("timeout_ms") = 2000, py::call_guard<py::gil_scoped_release>())
      .def("set_status", [](HostCtrl& h, int s) { h.set_status((Status)s); });
}
