// config.h — agent configuration: a parser for the libconfig subset the reference's SoC
// configuration files use (octep_cp_agent/*.cfg, app_config.c, SURVEY NAT3) and the typed
// PEM/PF/VF tree built from it.
//
// Grammar accepted: `name = value;` or `name : value;` settings; groups `{ ... }`; lists
// `( v, v )`; arrays `[ s, s ]`; integers (decimal, 0x hex, optional L suffix), floats,
// true/false, "strings" (adjacent literals concatenate); comments `/* */`, `//`, `#`.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "ctrl_net.h"

namespace agent {

struct CfgValue {
  enum class Kind { Int, Float, Bool, String, Array, List, Group } kind = Kind::Group;
  int64_t i = 0;
  double f = 0.0;
  std::string s;
  std::vector<CfgValue> items;                            // Array / List
  std::vector<std::pair<std::string, CfgValue>> members;  // Group

  const CfgValue* member(const std::string& name) const;
  bool lookup_int(const std::string& name, int64_t& out) const;
};

CfgValue parse_config(const std::string& text);  // throws std::runtime_error with line info

struct IfCfg {
  uint8_t mac[6]{};
  int64_t link_state = 0, rx_state = 0, autoneg = 0, pause_mode = 0, speed = 0;
  int64_t supported_modes = 0, advertised_modes = 0;
  int64_t dp_port = -1;  // MI355X addition: data-plane port backing this function
};
struct VfCfg {
  int idx = 0;
  IfCfg iface;
};
struct PfCfg {
  int idx = 0;
  IfCfg iface;
  FwInfo info{};
  std::vector<VfCfg> vfs;
};
struct PemCfg {
  int idx = 0;
  std::vector<PfCfg> pfs;
};
struct AgentConfig {
  std::vector<PemCfg> pems;
  uint64_t hb_interval_ms = 1000;
  uint64_t hb_miss_count = 20;
};

// soc = { pems = ( { idx; pfs = ( { idx; mac_addr; ...; hb_interval; hb_miss_count; vfs = (...) } ) } ) }
AgentConfig build_agent_config(const CfgValue& root);

}  // namespace agent
