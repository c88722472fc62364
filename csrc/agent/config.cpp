// config.cpp — libconfig-subset parser and the PEM/PF/VF tree (see config.h).
#include "config.h"

#include <cctype>
#include <cstdlib>
#include <stdexcept>

namespace agent {

const CfgValue* CfgValue::member(const std::string& name) const {
  for (const auto& m : members)
    if (m.first == name) return &m.second;
  return nullptr;
}

bool CfgValue::lookup_int(const std::string& name, int64_t& out) const {
  const CfgValue* v = member(name);
  if (!v) return false;
  if (v->kind == Kind::Int) { out = v->i; return true; }
  if (v->kind == Kind::Bool) { out = v->i; return true; }
  return false;
}

namespace {

class Parser {
 public:
  explicit Parser(const std::string& t) : t_(t) {}

  CfgValue file() {
    CfgValue root;
    root.kind = CfgValue::Kind::Group;
    skip();
    while (pos_ < t_.size()) {
      root.members.push_back(setting());
      skip();
    }
    return root;
  }

 private:
  [[noreturn]] void fail(const std::string& what) {
    int line = 1;
    for (size_t i = 0; i < pos_ && i < t_.size(); ++i) line += t_[i] == '\n';
    throw std::runtime_error("config line " + std::to_string(line) + ": " + what);
  }

  void skip() {
    for (;;) {
      while (pos_ < t_.size() && std::isspace((unsigned char)t_[pos_])) ++pos_;
      if (pos_ + 1 < t_.size() && t_[pos_] == '/' && t_[pos_ + 1] == '*') {
        const size_t e = t_.find("*/", pos_ + 2);
        if (e == std::string::npos) fail("unterminated comment");
        pos_ = e + 2;
      } else if ((pos_ + 1 < t_.size() && t_[pos_] == '/' && t_[pos_ + 1] == '/') ||
                 (pos_ < t_.size() && t_[pos_] == '#')) {
        while (pos_ < t_.size() && t_[pos_] != '\n') ++pos_;
      } else {
        return;
      }
    }
  }

  char peek() {
    skip();
    return pos_ < t_.size() ? t_[pos_] : '\0';
  }

  void expect(char c) {
    if (peek() != c) fail(std::string("expected '") + c + "'");
    ++pos_;
  }

  std::string name() {
    skip();
    const size_t b = pos_;
    if (pos_ >= t_.size() || !(std::isalpha((unsigned char)t_[pos_]) || t_[pos_] == '*')) fail("expected a setting name");
    while (pos_ < t_.size() && (std::isalnum((unsigned char)t_[pos_]) || t_[pos_] == '_' || t_[pos_] == '-' || t_[pos_] == '*'))
      ++pos_;
    return t_.substr(b, pos_ - b);
  }

  std::pair<std::string, CfgValue> setting() {
    std::string n = name();
    const char c = peek();
    if (c != '=' && c != ':') fail("expected '=' or ':' after " + n);
    ++pos_;
    CfgValue v = value();
    const char e = peek();
    if (e == ';' || e == ',') ++pos_;
    return {n, std::move(v)};
  }

  CfgValue value() {
    const char c = peek();
    CfgValue v;
    if (c == '{') {
      ++pos_;
      v.kind = CfgValue::Kind::Group;
      while (peek() != '}') {
        if (pos_ >= t_.size()) fail("unterminated group");
        v.members.push_back(setting());
      }
      ++pos_;
    } else if (c == '(' || c == '[') {
      const char close = c == '(' ? ')' : ']';
      ++pos_;
      v.kind = c == '(' ? CfgValue::Kind::List : CfgValue::Kind::Array;
      if (peek() != close) {
        for (;;) {
          v.items.push_back(value());
          if (peek() == ',') { ++pos_; if (peek() == close) break; continue; }
          break;
        }
      }
      expect(close);
    } else if (c == '"') {
      v.kind = CfgValue::Kind::String;
      while (peek() == '"') {
        ++pos_;
        while (pos_ < t_.size() && t_[pos_] != '"') {
          if (t_[pos_] == '\\' && pos_ + 1 < t_.size()) ++pos_;
          v.s.push_back(t_[pos_++]);
        }
        if (pos_ >= t_.size()) fail("unterminated string");
        ++pos_;
      }
    } else {
      scalar(v);
    }
    return v;
  }

  void scalar(CfgValue& v) {
    skip();
    const size_t b = pos_;
    while (pos_ < t_.size() && (std::isalnum((unsigned char)t_[pos_]) || t_[pos_] == '.' || t_[pos_] == '-' ||
                                t_[pos_] == '+'))
      ++pos_;
    std::string tok = t_.substr(b, pos_ - b);
    if (tok.empty()) fail("expected a value");
    std::string low;
    for (char ch : tok) low.push_back((char)std::tolower((unsigned char)ch));
    if (low == "true" || low == "false") {
      v.kind = CfgValue::Kind::Bool;
      v.i = low == "true";
      return;
    }
    while (!low.empty() && low.back() == 'l') low.pop_back();  // 64-bit suffix
    char* end = nullptr;
    const bool hex = low.size() > 2 && (low.compare(0, 2, "0x") == 0 || low.compare(0, 3, "-0x") == 0);
    if (hex || low.find_first_of(".e") == std::string::npos) {
      const long long x = std::strtoll(low.c_str(), &end, hex ? 16 : 10);
      if (!end || *end) fail("bad integer '" + tok + "'");
      v.kind = CfgValue::Kind::Int;
      v.i = x;
      return;
    }
    const double d = std::strtod(low.c_str(), &end);
    if (!end || *end) fail("bad number '" + tok + "'");
    v.kind = CfgValue::Kind::Float;
    v.f = d;
  }

  const std::string& t_;
  size_t pos_ = 0;
};

void fill_if(const CfgValue& g, IfCfg& c) {
  if (const CfgValue* m = g.member("mac_addr")) {
    for (size_t i = 0; i < m->items.size() && i < 6; ++i) c.mac[i] = (uint8_t)m->items[i].i;
  }
  g.lookup_int("link_state", c.link_state);
  g.lookup_int("rx_state", c.rx_state);
  g.lookup_int("autoneg", c.autoneg);
  g.lookup_int("pause_mode", c.pause_mode);
  g.lookup_int("speed", c.speed);
  g.lookup_int("supported_modes", c.supported_modes);
  g.lookup_int("advertised_modes", c.advertised_modes);
  g.lookup_int("dp_port", c.dp_port);
}

int req_idx(const CfgValue& g, const char* what) {
  int64_t idx;
  if (!g.lookup_int("idx", idx) || idx < 0) throw std::runtime_error(std::string(what) + " without a valid idx");
  return (int)idx;
}

}  // namespace

CfgValue parse_config(const std::string& text) { return Parser(text).file(); }

AgentConfig build_agent_config(const CfgValue& root) {
  AgentConfig out;
  const CfgValue* soc = root.member("soc");
  if (!soc) throw std::runtime_error("config: missing 'soc' group");
  const CfgValue* pems = soc->member("pems");
  if (!pems) throw std::runtime_error("config: missing soc.pems");
  bool hb_set = false;
  for (const CfgValue& pg : pems->items) {
    PemCfg pem;
    pem.idx = req_idx(pg, "pem");
    if (pem.idx > 15) throw std::runtime_error("config: pem idx > 15");
    if (const CfgValue* pfs = pg.member("pfs")) {
      for (const CfgValue& fg : pfs->items) {
        PfCfg pf;
        pf.idx = req_idx(fg, "pf");
        if (pf.idx > 511) throw std::runtime_error("config: pf idx > 511");
        fill_if(fg, pf.iface);
        int64_t v;
        if (fg.lookup_int("pkind", v)) pf.info.pkind = (uint32_t)v;
        pf.info.hb_interval_ms = fg.lookup_int("hb_interval", v) ? (uint64_t)v : 1000;
        pf.info.hb_miss_count = fg.lookup_int("hb_miss_count", v) ? (uint64_t)v : 20;
        if (!hb_set) {
          out.hb_interval_ms = pf.info.hb_interval_ms;
          out.hb_miss_count = pf.info.hb_miss_count;
          hb_set = true;
        }
        if (const CfgValue* vfs = fg.member("vfs")) {
          for (const CfgValue& vg : vfs->items) {
            VfCfg vf;
            vf.idx = req_idx(vg, "vf");
            fill_if(vg, vf.iface);
            pf.vfs.push_back(vf);
          }
        }
        pem.pfs.push_back(std::move(pf));
      }
    }
    out.pems.push_back(std::move(pem));
  }
  return out;
}

}  // namespace agent
