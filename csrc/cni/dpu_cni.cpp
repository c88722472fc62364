// dpu_cni.cpp — the `dpu-cni` CNI plugin as a self-contained native binary.
//
// Kubelet / Multus exec the plugin ON THE HOST (outside any container), so it must not depend on
// a Python runtime or this package being installed there: the daemon copies this static binary
// to the host CNI bin dir (daemon.prepare, reference internal/daemon/daemon.go:195-209).  Same
// wire protocol as the reference shim (dpu-cni/pkgs/cni/cnishim.go:20-139) and as
// dpu_operator_amd/cni/shim.py:
//   * snapshot the CNI_* environment + stdin config into {"env": {...}, "config": base64(stdin)}
//   * POST it as HTTP/1.1 to /cni over the daemon's unix socket (0600, root-only dir)
//   * ADD: print the daemon's Result with cniVersion set to the config's; DEL: ignore the result;
//     CHECK: no-op; VERSION: supported versions.  Failures print a CNI error object
//     {"cniVersion", "code", "msg"} and exit 1 (11 = cannot reach the daemon, 6 = bad config,
//     4 = unknown command, 999 = daemon error).
// Socket: $DPU_CNI_SOCKET, else /var/run/dpu-daemon/dpu-cni/dpu-cni-server.sock.
#include <sys/socket.h>
#include <sys/time.h>
#include <sys/un.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <iterator>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

extern char** environ;

namespace {

constexpr const char* kDefaultSocket = "/var/run/dpu-daemon/dpu-cni/dpu-cni-server.sock";
constexpr const char* kSupported = R"(["0.3.0","0.3.1","0.4.0","1.0.0"])";

struct CniError : std::runtime_error {
  int code;
  CniError(const std::string& m, int c) : std::runtime_error(m), code(c) {}
};

// ------------------------------------------------------------------------ minimal JSON DOM
struct Json {
  enum Type { Null, Bool, Num, Str, Arr, Obj } t = Null;
  bool b = false;
  std::string s;  // string value, or the raw number text
  std::vector<Json> a;
  std::vector<std::pair<std::string, Json>> o;

  Json* get(const std::string& k) {
    for (auto& kv : o)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  void set(const std::string& k, Json v) {
    if (Json* p = get(k)) *p = std::move(v);
    else o.emplace_back(k, std::move(v));
  }
  static Json str(std::string v) { Json j; j.t = Str; j.s = std::move(v); return j; }
};

class Parser {
 public:
  explicit Parser(const std::string& in) : s_(in) {}
  Json parse() {
    Json v = value();
    ws();
    if (i_ != s_.size()) fail("trailing data");
    return v;
  }

 private:
  [[noreturn]] void fail(const char* what) { throw std::invalid_argument(std::string(what) + " at offset " + std::to_string(i_)); }
  void ws() { while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\t' || s_[i_] == '\n' || s_[i_] == '\r')) ++i_; }
  bool lit(const char* w) {
    const size_t n = std::strlen(w);
    if (s_.compare(i_, n, w) == 0) { i_ += n; return true; }
    return false;
  }
  static void put_utf8(std::string& out, uint32_t cp) {
    if (cp < 0x80) out += (char)cp;
    else if (cp < 0x800) { out += (char)(0xC0 | (cp >> 6)); out += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12)); out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18)); out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F)); out += (char)(0x80 | (cp & 0x3F));
    }
  }
  uint32_t hex4() {
    if (i_ + 4 > s_.size()) fail("short \\u escape");
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = s_[i_++];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("bad \\u escape");
    }
    return v;
  }
  std::string string() {
    if (s_[i_] != '"') fail("expected string");
    ++i_;
    std::string out;
    while (true) {
      if (i_ >= s_.size()) fail("unterminated string");
      const char c = s_[i_++];
      if (c == '"') break;
      if ((unsigned char)c < 0x20) fail("control character in string");
      if (c != '\\') { out += c; continue; }
      if (i_ >= s_.size()) fail("bad escape");
      const char e = s_[i_++];
      switch (e) {
        case '"': out += '"'; break;
        case '\\': out += '\\'; break;
        case '/': out += '/'; break;
        case 'b': out += '\b'; break;
        case 'f': out += '\f'; break;
        case 'n': out += '\n'; break;
        case 'r': out += '\r'; break;
        case 't': out += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && s_.compare(i_, 2, "\\u") == 0) {
            i_ += 2;
            const uint32_t lo = hex4();
            if (lo < 0xDC00 || lo >= 0xE000) fail("bad surrogate pair");
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    return out;
  }
  Json value() {
    ws();
    if (i_ >= s_.size()) fail("unexpected end");
    Json v;
    const char c = s_[i_];
    if (c == '{') {
      v.t = Json::Obj;
      ++i_;
      ws();
      if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
      while (true) {
        ws();
        std::string k = string();
        ws();
        if (i_ >= s_.size() || s_[i_] != ':') fail("expected ':'");
        ++i_;
        v.o.emplace_back(std::move(k), value());
        ws();
        if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
        if (i_ < s_.size() && s_[i_] == '}') { ++i_; return v; }
        fail("expected ',' or '}'");
      }
    }
    if (c == '[') {
      v.t = Json::Arr;
      ++i_;
      ws();
      if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
      while (true) {
        v.a.push_back(value());
        ws();
        if (i_ < s_.size() && s_[i_] == ',') { ++i_; continue; }
        if (i_ < s_.size() && s_[i_] == ']') { ++i_; return v; }
        fail("expected ',' or ']'");
      }
    }
    if (c == '"') { v.t = Json::Str; v.s = string(); return v; }
    if (lit("true")) { v.t = Json::Bool; v.b = true; return v; }
    if (lit("false")) { v.t = Json::Bool; v.b = false; return v; }
    if (lit("null")) return v;
    const size_t st = i_;
    if (s_[i_] == '-') ++i_;
    while (i_ < s_.size() && (std::isdigit((unsigned char)s_[i_]) || s_[i_] == '.' || s_[i_] == 'e' || s_[i_] == 'E' ||
                              s_[i_] == '+' || s_[i_] == '-'))
      ++i_;
    if (i_ == st || (i_ == st + 1 && s_[st] == '-')) fail("unexpected character");
    v.t = Json::Num;
    v.s = s_.substr(st, i_ - st);
    return v;
  }
  const std::string& s_;
  size_t i_ = 0;
};

void quote(std::string& out, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) { out += "\\u00"; out += hex[c >> 4]; out += hex[c & 15]; }
        else out += (char)c;
    }
  }
  out += '"';
}

void dump(std::string& out, const Json& v) {
  switch (v.t) {
    case Json::Null: out += "null"; break;
    case Json::Bool: out += v.b ? "true" : "false"; break;
    case Json::Num: out += v.s; break;
    case Json::Str: quote(out, v.s); break;
    case Json::Arr:
      out += '[';
      for (size_t k = 0; k < v.a.size(); ++k) { if (k) out += ','; dump(out, v.a[k]); }
      out += ']';
      break;
    case Json::Obj:
      out += '{';
      for (size_t k = 0; k < v.o.size(); ++k) {
        if (k) out += ',';
        quote(out, v.o[k].first);
        out += ':';
        dump(out, v.o[k].second);
      }
      out += '}';
      break;
  }
}

std::string base64(const std::string& in) {
  static const char* tbl = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string out;
  out.reserve((in.size() + 2) / 3 * 4);
  size_t i = 0;
  for (; i + 2 < in.size(); i += 3) {
    const uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8) | (uint8_t)in[i + 2];
    out += tbl[v >> 18]; out += tbl[(v >> 12) & 63]; out += tbl[(v >> 6) & 63]; out += tbl[v & 63];
  }
  if (i + 1 == in.size()) {
    const uint32_t v = (uint8_t)in[i] << 16;
    out += tbl[v >> 18]; out += tbl[(v >> 12) & 63]; out += "==";
  } else if (i + 2 == in.size()) {
    const uint32_t v = ((uint8_t)in[i] << 16) | ((uint8_t)in[i + 1] << 8);
    out += tbl[v >> 18]; out += tbl[(v >> 12) & 63]; out += tbl[(v >> 6) & 63]; out += '=';
  }
  return out;
}

// ------------------------------------------------------------------------ HTTP over unix socket
std::pair<int, std::string> post_unix(const std::string& path, const std::string& body, int timeout_s) {
  const int fd = ::socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) throw CniError(std::string("failed to send CNI request: socket: ") + std::strerror(errno), 11);
  struct FdGuard { int fd; ~FdGuard() { ::close(fd); } } guard{fd};
  timeval tv{timeout_s, 0};
  ::setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
  ::setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
  sockaddr_un addr{};
  addr.sun_family = AF_UNIX;
  if (path.size() >= sizeof(addr.sun_path)) throw CniError("failed to send CNI request: socket path too long", 11);
  std::memcpy(addr.sun_path, path.c_str(), path.size() + 1);
  if (::connect(fd, reinterpret_cast<sockaddr*>(&addr), sizeof addr) != 0)
    throw CniError("failed to send CNI request: connect " + path + ": " + std::strerror(errno), 11);
  std::string req = "POST /cni HTTP/1.1\r\nHost: dummy\r\nContent-Type: application/json\r\nContent-Length: " +
                    std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body;
  for (size_t off = 0; off < req.size();) {
    const ssize_t n = ::send(fd, req.data() + off, req.size() - off, MSG_NOSIGNAL);
    if (n <= 0) throw CniError(std::string("failed to send CNI request: send: ") + std::strerror(errno), 11);
    off += (size_t)n;
  }
  std::string resp;
  char buf[65536];
  while (true) {
    const ssize_t n = ::recv(fd, buf, sizeof buf, 0);
    if (n < 0) throw CniError(std::string("failed to send CNI request: recv: ") + std::strerror(errno), 11);
    if (n == 0) break;
    resp.append(buf, (size_t)n);
  }
  const size_t hdr_end = resp.find("\r\n\r\n");
  if (hdr_end == std::string::npos || resp.compare(0, 5, "HTTP/") != 0)
    throw CniError("failed to send CNI request: malformed HTTP response", 11);
  const std::string head = resp.substr(0, hdr_end);
  std::string payload = resp.substr(hdr_end + 4);
  const size_t sp = head.find(' ');
  const int status = sp == std::string::npos ? 0 : std::atoi(head.c_str() + sp + 1);
  // honour Content-Length (case-insensitive header name)
  size_t ls = head.find("\r\n");
  while (ls != std::string::npos) {
    const size_t le = head.find("\r\n", ls + 2);
    std::string line = head.substr(ls + 2, (le == std::string::npos ? head.size() : le) - ls - 2);
    const size_t colon = line.find(':');
    if (colon != std::string::npos) {
      std::string k = line.substr(0, colon);
      for (char& ch : k) ch = (char)std::tolower((unsigned char)ch);
      if (k == "content-length") {
        const size_t n = (size_t)std::strtoull(line.c_str() + colon + 1, nullptr, 10);
        if (n < payload.size()) payload.resize(n);
      }
    }
    ls = le;
  }
  return {status, payload};
}

std::string trim(std::string s) {
  while (!s.empty() && std::isspace((unsigned char)s.back())) s.pop_back();
  size_t i = 0;
  while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  return s.substr(i);
}

Json post_request(const std::string& sock, const std::string& stdin_data) {
  Json env;
  env.t = Json::Obj;
  for (char** e = environ; e && *e; ++e) {
    const char* eq = std::strchr(*e, '=');
    if (!eq || std::strncmp(*e, "CNI_", 4) != 0) continue;
    env.set(std::string(*e, (size_t)(eq - *e)), Json::str(eq + 1));
  }
  Json req;
  req.t = Json::Obj;
  req.set("env", env);
  req.set("config", Json::str(base64(stdin_data)));
  std::string body;
  dump(body, req);
  auto [status, payload] = post_unix(sock, body, 120);
  if (status != 200)
    throw CniError("CNI request failed with status " + std::to_string(status) + ": '" + trim(payload) + "'", 999);
  if (trim(payload).empty()) return Json{};
  Json resp;
  try {
    resp = Parser(payload).parse();
  } catch (const std::exception& ex) {
    throw CniError(std::string("failed to parse CNI server response: ") + ex.what(), 999);
  }
  Json* r = resp.t == Json::Obj ? resp.get("Result") : nullptr;
  return r ? *r : Json{};
}

void print_error(const CniError& e) {
  std::string out = "{\"cniVersion\":\"1.0.0\",\"code\":" + std::to_string(e.code) + ",\"msg\":";
  quote(out, e.what());
  out += "}";
  std::cout << out << std::flush;
}

}  // namespace

int main() {
  const char* cmd_c = std::getenv("CNI_COMMAND");
  const std::string cmd = cmd_c ? cmd_c : "";
  const char* sock_c = std::getenv("DPU_CNI_SOCKET");
  const std::string sock = sock_c && *sock_c ? sock_c : kDefaultSocket;
  try {
    if (cmd == "VERSION") {
      std::cout << "{\"cniVersion\":\"1.0.0\",\"supportedVersions\":" << kSupported << "}" << std::flush;
      return 0;
    }
    const std::string data((std::istreambuf_iterator<char>(std::cin)), std::istreambuf_iterator<char>());
    if (cmd == "ADD") {
      Json conf;
      try {
        conf = Parser(data).parse();
      } catch (const std::exception& ex) {
        throw CniError(std::string("failed to parse network config: ") + ex.what(), 6);
      }
      if (conf.t != Json::Obj) throw CniError("network config must be a JSON object", 6);
      Json result = post_request(sock, data);
      if (result.t != Json::Obj || result.o.empty()) throw CniError("CNI server returned no result for ADD", 999);
      const Json* cv = conf.get("cniVersion");
      std::string ver = cv && cv->t == Json::Str && !cv->s.empty() ? cv->s : "";
      if (ver.empty()) {
        const Json* rv = result.get("cniVersion");
        ver = rv && rv->t == Json::Str ? rv->s : "1.0.0";
      }
      result.set("cniVersion", Json::str(ver));
      std::string out;
      dump(out, result);
      std::cout << out << std::flush;
      return 0;
    }
    if (cmd == "DEL") {
      (void)post_request(sock, data);  // result ignored (cnishim.go CmdDel)
      return 0;
    }
    if (cmd == "CHECK") return 0;
    throw CniError("unknown CNI_COMMAND: " + cmd, 4);
  } catch (const CniError& e) {
    print_error(e);
    return 1;
  }
}
