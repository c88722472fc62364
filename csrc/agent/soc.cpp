// soc.cpp — KFD-topology / PCI based accelerator detection (see soc.h).
#include "soc.h"

#include <dirent.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>

namespace agent {

namespace {

std::string join(const std::string& root, const std::string& p) {
  if (root.empty() || root == "/") return p;
  return (root.back() == '/' ? root.substr(0, root.size() - 1) : root) + p;
}

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

// KFD `properties` file: "name value" per line.
std::map<std::string, uint64_t> read_props(const std::string& path) {
  std::map<std::string, uint64_t> m;
  std::string text;
  if (!read_file(path, text)) return m;
  std::istringstream in(text);
  std::string k;
  while (in >> k) {
    std::string v;
    if (!(in >> v)) break;
    m[k] = std::strtoull(v.c_str(), nullptr, 0);
  }
  return m;
}

uint64_t get(const std::map<std::string, uint64_t>& m, const char* k, uint64_t dflt = 0) {
  auto it = m.find(k);
  return it == m.end() ? dflt : it->second;
}

std::vector<int> list_numeric_dirs(const std::string& dir) {
  std::vector<int> out;
  DIR* d = opendir(dir.c_str());
  if (!d) return out;
  while (dirent* e = readdir(d)) {
    const char* s = e->d_name;
    if (*s < '0' || *s > '9') continue;
    out.push_back(std::atoi(s));
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

std::string gfx_name(uint32_t v) {
  // gfx_target_version = major*10000 + minor*100 + stepping (stepping printed in hex)
  char buf[32];
  std::snprintf(buf, sizeof(buf), "gfx%u%u%x", v / 10000, (v / 100) % 100, v % 100);
  return buf;
}

}  // namespace

uint32_t model_from_device_id(uint32_t device_id, uint32_t gfx_target_version) {
  switch (device_id) {
    case 0x74a0: return kGpuMI300A;
    case 0x74a1: case 0x74b5: return kGpuMI300X;
    case 0x74a5: case 0x74b9: return kGpuMI325X;
    case 0x75a0: case 0x75b0: return kGpuMI350X;
    case 0x75a3: case 0x75b3: return kGpuMI355X;
    default: break;
  }
  if (gfx_target_version / 100 == 905) return kGpuMI355X;  // gfx950 part without a known id
  if (gfx_target_version / 100 == 904) return kGpuMI300X;
  return kGpuUnknown;
}

const char* model_name(uint32_t model) {
  switch (model) {
    case kGpuMI300X: return "MI300X";
    case kGpuMI300A: return "MI300A";
    case kGpuMI325X: return "MI325X";
    case kGpuMI350X: return "MI350X";
    case kGpuMI355X: return "MI355X";
    default: return "unknown";
  }
}

std::vector<GpuInfo> detect_gpus(const std::string& sys_root) {
  std::vector<GpuInfo> out;
  const std::string nodes = join(sys_root, "/sys/class/kfd/kfd/topology/nodes");
  for (int id : list_numeric_dirs(nodes)) {
    const std::string nd = nodes + "/" + std::to_string(id);
    const auto p = read_props(nd + "/properties");
    const uint32_t simd = (uint32_t)get(p, "simd_count");
    if (simd == 0) continue;  // CPU node
    GpuInfo g;
    g.node = id;
    g.gfx_target_version = (uint32_t)get(p, "gfx_target_version");
    g.gfx_arch = gfx_name(g.gfx_target_version);
    g.vendor_id = (uint32_t)get(p, "vendor_id");
    g.device_id = (uint32_t)get(p, "device_id");
    g.simd_count = simd;
    g.simd_per_cu = (uint32_t)get(p, "simd_per_cu", 4);
    g.cu_count = g.simd_per_cu ? simd / g.simd_per_cu : 0;
    g.num_xcc = (uint32_t)get(p, "num_xcc", 1);
    g.wave_front_size = (uint32_t)get(p, "wave_front_size", 64);
    g.lds_size_kb = (uint32_t)get(p, "lds_size_in_kb");
    g.numa_node = (int)(int64_t)get(p, "numa_node", (uint64_t)-1);
    g.unique_id_lo = (uint32_t)get(p, "unique_id");
    const uint64_t loc = get(p, "location_id");       // bus << 8 | dev << 3 | fn
    const uint64_t dom = get(p, "domain");
    char bdf[32];
    std::snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.%x", (unsigned)dom, (unsigned)((loc >> 8) & 0xFF),
                  (unsigned)((loc >> 3) & 0x1F), (unsigned)(loc & 7));
    g.pci = bdf;
    for (int b : list_numeric_dirs(nd + "/mem_banks")) {
      const auto mp = read_props(nd + "/mem_banks/" + std::to_string(b) + "/properties");
      const uint64_t heap = get(mp, "heap_type");
      if (heap == 1 || heap == 2) g.vram_bytes += get(mp, "size_in_bytes");  // private / public FB
    }
    g.model = model_from_device_id(g.device_id, g.gfx_target_version);
    g.model_name = model_name(g.model);
    // the PCI tree is authoritative for NUMA when KFD does not report it
    if (g.numa_node < 0) {
      std::string v;
      if (read_file(join(sys_root, "/sys/bus/pci/devices/" + g.pci + "/numa_node"), v)) g.numa_node = std::atoi(v.c_str());
    }
    out.push_back(g);
  }
  return out;
}

}  // namespace agent
