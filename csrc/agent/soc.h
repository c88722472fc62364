// soc.h — accelerator detection for the node agent.
//
// Role of the reference's SoC detection (octep_cp_lib soc/soc.c:116-378: MIDR + RVU sysfs ->
// CN9K/CN10K model bitmask) for the node that hosts THIS data plane: the agent identifies the
// AMD Instinct GPUs from the KFD topology (/sys/class/kfd/kfd/topology/nodes/N/properties) and
// the PCI device tree, and derives what the data plane is sized from: CU count (grid size),
// XCC count (XCD-aware block remaps), SIMDs, LDS per workgroup, HBM size, NUMA node and the PCI
// address (the device-plugin topology hint and the ctrl-net function's backing device).
// `sys_root` prefixes every path (tests pass a fake sysfs tree).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace agent {

enum GpuModel : uint32_t {
  kGpuUnknown = 0,
  kGpuMI300X = 1u << 0,
  kGpuMI300A = 1u << 1,
  kGpuMI325X = 1u << 2,
  kGpuMI350X = 1u << 3,
  kGpuMI355X = 1u << 4,
  kGpuCdna3 = kGpuMI300X | kGpuMI300A | kGpuMI325X,
  kGpuCdna4 = kGpuMI350X | kGpuMI355X,
};

struct GpuInfo {
  int node = -1;                 // KFD topology node id
  uint32_t gfx_target_version = 0;  // e.g. 90500 = gfx950
  std::string gfx_arch;          // "gfx950"
  uint32_t vendor_id = 0, device_id = 0;
  uint32_t model = kGpuUnknown;  // GpuModel bit
  std::string model_name;
  uint32_t simd_count = 0, cu_count = 0, num_xcc = 1, simd_per_cu = 4, wave_front_size = 64;
  uint32_t lds_size_kb = 0;
  uint64_t vram_bytes = 0;
  int numa_node = -1;
  std::string pci;               // domain:bus:dev.fn
  uint32_t unique_id_lo = 0;
};

// All GPU agents (nodes with simd_count > 0) under sys_root, ordered by node id.
std::vector<GpuInfo> detect_gpus(const std::string& sys_root = "/");
// Model bit for a PCI device id (0x74a1 MI300X, 0x74a5 MI325X, 0x75a0 MI350X, 0x75a3 MI355X, ...)
uint32_t model_from_device_id(uint32_t device_id, uint32_t gfx_target_version);
const char* model_name(uint32_t model);

}  // namespace agent
