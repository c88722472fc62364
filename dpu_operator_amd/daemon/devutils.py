"""Device-handler types and sysfs helpers (DH2).

Reference: internal/daemon/device-handler/types.go:7-12 (DeviceList) and utils.go:16-38
(GetDriverName via the `driver` symlink, GetNumaNode via `numa_node`).  Added for the MI355X
node: `gpu_topology()` reads the KFD topology through the native agent (csrc/agent/soc.cpp) so
the device plugin can advertise the NUMA node of the GPU that backs the data-plane vports, and
the data plane can size its grid from the CU / XCC counts.
"""
from __future__ import annotations

import os

# device id -> (id, health) as served to kubelet
DeviceList = dict[str, tuple[str, str]]


def _dev(sys_root: str, pci: str, *parts: str) -> str:
    return os.path.join(sys_root, "sys/bus/pci/devices", pci, *parts)


def get_driver_name(pci: str, sys_root: str = "/") -> str:
    try:
        return os.path.basename(os.readlink(_dev(sys_root, pci, "driver")))
    except OSError as e:
        raise FileNotFoundError(f"no driver bound to {pci}") from e


def get_numa_node(pci: str, sys_root: str = "/") -> int:
    """NUMA node of a PCI function; -1 when the platform does not report one."""
    try:
        with open(_dev(sys_root, pci, "numa_node")) as f:
            return int(f.read().strip())
    except (OSError, ValueError):
        return -1


def gpu_topology(sys_root: str = "/") -> list[dict]:
    """AMD Instinct GPUs (KFD topology): model, gfx arch, CUs, XCCs, LDS, VRAM, NUMA, PCI."""
    from ..native import agent

    return list(agent().detect_gpus(sys_root))


def data_plane_numa(sys_root: str = "/", gpu_index: int = 0) -> int:
    gpus = gpu_topology(sys_root)
    return gpus[gpu_index]["numa_node"] if gpu_index < len(gpus) else -1
