"""GPU detection from the KFD topology (native soc.cpp), device-handler utils and the device
plugin's NUMA topology hints."""
from __future__ import annotations

import os

import pytest

from dpu_operator_amd.daemon import devutils


def _kfd_node(root, nid, props, banks=()):
    d = os.path.join(root, "sys/class/kfd/kfd/topology/nodes", str(nid))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "properties"), "w") as f:
        for k, v in props.items():
            f.write(f"{k} {v}\n")
    for b, (heap, size) in enumerate(banks):
        bd = os.path.join(d, "mem_banks", str(b))
        os.makedirs(bd, exist_ok=True)
        with open(os.path.join(bd, "properties"), "w") as f:
            f.write(f"heap_type {heap}\nsize_in_bytes {size}\n")


@pytest.fixture
def sysfs(tmp_path):
    root = str(tmp_path)
    _kfd_node(root, 0, {"cpu_cores_count": 96, "simd_count": 0})
    for n in (1, 2):
        _kfd_node(root, n, {"simd_count": 1024, "simd_per_cu": 4, "gfx_target_version": 90500, "vendor_id": 4098,
                            "device_id": 0x75a3, "num_xcc": 8, "wave_front_size": 64, "lds_size_in_kb": 160,
                            "location_id": ((0x05 + n) << 8) | 0, "domain": 0, "numa_node": n - 1},
                  banks=[(1, 288 << 30)])
    pci = os.path.join(root, "sys/bus/pci/devices/0000:06:00.0")
    os.makedirs(pci)
    with open(os.path.join(pci, "numa_node"), "w") as f:
        f.write("0\n")
    os.makedirs(os.path.join(root, "sys/bus/pci/drivers/amdgpu"))
    os.symlink(os.path.join(root, "sys/bus/pci/drivers/amdgpu"), os.path.join(pci, "driver"))
    return root


def test_detect_gpus_from_kfd_topology(sysfs):
    gpus = devutils.gpu_topology(sysfs)
    assert len(gpus) == 2
    g = gpus[0]
    assert g["model"] == "MI355X" and g["gfx_arch"] == "gfx950"
    assert g["cu_count"] == 256 and g["num_xcc"] == 8 and g["lds_size_kb"] == 160
    assert g["vram_bytes"] == 288 << 30 and g["pci"] == "0000:06:00.0" and g["numa_node"] == 0
    assert gpus[1]["numa_node"] == 1 and devutils.data_plane_numa(sysfs, 1) == 1


def test_driver_and_numa_helpers(sysfs):
    assert devutils.get_driver_name("0000:06:00.0", sysfs) == "amdgpu"
    assert devutils.get_numa_node("0000:06:00.0", sysfs) == 0
    assert devutils.get_numa_node("0000:99:00.0", sysfs) == -1
    with pytest.raises(FileNotFoundError):
        devutils.get_driver_name("0000:99:00.0", sysfs)


def test_device_plugin_advertises_numa():
    from dpu_operator_amd.daemon.deviceplugin import DeviceHandler, DevicePluginServer

    h = DeviceHandler(vsp=None, dpu_mode=True, numa_of=lambda d: 1 if d.startswith("dpuvp") else -1)
    srv = DevicePluginServer(h)
    d1 = srv._device("dpuvp0", "Healthy")
    d2 = srv._device("other", "Healthy")
    assert [n.ID for n in d1.topology.nodes] == [1]
    assert not d2.HasField("topology")


def test_agent_binary_lists_gpus(sysfs):
    import json
    import subprocess

    from dpu_operator_amd.native.build import build_exe

    out = subprocess.run([str(build_exe("dpu-cp-agent")), "--list-gpus", sysfs], capture_output=True, text=True,
                         timeout=30, check=True).stdout.splitlines()
    gpus = [json.loads(x) for x in out]
    assert [g["model"] for g in gpus] == ["MI355X", "MI355X"] and gpus[0]["cus"] == 256 and gpus[1]["pci"] == "0000:07:00.0"
