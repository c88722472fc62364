"""SR-IOV sysfs helpers + NetConf cache (reference: dpu-cni/pkgs/sriovutils/sriovutils.go:15-420).

All paths are relative to a `root` so tests build a fake /sys tree with real files and symlinks.
"""
from __future__ import annotations

import json
import os
import re
import time

SYS_BUS_PCI = "/sys/bus/pci/devices"
USERSPACE_DRIVERS = ("vfio-pci", "uio_pci_generic", "igb_uio")
PCI_RE = re.compile(r"^[0-9a-fA-F]{4}:[0-9a-fA-F]{2}:[0-9a-fA-F]{2}\.[0-7]$")
DEFAULT_CNI_DIR = "/var/lib/cni/dpusriov"


class Sysfs:
    def __init__(self, root: str = "/"):
        self.root = root

    def p(self, *parts: str) -> str:
        path = os.path.join(*parts)
        return os.path.join(self.root, path.lstrip("/")) if self.root not in ("", "/") else path

    def dev(self, pci: str, *rest: str) -> str:
        return self.p(SYS_BUS_PCI, pci, *rest)

    # -------------------------------------------------------------- VF / PF topology
    def get_sriov_numvfs(self, ifname: str) -> int:
        with open(self.p("/sys/class/net", ifname, "device/sriov_numvfs")) as f:
            return int(f.read().strip() or 0)

    def set_sriov_numvfs(self, pci: str, n: int) -> None:
        """write 0 then N (the kernel rejects changing a non-zero count directly)."""
        path = self.dev(pci, "sriov_numvfs")
        with open(path, "w") as f:
            f.write("0")
        if n:
            with open(path, "w") as f:
                f.write(str(n))

    def get_total_vfs(self, pci: str) -> int:
        with open(self.dev(pci, "sriov_totalvfs")) as f:
            return int(f.read().strip() or 0)

    def get_pf_pci(self, vf_pci: str) -> str:
        return os.path.basename(os.readlink(self.dev(vf_pci, "physfn")))

    def get_pf_name(self, vf_pci: str) -> str:
        pf = self.get_pf_pci(vf_pci)
        names = os.listdir(self.dev(pf, "net"))
        if not names:
            raise FileNotFoundError(f"no netdev for PF {pf}")
        return names[0]

    def get_vfid(self, vf_pci: str) -> int:
        pf = self.get_pf_pci(vf_pci)
        for entry in os.listdir(self.dev(pf)):
            if entry.startswith("virtfn"):
                if os.path.basename(os.readlink(self.dev(pf, entry))) == vf_pci:
                    return int(entry[len("virtfn"):])
        raise FileNotFoundError(f"VF {vf_pci} not found under PF {pf}")

    def vf_pci_addresses(self, pf_pci: str) -> list[str]:
        out = []
        for entry in os.listdir(self.dev(pf_pci)):
            if entry.startswith("virtfn"):
                out.append((int(entry[6:]), os.path.basename(os.readlink(self.dev(pf_pci, entry)))))
        return [p for _, p in sorted(out)]

    def get_vf_link_name(self, pci: str) -> str:
        d = self.dev(pci, "net")
        if not os.path.isdir(d):
            return ""
        names = sorted(os.listdir(d))
        return names[0] if names else ""

    def driver_name(self, pci: str) -> str:
        link = self.dev(pci, "driver")
        return os.path.basename(os.readlink(link)) if os.path.islink(link) else ""

    def has_dpdk_driver(self, pci: str) -> bool:
        return self.driver_name(pci) in USERSPACE_DRIVERS

    def numa_node(self, pci: str) -> int:
        try:
            with open(self.dev(pci, "numa_node")) as f:
                return int(f.read().strip())
        except (OSError, ValueError):
            return -1


def is_valid_pci_address(addr: str) -> bool:
    return bool(PCI_RE.match(addr or ""))


def retry(n: int, delay: float, fn):
    last = None
    for _ in range(n):
        try:
            return fn()
        except Exception as e:  # noqa: BLE001
            last = e
            time.sleep(delay)
    raise last  # type: ignore[misc]


# ------------------------------------------------------------------ NetConf cache
def cache_path(cache_dir: str, container_id: str, ifname: str) -> str:
    return os.path.join(cache_dir, f"{container_id}-{ifname}")


def save_net_conf(container_id: str, cache_dir: str, ifname: str, conf: dict) -> None:
    os.makedirs(cache_dir, exist_ok=True)
    p = cache_path(cache_dir, container_id, ifname)
    with open(p + ".tmp", "w") as f:
        json.dump(conf, f)
    os.replace(p + ".tmp", p)


def read_scratch_net_conf(path: str) -> dict:
    with open(path) as f:
        return json.load(f)


def clean_cached_net_conf(path: str) -> None:
    try:
        os.unlink(path)
    except FileNotFoundError:
        pass
