"""Hardware platform view: PCI devices, NICs, product string, PCIe device serial numbers.

Reference: internal/platform/platform.go:13-129 (`Platform` interface over ghw, serial number =
8 bytes of PCI config space at offset 0x150, `FakePlatform` for tests).  `SysfsPlatform` reads
/sys/bus/pci/devices directly (vendor / device / class / physfn / net), under a relocatable root.
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field

PCI_CLASS_NAMES = {0x02: "Network controller", 0x03: "Display controller", 0x12: "Processing accelerators",
                   0x0B: "Processor"}
VENDOR_NAMES = {"8086": "Intel Corporation", "177d": "Cavium, Inc.", "1002": "Advanced Micro Devices, Inc. [AMD/ATI]"}


@dataclass
class PciDevice:
    address: str
    vendor_id: str
    device_id: str
    class_code: int = 0x020000
    product_name: str = ""
    vendor_name: str = ""
    is_vf: bool = False
    numa_node: int = -1
    serial: str = ""
    netdevs: list[str] = field(default_factory=list)

    @property
    def class_name(self) -> str:
        return PCI_CLASS_NAMES.get(self.class_code >> 16, "Unknown")


@dataclass
class Nic:
    name: str
    mac: str
    pci_address: str = ""
    is_virtual: bool = False


class Platform:
    def pci_devices(self) -> list[PciDevice]: ...
    def net_devs(self) -> list[Nic]: ...
    def product(self) -> str: ...
    def read_device_serial_number(self, dev: PciDevice) -> str: ...


class SysfsPlatform(Platform):
    def __init__(self, root: str = "/"):
        self.root = root

    def _p(self, *parts: str) -> str:
        path = os.path.join(*parts)
        return os.path.join(self.root, path.lstrip("/")) if self.root not in ("", "/") else path

    def _read(self, *parts: str, default: str = "") -> str:
        try:
            with open(self._p(*parts)) as f:
                return f.read().strip()
        except OSError:
            return default

    def pci_devices(self) -> list[PciDevice]:
        base = self._p("/sys/bus/pci/devices")
        out = []
        if not os.path.isdir(base):
            return out
        for addr in sorted(os.listdir(base)):
            d = os.path.join(base, addr)
            vid = self._read(d, "vendor")[2:].lower()
            did = self._read(d, "device")[2:].lower()
            cls = int(self._read(d, "class", default="0x0") or "0x0", 16)
            nets = sorted(os.listdir(os.path.join(d, "net"))) if os.path.isdir(os.path.join(d, "net")) else []
            try:
                numa = int(self._read(d, "numa_node", default="-1"))
            except ValueError:
                numa = -1
            out.append(PciDevice(addr, vid, did, cls, self._read(d, "label"), VENDOR_NAMES.get(vid, ""),
                                 os.path.islink(os.path.join(d, "physfn")), numa, "", nets))
        return out

    def net_devs(self) -> list[Nic]:
        base = self._p("/sys/class/net")
        out = []
        if not os.path.isdir(base):
            return out
        for n in sorted(os.listdir(base)):
            dev = os.path.join(base, n, "device")
            pci = os.path.basename(os.readlink(dev)) if os.path.islink(dev) else ""
            out.append(Nic(n, self._read(base, n, "address"), pci, not pci))
        return out

    def product(self) -> str:
        return self._read("/sys/class/dmi/id/product_name")

    def read_device_serial_number(self, dev: PciDevice) -> str:
        path = self._p("/sys/bus/pci/devices", dev.address, "config")
        with open(path, "rb") as f:
            f.seek(0x150)
            buf = f.read(8)
        if len(buf) != 8:
            raise OSError(f"short read of device serial number from {path}")
        return buf.hex()


class FakePlatform(Platform):
    """In-memory platform (reference: platform.go:79-129)."""

    def __init__(self, product: str = "", devices: list[PciDevice] | None = None, nics: list[Nic] | None = None):
        self._lock = threading.Lock()
        self._product = product
        self._devices = list(devices or [])
        self._nics = list(nics or [])

    def set_product(self, p: str) -> None:
        with self._lock:
            self._product = p

    def add_pci(self, dev: PciDevice) -> None:
        with self._lock:
            self._devices.append(dev)

    def remove_all(self) -> None:
        with self._lock:
            self._devices.clear()
            self._nics.clear()

    def pci_devices(self):
        with self._lock:
            return list(self._devices)

    def net_devs(self):
        with self._lock:
            return list(self._nics)

    def product(self):
        with self._lock:
            return self._product

    def read_device_serial_number(self, dev):
        return dev.serial or dev.address.replace(":", "").replace(".", "")
