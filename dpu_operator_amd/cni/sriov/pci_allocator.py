"""File-per-PCI allocation locks (reference: dpu-cni/pkgs/sriovutils/pci_allocator.go:18-97).

``<dir>/pci/<addr>`` holds the netns path of the pod that owns the VF.  A lock whose netns no longer
exists is stale and is released automatically (a crashed pod must not leak its VF).
"""
from __future__ import annotations

import os


class PCIAllocator:
    def __init__(self, data_dir: str, netns_exists=None):
        self.dir = os.path.join(data_dir, "pci")
        self._netns_exists = netns_exists or os.path.exists

    def _p(self, pci: str) -> str:
        return os.path.join(self.dir, pci)

    def save_allocated_pci(self, pci: str, netns: str) -> None:
        os.makedirs(self.dir, exist_ok=True)
        with open(self._p(pci), "w") as f:
            f.write(netns)

    def delete_allocated_pci(self, pci: str) -> None:
        try:
            os.unlink(self._p(pci))
        except FileNotFoundError:
            pass

    def is_allocated(self, pci: str) -> bool:
        p = self._p(pci)
        if not os.path.exists(p):
            return False
        with open(p) as f:
            netns = f.read().strip()
        if not netns or not self._netns_exists(netns):
            self.delete_allocated_pci(pci)  # stale: the owning netns is gone
            return False
        return True
