"""Offload-engine detection: which VSP to run and whether this node is the device side.

Reference: internal/platform/vendordetector.go:15-135 (DpuDetectorManager: for each detector, if
the node IS the offload device -> VSP in dpu mode; else scan PCI and the first matching device ->
VSP in host mode with its identifier), ipu.go:46-92, marvell-dpu.go:12-77,
netsec-accelerator.go:12-91.

Added detector: MI355X (AMD Instinct, vendor 1002, CDNA4 gfx950 device ids) — the GPU data
plane.  A GPU node is both sides at once: the node daemon runs the device-side manager (OPI
bridge-port server, NF CNI, SFC reconciler) and the host-side manager (workload VFs/vports) in one
process, and the VSP drives the node's GPUs.
"""
from __future__ import annotations

import json
from dataclasses import dataclass

from .. import images as I
from .platform import PciDevice, Platform

INTEL = "8086"
MARVELL = "177d"
AMD = "1002"
# Instinct MI350/MI355X (CDNA4, gfx950) PCI device ids (PF + VF)
MI355X_DEVICE_IDS = {"75a0", "75a3", "75b0", "75b3"}


@dataclass
class VspSpec:
    """How to run a VSP: image key + command/args for the VSP DaemonSet (vsp-ds bindata)."""
    vendor: str
    image_key: str
    command: list[str]
    args: list[str]
    dpu_mode: bool
    identifier: str = ""
    colocated: bool = False   # device side and host side on one node (GPU data plane)

    def template_vars(self, image_manager) -> dict:
        try:
            image = image_manager.get_image(self.image_key)
        except I.ImageNotFound:
            image = ""
        return {"VendorSpecificPluginImage": image, "Command": json.dumps(self.command),
                "Args": json.dumps(self.args)}


class VendorDetector:
    name = "base"
    vendor = ""

    def is_dpu_platform(self, platform: Platform) -> bool:
        return False

    def is_dpu(self, platform: Platform, pci: PciDevice, found: list[str]) -> bool:
        return False

    def get_dpu_identifier(self, platform: Platform, pci: PciDevice) -> str:
        return pci.address

    def vsp(self, dpu_mode: bool, identifier: str = "") -> VspSpec:
        raise NotImplementedError


class IntelIpuDetector(VendorDetector):
    name, vendor = "Intel IPU", "intel"

    def is_dpu_platform(self, platform):
        return "IPU Adapter E2100-CCQDA2" in (platform.product() or "")

    def is_dpu(self, platform, pci, found):
        return (not pci.is_vf and pci.class_name == "Network controller" and pci.vendor_id == INTEL
                and (pci.product_name == "Infrastructure Data Path Function" or pci.device_id == "1452"))

    def vsp(self, dpu_mode, identifier=""):
        mode = "ipu" if dpu_mode else "host"
        return VspSpec(self.vendor, I.VSP_IMAGE_INTEL, ["/ipuplugin"],
                       ["--bridgeType=ovs", f"--interface=enp0s1f0d3", f"--mode={mode}",
                        "--p4rtName=vsp-p4-service.openshift-dpu-operator.svc.cluster.local"], dpu_mode, identifier)


class MarvellDetector(VendorDetector):
    name, vendor = "Marvell DPU", "marvell"

    def is_dpu_platform(self, platform):
        return any(p.vendor_id == MARVELL and p.device_id == "a0f7" for p in platform.pci_devices())

    def is_dpu(self, platform, pci, found):
        return pci.vendor_id == MARVELL and pci.device_id == "b900"

    def vsp(self, dpu_mode, identifier=""):
        return VspSpec(self.vendor, I.VSP_IMAGE_MARVELL, ["/vsp-mrvl"], [], dpu_mode, identifier)


class NetsecAcceleratorDetector(VendorDetector):
    name, vendor = "Intel Netsec Accelerator", "intel-netsec"

    def is_dpu_platform(self, platform):
        return any(p.vendor_id == INTEL and p.device_id == "124c" for p in platform.pci_devices())

    def is_dpu(self, platform, pci, found):
        if not (pci.vendor_id == INTEL and pci.device_id == "1599"):
            return False
        # dual-port card: both ports share a serial number; count the card once
        return self.get_dpu_identifier(platform, pci) not in found

    def get_dpu_identifier(self, platform, pci):
        return platform.read_device_serial_number(pci)

    def vsp(self, dpu_mode, identifier=""):
        return VspSpec(self.vendor, I.VSP_IMAGE_INTEL_NETSEC, ["/vsp-intel-netsec"], [], dpu_mode, identifier)


class Mi355xDetector(VendorDetector):
    name, vendor = "AMD Instinct MI355X", "amd-gpu"

    def gpus(self, platform) -> list[PciDevice]:
        return [p for p in platform.pci_devices()
                if p.vendor_id == AMD and p.device_id in MI355X_DEVICE_IDS and not p.is_vf]

    def is_dpu_platform(self, platform):
        return bool(self.gpus(platform))

    # The VSP runs the live data path: pods' vports (veth pairs by default, node config
    # vport_kind) through the native I/O engine into the resident ring kernel of every MI355X of
    # the node (flows sharded by RSS owner).  The reference's detector likewise deploys its VSP
    # with the arguments its data plane needs (internal/platform/ipu.go:76-92).
    VSP_ARGS = ["--vendor", "amd-gpu", "--live", "--live-engine", "native", "--gpus", "all"]

    def vsp(self, dpu_mode, identifier=""):
        # the wire port (node config `uplink`: a host-side veth pair by default, or the node's data
        # NIC), as the reference's VSPs take their RPM / SFP port (marvell/main.go:104-154,
        # intel-netsec/main.go:183-199)
        from ..config import node_config

        return VspSpec(self.vendor, I.VSP_IMAGE_AMD_GPU, ["python3", "-m", "dpu_operator_amd.cmd.vsp"],
                       list(self.VSP_ARGS) + ["--uplink", node_config().uplink], True, identifier, colocated=True)


class DpuDetectorManager:
    def __init__(self, platform: Platform, detectors: list[VendorDetector] | None = None):
        self.platform = platform
        self.detectors = detectors if detectors is not None else [
            IntelIpuDetector(), MarvellDetector(), NetsecAcceleratorDetector(), Mi355xDetector()]

    def detect_dpu_platform(self, required: bool = False) -> VendorDetector | None:
        active = [d for d in self.detectors if d.is_dpu_platform(self.platform)]
        if len(active) > 1:
            raise RuntimeError(f"Failed to detect DPU platform unambiguously: {[d.name for d in active]}")
        if not active:
            if required:
                raise RuntimeError("Failed to detect any DPU platform")
            return None
        return active[0]

    def is_dpu(self) -> bool:
        return self.detect_dpu_platform() is not None

    def detect(self) -> VspSpec | None:
        """-> the VSP to run (dpu_mode says which side this node is), or None."""
        for det in self.detectors:
            if det.is_dpu_platform(self.platform):
                return det.vsp(True, "")
            found: list[str] = []
            for pci in self.platform.pci_devices():
                if det.is_dpu(self.platform, pci, found):
                    ident = det.get_dpu_identifier(self.platform, pci)
                    return det.vsp(False, ident)
        return None
