"""Intel NetSec Accelerator VSP, with the OvS bridge compiled onto the MI355X data plane.

Reference: internal/daemon/vendor-specific-plugins/intel-netsec/main.go:30-640.
Behaviour kept:
* comm channel: IPv6 link-local on the backplane PF 0000:f4:00.2 (DPU side, fe80::1) or on the
  card's function-0 PF found by serial number (host side, fe80::2); gRPC address `[fe80::1%if]`
  (`%25` escaped on the host), port 8085;
* DPU side: two NF veth pairs, bridge `br-secondary` with the second SFP port (0000:f4:00.1);
* SetNumVfs: sriov_numvfs 0 then N on the backplane (DPU) or the card PF (host), then per VF:
  VLAN = vf + 2 (isolation: every VF's traffic is forced through the accelerator), spoof-check
  off, trust on; host PF in VEPA hwmode; VF table keyed by (PF netdev, VF id);
* CreateBridgePort(host0-<vf>): the VF's netdev joins the bridge (pf != 0 unsupported);
* GetDevices: host -> VF PCI addresses on the card's bus (device 1889); DPU -> NF veth names.
MI355X additions: VF ports are programmed on the GPU with the K10 semantics (VLAN isolate + egress
tag with vf+2, trust); CreateNetworkFunction is implemented (the reference leaves it a TODO) with
the same steering as the Marvell VSP.
"""
from __future__ import annotations

import logging
import re
import threading

from ..cni.netlink import NetlinkManager
from ..dataplane import tables as T
from ..dataplane.ovs import OvsSwitch
from ..platform.platform import Platform
from ..utils.cmdrunner import Runner
from . import common
from .base import VspBase

log = logging.getLogger("dpu.vsp.netsec")

INTEL = "8086"
HOST_VF_DEVICE_ID = "1889"
HOST_DEVICE_ID = "1599"
DPU_SFP0 = "0000:f4:00.0"
DPU_SFP1 = "0000:f4:00.1"
DPU_BACKPLANE_F2 = "0000:f4:00.2"
DPU_BACKPLANE_F3 = "0000:f4:00.3"
VLAN_OFFSET = 2
NO_OF_VETH_PAIRS = 2
BRIDGE = "br-secondary"
DEFAULT_PORT = 8085
IPV6_DPU = "fe80::1"
IPV6_HOST = "fe80::2"


def _bus(addr: str) -> str:
    return addr.split(":")[1] if addr.count(":") >= 2 else ""


def _function(addr: str) -> str:
    return addr.rsplit(".", 1)[-1]


class NetsecVsp(VspBase):
    name = "intel-netsec-vsp"

    def __init__(self, platform: Platform, nl: NetlinkManager, runner: Runner, dataplane=None, path_manager=None,
                 sys_root: str = "/", uplink_port: int = 4000):
        super().__init__(path_manager)
        self.platform = platform
        self.nl = nl
        self.runner = runner
        self.root = sys_root
        self.dp = dataplane
        self.sw = OvsSwitch(dataplane) if dataplane is not None else None
        self.uplink_port = uplink_port
        self.dpu_mode = False
        self.identifier = ""
        self.dpu_pcie = ""
        self.vf_cnt = 0
        self.veths: list[common.VethPair] = []
        self.vf_devs: dict[tuple[str, int], common.VfDevice] = {}
        self.bridge_vfs: dict[str, str] = {}     # bridge port name -> VF netdev
        self._next_port = 0
        self._ports: dict[str, int] = {}
        self.nf: tuple[str, str] | None = None
        self._mu = threading.RLock()

    # -------------------------------------------------------------- helpers
    def _netdev(self, pci: str) -> str:
        for d in self.platform.pci_devices():
            if d.address == pci and d.netdevs:
                return d.netdevs[0]
        return common.netdev_from_pci(pci, self.root)

    def _dpu_pcie_address(self) -> str:
        if self.dpu_mode:
            return ""
        for d in self.platform.pci_devices():
            if d.vendor_id == INTEL and d.device_id == HOST_DEVICE_ID:
                if self.platform.read_device_serial_number(d) == self.identifier and _function(d.address) == "0":
                    return d.address
        raise LookupError(f"DPU PCIe address not found for identifier: {self.identifier}")

    def _vfs_on_card(self) -> list[str]:
        bus = _bus(self.dpu_pcie)
        return [d.address for d in self.platform.pci_devices()
                if _bus(d.address) == bus and d.vendor_id == INTEL and d.device_id == HOST_VF_DEVICE_ID]

    def _port(self, name: str) -> int:
        if name not in self._ports:
            self._ports[name] = self._next_port
            self._next_port += 1
        return self._ports[name]

    # -------------------------------------------------------------- hooks
    def init(self, dpu_mode, dpu_identifier):
        with self._mu:
            self.dpu_mode = dpu_mode
            self.identifier = dpu_identifier
            self.dpu_pcie = self._dpu_pcie_address()
            ifname = self._netdev(DPU_BACKPLANE_F2 if dpu_mode else self.dpu_pcie)
            common.enable_ipv6_link_local(self.runner, ifname, IPV6_DPU if dpu_mode else IPV6_HOST, self.root)
            ip = f"[{IPV6_DPU}%{ifname}]" if dpu_mode else f"[{IPV6_DPU}%25{ifname}]"
            if dpu_mode:
                self.veths = [common.create_nf_veth_pair(self.nl, i) for i in range(NO_OF_VETH_PAIRS)]
                if self.sw is not None:
                    br = self.sw.add_br(BRIDGE)
                    sfp = self._netdev(DPU_SFP1)
                    br.add_port(sfp, self.uplink_port)
                    self._ports[sfp] = self.uplink_port
                    self.dp.commit()
            return ip, DEFAULT_PORT

    def _set_vlan_ids_spoofchk(self, n: int) -> None:
        pf = self._netdev(DPU_BACKPLANE_F2 if self.dpu_mode else self.dpu_pcie)
        if not self.dpu_mode:
            common.set_pf_hwmode_vepa(self.runner, pf)
        self.vf_devs = {}
        for vf in range(n):
            vlan = vf + VLAN_OFFSET
            self.nl.link_set_vf(pf, vf, vlan=vlan, spoofchk=False, trust=True)
            pci = common.vf_pci_from_index(pf, vf, self.root)
            self.vf_devs[(pf, vf)] = common.VfDevice(pf, vf, pci, vlan)

    def set_num_vfs(self, n):
        with self._mu:
            common.set_sriov_numvfs(DPU_BACKPLANE_F2 if self.dpu_mode else self.dpu_pcie, n, self.root)
            self._set_vlan_ids_spoofchk(n)
            self.vf_cnt = n
            return n

    def _connected_vf(self, bp_name: str) -> common.VfDevice:
        m = re.fullmatch(r"host(\d+)-(\d+)", bp_name)
        if not m:
            raise ValueError("OPI BridgePortName does not match expected format")
        pfid, vf = int(m.group(1)), int(m.group(2))
        if pfid != 0:
            raise ValueError(f"PFID {pfid} is not supported")
        pf = self._netdev(DPU_BACKPLANE_F2)
        dev = self.vf_devs.get((pf, vf))
        if dev is None:
            raise LookupError(f"VF Device not found PFInterfaceName: {pf}, VFId: {vf}")
        return dev

    def create_bridge_port(self, name, mac, ptype, logical_bridges):
        with self._mu:
            dev = self._connected_vf(name)
            ifname = self._netdev(dev.pci)
            self.bridge_vfs[name] = ifname
            if self.sw is not None:
                br = self.sw.br(BRIDGE)
                idx = self._port(ifname)
                mac_s = ":".join(f"{b:02x}" for b in mac) if mac else None
                br.add_port(ifname, idx, mac=mac_s)
                # K10: per-VF VLAN isolation + egress tagging, trusted (spoof check off)
                self.dp.ports.update(idx, flags=int(T.PORT_VALID | T.PORT_VLAN_ISOLATE | T.PORT_TAG_EGRESS | T.PORT_TRUST),
                                     vlan=dev.vlan)
                if self.nf:
                    self._steer_vf(ifname, mac_s)
                self.dp.commit()
            dev.allocated = True

    def delete_bridge_port(self, name):
        with self._mu:
            dev = self._connected_vf(name)
            ifname = self.bridge_vfs.pop(name, self._netdev(dev.pci))
            if self.sw is not None:
                br = self.sw.br(BRIDGE)
                br.del_flows(f"in_port={ifname}")
                br.del_port(ifname)
                self.dp.commit()
            dev.allocated = False

    def _steer_vf(self, vf_if: str, mac: str | None) -> None:
        br = self.sw.br(BRIDGE)
        i_dp, o_dp = self.nf
        br.add_flow(f"priority=10,in_port={vf_if},actions=output:{i_dp}")
        if mac:
            br.add_flow(f"in_port={i_dp},dl_dst={mac},actions=output:{vf_if}")
            br.add_flow(f"priority=100,in_port={o_dp},dl_dst={mac},actions=in_port")

    def create_network_function(self, inp, out):
        with self._mu:
            by_mac = {v.if_mac: v for v in self.veths}
            if inp not in by_mac or out not in by_mac:
                raise KeyError("unknown NF interface MAC")
            if self.sw is None:
                return
            br = self.sw.br(BRIDGE)
            i_dp, o_dp = by_mac[inp].peer, by_mac[out].peer
            br.add_port(i_dp, self._port(i_dp))
            br.add_port(o_dp, self._port(o_dp))
            self.nf = (i_dp, o_dp)
            for ifname in self.bridge_vfs.values():
                mac = next((m for m, n in br.learned.items() if n == ifname), None)
                self._steer_vf(ifname, mac)
            sfp = self._netdev(DPU_SFP1)
            br.add_flow(f"priority=10,in_port={o_dp},actions=output:{sfp}")
            br.add_flow(f"priority=10,in_port={sfp},actions=output:{o_dp}")
            self.dp.commit()

    def delete_network_function(self, inp, out):
        with self._mu:
            if self.sw is None or self.nf is None:
                return
            br = self.sw.br(BRIDGE)
            i_dp, o_dp = self.nf
            for ifname in self.bridge_vfs.values():
                br.del_flows(f"in_port={ifname}")
            br.del_flows(f"in_port={self._netdev(DPU_SFP1)}")
            br.del_port(i_dp)
            br.del_port(o_dp)
            self.nf = None
            self.dp.commit()

    def get_devices(self):
        with self._mu:
            if not self.dpu_mode:
                return {vf: "Healthy" for vf in self._vfs_on_card()}
            return {v.ifname: "Healthy" for v in self.veths}
