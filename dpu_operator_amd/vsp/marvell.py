"""Marvell OCTEON VSP, with the OvS datapath replaced by the MI355X data plane.

Reference: internal/daemon/vendor-specific-plugins/marvell/main.go:32-823, ovs-dp
(V3), debug-dp (V4), mrvl-utils (V5), cp-agent launcher (V6).  Behaviour kept:
* Init(dpu): IPv6 link-local comm channel on the SDP interface (fe80::1 DPU / fe80::2 host,
  port 8085, address `[fe80::1%<if>]`), DPU side creates NoOfPortPairs=2 veth pairs
  nf_interfaceN/dp_interfaceN (devices keyed by the NF-side MAC) and the bridge `br-mrv0` with the
  RPM (uplink, device a063) port; host side loads the SDP VFs (device b903) as devices.
* CreateBridgePort(host<pf>-<vf>): VF = SDP VF number pf_count*(vf+1)+pfid, added to the bridge;
  with an NF present: `in_port=vf -> nf_in`, `in_port=nf_in,dl_dst=mac -> vf`, hairpin
  `priority=100,in_port=nf_out,dl_dst=mac,actions=in_port`.
* CreateNetworkFunction(in_mac, out_mac): dp sides of the two veth pairs join the bridge; the
  three flows for every known VF; `nf_out <-> RPM`.
* GetDevices: DPU -> NF-side veth names with link health; host -> VF PCI addresses.
* SetNumVfs: host only (sriov_numvfs 0 then N, then reload; count must match).
Changes: the flows are compiled onto the GPU tables by `dataplane.ovs.OvsBridge`
(`GpuOvsDataPlane`), or logged (`DebugDataPlane`) — no ovs-vsctl, no chroot; flow-delete
errors are reported instead of silently returning success (main.go:452-459).
"""
from __future__ import annotations

import logging
import os
import re
import threading
from dataclasses import dataclass, field

from ..cni.netlink import NetlinkManager
from ..platform.platform import Platform
from ..utils.cmdrunner import Runner
from . import common
from .base import VspBase

log = logging.getLogger("dpu.vsp.marvell")

VENDOR_ID = "177d"
DPU_SDP_PF_ID = "a0f7"     # DPU-side SDP interface
HOST_SDP_PF_ID = "b900"    # host-side SDP PF
HOST_VF_ID = "b903"        # host-side SDP VFs
DPI_PF_ID = "a080"
PEM_PF_ID = "a06c"
DPU_RPM_ID = "a063"        # uplink (RPM) interface
DEFAULT_PORT = 8085
IPV6_DPU = "fe80::1"
IPV6_HOST = "fe80::2"
NO_OF_PORT_PAIRS = 2
NUM_PFS = 1
PF_ID = 0
NF_NAME = "mrvl-nf1"
BRIDGE = "br-mrv0"


class NoSuchDevice(LookupError):
    pass


# ------------------------------------------------------------------------------------ mrvl utils
class MarvellUtils:
    """PCI discovery and platform setup helpers (mrvl-utils/mrvlutils.go:18-396)."""

    def __init__(self, platform: Platform, runner: Runner, sys_root: str = "/"):
        self.platform = platform
        self.runner = runner
        self.root = sys_root

    def all_by_device_id(self, device_id: str) -> list[str]:
        out = [d.address for d in self.platform.pci_devices() if d.vendor_id == VENDOR_ID and d.device_id == device_id]
        if not out:
            raise NoSuchDevice(f"No devices for PCI ID [{VENDOR_ID}:{device_id}] found")
        return out

    def pci_by_device_id(self, device_id: str) -> str:
        return self.all_by_device_id(device_id)[0]

    def name_by_pci(self, pci: str) -> str:
        for d in self.platform.pci_devices():
            if d.address == pci and d.netdevs:
                return d.netdevs[0]
        return common.netdev_from_pci(pci, self.root)

    def name_by_device_id(self, device_id: str) -> str:
        return self.name_by_pci(self.pci_by_device_id(device_id))

    def mapped_vf(self, pf_count: int, pfid: int, vfid: int) -> str:
        sdp = [d.address for d in self.platform.pci_devices() if d.vendor_id == VENDOR_ID and d.device_id == DPU_SDP_PF_ID]
        idx = pf_count * vfid + pfid
        if idx > len(sdp) - 1:
            raise IndexError("mapped VF out of bounds")
        return sdp[idx]

    def detect_platform_mode(self) -> str:
        return "dpu" if any(d.vendor_id == VENDOR_ID and d.device_id == DPU_SDP_PF_ID
                            for d in self.platform.pci_devices()) else "host"

    def bind_to_vfio(self, pci: str, current_driver: str = "") -> None:
        import os

        base = common._p(self.root, "/sys/bus/pci")
        if current_driver:
            with open(os.path.join(base, "drivers", current_driver, "unbind"), "w") as f:
                f.write(pci)
        with open(os.path.join(base, "devices", pci, "driver_override"), "w") as f:
            f.write("vfio-pci")
        with open(os.path.join(base, "drivers_probe"), "w") as f:
            f.write(pci)

    def setup_hugepages(self) -> None:
        self.runner.run(["mkdir", "-p", "/dev/huge"])
        self.runner.run(["mount", "-t", "hugetlbfs", "none", "/dev/huge"])

    def setup_host_interface(self, attempts: int = 9, wait=None) -> None:
        """Reload octeon_ep until the host SDP PF netdev appears (mrvlutils.go:323-346)."""
        import time

        wait = wait or time.sleep
        for _ in range(attempts):
            try:
                if self.name_by_device_id(HOST_SDP_PF_ID):
                    return
            except LookupError:
                pass
            self.runner.run(["rmmod", "octeon_ep_vf"], check=False, host=True)
            self.runner.run(["rmmod", "octeon_ep"], check=False, host=True)
            wait(20)
            self.runner.run(["modprobe", "octeon_ep"], host=True)
            self.runner.run(["modprobe", "octeon_ep_vf"], host=True)
            wait(5)
        raise RuntimeError("Failed to set up Host Interface")


# ---------------------------------------------------------------------------------- cp agent
CP_AGENT_UNIT = """[Unit]
Description=Control Plane Agent for the MI355X data plane node

[Service]
Restart=always
ExecStart={exe} {cfg} --mbox {mbox} --plugin-port {port}
ExecStop=/bin/kill -TERM $MAINPID

[Install]
WantedBy=multi-user.target
"""


def cp_agent_command(exe: str, cfg: str, mbox: str, plugin_port: int = 49500, dpi_dev: str = "",
                     pem_dev: str = "") -> list[str]:
    """The agent command line (cp-agent-run.go: `<agent> <cfg> -- --dpi_dev X --pem_dev Y`).  The native
    MI355X agent has no DPI/PEM engines to bind; those are accepted for parity and ignored."""
    argv = [exe, cfg, "--mbox", mbox, "--plugin-port", str(plugin_port)]
    if dpi_dev or pem_dev:
        log.info("dpi_dev=%s pem_dev=%s are not used by the MI355X agent", dpi_dev, pem_dev)
    return argv


def setup_dpu_service(runner: Runner, unit_text: str, unit_dir: str = "/etc/systemd/system") -> None:
    """Install + start the agent unit (mrvlutils.go:348-379 SetupDpuService)."""
    import os

    os.makedirs(unit_dir, exist_ok=True)
    with open(os.path.join(unit_dir, "cp-agent.service"), "w") as f:
        f.write(unit_text)
    runner.run(["systemctl", "enable", "cp-agent"], host=True)
    runner.run(["systemctl", "daemon-reload"], host=True)
    runner.run(["systemctl", "start", "cp-agent"], host=True)


# ---------------------------------------------------------------------------------- data planes
class MarvellDataPlane:
    def init_data_plane(self, bridge: str) -> None: ...
    def add_port(self, bridge: str, port: str, pci: str = "", dpdk: bool = False) -> None: ...
    def delete_port(self, bridge: str, port: str) -> None: ...
    def add_flow_rule(self, bridge: str, in_port: str, out_port: str, dst_mac: str = "") -> None: ...
    def delete_flow_rule(self, bridge: str, in_port: str, out_port: str = "", dst_mac: str = "") -> None: ...
    def read_all_ports(self, bridge: str) -> list[str]: ...


class DebugDataPlane(MarvellDataPlane):
    """Log-only data plane (debug-dp/debugdp.go)."""

    def __init__(self):
        self.ops: list[tuple] = []

    def init_data_plane(self, bridge):
        self.ops.append(("init", bridge))

    def add_port(self, bridge, port, pci="", dpdk=False):
        self.ops.append(("add_port", bridge, port, pci, dpdk))

    def delete_port(self, bridge, port):
        self.ops.append(("del_port", bridge, port))

    def add_flow_rule(self, bridge, in_port, out_port, dst_mac=""):
        self.ops.append(("add_flow", bridge, in_port, out_port, dst_mac))

    def delete_flow_rule(self, bridge, in_port, out_port="", dst_mac=""):
        self.ops.append(("del_flow", bridge, in_port, out_port, dst_mac))

    def read_all_ports(self, bridge):
        return [o[2] for o in self.ops if o[0] == "add_port" and o[1] == bridge]


class GpuOvsDataPlane(MarvellDataPlane):
    """OvS-compatible bridge semantics compiled onto the MI355X DataPlane (dataplane/ovs.py)."""

    def __init__(self, dataplane, uplink_name: str | None = None, uplink_port: int = 4000, first_port: int = 0,
                 mac_of=None, live_factory=None):
        """live_factory(dataplane) -> a started NativeLivePath: the bridge's netdev ports then
        carry live traffic (each OvS port an AF_PACKET port of the native I/O engine), the way
        the reference's OvS-DPDK bridge forwards between its DPDK ports (ovsdp.go:39-55)."""
        from ..dataplane.ovs import OvsSwitch

        self.dp = dataplane
        self.sw = OvsSwitch(dataplane)
        self.live_factory = live_factory
        self.live = None
        self.uplink_name = uplink_name
        self.uplink_port = uplink_port
        self._next = first_port
        self._index: dict[str, int] = {}
        self.mac_of = mac_of or (lambda name: None)

    def _idx(self, port: str) -> int:
        if port == self.uplink_name:
            return self.uplink_port
        if port not in self._index:
            self._index[port] = self._next
            self._next += 1
        return self._index[port]

    def init_data_plane(self, bridge):
        br = self.sw.add_br(bridge, "netdev")
        if self.uplink_name:
            br.add_port(self.uplink_name, self.uplink_port)
        self.dp.commit()
        if self.live_factory is not None and self.live is None:
            self.live = self.live_factory(self.dp)
        if self.uplink_name:
            self._live_add(self.uplink_name, self.uplink_port)

    def _live_add(self, port: str, idx: int) -> None:
        """A netdev bridge port joins the native engine (ports that are not netdevs here, e.g.
        DPDK PCI devices bound elsewhere, stay table-only)."""
        if self.live is not None and os.path.exists(f"/sys/class/net/{port}"):
            from ..dataplane.native_io import PacketVport

            self.live.add_port(idx, PacketVport(port))

    def add_port(self, bridge, port, pci="", dpdk=False):
        self.sw.br(bridge).add_port(port, self._idx(port), mac=self.mac_of(port), pci=pci or None, dpdk=dpdk)
        self.dp.commit()
        self._live_add(port, self._idx(port))

    def delete_port(self, bridge, port):
        self.sw.br(bridge).del_port(port)
        if self.live is not None and port in self._index:
            self.live.remove_port(self._index[port])
        self.dp.commit()

    def close(self) -> None:
        if self.live is not None:
            self.live.stop()
            self.live = None

    def add_flow_rule(self, bridge, in_port, out_port, dst_mac=""):
        br = self.sw.br(bridge)
        if dst_mac:
            if in_port == out_port:
                br.add_flow(f"priority=100,in_port={in_port},dl_dst={dst_mac},actions=in_port")
            else:
                br.add_flow(f"in_port={in_port},dl_dst={dst_mac},actions=output:{out_port}")
        else:
            br.add_flow(f"priority=10,in_port={in_port},actions=output:{out_port}")
        self.dp.commit()

    def delete_flow_rule(self, bridge, in_port, out_port="", dst_mac=""):
        spec = f"in_port={in_port}" + (f",dl_dst={dst_mac}" if dst_mac else "")
        self.sw.br(bridge).del_flows(spec)
        self.dp.commit()

    def read_all_ports(self, bridge):
        return self.sw.br(bridge).list_ports()

    def port_index(self, port: str) -> int:
        return self._idx(port)


# ---------------------------------------------------------------------------------------- VSP
@dataclass
class _Dev:
    sec_if: str = ""
    dp_if: str = ""
    dp_mac: str = ""
    pci: str = ""
    health: str = "Healthy"
    ptype: str = "veth"


@dataclass
class _NfPorts:
    vfs: list[tuple[str, str]] = field(default_factory=list)   # (vf netdev, pod mac)
    inp: str = ""
    out: str = ""


class MarvellVsp(VspBase):
    name = "marvell-vsp"

    def __init__(self, platform: Platform, nl: NetlinkManager, runner: Runner, data_plane: MarvellDataPlane,
                 path_manager=None, sys_root: str = "/", port_type: str = "veth", port_pairs: int = NO_OF_PORT_PAIRS):
        super().__init__(path_manager)
        self.utils = MarvellUtils(platform, runner, sys_root)
        self.nl = nl
        self.runner = runner
        self.mdp = data_plane
        self.root = sys_root
        self.port_type = port_type
        self.port_pairs = port_pairs
        self.dpu_mode = False
        self.devices: dict[str, _Dev] = {}
        self.store: dict[str, _NfPorts] = {}
        self.is_nf = False
        self.bridge = ""
        self._mu = threading.RLock()

    # -------------------------------------------------------------- helpers
    def _health(self, ifname: str) -> str:
        try:
            return "Healthy" if self.nl.link_by_name(ifname).up else "Unhealthy"
        except KeyError:
            return "Unhealthy"

    def _configure_ip(self, dpu_mode: bool) -> tuple[str, int]:
        addr, dev = (IPV6_DPU, DPU_SDP_PF_ID) if dpu_mode else (IPV6_HOST, HOST_SDP_PF_ID)
        ifname = self.utils.name_by_device_id(dev)
        common.enable_ipv6_link_local(self.runner, ifname, addr, self.root)
        # both sides dial / serve the DPU address; the host escapes '%' for the gRPC target
        return (f"[{IPV6_DPU}%{ifname}]" if dpu_mode else f"[{IPV6_DPU}%25{ifname}]"), DEFAULT_PORT

    def _configure_network_interfaces(self) -> None:
        if self.port_type != "veth":
            raise RuntimeError("currently only veth pairs are supported")
        made = []
        try:
            for i in range(self.port_pairs):
                pair = common.create_nf_veth_pair(self.nl, i)
                made.append(pair)
                self.devices[pair.if_mac] = _Dev(pair.ifname, pair.peer, pair.peer_mac, health=self._health(pair.ifname))
        except Exception:
            for p in made:
                try:
                    common.destroy_veth_pair(self.nl, p)
                except Exception:  # noqa: BLE001
                    pass
            self.devices.clear()
            raise

    def _reload_vfs(self) -> None:
        try:
            vfs = self.utils.all_by_device_id(HOST_VF_ID)
        except NoSuchDevice:
            vfs = []
        self.devices = {pci: _Dev(pci=pci, health="Healthy", ptype="sriov") for pci in vfs}

    def _vf_details(self, bp_name: str) -> tuple[str, str]:
        m = re.search(r"host(\d+)-(\d+)", bp_name)
        if not m:
            raise ValueError("no VFId Match Found")
        pfid, vfid = int(m.group(1)), int(m.group(2)) + 1  # VF 0 is the PF
        pci = self.utils.mapped_vf(NUM_PFS, PF_ID, vfid)
        return self.utils.name_by_pci(pci), pci

    # -------------------------------------------------------------- VSP hooks
    def init(self, dpu_mode, dpu_identifier):
        with self._mu:
            self.dpu_mode = dpu_mode
            self.devices = {}
            ip, port = self._configure_ip(dpu_mode)
            if dpu_mode:
                self._configure_network_interfaces()
                self.bridge = BRIDGE
                self.mdp.init_data_plane(self.bridge)
            else:
                self.utils.all_by_device_id(HOST_SDP_PF_ID)
                self._reload_vfs()
                self.port_type = "sriov"
            return ip, port

    def create_bridge_port(self, name, mac, ptype, logical_bridges):
        with self._mu:
            vf, pci = self._vf_details(name)
            self.mdp.add_port(self.bridge, vf, pci, False)
            mac_s = ":".join(f"{b:02x}" for b in mac)
            nf = self.store.setdefault(NF_NAME, _NfPorts())
            nf.vfs.append((vf, mac_s))
            if self.is_nf:
                self.mdp.add_flow_rule(self.bridge, vf, nf.inp)
                self.mdp.add_flow_rule(self.bridge, nf.inp, vf, mac_s)
                self.mdp.add_flow_rule(self.bridge, nf.out, nf.out, mac_s)

    def delete_bridge_port(self, name):
        with self._mu:
            vf, _ = self._vf_details(name)
            nf = self.store.get(NF_NAME)
            if self.is_nf and nf is not None:
                vf_mac = next((m for v, m in nf.vfs if v == vf), "")
                self.mdp.delete_flow_rule(self.bridge, vf)
                self.mdp.delete_flow_rule(self.bridge, nf.out, nf.out, vf_mac)
                self.mdp.delete_flow_rule(self.bridge, nf.inp, vf, vf_mac)
            self.mdp.delete_port(self.bridge, vf)
            if nf is not None:
                nf.vfs = [(v, m) for v, m in nf.vfs if v != vf]

    def create_network_function(self, inp, out):
        with self._mu:
            if inp not in self.devices or out not in self.devices:
                raise KeyError(f"unknown NF device MAC(s): {inp}, {out}")
            self.is_nf = True
            i_dp, o_dp = self.devices[inp].dp_if, self.devices[out].dp_if
            self.mdp.add_port(self.bridge, i_dp)
            self.mdp.add_port(self.bridge, o_dp)
            nf = self.store.setdefault(NF_NAME, _NfPorts())
            nf.inp, nf.out = i_dp, o_dp
            for vf, mac in nf.vfs:
                self.mdp.add_flow_rule(self.bridge, vf, i_dp)
                self.mdp.add_flow_rule(self.bridge, i_dp, vf, mac)
                self.mdp.add_flow_rule(self.bridge, o_dp, o_dp, mac)
            rpm = self.utils.name_by_device_id(DPU_RPM_ID)
            self.mdp.add_flow_rule(self.bridge, o_dp, rpm)
            self.mdp.add_flow_rule(self.bridge, rpm, o_dp)

    def delete_network_function(self, inp, out):
        with self._mu:
            self.is_nf = False
            i_dp, o_dp = self.devices[inp].dp_if, self.devices[out].dp_if
            nf = self.store.get(NF_NAME, _NfPorts())
            for vf, _ in nf.vfs:
                self.mdp.delete_flow_rule(self.bridge, vf, i_dp)
            self.mdp.delete_flow_rule(self.bridge, i_dp)
            self.mdp.delete_flow_rule(self.bridge, o_dp)
            self.mdp.delete_flow_rule(self.bridge, self.utils.name_by_device_id(DPU_RPM_ID))
            self.mdp.delete_port(self.bridge, i_dp)
            self.mdp.delete_port(self.bridge, o_dp)
            nf.inp = nf.out = ""

    def get_devices(self):
        with self._mu:
            if self.dpu_mode:
                return {d.sec_if: self._health(d.sec_if) for d in self.devices.values()}
            return {d.pci: d.health for d in self.devices.values()}

    def set_num_vfs(self, n):
        with self._mu:
            if self.dpu_mode:
                raise RuntimeError("SetNumVfs is not supported in DPU Mode")
            if n < 0:
                raise ValueError("invalid VF Count")
            pci = self.utils.pci_by_device_id(HOST_SDP_PF_ID)
            common.set_sriov_numvfs(pci, n, self.root)
            self._reload_vfs()
            if len(self.devices) != n:
                raise RuntimeError(f"failed to load expected number {n} of VFs but got {len(self.devices)}")
            return n
