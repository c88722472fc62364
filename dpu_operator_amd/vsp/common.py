"""Network helpers shared by the vendor VSPs.

Reference: internal/daemon/vendor-specific-plugins/common/vspnetutils.go:44-282:
* set_sriov_numvfs: write 0, then N, to /sys/bus/pci/devices/<addr>/sriov_numvfs
* enable_ipv6_link_local: NetworkManager unmanaged (nsenter into pid 1), optimistic DAD,
  addrgenmode eui64 + link toggle unless already eui64, link up, `ip addr replace <ll>/64 optimistic`
* veth pairs for NF ports, VF PCI address from (PF, index) via the `virtfn<N>` link,
  PF `bridge link set hwmode vepa`, OvS bridge/port helpers.
All sysfs/procfs access is relative to a root (tests use a temp tree), every command goes through
a Runner, and links through a NetlinkManager.
"""
from __future__ import annotations

import logging
import os
from dataclasses import dataclass

from ..cni.netlink import NetlinkManager
from ..utils.cmdrunner import CommandError, Runner

log = logging.getLogger("dpu.vsp.common")

NET_SYS_DIR = "/sys/class/net"


@dataclass
class VethPair:
    ifname: str
    peer: str
    if_mac: str = ""
    peer_mac: str = ""


@dataclass
class VfDevice:
    pf: str
    vf_id: int
    pci: str
    vlan: int = 0
    allocated: bool = False


def _p(root: str, path: str) -> str:
    return os.path.join(root, path.lstrip("/")) if root not in ("", "/") else path


def set_sriov_numvfs(pci_addr: str, num_vfs: int, root: str = "/") -> None:
    path = _p(root, f"/sys/bus/pci/devices/{pci_addr}/sriov_numvfs")
    # the kernel refuses N -> M directly; always reset to 0 first
    with open(path, "w") as f:
        f.write("0")
    if num_vfs:
        with open(path, "w") as f:
            f.write(str(num_vfs))


def enable_ipv6_link_local(runner: Runner, ifname: str, addr: str, root: str = "/") -> None:
    try:
        runner.run(["nsenter", "-t", "1", "-m", "-u", "-n", "-i", "--", "nmcli", "device", "set", ifname,
                    "managed", "no"])
    except CommandError as e:  # the node may not run NetworkManager at all
        log.info("nmcli unmanaged failed (ignored): %s", e)
    try:
        with open(_p(root, f"/proc/sys/net/ipv6/conf/{ifname}/optimistic_dad"), "w") as f:
            f.write("1")
    except OSError as e:
        log.error("setting optimistic_dad on %s: %s", ifname, e)
    out = ""
    try:
        out = runner.run(["ip", "-d", "link", "show", "dev", ifname])
    except CommandError:
        pass
    if "addrgenmode eui64" not in out:
        runner.run(["ip", "link", "set", ifname, "addrgenmode", "eui64"])
        runner.run(["ip", "link", "set", ifname, "down"])
    runner.run(["ip", "link", "set", ifname, "up"])
    runner.run(["ip", "addr", "replace", f"{addr}/64", "dev", ifname, "optimistic"])


def netdev_from_pci(pci_addr: str, root: str = "/") -> str:
    d = _p(root, f"/sys/bus/pci/devices/{pci_addr}/net")
    try:
        names = sorted(os.listdir(d))
    except OSError as e:
        raise LookupError(f"no netdev for PCI {pci_addr}") from e
    if not names:
        raise LookupError(f"no netdev for PCI {pci_addr}")
    return names[0]


def create_veth_pair(nl: NetlinkManager, ifname: str, peer: str) -> VethPair:
    try:
        a, b = nl.link_by_name(ifname), nl.link_by_name(peer)
    except KeyError:
        nl.link_add_veth(ifname, peer)
        a, b = nl.link_by_name(ifname), nl.link_by_name(peer)
    nl.link_set_up(ifname)
    nl.link_set_up(peer)
    return VethPair(ifname, peer, a.mac, b.mac)


def create_nf_veth_pair(nl: NetlinkManager, idx: int, nf_prefix: str = "nf_interface",
                        dp_prefix: str = "dp_interface") -> VethPair:
    return create_veth_pair(nl, f"{nf_prefix}{idx}", f"{dp_prefix}{idx}")


def destroy_veth_pair(nl: NetlinkManager, dev: VethPair) -> None:
    nl.link_del(dev.ifname)


def vf_pci_from_index(pf: str, vf_id: int, root: str = "/") -> str:
    link = _p(root, f"{NET_SYS_DIR}/{pf}/device/virtfn{vf_id}")
    try:
        return os.path.basename(os.readlink(link))
    except OSError as e:
        raise LookupError(f"cannot read {link} for VF virtfn{vf_id} of PF {pf}") from e


def set_pf_hwmode_vepa(runner: Runner, pf: str) -> None:
    runner.run(["bridge", "link", "set", "dev", pf, "hwmode", "vepa"])
