"""Host-side SR-IOV attach/detach (reference: dpu-cni/pkgs/sriov/sriov.go:20-583 and
dpu-cni/pkgs/sriovconfig/sriovconfig.go:13-171).

ADD: LoadConf (VF PCI -> PF + VF id; reject an allocated VF; netdev or DPDK driver; validate
vlan 0-4094, QoS 0-7 (needs vlan), proto 802.1q/802.1ad (802.1ad needs vlan), link_state) ->
ApplyVFConfig (MAC, rate, spoofchk, trust, link state; VLAN left to the data plane because the
device side owns VLAN isolation, the reference's host_vlans=false) -> SetupVF (down, temp name,
move into pod netns, rename, MAC, up) -> IPAM -> announce -> cache NetConf -> PCI allocation file.
DEL: idempotent when the cache is gone; restores name/MAC/VF state, releases IPAM and the PCI lock.
Each ADD step is undone on failure.
"""
from __future__ import annotations

import copy
import json
import os
import secrets

from .. import logging as clog
from ..ipam import HostLocalIpam
from ..netlink import LinkNotFound, NetlinkManager
from ..types import PROTO_8021AD, PROTO_8021Q, VLAN_PROTO_INT, NetConf, PodRequest, VfState, result_json
from . import utils as U
from .packet import announce
from .pci_allocator import PCIAllocator


def load_conf(conf: NetConf, sysfs: U.Sysfs, allocator: PCIAllocator) -> NetConf:
    if not conf.deviceID:
        raise ValueError("LoadConf(): VF pci addr is required")
    try:
        conf.Master = sysfs.get_pf_name(conf.deviceID)
        conf.VFID = sysfs.get_vfid(conf.deviceID)
    except OSError as e:
        raise ValueError(f"LoadConf(): failed to get VF information: {e}") from e
    if allocator.is_allocated(conf.deviceID):
        raise ValueError(f"pci address {conf.deviceID} is already allocated")
    host_if = sysfs.get_vf_link_name(conf.deviceID)
    if not host_if:
        conf.DPDKMode = sysfs.has_dpdk_driver(conf.deviceID)
    else:
        conf.OrigVfState.HostIFName = host_if
    if not host_if and not conf.DPDKMode:
        raise ValueError(f"LoadConf(): the VF {conf.deviceID} does not have a interface name or a dpdk driver")
    if conf.vlan is None:
        conf.vlan = 0
    if not 0 <= conf.vlan <= 4094:
        raise ValueError(f"LoadConf(): vlan id {conf.vlan} invalid: value must be in the range 0-4094")
    if conf.vlanQoS is None:
        conf.vlanQoS = 0
    if not 0 <= conf.vlanQoS <= 7:
        raise ValueError(f"LoadConf(): vlan QoS PCP {conf.vlanQoS} invalid: value must be in the range 0-7")
    if conf.vlanQoS != 0 and conf.vlan == 0:
        raise ValueError("LoadConf(): non-zero vlan id must be configured to set vlan QoS to a non-zero value")
    conf.vlanProto = (conf.vlanProto or PROTO_8021Q).lower()
    if conf.vlanProto not in (PROTO_8021Q, PROTO_8021AD):
        raise ValueError(f"LoadConf(): vlan Proto {conf.vlanProto} invalid: value must be '802.1Q' or '802.1ad'")
    if conf.vlanProto == PROTO_8021AD and conf.vlan == 0:
        raise ValueError("LoadConf(): non-zero vlan id must be configured to set vlan proto 802.1ad")
    if conf.link_state not in ("", "auto", "enable", "disable"):
        raise ValueError(f"LoadConf(): invalid link_state value: {conf.link_state}")
    return conf


class SriovManager:
    def __init__(self, nl: NetlinkManager, sysfs: U.Sysfs | None = None, cache_dir: str = U.DEFAULT_CNI_DIR,
                 ipam: HostLocalIpam | None = None, netns_exists=None):
        self.nl = nl
        self.sysfs = sysfs or U.Sysfs("/")
        self.cache_dir = cache_dir
        self.allocator = PCIAllocator(cache_dir, netns_exists)
        self.ipam = ipam

    # -------------------------------------------------------------------------- VF config
    def _fill_orig_state(self, conf: NetConf) -> None:
        pf = self.nl.link_by_name(conf.Master)
        vf = pf.vfs[conf.VFID] if conf.VFID < len(pf.vfs) else None
        if vf is not None:
            conf.OrigVfState.AdminMAC = vf.mac
            conf.OrigVfState.SpoofChk = vf.spoofchk
            conf.OrigVfState.Trust = vf.trust
            conf.OrigVfState.Vlan = vf.vlan
            conf.OrigVfState.VlanQoS = vf.qos
            conf.OrigVfState.VlanProto = vf.vlan_proto
            conf.OrigVfState.MinTxRate = vf.min_tx_rate
            conf.OrigVfState.MaxTxRate = vf.max_tx_rate
            conf.OrigVfState.LinkState = vf.link_state
        if conf.OrigVfState.HostIFName:
            conf.OrigVfState.EffectiveMAC = self.nl.link_by_name(conf.OrigVfState.HostIFName).mac

    def apply_vf_config(self, conf: NetConf) -> None:
        attrs = {}
        mac = conf.MAC or (conf.runtimeConfig or {}).get("mac", "")
        if mac:
            attrs["mac"] = mac.lower()
        if conf.min_tx_rate is not None:
            attrs["min_tx_rate"] = conf.min_tx_rate
        if conf.max_tx_rate is not None:
            attrs["max_tx_rate"] = conf.max_tx_rate
        if conf.spoofchk:
            attrs["spoofchk"] = conf.spoofchk == "on"
        if conf.trust:
            attrs["trust"] = conf.trust == "on"
        if conf.link_state:
            attrs["link_state"] = {"auto": 0, "enable": 1, "disable": 2}[conf.link_state]
        if attrs:
            self.nl.link_set_vf(conf.Master, conf.VFID, **attrs)

    def reset_vf_config(self, conf: NetConf) -> None:
        o = conf.OrigVfState
        self.nl.link_set_vf(conf.Master, conf.VFID, mac=o.AdminMAC or "00:00:00:00:00:00", spoofchk=o.SpoofChk,
                            trust=o.Trust, vlan=o.Vlan, qos=o.VlanQoS,
                            vlan_proto=o.VlanProto or VLAN_PROTO_INT[PROTO_8021Q], min_tx_rate=o.MinTxRate,
                            max_tx_rate=o.MaxTxRate, link_state=o.LinkState)

    def setup_vf(self, conf: NetConf, ifname: str, netns: str) -> str:
        host_if = conf.OrigVfState.HostIFName
        tmp = "dpu" + secrets.token_hex(4)
        self.nl.link_set_down(host_if)
        self.nl.link_set_name(host_if, tmp)
        try:
            self.nl.link_set_ns(tmp, netns)
        except Exception:
            self.nl.link_set_name(tmp, host_if)
            raise
        self.nl.link_set_name(tmp, ifname, netns)
        mac = conf.MAC or (conf.runtimeConfig or {}).get("mac", "")
        if mac:
            self.nl.link_set_hw_addr(ifname, mac, netns)
        self.nl.link_set_up(ifname, netns)
        return self.nl.link_by_name(ifname, netns).mac

    def release_vf(self, conf: NetConf, ifname: str, netns: str) -> None:
        host_if = conf.OrigVfState.HostIFName
        try:
            self.nl.link_by_name(ifname, netns)
        except (LinkNotFound, KeyError):
            return
        self.nl.link_set_down(ifname, netns)
        self.nl.link_set_name(ifname, host_if, netns)
        if conf.OrigVfState.EffectiveMAC:
            self.nl.link_set_hw_addr(host_if, conf.OrigVfState.EffectiveMAC, netns)
        self.nl.link_set_ns(host_if, "", netns)

    # -------------------------------------------------------------------------- CNI verbs
    def cmd_add(self, req: PodRequest) -> dict:
        conf = load_conf(copy.deepcopy(req.cni_conf), self.sysfs, self.allocator)
        self._fill_orig_state(conf)
        req.cni_conf.VFID = conf.VFID
        req.cni_conf.OrigVfState = conf.OrigVfState
        undo = []
        try:
            self.apply_vf_config(conf)
            undo.append(lambda: self.reset_vf_config(conf))
            ifaces, ips = [], []
            if not conf.DPDKMode:
                mac = self.setup_vf(conf, req.ifname, req.netns)
                undo.append(lambda: self.release_vf(conf, req.ifname, req.netns))
                conf.MAC = mac
                ifaces.append({"name": req.ifname, "mac": mac, "sandbox": req.netns})
                if self.ipam is not None and conf.ipam:
                    if conf.ipam.get("subnet"):
                        self.ipam.configure(conf.name, conf.ipam["subnet"])
                    ip = self.ipam.allocate(conf.name, req.container_id, req.ifname)
                    undo.append(lambda: self.ipam.release(conf.name, req.container_id, req.ifname))
                    self.nl.addr_add(req.ifname, ip["address"], req.netns)
                    ips.append(dict(ip, interface=0))
                    # GARP / NA from inside the pod netns, where the VF now lives (packet.go:166-198)
                    try:
                        self.nl.run_in_ns(req.netns, lambda: announce(req.ifname, mac, [ip["address"]]))
                    except OSError as e:
                        clog.warning(f"announce {req.ifname} in {req.netns}: {e}")
            U.save_net_conf(req.container_id, self.cache_dir, req.ifname, conf.to_json())
            undo.append(lambda: U.clean_cached_net_conf(U.cache_path(self.cache_dir, req.container_id, req.ifname)))
            self.allocator.save_allocated_pci(conf.deviceID, req.netns)
        except Exception:
            for fn in reversed(undo):
                try:
                    fn()
                except Exception as e:  # noqa: BLE001
                    clog.error("sriov rollback step failed", err=repr(e))
            raise
        req.cni_conf.MAC = conf.MAC
        clog.info("sriov ADD done", vf=conf.VFID, pf=conf.Master, mac=conf.MAC)
        return result_json(conf.cniVersion, interfaces=ifaces, ips=ips)

    def cmd_del(self, req: PodRequest) -> None:
        path = U.cache_path(self.cache_dir, req.container_id, req.ifname)
        if not os.path.exists(path):
            clog.info("sriov DEL: no cached NetConf (already released)")
            return  # idempotent (sriov.go:508-519)
        from ..helper import read_cni_config

        conf = read_cni_config(json.dumps(U.read_scratch_net_conf(path)).encode())
        req.cni_conf.VFID = conf.VFID
        req.cni_conf.OrigVfState = conf.OrigVfState
        if self.ipam is not None and conf.ipam:
            self.ipam.release(conf.name, req.container_id, req.ifname)
        if not conf.DPDKMode:
            self.release_vf(conf, req.ifname, req.netns)
        self.reset_vf_config(conf)
        self.allocator.delete_allocated_pci(conf.deviceID)
        U.clean_cached_net_conf(path)


class SriovManagerStub:
    """Test stub (the reference's SriovManagerStub, hostsidemanager_test.go:33-60)."""

    def __init__(self):
        self.added, self.deleted = [], []

    def cmd_add(self, req: PodRequest) -> dict:
        self.added.append(req)
        req.cni_conf.VFID = int(req.cni_conf.raw.get("VFID", 0) or 0)
        req.cni_conf.OrigVfState = VfState(EffectiveMAC="00:11:22:33:44:55")
        return result_json(req.cni_conf.cniVersion, interfaces=[{"name": req.ifname, "mac": "00:11:22:33:44:55"}])

    def cmd_del(self, req: PodRequest) -> None:
        self.deleted.append(req)
        req.cni_conf.OrigVfState = VfState(EffectiveMAC="00:11:22:33:44:55")
