"""NF-side CNI: move a device-side netdev into the NF pod's namespace (and back on DEL).

Reference: dpu-cni/pkgs/networkfn/networkfn.go:16-349.  ADD: the NetConf's ``deviceID`` names a
netdev (not a PCI address) on the device side; it is moved into the pod netns under a temporary
name, its alias set to the original name, renamed to CNI_IFNAME and brought up; optional IPAM.
Every step rolls back on failure.  DEL moves it back to the root namespace and restores the
original name from the alias.  On the MI355X data plane the netdev is the NF's vport tap (the
GPU VSP's NF in/out ports), so the NF container sees ordinary interfaces.
"""
from __future__ import annotations

import secrets

from . import logging as clog
from .ipam import HostLocalIpam
from .netlink import LinkNotFound, NetlinkManager
from .types import PodRequest, result_json


def _tmp_name() -> str:
    return "tmp" + secrets.token_hex(4)


def cmd_add(req: PodRequest, nl: NetlinkManager, ipam: HostLocalIpam | None = None) -> dict:
    conf = req.cni_conf
    if conf is None or not conf.deviceID:
        raise ValueError("networkfn: deviceID (netdev name) is required")
    dev = conf.deviceID
    link = nl.link_by_name(dev)
    conf.MAC = link.mac
    tmp = _tmp_name()
    undo = []
    try:
        nl.link_set_down(dev)
        nl.link_set_name(dev, tmp)
        undo.append(lambda: nl.link_set_name(tmp, dev))
        nl.link_set_ns(tmp, req.netns)
        undo.append(lambda: (nl.link_set_ns(tmp, "", req.netns)))
        nl.link_set_alias(tmp, dev, req.netns)
        nl.link_set_name(tmp, req.ifname, req.netns)
        undo.append(lambda: nl.link_set_name(req.ifname, tmp, req.netns))
        nl.link_set_up(req.ifname, req.netns)
        ips = []
        if ipam is not None and conf.ipam:
            ip = ipam.allocate(conf.name, req.container_id, req.ifname)
            undo.append(lambda: ipam.release(conf.name, req.container_id, req.ifname))
            nl.addr_add(req.ifname, ip["address"], req.netns)
            ips.append(dict(ip, interface=0))
    except Exception:
        for fn in reversed(undo):
            try:
                fn()
            except Exception as e:  # noqa: BLE001
                clog.error("networkfn rollback step failed", err=repr(e))
        raise
    clog.info("networkfn ADD done", dev=dev, ifname=req.ifname, mac=link.mac)
    return result_json(conf.cniVersion, interfaces=[{"name": req.ifname, "mac": link.mac, "sandbox": req.netns}],
                       ips=ips)


def cmd_del(req: PodRequest, nl: NetlinkManager, ipam: HostLocalIpam | None = None) -> None:
    conf = req.cni_conf
    if ipam is not None and conf is not None and conf.ipam:
        ipam.release(conf.name, req.container_id, req.ifname)
    try:
        link = nl.link_by_name(req.ifname, req.netns)
    except (LinkNotFound, KeyError):
        clog.info("networkfn DEL: interface already gone", ifname=req.ifname)
        return  # idempotent
    orig = link.alias or (conf.deviceID if conf else "")
    tmp = _tmp_name()
    nl.link_set_down(req.ifname, req.netns)
    nl.link_set_name(req.ifname, tmp, req.netns)
    nl.link_set_ns(tmp, "", req.netns)
    nl.link_set_name(tmp, orig)
    nl.link_set_up(orig)
