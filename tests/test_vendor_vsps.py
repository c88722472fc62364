"""Vendor VSPs re-expressed on the MI355X data plane: OpenFlow-subset bridge compile, Marvell and
Intel NetSec VSP behaviour (reference: marvell/main.go, ovs-dp/ovsdp.go, intel-netsec/main.go,
common/vspnetutils.go).  The data plane runs as the bit-exact CPU oracle here; the flows' effect
is checked by sending frames through it.
"""
from __future__ import annotations

import os
import shutil
import tempfile

import numpy as np
import pytest

from dpu_operator_amd.cni.netlink import FakeNetlink, Link
from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.dataplane.ovs import OvsSwitch, parse_flow
from dpu_operator_amd.ops import packets as P
from dpu_operator_amd.platform.platform import FakePlatform, PciDevice
from dpu_operator_amd.utils.cmdrunner import FakeRunner
from dpu_operator_amd.vsp import common
from dpu_operator_amd.vsp.marvell import (DebugDataPlane, GpuOvsDataPlane, MarvellUtils, MarvellVsp, cp_agent_command)
from dpu_operator_amd.vsp.netsec import NetsecVsp

M_A, M_B, M_GW = "02:aa:00:00:00:01", "02:aa:00:00:00:02", "02:00:00:00:ff:01"


def send(dp, in_port, dmac, smac=M_A):
    frames, lens = P.craft(1, dmac=dmac, smac=smac, src_ip=0x0A000001, dst_ip=0x0A000002, sport=1, dport=2)
    r = dp.run(frames, P.inmeta(np.array([in_port]), lens))
    op, _, reason = P.meta_fields(r.meta)
    return int(op[0]), int(reason[0]), r.out[0]


@pytest.fixture
def dp():
    d = DataPlane(device="cpu", flow_buckets=1 << 6)
    d.commit(full=True)
    return d


def test_parse_flow_syntax():
    f = parse_flow("priority=100,in_port=dp1,dl_dst=02:AA:00:00:00:01,actions=in_port")
    assert (f.priority, f.in_port, f.dl_dst, f.action) == (100, "dp1", M_A, "in_port")
    assert parse_flow("in_port=a actions=output:b").priority == 32768
    for bad in ("in_port=a", "nw_src=1.2.3.4,actions=drop", "in_port=a,actions=mod_vlan_vid:3"):
        with pytest.raises(ValueError):
            parse_flow(bad)


def test_ovs_bridge_semantics(dp):
    br = OvsSwitch(dp).add_br("br0")
    for i, (n, mac) in enumerate((("vf0", M_A), ("vf1", M_B), ("nfin", None), ("nfout", None))):
        br.add_port(n, i, mac=mac)
    br.add_port("uplink", 4000)
    dp.commit()
    # no flows: actions=normal learning bridge between known MACs
    assert send(dp, 0, M_B)[:2] == (1, 0)
    assert send(dp, 0, M_GW)[1] == 5  # unknown destination, no default output: no route (punt)
    br.add_flow("priority=10,in_port=vf0,actions=output:nfin")
    br.add_flow(f"in_port=nfin,dl_dst={M_A},actions=output:vf0")
    br.add_flow(f"priority=100,in_port=nfout,dl_dst={M_A},actions=in_port")
    br.add_flow("priority=10,in_port=nfout,actions=output:uplink")
    br.add_flow("priority=10,in_port=uplink,actions=output:nfout")
    dp.commit()
    assert send(dp, 0, M_B)[0] == 2           # VF -> NF in (even for a local destination)
    assert send(dp, 2, M_A)[0] == 0           # NF in -> VF by dst MAC
    assert send(dp, 3, M_A)[0] == 3           # hairpin
    assert send(dp, 3, M_GW)[0] == 4000       # NF out -> uplink
    assert send(dp, 4000, M_A)[0] == 3        # uplink -> NF out
    assert send(dp, 1, M_A)[0] == 0           # vf1 still on the normal bridge
    assert f"priority=100,in_port=nfout,dl_dst={M_A} actions=in_port" in br.dump_flows()
    # shadowed: a dl_dst flow below the in_port flow never matches
    br.add_flow(f"priority=5,in_port=vf0,dl_dst={M_B},actions=output:vf1")
    dp.commit()
    assert send(dp, 0, M_B)[0] == 2
    # non-strict delete by in_port removes both vf0 flows; vf0 falls back to normal
    assert br.del_flows("in_port=vf0") == 2
    dp.commit()
    assert send(dp, 0, M_B)[0] == 1
    br.add_flow(f"in_port=vf1,dl_dst={M_A},actions=drop")
    dp.commit()
    assert send(dp, 1, M_A, smac=M_B)[1] == 1  # dropped (bad-port reason)
    br.del_port("nfout")
    dp.commit()
    assert all("nfout" not in f for f in br.dump_flows())
    with pytest.raises(KeyError):
        br.add_flow("in_port=nope,actions=drop")


def test_mac_table_tombstones(dp):
    mt = T.MacTable(16)
    macs = [f"02:00:00:00:00:{i:02x}" for i in range(12)]
    for i, m in enumerate(macs):
        mt.insert(7, m, i)
    for m in macs[::2]:
        assert mt.remove(7, m)
    for i, m in enumerate(macs):
        assert mt.lookup(7, m) == (-1 if i % 2 == 0 else i)
    for i, m in enumerate(macs[::2]):
        mt.insert(7, m, 100 + i)
    assert mt.lookup(7, macs[4]) == 102
    assert not mt.remove(7, "02:ff:ff:ff:ff:ff")


# ------------------------------------------------------------------------------------ Marvell
def marvell_platform():
    devs = [PciDevice(f"0002:1f:00.{i}", "177d", "a0f7", netdevs=[f"sdp{i}"]) for i in range(4)]
    devs.append(PciDevice("0002:02:00.0", "177d", "a063", netdevs=["rpm0"]))
    return FakePlatform("Marvell CN106", devs)


@pytest.fixture
def sysroot():
    d = tempfile.mkdtemp(prefix="sys", dir="/tmp")
    yield d
    shutil.rmtree(d, ignore_errors=True)


def test_marvell_utils(sysroot):
    u = MarvellUtils(marvell_platform(), FakeRunner(), sysroot)
    assert u.detect_platform_mode() == "dpu"
    assert u.mapped_vf(1, 0, 2) == "0002:1f:00.2"
    with pytest.raises(IndexError):
        u.mapped_vf(1, 0, 9)
    assert u.name_by_device_id("a063") == "rpm0"
    base = os.path.join(sysroot, "sys/bus/pci")
    os.makedirs(os.path.join(base, "devices/0002:1f:00.1"))
    os.makedirs(os.path.join(base, "drivers/rvu_nicvf"))
    u.bind_to_vfio("0002:1f:00.1", "rvu_nicvf")
    assert open(os.path.join(base, "devices/0002:1f:00.1/driver_override")).read() == "vfio-pci"
    assert open(os.path.join(base, "drivers_probe")).read() == "0002:1f:00.1"
    argv = cp_agent_command("/bin/dpu-cp-agent", "/etc/a.cfg", "/run/mbox", 49500, "dpi", "pem")
    assert argv == ["/bin/dpu-cp-agent", "/etc/a.cfg", "--mbox", "/run/mbox", "--plugin-port", "49500"]


def test_marvell_vsp_flows_match_reference_sequence(sysroot):
    nl, runner, ddp = FakeNetlink(), FakeRunner(), DebugDataPlane()
    vsp = MarvellVsp(marvell_platform(), nl, runner, ddp, sys_root=sysroot)
    ip, port = vsp.init(True, "")
    assert (ip, port) == ("[fe80::1%sdp0]", 8085)
    assert "ip addr replace fe80::1/64 dev sdp0 optimistic" in runner.commands()
    assert sorted(vsp.get_devices()) == ["nf_interface0", "nf_interface1"]
    vsp.create_bridge_port("host0-0", bytes.fromhex("02aa00000001"), 0, ["2"])
    macs = list(vsp.devices)
    vsp.create_network_function(macs[0], macs[1])
    flows = [o for o in ddp.ops if o[0] == "add_flow"]
    assert flows == [
        ("add_flow", "br-mrv0", "sdp1", "dp_interface0", ""),
        ("add_flow", "br-mrv0", "dp_interface0", "sdp1", M_A),
        ("add_flow", "br-mrv0", "dp_interface1", "dp_interface1", M_A),
        ("add_flow", "br-mrv0", "dp_interface1", "rpm0", ""),
        ("add_flow", "br-mrv0", "rpm0", "dp_interface1", ""),
    ]
    vsp.delete_bridge_port("host0-0")
    vsp.delete_network_function(macs[0], macs[1])
    assert ("del_port", "br-mrv0", "dp_interface1") in ddp.ops
    with pytest.raises(RuntimeError, match="not supported in DPU Mode"):
        vsp.set_num_vfs(4)


def test_marvell_vsp_on_gpu_dataplane(dp, sysroot):
    nl, runner = FakeNetlink(), FakeRunner()
    gdp = GpuOvsDataPlane(dp, uplink_name="rpm0")
    vsp = MarvellVsp(marvell_platform(), nl, runner, gdp, sys_root=sysroot)
    vsp.init(True, "")
    vsp.create_bridge_port("host0-0", bytes.fromhex("02aa00000001"), 0, ["2"])
    macs = list(vsp.devices)
    vsp.create_network_function(macs[0], macs[1])
    vf, nfin, nfout = (gdp.port_index(n) for n in ("sdp1", "dp_interface0", "dp_interface1"))
    assert send(dp, vf, M_GW)[0] == nfin
    assert send(dp, nfin, M_A)[0] == vf
    assert send(dp, nfout, M_A)[0] == nfout
    assert send(dp, nfout, M_GW)[0] == 4000
    assert send(dp, 4000, M_A)[0] == nfout
    vsp.delete_network_function(macs[0], macs[1])
    assert not dp.ports.valid(nfin)


def test_marvell_host_mode_set_num_vfs(sysroot):
    plat = FakePlatform("host", [PciDevice("0000:81:00.0", "177d", "b900", netdevs=["enp129s0"])])
    os.makedirs(os.path.join(sysroot, "sys/bus/pci/devices/0000:81:00.0"))
    vsp = MarvellVsp(plat, FakeNetlink(), FakeRunner(), DebugDataPlane(), sys_root=sysroot)
    assert vsp.init(False, "")[0] == "[fe80::1%25enp129s0]"
    for i in range(3):
        plat.add_pci(PciDevice(f"0000:81:00.{i + 1}", "177d", "b903", is_vf=True))
    assert vsp.set_num_vfs(3) == 3
    assert open(os.path.join(sysroot, "sys/bus/pci/devices/0000:81:00.0/sriov_numvfs")).read() == "3"
    assert sorted(vsp.get_devices()) == ["0000:81:00.1", "0000:81:00.2", "0000:81:00.3"]
    with pytest.raises(RuntimeError, match="expected number 5"):
        vsp.set_num_vfs(5)


# ------------------------------------------------------------------------------------ NetSec
def netsec_setup(sysroot, n_vfs=4):
    devs = [PciDevice("0000:f4:00.1", "8086", "124c", netdevs=["sfp1"]),
            PciDevice("0000:f4:00.2", "8086", "124c", netdevs=["bp2"])]
    plat = FakePlatform("netsec", devs)
    pf_dev = os.path.join(sysroot, "sys/class/net/bp2/device")
    os.makedirs(pf_dev)
    os.makedirs(os.path.join(sysroot, "sys/bus/pci/devices/0000:f4:00.2"))
    for i in range(n_vfs):
        pci = f"0000:f4:01.{i}"
        os.symlink(f"../../../../bus/pci/devices/{pci}", os.path.join(pf_dev, f"virtfn{i}"))
        plat.add_pci(PciDevice(pci, "8086", "1889", is_vf=True, netdevs=[f"bp2v{i}"]))
    nl = FakeNetlink()
    nl.add_link(Link(name="bp2"))
    return plat, nl


def test_netsec_vsp_dpu_side(dp, sysroot):
    plat, nl = netsec_setup(sysroot)
    runner = FakeRunner()
    vsp = NetsecVsp(plat, nl, runner, dp, sys_root=sysroot)
    assert vsp.init(True, "") == ("[fe80::1%bp2]", 8085)
    assert vsp.set_num_vfs(4) == 4
    vfs = nl.link_by_name("bp2").vfs
    assert [(v.vlan, v.spoofchk, v.trust) for v in vfs] == [(i + 2, False, True) for i in range(4)]
    vsp.create_bridge_port("host0-1", bytes.fromhex("02aa00000001"), 0, [])
    idx = vsp._ports["bp2v1"]
    pe = dp.ports.a[idx]
    assert pe["vlan"] == 3 and pe["flags"] & T.PORT_VLAN_ISOLATE and pe["flags"] & T.PORT_TAG_EGRESS
    with pytest.raises(ValueError, match="PFID 1"):
        vsp.create_bridge_port("host1-0", b"", 0, [])
    # NF steering (implemented here; a TODO in the reference)
    vsp.create_network_function(vsp.veths[0].if_mac, vsp.veths[1].if_mac)
    nfin, nfout = vsp._ports["dp_interface0"], vsp._ports["dp_interface1"]
    assert send(dp, idx, M_GW)[0] == nfin
    op, reason, out = send(dp, nfin, M_A)
    assert (op, reason) == (idx, 0) and out[12] == 0x81 and out[15] == 3  # tagged with vf+2
    assert send(dp, 4000, M_A)[0] == nfout
    vsp.delete_network_function(vsp.veths[0].if_mac, vsp.veths[1].if_mac)
    vsp.delete_bridge_port("host0-1")
    assert not dp.ports.valid(idx)
    assert sorted(vsp.get_devices()) == ["nf_interface0", "nf_interface1"]


def test_netsec_vsp_host_side(sysroot):
    plat = FakePlatform("host", [PciDevice("0000:17:00.0", "8086", "1599", serial="abc", netdevs=["ens1f0"]),
                                 PciDevice("0000:17:00.1", "8086", "1599", serial="abc", netdevs=["ens1f1"]),
                                 PciDevice("0000:17:02.0", "8086", "1889", is_vf=True),
                                 PciDevice("0000:18:02.0", "8086", "1889", is_vf=True)])
    os.makedirs(os.path.join(sysroot, "sys/bus/pci/devices/0000:17:00.0"))
    runner = FakeRunner()
    vsp = NetsecVsp(plat, FakeNetlink(), runner, None, sys_root=sysroot)
    assert vsp.init(False, "abc")[0] == "[fe80::1%25ens1f0]"
    assert vsp.dpu_pcie == "0000:17:00.0"
    assert list(vsp.get_devices()) == ["0000:17:02.0"]  # VFs on the card's bus only
    with pytest.raises(LookupError):
        NetsecVsp(plat, FakeNetlink(), runner, None, sys_root=sysroot).init(False, "nope")


def test_vsp_common_helpers(sysroot):
    r = FakeRunner(responses={("ip", "-d", "link", "show"): (0, "... addrgenmode eui64 ...")})
    os.makedirs(os.path.join(sysroot, "proc/sys/net/ipv6/conf/eth9"))
    common.enable_ipv6_link_local(r, "eth9", "fe80::2", sysroot)
    cmds = r.commands()
    assert not any("addrgenmode eui64" in c and c.startswith("ip link set") for c in cmds)
    assert cmds[-1] == "ip addr replace fe80::2/64 dev eth9 optimistic"
    assert open(os.path.join(sysroot, "proc/sys/net/ipv6/conf/eth9/optimistic_dad")).read() == "1"
    r2 = FakeRunner(responses={("nsenter",): (1, "no NetworkManager")})
    common.enable_ipv6_link_local(r2, "eth9", "fe80::2", sysroot)  # nmcli failure tolerated
    assert "ip link set eth9 addrgenmode eui64" in r2.commands()
    nl = FakeNetlink()
    pair = common.create_nf_veth_pair(nl, 3)
    assert (pair.ifname, pair.peer) == ("nf_interface3", "dp_interface3") and nl.link_by_name("dp_interface3").up
    assert common.create_nf_veth_pair(nl, 3).if_mac == pair.if_mac  # idempotent
    common.destroy_veth_pair(nl, pair)
    with pytest.raises(KeyError):
        nl.link_by_name("dp_interface3")
