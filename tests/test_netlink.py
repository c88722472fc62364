"""Production netlink (cni/netlink.py RtNetlink) and the in-memory model (FakeNetlink) implement
the whole NetlinkManager interface; IFLA_VF_* encoding; privileged round trips against the real
kernel (veth, netns move, addresses, MTU, alias, delete) and GARP sent from inside a pod netns
(SR6), skipped without CAP_NET_ADMIN / CAP_SYS_ADMIN."""
import socket
import struct

import pytest

from dpu_operator_amd.cni import netlink as N
from dpu_operator_amd.testutils import netns as NS


def _ops():
    return [n for n, v in vars(N.NetlinkManager).items() if callable(v) and not n.startswith("_")]


@pytest.mark.parametrize("cls", [N.RtNetlink, N.FakeNetlink])
def test_every_operation_is_implemented(cls):
    missing = [n for n in _ops() if getattr(cls, n) is getattr(N.NetlinkManager, n)]
    assert not missing, f"{cls.__name__} does not implement {missing}"
    assert len(_ops()) >= 14


def test_base_class_refuses_silently():
    with pytest.raises(NotImplementedError):
        N.NetlinkManager().addr_add("x", "10.0.0.1/24")


def test_vf_attribute_encoding(monkeypatch):
    nl = N.RtNetlink()
    sent = {}
    monkeypatch.setattr(nl, "link_by_name", lambda name, ns="": N.Link(name=name, index=7))
    monkeypatch.setattr(nl, "_link_msg", lambda t, f, idx=0, fl=0, ch=0, attrs=b"": sent.update(t=t, idx=idx, a=attrs) or [])
    nl.link_set_vf("pf0", 3, mac="02:00:00:00:00:09", vlan=2, qos=1, spoofchk=False, trust=True,
                   min_tx_rate=10, max_tx_rate=100, link_state=2)
    assert sent["t"] == N.RTM_NEWLINK and sent["idx"] == 7
    a = sent["a"]
    ln, t = struct.unpack_from("HH", a, 0)
    assert t == N.IFLA_VFINFO_LIST | N.NLA_F_NESTED and ln == len(a)
    inner = dict((t2, v) for t2, v in nl._attrs(a[4:], 4))  # children of IFLA_VF_INFO
    assert struct.unpack("I", inner[N.IFLA_VF_MAC][:4])[0] == 3 and inner[N.IFLA_VF_MAC][4:10] == bytes.fromhex("020000000009")
    assert struct.unpack("III", inner[N.IFLA_VF_VLAN]) == (3, 2, 1)
    assert struct.unpack("II", inner[N.IFLA_VF_SPOOFCHK]) == (3, 0)
    assert struct.unpack("II", inner[N.IFLA_VF_TRUST]) == (3, 1)
    assert struct.unpack("III", inner[N.IFLA_VF_RATE]) == (3, 10, 100)
    assert struct.unpack("II", inner[N.IFLA_VF_LINK_STATE]) == (3, 2)
    with pytest.raises(AttributeError):
        nl.link_set_vf("pf0", 0, bogus=1)


priv = pytest.mark.skipif(not NS.privileged(), reason="needs CAP_NET_ADMIN + CAP_SYS_ADMIN")


@priv
def test_real_kernel_round_trip():
    nl = N.RtNetlink()
    ns = N.create_netns("/var/run/netns/nlt-pod")
    try:
        nl.link_add_veth("nltA", "nltB")
        assert nl.link_by_name("nltA").kind == "veth"
        nl.link_set_ns("nltB", ns)
        assert "nltB" in [x.name for x in nl.link_list(ns)] and "nltB" not in [x.name for x in nl.link_list()]
        nl.link_set_name("nltB", "eth7", ns)
        nl.link_set_alias("eth7", "nltB", ns)
        nl.link_set_mtu("eth7", 9000, ns)
        nl.link_set_hw_addr("eth7", "02:11:22:33:44:55", ns)
        nl.addr_add("eth7", "10.95.0.2/24", ns)
        nl.link_set_up("eth7", ns)
        l7 = nl.link_by_name("eth7", ns)
        assert (l7.alias, l7.mtu, l7.mac, l7.up) == ("nltB", 9000, "02:11:22:33:44:55", True)
        assert "10.95.0.2/24" in nl.addr_list("eth7", ns)
        nl.link_set_down("eth7", ns)
        assert not nl.link_by_name("eth7", ns).up
        nl.link_del("nltA")
        assert "eth7" not in [x.name for x in nl.link_list(ns)]  # the peer goes with it
    finally:
        N.delete_netns(ns)


@priv
def test_garp_is_sent_inside_the_pod_namespace():
    from dpu_operator_amd.cni.sriov.packet import announce

    nl = N.RtNetlink()
    ns = N.create_netns("/var/run/netns/nlt-garp")
    try:
        nl.link_add_veth("garpH", "garpP")
        nl.link_set_ns("garpP", ns)
        nl.link_set_up("garpH")
        nl.link_set_up("garpP", ns)
        rx = socket.socket(socket.AF_PACKET, socket.SOCK_RAW, socket.htons(0x0806))
        rx.bind(("garpH", 0))
        rx.settimeout(2)
        mac = nl.link_by_name("garpP", ns).mac
        assert nl.run_in_ns(ns, lambda: announce("garpP", mac, ["10.95.1.7/24"])) == 1
        assert announce("garpP", mac, ["10.95.1.7/24"]) == 0  # not in the daemon's namespace
        f = rx.recv(2048)
        assert f[12:14] == b"\x08\x06" and socket.inet_ntoa(f[28:32]) == "10.95.1.7" and f[6:12].hex() == mac.replace(":", "")
        rx.close()
    finally:
        try:
            nl.link_del("garpH")
        except Exception:
            pass
        N.delete_netns(ns)
