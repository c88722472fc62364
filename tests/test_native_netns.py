"""Kernel-netdev pods on the native I/O engine (csrc/nfdp/iox.cpp PacketPort / FdPort): real network
namespaces, one per pod, each holding the pod end of a veth pair (AF_PACKET TPACKET_V2 rings on the
data-plane end) or a TAP netdev (its fd kept by the engine).  Pods put the SFC's frames on their
interfaces with raw sockets; what comes out on every pod must be, byte for byte, what the batch
path of an identical data plane makes of the same frames.

(The deployed product path, daemon + device plugin + CNI + GPU VSP with a wire port and an NF pod,
is tests/test_deployed_node.py.)  Skipped without CAP_NET_ADMIN / CAP_SYS_ADMIN (namespaces, veth, TAP)."""
import os
import time

import numpy as np
import pytest

from dpu_operator_amd.testutils import netns as NS

pytestmark = pytest.mark.skipif(not NS.privileged(), reason="needs CAP_NET_ADMIN + CAP_SYS_ADMIN (netns, veth, TAP)")


def _until(fn, t=10.0):
    end = time.monotonic() + t
    while time.monotonic() < end:
        v = fn()
        if v:
            return v
        time.sleep(0.005)
    return fn()


def _expected(ref, slots, im):
    from dpu_operator_amd.ops import packets as P

    r = ref.run(slots, im)
    port, _, reason = P.meta_fields(r.meta)
    lens = im >> 16
    exp: dict[int, list[bytes]] = {}
    for i in np.nonzero(reason == 0)[0]:
        exp.setdefault(int(port[i]), []).append(P.assemble(r.out[i], int(r.meta[i]), slots[i], int(lens[i])))
    return exp


@pytest.mark.parametrize("kind", ["veth", "tap", "xdp"])
def test_netns_pods_through_the_native_engine_bit_exact(kind):
    from dpu_operator_amd.cni.netlink import RtNetlink
    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.dataplane.native_io import NativeLivePath, PacketVport, XdpVport
    from dpu_operator_amd.dataplane.netio import TapPort

    nl = RtNetlink()
    tag = {"veth": "v", "tap": "t", "xdp": "x"}[kind]
    n_pods = 4
    dp = DataPlane(device="cpu", flow_buckets=1 << 12)
    sc = S.build_sfc(dp, n_pods=n_pods, n_flows=2048, n_acl=32, seed=0)
    dp.commit(full=True)
    ref = DataPlane(device="cpu", flow_buckets=1 << 12)
    S.build_sfc(ref, n_pods=n_pods, n_flows=2048, n_acl=32, seed=0)
    ref.commit(full=True)
    ports, pods, taps, vps = {}, {}, [], []
    live = None
    try:
        for i in range(n_pods):
            name = f"nn{tag}{os.getpid() % 1000}p{i}"
            if kind in ("veth", "xdp"):   # (xdp: the engine's ends through AF_XDP, iox.h XdpPort)
                vp = (XdpVport if kind == "xdp" else PacketVport).create_veth(nl, name)
                vps.append(vp)
                ports[int(sc.pod_port[i])] = vp
            else:
                t = TapPort(name)
                nl.link_set_up(name)
                taps.append(t)
                ports[int(sc.pod_port[i])] = t
            pods[int(sc.pod_port[i])] = NS.RawPod(f"{name}-ns", name, nl)
        live = NativeLivePath(dp, ports, burst=64, ring_capacity=1024, queues=2).start()
        slots, im = S.traffic(sc, 1200, seed=4)
        exp = _expected(ref, slots, im)
        src = im & 0xFFFF
        for p, pod in pods.items():
            fr = [bytes(slots[k, : int(im[k] >> 16)]) for k in np.nonzero(src == p)[0]]
            # the kernel's queues are finite (socket, per-CPU backlog behind a TAP write): pace, so
            # a loaded box (parallel test workers) cannot make it drop
            for k in range(0, len(fr), 32):
                assert pod.send(fr[k:k + 32]) == len(fr[k:k + 32])
                time.sleep(0.002)
        got = {p: [] for p in pods}

        def done():
            for p, pod in pods.items():
                got[p] += pod.recv()
            return all(len(got[p]) >= len(exp.get(p, [])) for p in pods)

        assert _until(done, 30.0), ({p: (len(got[p]), len(exp.get(p, []))) for p in pods}, live.stats, live.error)
        for p, frames in exp.items():
            rest = list(got[p])
            for f in frames:        # every expected frame arrived, bit for bit (nothing else was sent)
                assert f in rest, p
                rest.remove(f)
            assert not rest, (p, len(rest))
        assert live.error is None
        # (>=: a netdev's kernel may emit a few frames of its own - IPv6 DAD / MLD before the
        # pod's IPv6 is off - which the engine reads too and the pipeline drops or punts)
        assert live.stats["rx"] >= len(slots)
    finally:
        if live is not None:
            live.stop()
        for pod in pods.values():
            pod.close()
        for t in taps:
            t.close()
        for vp in vps:
            vp.close()


@pytest.mark.parametrize("mode", ["linux-bridge", "engine"])
def test_veth_comparator_same_generator(mode):
    """tools/live_bench.py --veth: netns pods on veth pairs driven by the C++ generator / sink
    (trafgen_pkt.h, AF_PACKET rings opened inside each namespace), switched by a Linux bridge
    (the comparator) or by the native engine; every measured frame carries a valid send time and
    the report has loaded / half-load / idle latency."""
    import importlib.util

    spec = importlib.util.spec_from_file_location(
        "live_bench", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "live_bench.py"))
    lb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lb)
    r = lb.run_veth(mode, n_pods=3, duration=0.5, threads=1, queues=1)   # (long enough on a loaded box)
    assert r["switch"] == mode and r["mpps"] > 0 and r["p50_us"] is not None
    assert r["half_p99_us"] is not None and r["idle_p50_us"] is not None
    if mode == "engine":
        assert r["error"] is None and r["engine"]["rx"] > 0


@pytest.mark.parametrize("planes", [1, 2])
def test_marvell_ovs_bridge_live_on_the_native_engine(planes):
    """The Marvell VSP's OvS bridge on the GPU data plane with live I/O (`vsp --vendor marvell
    --live [--gpus N]`): every OvS port that is a netdev joins the native engine as an AF_PACKET
    port, OpenFlow rules program the tables, frames from one netns pod reach the other only where a
    rule sends them; with two planes (MultiDataPlane) the flows and rules span both."""
    from dpu_operator_amd.cni.netlink import RtNetlink
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.dataplane.multi import MultiDataPlane
    from dpu_operator_amd.dataplane.native_io import NativeLivePath, PacketVport
    from dpu_operator_amd.vsp.marvell import GpuOvsDataPlane

    nl = RtNetlink()
    dp = MultiDataPlane(["cpu"] * planes, flow_buckets=1 << 10) if planes > 1 else DataPlane(device="cpu", flow_buckets=1 << 10)
    dp.commit(full=True)
    tag = f"mv{planes}{os.getpid() % 1000}"
    vps, pods = [], []
    ovs = GpuOvsDataPlane(dp, live_factory=lambda d: NativeLivePath(d, {}, burst=64, ring_capacity=1024, queues=2).start())
    try:
        names = [f"{tag}a", f"{tag}b"]
        for n in names:
            vp = PacketVport.create_veth(nl, n)       # pod end n, bridge end n + "d"
            vps.append(vp)
            pods.append(NS.RawPod(f"{n}-ns", n, nl))
        ovs.init_data_plane("br-test")
        for n in names:
            ovs.add_port("br-test", n + "d")
        a, b = ovs.port_index(names[0] + "d"), ovs.port_index(names[1] + "d")
        assert ovs.live is not None and ovs.live.port(a) is not None and ovs.live.port(b) is not None
        ovs.add_flow_rule("br-test", names[0] + "d", names[1] + "d")      # a -> b only
        frame = bytes.fromhex("02000000000b" "02000000000a" "0800") + bytes(46)
        frames = [frame[:-1] + bytes([i]) for i in range(20)]
        assert pods[0].send(frames) == 20
        got = []
        assert _until(lambda: got.extend(pods[1].recv()) or len(got) >= 20, 5.0), (len(got), ovs.live.stats)
        assert sorted(got) == sorted(frames)
        assert pods[1].send(frames[:5]) == 5          # b -> a: no rule, nothing arrives
        time.sleep(0.3)
        assert pods[0].recv() == []
        ovs.delete_port("br-test", names[1] + "d")
        assert ovs.live.port(b) is None
    finally:
        ovs.close()
        for p in pods:
            p.close()
        for v in vps:
            v.close()
