"""The deployed MI355X node, end to end, with real traffic (the reference's e2e traffic suite,
e2e_test/e2e_test.go:399-512, on one node).

What the daemon deploys is what runs: the GPU VSP is built from `Mi355xDetector().vsp()`'s own
argument list (`--live --live-engine native --gpus all --uplink <node config>`: veth vports, the
native I/O engine, the resident ring kernel on every GPU, a wire port), behind the node daemon,
the device plugin and the CNI server.  Around it, network namespaces stand in for the pods and the
external host:

  pod0, pod1     workload pods: a vport each (device plugin Allocate, CNI ADD moves the netdev in,
                 CreateBridgePort programs it), addresses 10.97.0.1 / .2
  ext            the external host, on the far end of the wire port (the uplink veth's host end
                 moved into it), 10.97.1.200
  nf             an SFC network-function pod: two vports (CNI ADD in the operator namespace,
                 CreateNetworkFunction on the second MAC), a bump-in-the-wire forwarder between
                 them, net1 10.97.0.3 (toward the pods) and net2 10.97.2.3 (toward the wire)

Checks (each a key of the result):
  pod_pod, pod_pod_udp        pod <-> pod before any NF (ICMP both ways; a UDP datagram through
                              both kernels' UDP stacks, so checksums are verified on receipt)
  pod_ext, ext_pod, ext_udp   pod <-> external through the wire port (learned external MAC)
  nf_pod_pod                  pod <-> pod with the NF deployed (hairpin through the NF)
  pod_nf, nf_pod              pod <-> the NF's pod-side interface
  nf_ext                      NF -> external out of its wire-side interface
  pod_ext_nf                  pod -> external through the NF (frames counted by the forwarder)
  after_nf_del                pod <-> pod after the NF pod's CNI DEL (plain bridge again)

`python -m dpu_operator_amd.testutils.deployed --device cuda:0 --json` runs it and prints one
JSON line; without CAP_NET_ADMIN it can run in a user + network + mount namespace of its own
(`unshare -Urnm`, what `tests/test_deployed_node.py` does on the GPU box, where tests run as an
ordinary user): namespaces are then bound under DPU_NETNS_DIR.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import threading
import time


def _wait(fn, t: float = 10.0, step: float = 0.02):
    end = time.monotonic() + t
    while time.monotonic() < end:
        v = fn()
        if v:
            return v
        time.sleep(step)
    return fn()


def run(device: str = "cpu", queues: int = 2, log=None) -> dict:
    from .. import vars as V
    from ..cmd import vsp as vspcmd
    from ..cni.netlink import RtNetlink
    from ..config import NodeConfig, node_config, set_node_config
    from ..daemon.daemon import Daemon
    from ..k8s.apiserver import ApiServer
    from ..platform.detectors import Mi355xDetector
    from ..platform.platform import FakePlatform, PciDevice
    from ..utils.fileutils import touch
    from ..utils.paths import PathManager
    from . import netns as NS
    from .kubelet import FakeKubelet, cni_call

    say = log or (lambda *_: None)
    tag = f"{os.getpid() % 1000}"
    root = tempfile.mkdtemp(prefix="dpdep", dir="/tmp")
    pm = PathManager(root)
    nl = RtNetlink()
    saved = node_config()
    set_node_config(NodeConfig(**{**saved.__dict__, "uplink": "veth", "uplink_host_ifname": f"dw{tag}"}))
    res: dict = {"device": device, "queues": queues}
    gvsp = kubelet = d = nf = None
    nss: list[str] = []
    try:
        args = list(Mi355xDetector().vsp(True).args)
        res["vsp_args"] = args
        a = vspcmd.parse_args(args + ["--device", device, "--flow-buckets", "4096", "--root", root,
                                      "--io-queues", str(queues)])
        gvsp = vspcmd.build_vsp(a, pm)
        gvsp.prefix = f"d{tag}p"
        assert gvsp.live and gvsp.live_engine == "native" and gvsp.vport_kind == "veth", "not the deployed live path"
        touch(pm.wrap("/dpu-cni"))
        api = ApiServer()
        kubelet = FakeKubelet(pm, api).start()
        gvsp.start()
        plat = FakePlatform("AMD server", [PciDevice("0000:05:00.0", "1002", "75a3", class_code=0x120000)])
        d = Daemon(plat, "auto", api, None, pm, nl=nl, tick=0.05, manager_kw={"dp_poll": 0.05})
        threading.Thread(target=d.serve, daemon=True).start()
        assert _wait(lambda: kubelet.allocatable() == 8, 30), f"devices never advertised: {kubelet.devices}"
        lp = gvsp.livepath
        res["ring_on_gpu"] = bool(lp.gpu)
        sock = pm.cni_server_path()
        host_if = node_config().uplink_host_ifname

        def ns(name):
            p = NS.create_netns(NS.netns_path(f"{name}{tag}"))
            nss.append(p)
            return p

        def add(dev, netns, ifname, pod_ns, pod_name, cid):
            conf = {"cniVersion": "0.4.0", "name": "dpucni", "type": "dpucni", "deviceID": dev}
            return cni_call(sock, "ADD", conf, netns=netns, ifname=ifname, pod_ns=pod_ns, pod_name=pod_name,
                            container_id=cid)

        def delete(dev, netns, ifname, pod_ns, pod_name, cid):
            conf = {"cniVersion": "0.4.0", "name": "dpucni", "type": "dpucni", "deviceID": dev}
            return cni_call(sock, "DEL", conf, netns=netns, ifname=ifname, pod_ns=pod_ns, pod_name=pod_name,
                            container_id=cid)

        # --- workload pods
        devs = [f"{gvsp.prefix}0", f"{gvsp.prefix}1"]
        envs = kubelet.allocate(devs).container_responses[0].envs
        assert envs["NF-DEV"] == ",".join(devs) + ",", envs
        pods = []
        for i, dev in enumerate(devs):
            p = ns(f"pod{i}-")
            pods.append(p)
            add(dev, p, "eth1", "default", f"pod{i}", f"c{i}")
            nl.addr_add("eth1", f"10.97.0.{i + 1}/16", p)
        assert _wait(lambda: {"host0-0", "host0-1"} <= set(gvsp.bridge_ports), 10), gvsp.bridge_ports
        # --- the external host behind the wire port
        ext = ns("ext-")
        nl.link_set_ns(host_if, ext)
        nl.link_set_up("lo", ext)
        nl.addr_add(host_if, "10.97.1.200/16", ext)
        nl.link_set_up(host_if, ext)
        say("pods and external host up")

        def ping(src, dst, dev=None):
            return NS.ping(src, dst, timeout=5, dev=dev) is not None

        res["pod_pod"] = ping(pods[0], "10.97.0.2") and ping(pods[1], "10.97.0.1")
        res["pod_pod_udp"] = NS.udp_exchange(pods[0], pods[1], "10.97.0.2", os.urandom(1200)) is not None
        res["pod_ext"] = ping(pods[0], "10.97.1.200")
        res["ext_pod"] = ping(ext, "10.97.0.2")
        res["ext_udp"] = NS.udp_exchange(ext, pods[0], "10.97.0.1", os.urandom(900), port=47001) is not None
        say("plain bridge", {k: res[k] for k in ("pod_pod", "pod_pod_udp", "pod_ext", "ext_pod", "ext_udp")})
        # --- the SFC's network function pod: two vports, CreateNetworkFunction on the second MAC
        nfdevs = [f"{gvsp.prefix}2", f"{gvsp.prefix}3"]
        kubelet.allocate(nfdevs)
        nfns = ns("nf-")
        for i, dev in enumerate(nfdevs):
            add(dev, nfns, f"net{i + 1}", V.NAMESPACE, "nf", "cnf")
        assert _wait(lambda: len(gvsp.nfs) == 1, 10), gvsp.nfs
        nf = NS.WireNF("", "net1", "net2", nl, existing_ns=nfns)
        nl.link_set_up("lo", nfns)
        nl.addr_add("net1", "10.97.0.3/16", nfns)
        nl.addr_add("net2", "10.97.2.3/16", nfns)
        res["nf_pod_pod"] = ping(pods[0], "10.97.0.2") and ping(pods[1], "10.97.0.1")
        res["pod_nf"] = ping(pods[0], "10.97.0.3") and ping(pods[1], "10.97.0.3")
        res["nf_pod"] = ping(nfns, "10.97.0.1", dev="net1") and ping(nfns, "10.97.0.2", dev="net1")
        res["nf_ext"] = ping(nfns, "10.97.1.200", dev="net2")
        before = nf.forwarded
        res["pod_ext_nf"] = ping(pods[0], "10.97.1.200") and ping(pods[1], "10.97.1.200")
        res["nf_forwarded"] = nf.forwarded - before
        res["pod_ext_nf"] = res["pod_ext_nf"] and res["nf_forwarded"] > 0
        say("with the NF", {k: res[k] for k in ("nf_pod_pod", "pod_nf", "nf_pod", "nf_ext", "pod_ext_nf")})
        nf.close()
        nf = None
        for i, dev in enumerate(nfdevs):
            delete(dev, nfns, f"net{i + 1}", V.NAMESPACE, "nf", "cnf")
        assert _wait(lambda: not gvsp.nfs, 10), gvsp.nfs
        res["after_nf_del"] = ping(pods[0], "10.97.0.2")
        for i, dev in enumerate(devs):
            delete(dev, pods[i], "eth1", "default", f"pod{i}", f"c{i}")
        assert _wait(lambda: not gvsp.bridge_ports, 10), gvsp.bridge_ports
        st = lp.stats
        res["engine"] = {k: int(st.get(k, 0)) for k in ("rx", "tx", "drop", "replicas", "learn_events", "queues")}
        res["error"] = lp.error
        checks = ["pod_pod", "pod_pod_udp", "pod_ext", "ext_pod", "ext_udp", "nf_pod_pod", "pod_nf", "nf_pod",
                  "nf_ext", "pod_ext_nf", "after_nf_del"]
        res["ok"] = all(bool(res.get(k)) for k in checks) and lp.error is None
        return res
    finally:
        if nf is not None:
            nf.close()
        if d is not None and hasattr(d, "stop"):
            d.stop()
        if kubelet is not None:
            kubelet.stop()
        if gvsp is not None:
            gvsp.stop_live()
        for p in nss:
            NS.delete_netns(p)
        set_node_config(saved)
        shutil.rmtree(root, ignore_errors=True)


def run_memif(device: str = "cpu", queues: int = 2, log=None) -> dict:
    """The same node and checks without kernel netdevs (the GPU box runs tests with no
    CAP_NET_ADMIN and no user namespaces): the detector's VSP arguments with shared-memory vports
    and a shared-memory wire (`--vport-kind memif --uplink memif`) on `device`, the VSP's RPCs as
    the daemon's CNI / OPI paths issue them, and memif endpoints as pods, external host and NF
    (which forwards what arrives on its ingress vport to its egress vport).  Frames are IPv4 / UDP
    between the pods' MACs; every check asserts exactly which endpoints receive them, unchanged."""
    import numpy as np

    from ..cmd import vsp as vspcmd
    from ..native import nfdp
    from ..ops import packets as P
    from ..platform.detectors import Mi355xDetector
    from ..utils.paths import PathManager

    say = log or (lambda *_: None)
    nf = nfdp()
    root = tempfile.mkdtemp(prefix="dpdepm", dir="/tmp")
    pm = PathManager(root)
    res: dict = {"device": device, "queues": queues, "vports": "memif"}
    gvsp = None
    try:
        args = list(Mi355xDetector().vsp(True).args)
        a = vspcmd.parse_args(args + ["--device", device, "--flow-buckets", "4096", "--root", root,
                                      "--io-queues", str(queues), "--vport-kind", "memif", "--uplink", "memif"])
        res["vsp_args"] = args + ["--vport-kind", "memif", "--uplink", "memif"]
        gvsp = vspcmd.build_vsp(a, pm)
        gvsp.init(True, "gpu")
        gvsp.set_num_vfs(8)
        lp = gvsp.livepath
        res["ring_on_gpu"] = bool(lp.gpu)
        mac = {i: gvsp.vports[i]["mac"] for i in range(8)}
        # workload pods on vports 0 / 1 (CreateBridgePort with the vport's own MAC), NF on 2 / 3
        for i in (0, 1):
            gvsp.create_bridge_port(f"host0-{i}", bytes.fromhex(mac[i].replace(":", "")), 0, [str(i + 2)])
        ep = {i: nf.MemifEndpoint(gvsp.vport_path(i)) for i in range(4)}
        wire = nf.MemifEndpoint(gvsp._wire_vport().path)
        EXT = "02:ee:00:00:00:01"

        def frames(src, dst, n, sport0):
            fr, ln = P.craft(n, dmac=dst, smac=src, src_ip=0x0A610001, dst_ip=0x0A610002,
                             sport=np.arange(n) + sport0, dport=4789 + 1)
            return [bytes(fr[k, : ln[k]]) for k in range(n)]

        def deliver(sender, fr, want: dict, quiet_s: float = 0.15) -> bool:
            """send `fr` from endpoint `sender`; True when exactly `want` ({endpoint: frames})
            arrive (every other endpoint gets nothing)."""
            every = {**{k: v for k, v in ep.items()}, "wire": wire}
            for e in every.values():
                e.recv()
            assert sender.send(fr) == len(fr)
            got = {k: [] for k in every}
            end = time.monotonic() + 10
            while time.monotonic() < end:
                for k, e in every.items():
                    got[k] += e.recv()
                if all(len(got[k]) >= len(v) for k, v in want.items()):
                    break
                time.sleep(0.002)
            time.sleep(quiet_s)
            for k, e in every.items():
                got[k] += e.recv()
            ok = all(sorted(got[k]) == sorted(want.get(k, [])) for k in every)
            if not ok:
                say("mismatch", {k: (len(got[k]), len(want.get(k, []))) for k in every})
            return ok

        f01 = frames(mac[0], mac[1], 64, 1000)
        res["pod_pod"] = deliver(ep[0], f01, {1: f01}) and deliver(ep[1], frames(mac[1], mac[0], 64, 2000),
                                                                      {0: frames(mac[1], mac[0], 64, 2000)})
        # an unknown destination floods (wire first, then the other VFs); the external host's reply
        # teaches the wire port its MAC, after which pod -> external is forwarded to the wire only
        fx = frames(mac[0], EXT, 8, 3000)
        res["pod_ext_flood"] = deliver(ep[0], fx, {"wire": fx, 1: fx})
        fr = frames(EXT, mac[0], 8, 4000)
        res["ext_pod"] = deliver(wire, fr, {0: fr})
        lp.flush_learning()
        time.sleep(0.05)
        fx2 = frames(mac[0], EXT, 32, 5000)
        res["pod_ext_learned"] = deliver(ep[0], fx2, {"wire": fx2})
        # the SFC's network function on vports 2 (in) / 3 (out)
        gvsp.create_network_function(mac[2], mac[3])
        fn = frames(mac[0], EXT, 32, 6000)
        res["pod_to_nf_in"] = deliver(ep[0], fn, {2: fn})
        res["nf_out_to_ext"] = deliver(ep[3], fn, {"wire": fn})         # the NF passed them on
        fb = frames(EXT, mac[1], 16, 7000)
        res["ext_to_nf_out"] = deliver(wire, fb, {3: fb})
        res["nf_in_to_pod"] = deliver(ep[2], fb, {1: fb})              # (NF-in bridge, pod MAC) -> VF
        fp = frames(mac[0], mac[1], 16, 8000)
        res["nf_pod_pod_via_nf"] = deliver(ep[0], fp, {2: fp})          # pod -> pod enters the NF too
        res["nf_hairpin"] = deliver(ep[3], fp, {3: fp})                # NF-out, dst pod MAC: hairpin
        gvsp.delete_network_function(mac[2], mac[3])
        fz = frames(mac[0], mac[1], 16, 9000)
        res["after_nf_del"] = deliver(ep[0], fz, {1: fz})
        st = lp.stats
        res["engine"] = {k: int(st.get(k, 0)) for k in ("rx", "tx", "drop", "replicas", "learn_events", "queues")}
        res["error"] = lp.error
        checks = ["pod_pod", "pod_ext_flood", "ext_pod", "pod_ext_learned", "pod_to_nf_in", "nf_out_to_ext",
                  "ext_to_nf_out", "nf_in_to_pod", "nf_pod_pod_via_nf", "nf_hairpin", "after_nf_del"]
        res["checks"] = checks
        res["ok"] = all(bool(res.get(k)) for k in checks) and lp.error is None
        return res
    finally:
        if gvsp is not None:
            gvsp.stop_live()
        shutil.rmtree(root, ignore_errors=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="deployed")
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--queues", type=int, default=2)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    if "DPU_NETNS_DIR" in os.environ:
        # a namespace of our own (unshare -Urnm): its loopback starts down, and the daemon's host
        # side reaches the device side's OPI server over 127.0.0.1
        os.makedirs(os.environ["DPU_NETNS_DIR"], exist_ok=True)
        from ..cni.netlink import RtNetlink

        RtNetlink().link_set_up("lo")
    res = run(a.device, a.queues, log=(lambda *x: print(*x, file=sys.stderr, flush=True)))
    print(json.dumps(res) if a.json else res, flush=True)
    return 0 if res.get("ok") else 1


if __name__ == "__main__":
    sys.exit(main())
