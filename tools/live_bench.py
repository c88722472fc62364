"""Live pod-to-pod benchmark of the native packet path (csrc/nfdp/iox + memif vports).

Pods are shared-memory vports (csrc/nfdp/memif.h) driven by the C++ generator / sink
(csrc/nfdp/trafgen.h: every frame carries its send time, so one-way pod -> pod latency is read on
one clock).  Between them: the native I/O engine and the headline pipeline (1M flows, 256-rule
ACL -> SNAT -> L2 steer) on the persistent ring kernel of the GPU, or the C++ oracle on the CPU
(`--device cpu`, the comparator: same I/O engine, CPU pipeline), or nothing at all (`--backend wire`:
a zero-cost pipeline that forwards every frame by destination MAC — the ceiling of the I/O engine
and the pods themselves, what any pipeline behind the engine is held to).

Measured, per device:
  * `mpps`          : aggregate frames delivered per second with every pod sending as fast as its
                      vport accepts (64-B frames, 8 pods, random pod -> pod flows);
  * `p50/p99_us`    : one-way latency of that saturated run (queueing in the pod rings included);
  * `loaded_*`      : closed loop with `loaded_window` frames in flight: saturated throughput with
                      the queueing bounded (the loaded latency);
  * `idle_p50/p99`  : closed loop, one frame in flight (the unloaded pod -> pod latency);
  * `load90_*`, `half_*` : offered load at 90 % / 50 % of the measured maximum.

    python tools/live_bench.py [--device cuda|cpu] [--duration 1.0] [--flows 1048576]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.dataplane.native_io import MemifVport, NativeLivePath, memif_dir  # noqa: E402
from dpu_operator_amd.native import nfdp  # noqa: E402
from dpu_operator_amd.utils import cpuquota  # noqa: E402


def _pct(x, q):
    return round(float(np.percentile(x, q)), 2) if len(x) else None


def drain(nf, pods, stats, quiet_s: float = 0.05, limit_s: float = 10.0) -> int:
    """Let the engine deliver what the previous phase left queued; empty the pods' rx rings."""
    eps = [nf.MemifEndpoint(p[0]) for p in pods]
    n, last, t_end = 0, time.perf_counter(), time.perf_counter() + limit_s
    prev = stats().get("tx", 0)
    while time.perf_counter() < t_end:
        k = sum(len(e.recv()) for e in eps)
        cur = stats().get("tx", 0)
        n += k
        if k or cur != prev:
            last, prev = time.perf_counter(), cur
        elif time.perf_counter() - last > quiet_s:
            break
        time.sleep(0.002)
    return n


class _WireLive:
    """The I/O engine over a zero-cost pipeline (nf.WireBackend): pods are port i, MAC 02:00:00:00:00:i+1."""

    def __init__(self, nf, d: str, n_pods: int, burst: int, inflight: int, tx_workers: int, queues: int,
                 max_inflight_frames: int, ring_capacity: int, pod_ring: int, coalesce_us: float):
        self.eng = nf.IoEngine(burst, inflight, tx_workers, queues, max_inflight_frames)
        self.eng.set_coalesce(64, coalesce_us)
        macs = [(int.from_bytes(self.mac(i), "little"), i) for i in range(n_pods)]
        self.eng.add_backend(nf.WireBackend(ring_capacity, queues, macs))
        self.paths = [os.path.join(d, f"pod{i}") for i in range(n_pods)]
        for i, p in enumerate(self.paths):
            self.eng.add_port(i, nf.MemifPort(p, pod_ring, int(os.environ.get("WIRE_BUF", 2048)), queues))
        self.eng.start()

    @staticmethod
    def mac(i: int) -> bytes:
        return bytes([2, 0, 0, 0, 0, i + 1])

    def frames(self, i: int, n_pods: int, k: int = 4096, seed: int = 0, broadcast: bool = False):
        """k 60-B IPv4 / UDP frames from pod i to random other pods (distinct 5-tuples); with
        `broadcast` to ff:ff:ff:ff:ff:ff."""
        rng = np.random.default_rng(seed)
        f = np.zeros((k, 64), np.uint8)
        dst = (i + 1 + rng.integers(0, n_pods - 1, k)) % n_pods
        for j in range(k):
            d = int(dst[j])
            f[j, 0:6] = 0xFF if broadcast else np.frombuffer(self.mac(d), np.uint8)
            f[j, 6:12] = np.frombuffer(self.mac(i), np.uint8)
            f[j, 12:14] = (8, 0)
            f[j, 14:24] = (0x45, 0, 0, 46, 0, 0, 0, 0, 64, 17)
            f[j, 26:30] = (10, 0, 0, i + 1)
            f[j, 30:34] = (10, 0, 0, d + 1)
            f[j, 34:38] = (0x10, (j >> 8) & 0xFF, 0x00, 0x50 + (j & 0x0F))
            f[j, 38:40] = (0, 26)
            w = f[j, 14:34].astype(np.uint32)
            c = int(np.sum((w[0::2] << 8) | w[1::2]))
            c = (c & 0xFFFF) + (c >> 16)
            c = ~((c & 0xFFFF) + (c >> 16)) & 0xFFFF
            f[j, 24:26] = (c >> 8, c & 0xFF)       # a valid IPv4 header (a kernel bridge checks it)
        return f, np.full(k, 60, np.uint32)

    @property
    def stats(self) -> dict:
        return dict(self.eng.stats())

    def latency_us(self):
        return np.asarray(self.eng.take_latency_us())

    @property
    def error(self):
        return self.eng.error() or None

    def stop(self):
        self.eng.stop()


def run(device: str = "cuda", n_pods: int = 8, flows: int = 1 << 20, n_acl: int = 256, duration: float = 1.0,
        threads: int = 8, burst: int = 512, inflight: int = 64, ring_capacity: int = 16384,
        hash_mode: str = "lds", tx_workers: int = 0, queues: int = 6, max_inflight_frames: int = 4096,
        pod_ring: int = 1024, backend: str = "pipeline", coalesce_us: float = 8.0, loaded_window: int = 2048,
        traffic: str = "plain", zero_copy: bool = False, saturated_only: bool = False, gpu_egress: bool = False,
        trials: int = 1, split: str = "", planes: str = "", idle_only: bool = False) -> dict:
    """traffic: "plain" (the headline SFC), "vxlan-egress" (every pod's VF a VXLAN tunnel port:
    all frames leave encapsulated through one underlay vport, outer headers from the per-burst
    side pass) or "broadcast" (pods on one learning bridge sending to ff:ff:ff:ff:ff:ff: every
    frame floods to the other pods, one copy from the GPU and the rest from the side pass;
    `mpps` counts delivered copies).  zero_copy: the ring reads the pods' frames in their memif
    regions (NativeLivePath zero_copy) instead of header copies in its slots.  trials: saturated
    runs of `duration` each; `mpps` is their median (`mpps_trials` all of them, each with the CPU
    time it cost), the saturated latencies those of the median trial.  tx_workers = 0: run to
    completion (each queue's rx thread delivers its own bursts).  split: the SFC's hops with
    GPU placements, e.g. "acl,nat,l2fwd@1" (SFC hops across GPUs in the live path: two ring planes,
    `planes` "cuda:0,cuda:1" or by default the device twice, flows sharded by owner; frames cross
    to the other plane's grid mid-chain, ring.h XferEntry)."""
    nf = nfdp()
    t0 = time.perf_counter()
    d = tempfile.mkdtemp(prefix="dpu-live-", dir=memif_dir())
    pods = []
    if backend == "wire":
        live = _WireLive(nf, d, n_pods, burst, inflight, tx_workers, queues, max_inflight_frames, ring_capacity,
                         pod_ring, coalesce_us)
        for i in range(n_pods):
            fr, ln = live.frames(i, n_pods, seed=100 + i)
            pods.append((live.paths[i], fr, ln))
        device, flows, n_acl = "none", n_pods * 4096, 0
    elif traffic == "broadcast":
        from dpu_operator_amd.dataplane import tables as T

        dp = DataPlane(device=device, flow_buckets=1 << 12, mac_slots=1 << 12,
                       hash_mode=hash_mode if device != "cpu" else "mfma")
        for p in range(n_pods):
            dp.ports.set(p, flags=T.PORT_VALID | T.PORT_LEARN, bridge_id=5)
        dp.flood.set_members(5, list(range(n_pods)))
        dp.commit(full=True)
        ports = {p: MemifVport(os.path.join(d, f"pod{p}"), ring_size=pod_ring) for p in range(n_pods)}
        live = NativeLivePath(dp, ports, burst=burst, ring_capacity=ring_capacity, inflight=inflight,
                              tx_workers=tx_workers, queues=queues, max_inflight_frames=max_inflight_frames,
                              coalesce_us=coalesce_us, zero_copy=zero_copy, gpu_egress=gpu_egress).start()
        gen = _WireLive.__new__(_WireLive)
        for i in range(n_pods):
            fr, ln = gen.frames(i, n_pods, k=1024, seed=100 + i, broadcast=True)
            pods.append((ports[i].path, fr, ln))
        flows, n_acl = 0, 0
    else:
        buckets = max(1 << 12, 1 << int(np.ceil(np.log2(max(flows, 1) / 2))))
        if split:
            from dpu_operator_amd.dataplane.multi import MultiDataPlane

            devs = planes.split(",") if planes else [device, device]
            dp = MultiDataPlane(devs, placement="flow", flow_buckets=buckets,
                                hash_mode=hash_mode if device != "cpu" else "mfma")
            sc = S.build_sfc(dp, n_pods=n_pods, n_flows=flows, n_acl=n_acl, seed=0, hops=tuple(split.split(",")))
        else:
            dp = DataPlane(device=device, flow_buckets=buckets, hash_mode=hash_mode if device != "cpu" else "mfma")
            sc = S.build_sfc(dp, n_pods=n_pods, n_flows=flows, n_acl=n_acl, seed=0)
        underlay = S.install_vxlan_egress(dp, sc)["underlay"] if traffic == "vxlan-egress" else None
        dp.commit(full=True)
        ports = {int(sc.pod_port[i]): MemifVport(os.path.join(d, f"pod{i}"), ring_size=pod_ring) for i in range(n_pods)}
        if underlay is not None:
            ports[underlay] = MemifVport(os.path.join(d, "underlay"), ring_size=4 * pod_ring)
        live = NativeLivePath(dp, ports, burst=burst, ring_capacity=ring_capacity, inflight=inflight,
                              tx_workers=tx_workers, queues=queues, max_inflight_frames=max_inflight_frames,
                              coalesce_us=coalesce_us, zero_copy=zero_copy, gpu_egress=gpu_egress).start()
        for i in range(n_pods):
            slots, im = S.traffic(sc, 4096, seed=100 + i, src_pods=np.array([i]))
            pods.append((ports[int(sc.pod_port[i])].path, slots, (im >> 16).astype(np.uint32)))
        if underlay is not None:   # the VTEP's pod only receives
            pods.append((ports[underlay].path, np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32)))
        flows = int(len(sc.keys))
    setup_s = time.perf_counter() - t0
    stats = lambda: live.stats  # noqa: E731
    try:
        out = {"backend": backend, "traffic": traffic, "zero_copy": zero_copy, "device": device, "queues": queues, "coalesce_us": coalesce_us, "tx_workers": tx_workers, "inflight_bursts": inflight,
               **({"split": split, "planes": [str(getattr(p, "tdev", "cpu")) for p in dp.planes],
                   "xfer_active": live.xfer_active() if hasattr(live, "xfer_active") else None} if split else {}),
               "max_inflight_frames": max_inflight_frames, "pod_ring": pod_ring, "gen_threads": threads,
               "pods": n_pods, "flows": flows, "acl_rules": n_acl, "frame_bytes": 64,
               "setup_s": round(setup_s, 1)}
        if split and idle_only:
            # the split chain's hand-off, unloaded: one frame in flight, then the inbox's timing
            # (ring.h XferInbox: send -> picked up, picked up -> written back) per plane
            r1 = nf.trafgen_run(pods, duration_s=min(duration, 0.5), warmup_s=0.05, threads=1, burst=1, inflight=1)
            out.update(idle_p50_us=_pct(r1["lat_us"], 50), idle_p99_us=_pct(r1["lat_us"], 99),
                       idle_frames=int(r1["received"]))
            rings = list(live._rings)
            live.stop()
            xs = []
            for rg in rings:
                x = list(map(int, rg.eng.xfer_stats()))
                n = max(x[4], 1) if len(x) >= 5 else 1
                xs.append({"entries": x[0], "samples": x[4] if len(x) >= 5 else 0,
                           "send_to_pickup_us": round(x[2] / n * 0.01, 2) if len(x) >= 5 else None,
                           "pickup_to_back_us": round(x[3] / n * 0.01, 2) if len(x) >= 5 else None,
                           **({"entry_load_us": round(x[5] / n * 0.01, 2), "stages_us": round(x[6] / n * 0.01, 2),
                               "write_back_us": round(x[7] / n * 0.01, 2)} if len(x) >= 8 else {})})
            out["xfer"] = xs
            out["error"] = live.error
            return out
        # saturated: every pod as fast as its vport takes frames (with what each trial cost in CPU
        # time: the rate is host-CPU work, bounded by the box's CPU share)
        runs = []
        if int(trials) > 1:
            # one untimed run first: the first trial after setup ran 10-25 % low on several boxes
            # (page faults in fresh pod rings, cold caches; r6_s24, r6_s25)
            nf.trafgen_run(pods, duration_s=0.3, warmup_s=0.1, threads=threads, burst=32)
            drain(nf, pods, stats)
        for _ in range(max(1, int(trials))):
            with cpuquota.Meter() as cm:
                r = nf.trafgen_run(pods, duration_s=duration, warmup_s=0.2, threads=threads, burst=32)
            runs.append((r["received"] / duration / 1e6, r, cm.result))
            drain(nf, pods, stats)
        order = sorted(range(len(runs)), key=lambda k: runs[k][0])
        mpps, r, cpu = runs[order[len(order) // 2]]
        out["cpu"] = cpu
        out.update(mpps=round(mpps, 3), offered_mpps=round(r["sent"] / duration / 1e6, 3),
                   p50_us=_pct(r["lat_us"], 50), p99_us=_pct(r["lat_us"], 99))
        if len(runs) > 1:
            ms = [x[0] for x in runs]
            out.update(trials=len(runs), trial_s=duration, mpps_trials=[round(x, 3) for x in ms],
                       mpps_min=round(min(ms), 3), mpps_max=round(max(ms), 3),
                       mpps_spread=round((max(ms) - min(ms)) / max(mpps, 1e-9), 3),
                       cpus_used_trials=[x[2].get("process_cpus_used") for x in runs])
        if saturated_only:   # (the queue curve: saturated rate only)
            st = live.stats
            out["engine"] = {k: int(st.get(k, 0)) for k in ("rx", "tx", "gpu_tx", "tx_full", "drop")}
            out["error"] = live.error
            if gpu_egress and live._rings:   # GPU-direct egress diagnostics (ring.h RingDevState, after stop)
                rings = list(live._rings)
                live.stop()
                out["gde"] = [list(map(int, r.eng.gde_stats())) for r in rings]
            return out
        # loaded, closed loop: `loaded_window` frames in flight over all pods (the generator
        # refills as frames arrive): the throughput of a saturated path with its queueing bounded
        # by the window, not by the pod rings (one-way latency = window / rate, Little's law)
        rl = nf.trafgen_run(pods, duration_s=duration, warmup_s=0.2, threads=threads, burst=32, inflight=loaded_window)
        out.update(loaded_window=loaded_window, loaded_mpps=round(rl["received"] / duration / 1e6, 3),
                   loaded_p50_us=_pct(rl["lat_us"], 50), loaded_p99_us=_pct(rl["lat_us"], 99))
        drain(nf, pods, stats)
        # unloaded: closed loop, one frame in flight
        r1 = nf.trafgen_run(pods, duration_s=min(duration, 0.5), warmup_s=0.05, threads=1, burst=1, inflight=1)
        out.update(idle_p50_us=_pct(r1["lat_us"], 50), idle_p99_us=_pct(r1["lat_us"], 99),
                   idle_frames=int(r1["received"]))
        drain(nf, pods, stats)
        # offered loads below saturation: 90 % and 50 % of the measured maximum (of frames IN: with
        # broadcast every frame sent comes out as several delivered copies)
        fan = (r["received"] / r["sent"]) if (traffic == "broadcast" and r["sent"]) else 1.0
        out["copies_per_frame"] = round(fan, 2)
        if mpps > 0:
            for tag, frac in (("load90", 0.9), ("half", 0.5)):
                r2 = nf.trafgen_run(pods, duration_s=duration, warmup_s=0.1, threads=threads, burst=8,
                                    rate_pps=frac * mpps / max(fan, 1.0) * 1e6)
                out.update({f"{tag}_mpps": round(r2["received"] / duration / 1e6, 3),
                            f"{tag}_p50_us": _pct(r2["lat_us"], 50), f"{tag}_p99_us": _pct(r2["lat_us"], 99)})
                drain(nf, pods, stats)
            out["half_load_mpps"] = out.pop("half_mpps")
        st = live.stats
        out["engine"] = {k: int(v) for k, v in st.items() if k in ("rx", "tx", "drop", "bursts", "tx_full",
                                                                    "side_passes", "punt", "rx_wait_tx",
                                                                    "rx_idle_polls", "publish_ns", "deliver_ns",
                                                                    "zero_copy_frames")}
        if st.get("bursts"):
            out["engine"]["frames_per_burst"] = round(st["rx"] / st["bursts"], 1)
        lat = live.latency_us()
        out["engine_burst_p50_us"] = _pct(lat, 50)
        out["error"] = live.error
        return out
    except BaseException:
        print(json.dumps({"error": live.error, "stats": {k: int(v) for k, v in live.stats.items()}}), file=sys.stderr)
        raise
    finally:
        try:
            live.stop()
        except Exception as e:  # noqa: BLE001 - report, the measurement above stands
            print(f"stop: {e}", file=sys.stderr)
        shutil.rmtree(d, ignore_errors=True)


def run_veth(mode: str = "linux-bridge", n_pods: int = 4, duration: float = 1.0, threads: int = 2,
             queues: int = 2, tx_workers: int = 1, burst: int = 256, inflight: int = 64, ring_capacity: int = 16384,
             max_inflight_frames: int = 4096, coalesce_us: float = 8.0, device: str = "cuda", rx_frames: int = 0,
             pod_xdp: bool = False) -> dict:
    """Kernel-netdev pods: every pod a network namespace holding one end of a veth pair, driven by
    the same C++ generator / sink through AF_PACKET rings opened inside the namespace
    (csrc/nfdp/trafgen_pkt.h).  The host ends go to
      * `linux-bridge`: a Linux bridge (the kernel's own L2 switch, the comparator);
      * `engine`: the native I/O engine as PacketPorts over the zero-cost wire pipeline (the
        engine's own ceiling on veth);
      * `pipeline`: the native I/O engine over the data plane on `device` (the resident ring
        kernel on a GPU): the deployed GPU node's default, its pods on one L2 bridge with their
        MACs programmed (what the VSP does without an NF), frames switched by the pipeline;
    so all three switch identical pods with identical frames.  A "-xdp" mode ("engine-xdp",
    "pipeline-xdp") serves the engine's ends through AF_XDP (native_io.XdpVport) instead of AF_PACKET
    rings; pod_xdp: the pods' own application uses AF_XDP on its veth (an af_xdp PMD) instead of
    AF_PACKET.  rx_frames: the engine's rx ring per port (0: the vport kind's default)."""
    from dpu_operator_amd.cni.netlink import RtNetlink, create_netns, delete_netns
    from dpu_operator_amd.dataplane.native_io import PacketVport, XdpVport

    nf = nfdp()
    xdp = mode.endswith("-xdp")          # the engine's ends through AF_XDP instead of AF_PACKET rings
    mode = mode[:-4] if xdp else mode
    VP = XdpVport if xdp else PacketVport
    rx_frames = rx_frames or VP.DEFAULT_FRAMES
    live = None
    nl = RtNetlink()
    tag = f"{os.getpid() % 10000}"
    br = f"lbbr{tag}"
    nss, hosts, eng = [], [], None   # (IPv6 autoconfiguration frames of the pods count as `bad`)
    wire = _WireLive.__new__(_WireLive)
    try:
        if mode == "linux-bridge":
            nl.link_add_bridge(br)
            nl.link_set_up(br)
        for i in range(n_pods):
            pod, host = f"lb{tag}p{i}", f"lb{tag}p{i}d"
            nl.link_add_veth(pod, host)
            hosts.append(host)
            ns = create_netns(os.path.join(os.environ.get("DPU_NETNS_DIR", "/var/run/netns"), f"lb{tag}-{i}"))
            nss.append(ns)
            nl.link_set_hw_addr(pod, ":".join(f"{b:02x}" for b in _WireLive.mac(i)))
            nl.link_set_ns(pod, ns)
            nl.link_set_up(pod, ns)
            if mode == "linux-bridge":
                nl.link_set_master(host, br)
            nl.link_set_up(host)
        if mode == "engine":
            eng = nf.IoEngine(burst, inflight, tx_workers, queues, max_inflight_frames)
            eng.set_coalesce(64, coalesce_us)
            macs = [(int.from_bytes(_WireLive.mac(i), "little"), i) for i in range(n_pods)]
            eng.add_backend(nf.WireBackend(ring_capacity, queues, macs))
            for i, h in enumerate(hosts):
                eng.add_port(i, VP(h, frames=rx_frames).make(nf))
            eng.start()
        elif mode == "pipeline":
            from dpu_operator_amd.dataplane import tables as T

            dp = DataPlane(device=device, flow_buckets=1 << 12, hash_mode="lds" if device != "cpu" else "mfma")
            for i in range(n_pods):
                mac = ":".join(f"{b:02x}" for b in _WireLive.mac(i))
                dp.ports.set(i, flags=T.PORT_VALID | T.PORT_SPOOFCHK, bridge_id=1, mac=mac, peer_mac=mac)
                dp.macs.insert(1, mac, i)
            dp.flood.set_members(1, list(range(n_pods)))
            dp.commit(full=True)
            live = NativeLivePath(dp, {i: VP(h, frames=rx_frames) for i, h in enumerate(hosts)}, burst=burst,
                                  ring_capacity=ring_capacity, inflight=inflight, tx_workers=tx_workers, queues=queues,
                                  max_inflight_frames=max_inflight_frames, coalesce_us=coalesce_us).start()
            eng = live._eng
        pods = []
        for i in range(n_pods):
            fr, ln = wire.frames(i, n_pods, k=1024, seed=100 + i)
            pods.append((nss[i], f"lb{tag}p{i}", fr, ln))
        out = {"vports": "veth", "switch": mode, "engine_io": "af_xdp" if xdp else "af_packet",
               "pod_io": "af_xdp" if pod_xdp else "af_packet", "pods": n_pods,
               "gen_threads": threads, "frame_bytes": 64}
        if mode != "linux-bridge":
            out.update(queues=queues, tx_workers=tx_workers, coalesce_us=coalesce_us, rx_frames=rx_frames,
                       device=device if mode == "pipeline" else "none")
        # warm-up (the bridge learns every MAC), then saturated
        nf.trafgen_run_netns(pods, duration_s=0.2, warmup_s=0.0, threads=threads, burst=32, xdp=pod_xdp)
        time.sleep(0.1)
        r = nf.trafgen_run_netns(pods, duration_s=duration, warmup_s=0.2, threads=threads, burst=32, xdp=pod_xdp)
        mpps = r["received"] / duration / 1e6
        out.update(mpps=round(mpps, 3), offered_mpps=round(r["sent"] / duration / 1e6, 3),
                   p50_us=_pct(r["lat_us"], 50), p99_us=_pct(r["lat_us"], 99), bad=int(r["bad"]))
        time.sleep(0.1)
        for tag_, frac in (("load90", 0.9), ("half", 0.5)):
            if eng is not None:
                eng.take_latency_us()
            r2 = nf.trafgen_run_netns(pods, duration_s=min(duration, 0.5), warmup_s=0.1, threads=threads, burst=8,
                                      rate_pps=frac * mpps * 1e6, xdp=pod_xdp)
            out.update({f"{tag_}_mpps": round(r2["received"] / min(duration, 0.5) / 1e6, 3),
                        f"{tag_}_p50_us": _pct(r2["lat_us"], 50), f"{tag_}_p99_us": _pct(r2["lat_us"], 99)})
            if eng is not None:   # the engine's own share: rx read -> burst delivered
                el = np.asarray(eng.take_latency_us())
                out.update({f"{tag_}_engine_p50_us": _pct(el, 50), f"{tag_}_engine_p99_us": _pct(el, 99)})
            time.sleep(0.1)
        # unloaded: a slow trickle (1 kpps): no queueing anywhere
        r3 = nf.trafgen_run_netns(pods, duration_s=min(duration, 0.5), warmup_s=0.05, threads=1, burst=1,
                                  rate_pps=1000.0, xdp=pod_xdp)
        out.update(idle_p50_us=_pct(r3["lat_us"], 50), idle_p99_us=_pct(r3["lat_us"], 99))
        if eng is not None:
            st = dict(live.stats if live is not None else eng.stats())
            out["engine"] = {k: int(st.get(k, 0)) for k in ("rx", "tx", "drop", "bursts", "tx_full")}
            out["error"] = (live.error if live is not None else eng.error()) or None
        return out
    finally:
        if live is not None:
            live.stop()
        elif eng is not None:
            eng.stop()
        for ns in nss:
            delete_netns(ns)
        for h in hosts:
            try:
                nl.link_del(h)
            except Exception:  # noqa: BLE001 - went with its namespace peer
                pass
        if mode == "linux-bridge":
            try:
                nl.link_del(br)
            except Exception:  # noqa: BLE001
                pass


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--duration", type=float, default=1.0)
    ap.add_argument("--flows", type=int, default=1 << 20)
    ap.add_argument("--pods", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--burst", type=int, default=512)
    ap.add_argument("--inflight", type=int, default=64)
    ap.add_argument("--tx-workers", type=int, default=0, help="0: run to completion (the rx threads deliver)")
    ap.add_argument("--queues", type=int, default=6)
    ap.add_argument("--max-inflight-frames", type=int, default=4096)
    ap.add_argument("--pod-ring", type=int, default=1024)
    ap.add_argument("--backend", choices=("pipeline", "wire"), default="pipeline")
    ap.add_argument("--traffic", choices=("plain", "vxlan-egress", "broadcast"), default="plain")
    ap.add_argument("--coalesce-us", type=float, default=8.0)
    ap.add_argument("--loaded-window", type=int, default=2048, help="frames in flight of the closed-loop loaded run")
    ap.add_argument("--zero-copy", action="store_true", help="the ring reads frames in the pods' memif regions")
    ap.add_argument("--gpu-egress", action="store_true", help="the ring grid writes frames into the pods' rings itself")
    ap.add_argument("--trials", type=int, default=1, help="saturated runs (median reported)")
    ap.add_argument("--split", default="", help='SFC hops with GPU placements, e.g. "acl,nat,l2fwd@1" (two planes)')
    ap.add_argument("--planes", default="", help='--split: the planes\' devices, e.g. "cuda:0,cuda:1"')
    ap.add_argument("--idle-only", action="store_true", help="--split: the unloaded run and the inbox timing only")
    ap.add_argument("--veth", choices=("linux-bridge", "engine", "pipeline", "engine-xdp", "pipeline-xdp"), default=None,
                    help="netns pods on veth pairs, switched by a Linux bridge, by the native engine alone or by the "
                         "native engine in front of the data plane on --device (the deployed default)")
    ap.add_argument("--rx-frames", type=int, default=0, help="--veth: the engine's rx ring per port")
    ap.add_argument("--pod-xdp", action="store_true", help="--veth: the pods' application uses AF_XDP on its veth")
    a = ap.parse_args()
    if a.veth:
        if "DPU_NETNS_DIR" in os.environ:   # a namespace of our own (unshare -Urnm): loopback starts down
            os.makedirs(os.environ["DPU_NETNS_DIR"], exist_ok=True)
        print(json.dumps(run_veth(a.veth, n_pods=min(a.pods, 8), duration=a.duration, threads=min(a.threads, a.pods),
                                  queues=a.queues, tx_workers=a.tx_workers, coalesce_us=a.coalesce_us,
                                  device=a.device, rx_frames=a.rx_frames, pod_xdp=a.pod_xdp)), flush=True)
        return
    print(json.dumps(run(a.device, a.pods, a.flows, duration=a.duration, threads=a.threads, burst=a.burst,
                         inflight=a.inflight, tx_workers=a.tx_workers, queues=a.queues,
                         max_inflight_frames=a.max_inflight_frames, pod_ring=a.pod_ring,
                         backend=a.backend, coalesce_us=a.coalesce_us, loaded_window=a.loaded_window,
                         traffic=a.traffic, zero_copy=a.zero_copy, gpu_egress=a.gpu_egress, trials=a.trials,
                         split=a.split, planes=a.planes, idle_only=a.idle_only)),
          flush=True)


if __name__ == "__main__":
    main()
