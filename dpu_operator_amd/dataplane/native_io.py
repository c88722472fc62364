"""Native live packet path: the C++ I/O engine (csrc/nfdp/iox.{h,cpp}) between vports and the data
plane, with Python only configuring it.

``netio.LivePath`` moves every frame through a Python loop (os.read / os.write per frame, header
slots copied in Python).  ``NativeLivePath`` hands the same job to the native engine, organised
like a multi-queue NIC driver:

    vports (memif shared-memory rings, AF_PACKET rings on veth ends, TAP fds), split over
    `queues` rx threads
      -> rx thread q: 64-B header slots + ingress meta straight into ring queue q of the owner
         GPU's persistent ring kernel (pinned host slots; RSS owner = owner_of(toeplitz(FlowKey), N))
      -> tx workers of queue q: completion -> egress frames assembled from the rewritten header
         and the payload still in the rx buffer; replicas / learn events / outer headers from a
         per-burst CPU side pass (no ring drain); recirculation re-enters natively; slow-path
         frames come back here (`on_punt`).

One engine drives every data plane it is given: ``NativeLivePath([dp_gpu0, dp_gpu1, ...], ports)``
steers each flow to its owner GPU (the flow table of a multi-GPU data plane is sharded the same
way, dataplane/multi.py).  Without a GPU the backends are the bit-exact C++ oracle, so the whole
native path is tested on CPU (tests/test_native_io.py).

Table commits (DataPlane.commit hooks):
  * GPU planes with running coop rings: the commit is applied under traffic; the engine only
    holds publication for the epoch switch (`hold` / `release`: microseconds, nothing drained)
    and swaps its own configuration (steering, tunnel redirects, side ports, side-pass table
    snapshot) copy-on-write at the same moment;
  * otherwise (CPU oracle planes, ring relaunches): the engine is paused around the commit
    (`pre_commit` / `post_commit`: nothing in flight while tables move).

Health: a failed engine (a ring that stopped completing, an I/O error) sets ``error`` and
``healthy = False``; with ``auto_restart`` the supervisor thread rebuilds the engine in place.
"""
from __future__ import annotations

import logging
import os
import threading
import time

import numpy as np

from . import tables as T

log = logging.getLogger("dpu.native_io")

SIDE_PORT_FLAGS = T.PORT_LEARN | T.PORT_ARP_TRAP | T.PORT_MIRROR


class MemifVport:
    """A shared-memory vport (csrc/nfdp/memif.h): the data plane owns the region file; the pod
    (or NF) side attaches to `path` (nf.MemifEndpoint, the trafgen tool, a DPDK memif-style app).
    The region has one data-plane -> pod ring per engine queue (`tx_rings`, 0: the engine's
    queue count), so the queues' tx threads never contend for a pod."""

    def __init__(self, path: str, ring_size: int = 1024, buf_size: int = 2048, tx_rings: int = 0):
        self.path, self.ring_size, self.buf_size = path, int(ring_size), int(buf_size)
        self.tx_rings = int(tx_rings)

    MAX_RINGS = 16   # data plane -> pod rings a region can have (iox.h Port::kMaxTxQueues)

    def make(self, nf, queues: int = 1, gpu_rings: int = 0):
        """gpu_rings: extra rings the GPUs' grids write themselves (GPU-direct egress, one per engine
        lane, after the host queues' rings); as many as fit MAX_RINGS."""
        host = self.tx_rings or max(1, int(queues))
        return nf.MemifPort(self.path, self.ring_size, self.buf_size, min(self.MAX_RINGS, host + max(0, int(gpu_rings))))


class PacketVport:
    """The VSP-side end of a veth pair, read and written through AF_PACKET TPACKET_V2 rings.

    `VethVport.create` makes the pair: the pod end (`name`, the device the device plugin hands
    out and the CNI moves into the pod, networkfn.cmd_add) and the data-plane end (`name` + "d")
    this port opens."""

    # AF_PACKET rx ring per port: what an overloaded port can queue.  A NIC-like depth: deep enough
    # to absorb bursts, shallow enough that overload drops instead of building milliseconds of
    # standing queue (at ~100 kpps per veth, 512 frames are ~5 ms)
    DEFAULT_FRAMES = 512

    def __init__(self, ifname: str, frames: int = DEFAULT_FRAMES, frame_size: int = 2048):
        self.ifname, self.frames, self.frame_size = ifname, int(frames), int(frame_size)
        self._nl = None
        self.name = None

    @classmethod
    def create_veth(cls, nl, name: str, mac: str | None = None, frames: int = DEFAULT_FRAMES) -> "PacketVport":
        """A veth pair for a kernel-netdev pod: `name` (pod end) and `name`d (data-plane end)."""
        peer = name + "d"
        if len(peer) > 15:
            raise ValueError("interface names are at most 15 characters")
        nl.link_add_veth(name, peer)
        if mac:
            nl.link_set_hw_addr(name, mac)
        # The engine re-sends every frame as a plain frame: whatever the pod's stack left for the
        # hardware (checksum-partial UDP / TCP, TSO / GSO super-frames) would reach the next pod
        # unfinished.  The pod end computes checksums and segments itself; the engine end takes no
        # GRO aggregates.  (Features move with the netdev into the pod's namespace.)
        set_offloads(name, tx_csum=False, sg=False, tso=False, gso=False)
        set_offloads(peer, gro=False)
        _quiet_ipv6(peer)
        nl.link_set_up(peer)
        nl.link_set_up(name)
        vp = cls(peer, frames=frames)
        vp._nl, vp.name = nl, name
        return vp

    @classmethod
    def attach(cls, ifname: str, frames: int = 4096) -> "PacketVport":
        """An existing netdev as a data-plane port (the node's uplink NIC): opened through the same
        AF_PACKET rings, promiscuous while the engine holds it (the socket's membership), with
        receive offloads that would hand the engine super-frames (GRO) turned off."""
        set_offloads(ifname, gro=False)
        return cls(ifname, frames=frames)

    def make(self, nf, queues: int = 1):
        return nf.PacketPort(self.ifname, self.frames, self.frame_size)

    def close(self) -> None:
        """Delete the pair (the pod end goes with it, wherever it is); an attached netdev is only
        let go of (the engine's socket closes with the port)."""
        if self._nl is not None:
            try:
                self._nl.link_del(self.ifname)
            except Exception:  # noqa: BLE001 - already gone with its namespace
                pass
            self._nl = None


class XdpVport(PacketVport):
    """The VSP-side end of a veth pair served through AF_XDP (iox.h XdpPort): an XSK socket and
    a redirect XDP program on the netdev instead of AF_PACKET rings, so frames reach the engine
    without an skb or a packet socket.  Same pair creation as PacketVport (vport_kind "xdp")."""

    DEFAULT_FRAMES = 2048

    def __init__(self, ifname: str, frames: int = DEFAULT_FRAMES, frame_size: int = 2048):
        super().__init__(ifname, frames, frame_size)

    @classmethod
    def create_veth(cls, nl, name: str, mac: str | None = None, frames: int = DEFAULT_FRAMES) -> "XdpVport":
        return super().create_veth(nl, name, mac, frames)

    def make(self, nf, queues: int = 1):
        return nf.XdpPort(self.ifname, self.frames, self.frame_size)


_ETHTOOL = {"tx_csum": 0x17, "sg": 0x19, "tso": 0x1F, "gso": 0x24, "gro": 0x2C}   # ETHTOOL_S* (linux/ethtool.h)


def set_offloads(ifname: str, ns: str = "", **features: bool) -> dict:
    """Legacy ethtool feature switches on `ifname` (SIOCETHTOOL, what `ethtool -K` does), best
    effort: {feature: applied}.  Features: tx_csum, sg, tso, gso, gro."""
    import ctypes
    import fcntl
    import socket
    import struct

    from ..cni.netlink import in_netns

    def run():
        out = {}
        s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        try:
            for name, on in features.items():
                val = ctypes.create_string_buffer(struct.pack("II", _ETHTOOL[name], 1 if on else 0))
                ifr = struct.pack("16sP", ifname.encode()[:15], ctypes.addressof(val)) + bytes(16)
                try:
                    fcntl.ioctl(s.fileno(), 0x8946, ifr)          # SIOCETHTOOL
                    out[name] = True
                except OSError:
                    out[name] = False
        finally:
            s.close()
        return out

    return in_netns(ns, run)


def _quiet_ipv6(ifname: str) -> None:
    """No IPv6 autoconfiguration traffic from the data-plane end of a vport (best effort)."""
    try:
        with open(f"/proc/sys/net/ipv6/conf/{ifname}/disable_ipv6", "w") as f:
            f.write("1")
    except OSError:
        pass


def _make_port(nf, spec, queues: int = 1, gpu_rings: int = 0):
    if isinstance(spec, MemifVport):
        return spec.make(nf, queues, gpu_rings)
    if hasattr(spec, "make"):
        return spec.make(nf, queues)
    if hasattr(spec, "fd"):            # netio.TapPort and anything else with a packet fd
        return nf.FdPort(int(spec.fd))
    raise TypeError(f"unsupported vport {spec!r}")


def parse_cpulist(text: str) -> list[int]:
    """sysfs cpulist ("0-3,8,10-11") -> [0, 1, 2, 3, 8, 10, 11]."""
    out: list[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def device_local_cpus(dev, sys_root: str = "/") -> list[int]:
    """CPUs NUMA-local to GPU `dev` (its PCI function's local_cpulist) that this process may run
    on; [] when unknown or when that is every CPU this process has (nothing to pin)."""
    try:
        import torch

        d = torch.device(dev)
        if d.type != "cuda":
            return []
        pr = torch.cuda.get_device_properties(d.index or 0)
        pci = f"{getattr(pr, 'pci_domain_id', 0):04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        with open(os.path.join(sys_root, "sys/bus/pci/devices", pci, "local_cpulist")) as f:
            local = set(parse_cpulist(f.read()))
    except Exception:  # noqa: BLE001 - no such attribute / file: leave the threads unpinned
        return []
    allowed = os.sched_getaffinity(0)
    cpus = sorted(local & allowed)
    return cpus if cpus and set(cpus) != allowed else []


class NativeLivePath:
    def __init__(self, dps, ports: dict, burst: int = 256, ring_capacity: int = 4096, inflight: int = 64,
                 on_punt=None, auto_restart: bool = True, tx_workers: int = 1, queues: int = 1,
                 max_inflight_frames: int = 0, port_queues: dict | None = None, coalesce_us: float = 8.0,
                 coalesce_frames: int = 64, ring_cus: int = 0, zero_copy: bool = False, lane_groups: bool = False,
                 pin_cpus: bool = False, max_deferred_unmaps: int = 16, gpu_egress: bool = False):
        """dps: one data plane or a list (one per GPU, or a MultiDataPlane's planes); ports:
        {port id: vport spec}; queues: rx threads (each with a ring queue on every GPU) — with
        `lane_groups`, per data plane: every plane brings `queues` rx threads (and their tx
        workers) of its own, so the engine's I/O capacity grows with the GPU count, and a port
        placed on a plane (MultiDataPlane placement="port") is served by a queue of that plane's
        group; pin_cpus: each group's threads run on its GPU's NUMA-local CPUs (or {group: CPUs});
        port_queues: {port id: queue} (default: least loaded); max_inflight_frames: per lane
        bound of the engine's own queueing (0: the ring capacity); coalesce_us / coalesce_frames:
        with bursts of a lane in flight, frames gather into one publish until that many are read
        or the oldest waited that long (an idle lane publishes at once); zero_copy: the pipelines
        read memif frames where the pods wrote them (the regions pinned and mapped for the GPUs)
        instead of from copies of their headers in the ring slots.  A removed zero-copy vport's
        region stays pinned until no ring grid of the process runs (hipHostUnregister waits for
        the device): when more than `max_deferred_unmaps` pile up, the supervisor restarts the
        rings (a maintenance restart: traffic pauses for the relaunch) and they are released, so
        pinned memory stays bounded under vport churn.  gpu_egress (GPU planes): the ring grids
        write frames bound for memif vports straight into those pods' rings (ring.h GdeRing, one ring
        per engine lane in each region after the host queues' rings); the tx threads only see the
        frames that need the host (drops aside: side work, frames longer than the 64-B slot, a full
        GPU ring)."""
        from ..native import nfdp

        self.nf = nfdp()
        self.dps = list(dps) if isinstance(dps, (list, tuple)) else list(getattr(dps, "planes", [dps]))
        if not self.dps:
            raise ValueError("at least one data plane")
        self._port_owner = getattr(self.dps[0], "_port_owner", None)   # (MultiDataPlane placement="port")
        self.lane_groups = bool(lane_groups)
        self.group_queues = int(queues)
        if self.lane_groups:
            queues = int(queues) * len(self.dps)
        self.pin_cpus = pin_cpus if isinstance(pin_cpus, dict) else bool(pin_cpus)
        self.max_deferred_unmaps = int(max_deferred_unmaps)
        self.unmap_restarts = 0
        self.gpu = self.dps[0].gpu
        if any(d.gpu != self.gpu for d in self.dps):
            raise ValueError("data planes must all be GPU or all CPU")
        if ring_capacity < 64 or ring_capacity & (ring_capacity - 1):
            raise ValueError("ring_capacity must be a power of two >= 64")
        self.burst, self.capacity, self.inflight = int(burst), int(ring_capacity), int(inflight)
        self.tx_workers, self.queues = int(tx_workers), int(queues)
        self.max_inflight_frames = int(max_inflight_frames)
        self.coalesce_us, self.coalesce_frames = float(coalesce_us), int(coalesce_frames)
        self.ring_cus = int(ring_cus)   # CUs of each ring grid (0: the GPU's, split between planes sharing it)
        self.zero_copy = bool(zero_copy)
        self.gpu_egress = bool(gpu_egress) and self.gpu
        self.specs = dict(ports)
        self.port_queues = dict(port_queues or {})
        self.on_punt = on_punt
        self.auto_restart = auto_restart
        self.error: str | None = None
        self.healthy = True
        self.restarts = 0
        self._lock = threading.RLock()
        self._eng = None
        self._ports: dict[int, object] = {}
        self._rings = []
        self._backends = []
        self.xfer = False               # rings wired for cross-GPU hops (_wire_xfer)
        self._sup: threading.Thread | None = None
        self._stop = threading.Event()
        self._totals: dict[str, int] = {}
        self._side_base = None          # side counters of engines that were torn down
        self.punts = 0

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "NativeLivePath":
        with self._lock:
            self._build()
        self._stop.clear()
        self._sup = threading.Thread(target=self._supervise, daemon=True, name="dpu-native-io")
        self._sup.start()
        return self

    def _build(self) -> None:
        nf = self.nf
        eng = nf.IoEngine(self.burst, self.inflight, self.tx_workers, self.queues, self.max_inflight_frames)
        eng.set_coalesce(self.coalesce_frames, self.coalesce_us)
        self._rings, self._backends = [], []
        # planes sharing a GPU split its CUs between their resident grids (a resident grid never
        # yields: a second full-size grid on the same device would never be scheduled)
        per_dev: dict = {}
        for dp in self.dps:
            per_dev[str(getattr(dp, "tdev", ""))] = per_dev.get(str(getattr(dp, "tdev", "")), 0) + 1
        for dp in self.dps:
            if self.gpu:
                import torch

                from .ring import RingPath

                share = per_dev[str(dp.tdev)]
                with torch.cuda.device(dp.tdev):
                    ring = RingPath(dp, capacity=self.capacity, host_slots=True, coop=True, side=False,
                                    deadline_s=3600.0, queues=self.queues,
                                    cus=self.ring_cus or max(1, int(dp.num_cus) // share))
                    ring.eng.set_frame_addrs(self.zero_copy)
                    ring.eng.gde_enable(self.gpu_egress)
                self._rings.append(ring)   # (started below, after the cross-GPU hop wiring)
                be = nf.GpuBackend(ring.eng)
            else:
                be = nf.OracleBackend(self.capacity, self.queues)
                be.set_frame_addrs(self.zero_copy)
            self._backends.append(be)
            eng.add_backend(be)
            if self not in getattr(dp, "_io_hooks", []):
                dp._io_hooks = getattr(dp, "_io_hooks", []) + [self]
            dp._learned_on_device = True     # the engine learns into the device MAC table: commits pull first
        if self.gpu:
            self._wire_xfer()
            import torch

            for ring in self._rings:
                with torch.cuda.device(ring.dp.tdev):
                    ring.start()
        # replica counters appear in the first plane's counters (a MultiDataPlane sums its planes)
        eng.set_zero_copy(self.zero_copy)
        eng.set_gpu_egress(self.gpu_egress)
        hooks = getattr(self.dps[0], "_ctr_hooks", [])
        if self not in hooks:
            self.dps[0]._ctr_hooks = hooks + [self]
        if self.pin_cpus:
            for q in range(self.queues):
                g = self.group_of(q)
                cpus = (self.pin_cpus.get(g, []) if isinstance(self.pin_cpus, dict)
                        else device_local_cpus(getattr(self.dps[g], "tdev", "cpu")))
                if cpus:
                    eng.set_queue_cpus(q, list(cpus))
        for idx, spec in self.specs.items():
            p = self._ports.get(idx)
            if p is None:
                p = self._ports[idx] = _make_port(nf, spec, self.queues, self._gpu_rings())
            eng.add_port(int(idx), p, self._queue_for(idx))
        eng.learn_stamp = max(int(getattr(d, "stamp", 0)) for d in self.dps) + 1
        self._eng = eng
        self._applied = {}   # a new engine holds no configuration yet
        self._refresh()
        eng.start()

    # SFC hops across GPUs (ring.h XferEntry): with two or more GPU planes, every ring gets an inbox
    # that the other planes' grids hand split-chain frames to, and its grid resumes them there and
    # stores the final header straight into the entry ring's out slot; the engine delivers a burst
    # once every frame of it is back (no host hop, no launch).  Not with GPU-direct egress (its
    # instances do not hand off) nor IPv6 tables (the V6 instances run a split chain where it entered).
    # The inbox holds 128-B entries (16 MB at 1<<17): room for every frame a saturated entry plane
    # can have in flight; an eighth of each grid's workgroups serve it (every wave on its own ticket
    # of 64 entries), so a hand-off is picked up within a poll period however many queues feed it.
    XFER_ENTRIES = 1 << 17
    XFER_WG_SHARE = 8

    def _wire_xfer(self) -> None:
        self.xfer = len(self._rings) > 1 and not self.gpu_egress
        if not self.xfer:
            return
        devs = sorted({int(r.dp.tdev.index or 0) for r in self._rings})
        for a in devs:
            for b in devs:
                if a != b and not self.nf.enable_peer_access(a, b):
                    raise RuntimeError(f"cuda:{a} cannot store into cuda:{b}'s memory (no peer access)")
        for r in self._rings:
            wgs = max(1, min(int(r.cus) - self.queues, int(r.cus) // self.XFER_WG_SHARE))
            r.eng.xfer_enable(self.XFER_ENTRIES, wgs)
        descs = [r.eng.xfer_desc() for r in self._rings]
        for k, r in enumerate(self._rings):
            r.eng.xfer_set_peers(k, descs)

    def xfer_active(self) -> list[bool]:
        """Per plane: its running grid hands split-chain frames to the next plane (XF instance)."""
        return [bool(r.eng.xfer_active) for r in self._rings]

    def stop(self) -> None:
        self._stop.set()
        if self._sup is not None:
            self._sup.join(timeout=5)
            self._sup = None
        with self._lock:
            self._teardown()
        for dp in self.dps:
            hooks = getattr(dp, "_io_hooks", [])
            if self in hooks:
                hooks.remove(self)
            ch = getattr(dp, "_ctr_hooks", [])
            if self in ch:
                ch.remove(self)

    def _teardown(self) -> None:
        if self._eng is not None:
            self._accumulate()
            self._eng.stop()
            self._sync_stamps()
            sp, sd = np.asarray(self._eng.side_port_counters()), np.asarray(self._eng.side_drop_counters())
            self._side_base = (sp, sd) if self._side_base is None else (self._side_base[0] + sp, self._side_base[1] + sd)
        errs = []
        for r in self._rings:
            try:
                r.close()
            except Exception as e:  # noqa: BLE001 - close every ring, report the first failure
                errs.append(e)
        self._rings = []
        self._eng = None
        if errs:
            raise errs[0]

    def _sync_stamps(self) -> None:
        st = int(self._eng.learn_stamp)
        for dp in self.dps:
            dp.stamp = max(dp.stamp, st)

    # ------------------------------------------------------------------ table commits (DataPlane hooks)
    def pre_commit(self, dp) -> None:
        """Tables move with nothing in flight (oracle planes, ring relaunches)."""
        if self._eng is not None and self._eng.running:
            self._eng.flush_learning()
            self._eng.pause()

    def post_commit(self, dp) -> None:
        if self._eng is None:
            return
        self._refresh()
        self._eng.resume()

    def hold(self, dp) -> None:
        """A live commit's epoch switch: publication stops between two bursts (no drain).  The
        engine's new configuration (side-table snapshots, side ports, redirects, steering) is
        built BEFORE publication stops; only pointer swaps happen inside the hold."""
        if self._eng is not None and self._eng.running:
            self._staged = self._collect()
            self._eng.hold()

    def release(self, dp) -> None:
        if self._eng is None:
            return
        staged, self._staged = getattr(self, "_staged", None), None
        self._apply(staged if staged is not None else self._collect())
        self._eng.release()

    def switch(self, dp, engs, flows, sets) -> None:
        """A live commit's switch (engine.live_switch): the new configuration is built first, then
        ONE native call holds publication, changes every ring's epoch, swaps the configuration
        in and releases."""
        if self._eng is None or not self._eng.running:
            for e, f, st in zip(engs, flows, sets):
                e.change_epoch(f, st)
            if self._eng is not None:
                self._refresh()
            return
        c = self._collect()
        last = getattr(self, "_applied", {})
        st = c["steer"]
        old = last.get("steer")
        if st is not None and (old is None or old[1:] != st[1:] or not np.array_equal(old[0], st[0])):
            self._eng.set_steering(*st)   # (steering only picks the GPU: any burst may take either)
        sp = c["side_ports"] if last.get("side_ports") != c["side_ports"] else None
        rd = c["redirects"] if last.get("redirects") != c["redirects"] else None
        self._eng.switch_tables(list(engs), list(flows), list(sets), c["side"], sp, rd)
        self._applied = {"side_ports": c["side_ports"], "redirects": c["redirects"], "steer": st}

    def refresh(self, dp) -> None:
        """Rebuild and swap the engine's configuration now (copy-on-write, no hold): after table
        writes that went through the rings' control mailbox (DataPlane.ctrl_ports)."""
        if self._eng is not None:
            self._apply(self._collect())

    def _refresh(self) -> None:
        """Point the oracle backends at the current tables; the side-pass table snapshots, side
        ports, tunnel redirects and steering (copy-on-write in the engine)."""
        self._apply(self._collect())

    def _collect(self) -> dict:
        side = [self.nf.SideTables(**dp.side_tables_host()) for dp in self.dps]
        dp0 = self.dps[0]
        a = dp0.ports.a
        flags = a["flags"].astype(np.uint32)
        side_ports = [int(i) for i in np.nonzero(flags & np.uint32(SIDE_PORT_FLAGS))[0]]
        red = []
        for i in np.nonzero(flags & np.uint32(T.PORT_TUNNEL))[0]:
            tab = dp0.tunnels6 if flags[i] & T.PORT_TUNNEL6 else dp0.tunnels
            lag = int(a[i]["lag"])
            if lag < len(tab.a):
                red.append((int(i), int(tab.a[lag]["out_port"])))
        steer = None
        if len(self.dps) > 1:
            v6 = any(d._v6_keys() for d in self.dps)   # IPv6 frames steer by their folded 5-tuple
            po = getattr(dp0, "_port_owner", None)   # MultiDataPlane placement="port"
            steer = (np.ascontiguousarray(a).copy(), bytes(dp0.rss_key), v6,
                     [int(x) for x in po] if po is not None else [])
        return {"side": side, "side_ports": side_ports, "redirects": red, "steer": steer}

    def _apply(self, c: dict) -> None:
        eng = self._eng
        for g, (dp, be) in enumerate(zip(self.dps, self._backends)):
            if not self.gpu:
                be.configure(dp.tables_ptrs(), dp._ptr("flow_ctr"), dp._ptr("port_ctr"), dp._ptr("drop_ctr"))
            eng.set_side_tables(g, c["side"][g])
        last = getattr(self, "_applied", {})
        if last.get("side_ports") != c["side_ports"]:
            eng.set_side_ports(c["side_ports"])
        if last.get("redirects") != c["redirects"]:
            eng.set_redirects(c["redirects"])   # the whole map: a port that stopped being a tunnel loses its entry
        st = c["steer"]
        old = last.get("steer")
        if st is not None and (old is None or old[1:] != st[1:] or not np.array_equal(old[0], st[0])):
            eng.set_steering(*st)
        self._applied = {"side_ports": c["side_ports"], "redirects": c["redirects"], "steer": st}

    # ------------------------------------------------------------------ counters (DataPlane._ctr_hooks)
    def side_port_counters(self) -> np.ndarray:
        v = np.asarray(self._eng.side_port_counters()) if self._eng is not None else np.zeros(0, np.uint64)
        if self._side_base is not None:
            v = self._side_base[0] + v if len(v) else self._side_base[0]
        return v

    def side_drop_counters(self) -> np.ndarray:
        v = np.asarray(self._eng.side_drop_counters()) if self._eng is not None else np.zeros(0, np.uint64)
        if self._side_base is not None:
            v = self._side_base[1] + v if len(v) else self._side_base[1]
        return v

    def flush_learning(self) -> None:
        """Block until every MAC the engine has seen so far is in every plane's table."""
        if self._eng is not None:
            self._eng.flush_learning()

    # ------------------------------------------------------------------ ports
    def group_of(self, q: int) -> int:
        """The data plane (lane group) whose threads queue q is (0 without lane groups)."""
        return q // self.group_queues if self.lane_groups else 0

    def _queue_for(self, idx: int) -> int:
        """The queue serving port idx: an explicit choice, else with lane groups and a port placed
        on a plane the least loaded queue of that plane's group, else the engine's least loaded."""
        if idx in self.port_queues:
            return int(self.port_queues[idx])
        po = self._port_owner
        if self.lane_groups and po is not None and 0 <= int(idx) < len(po) and self._eng is not None:
            g = int(po[int(idx)]) % len(self.dps)
            group = range(g * self.group_queues, (g + 1) * self.group_queues)
            load = {q: 0 for q in group}
            for other in self._ports:
                if other != idx:
                    q = self.port_queue(other)
                    if q in load:
                        load[q] += 1
            return min(group, key=lambda q: (load[q], q))
        return -1

    def _gpu_rings(self) -> int:
        """GPU-direct egress rings a new memif region gets: one per engine lane (queue x plane)."""
        return self.queues * len(self.dps) if self.gpu_egress else 0

    def add_port(self, idx: int, spec, queue: int = -1) -> None:
        with self._lock:
            self.specs[idx] = spec
            if queue >= 0:
                self.port_queues[idx] = queue
            p = self._ports[idx] = _make_port(self.nf, spec, self.queues, self._gpu_rings())
            if self._eng is not None:
                self._eng.add_port(int(idx), p, self._queue_for(idx))

    def remove_port(self, idx: int):
        with self._lock:
            self.specs.pop(idx, None)
            self.port_queues.pop(idx, None)
            self._ports.pop(idx, None)
            if self._eng is not None:
                return self._eng.remove_port(int(idx))

    def port(self, idx: int):
        return self._ports.get(idx)

    def port_queue(self, idx: int) -> int:
        return int(self._eng.port_queue(int(idx))) if self._eng is not None else -1

    # ------------------------------------------------------------------ slow path + supervision
    def poll_punts(self) -> int:
        eng = self._eng
        if eng is None:
            return 0
        n = 0
        for frame, in_port, reason in eng.take_punts(1024):
            n += 1
            if reason == 14:        # IPv6-underlay tunnel to the local VTEP: the VNI needs the whole frame
                r6 = self.dps[0].resolve_recirc6(frame)
                if r6 is not None:
                    eng.inject(int(r6[0]), bytes(r6[1]))
                    continue
                reason = 5
            self.punts += 1
            if self.on_punt is not None:
                try:
                    self.on_punt(frame, in_port, reason)
                except Exception:  # noqa: BLE001 - a slow-path handler must not stop the path
                    log.exception("punt handler failed")
        return n

    def _supervise(self) -> None:
        while not self._stop.wait(0.005):
            self.poll_punts()
            eng = self._eng
            if eng is None:
                continue
            if self.gpu and self.zero_copy and self.nf.deferred_host_unmaps() > self.max_deferred_unmaps:
                from .engine import commit_guard

                with commit_guard(self.dps), self._lock:   # (no commit flips rings being replaced)
                    log.warning("native I/O engine: %d removed zero-copy regions still pinned: restarting the rings "
                                "to release them", self.nf.deferred_host_unmaps())
                    self._teardown()          # (the last grid's stop unregisters them)
                    self._build()
                    self.unmap_restarts += 1
                continue
            err = eng.error()
            if err:
                self.error = err
                self.healthy = False
                log.error("native I/O engine failed: %s", err)
                if not self.auto_restart:
                    continue
                with self._lock:
                    try:
                        self._teardown()
                        self._build()
                        self.restarts += 1
                        self.healthy = True
                        log.warning("native I/O engine restarted (%d)", self.restarts)
                    except Exception as e:  # noqa: BLE001
                        self.error = f"restart failed: {e}"
                        log.exception("native I/O engine restart failed")
                        time.sleep(0.5)

    # ------------------------------------------------------------------ observability
    def _accumulate(self) -> None:
        if self._eng is None:
            return
        for k, v in self._eng.stats().items():
            if k != "queues":
                self._totals[k] = self._totals.get(k, 0) + int(v)

    @property
    def stats(self) -> dict:
        s = dict(self._totals)
        if self._eng is not None:
            for k, v in self._eng.stats().items():
                s[k] = (s.get(k, 0) if k != "queues" else 0) + int(v)
        s["punt_handled"] = self.punts
        s["restarts"] = self.restarts
        return s

    def latency_us(self) -> np.ndarray:
        """Engine-side rx -> tx time of every burst since the last call (µs)."""
        return np.asarray(self._eng.take_latency_us()) if self._eng is not None else np.zeros(0)

    def fault(self, what: str = "injected") -> None:
        """Test hook: make the engine fail as an I/O error would (the supervisor restarts it)."""
        if self._eng is not None:
            self._eng.inject_failure(what)


def memif_dir() -> str:
    d = os.environ.get("DPU_MEMIF_DIR") or ("/dev/shm" if os.path.isdir("/dev/shm") else "/tmp")
    return d
