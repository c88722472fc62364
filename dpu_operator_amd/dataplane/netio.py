"""Live packet path: vport netdevs <-> the data plane.

The reference moves real frames between pod netdevs through veth pairs and the OvS bridge
(vspnetutils.go:141-208, marvell/main.go:105-154).  Here every data-plane port that
faces a pod or an NF is a TAP netdev owned by the VSP: the CNI moves it into the pod's network
namespace like any DPU netdev (networkfn.go:233-317), and the VSP keeps its file descriptor, so
what the pod sends arrives on that fd and what the VSP writes to it is what the pod receives.

``LivePath`` is the loop between those fds and the pipeline:

    poll(all vport fds) -> read bursts (up to `burst` frames, every port) -> header slots
      (first 64 B) + ingress meta (port | len << 16); the frames stay in host memory
    -> DataPlane.run: the fused HIP kernel on the GPU (batch uploaded to HBM) or the oracle
    -> every forwarded frame: ohdr[:hl] ++ frame[to:len] (nfdp.h out_tail) written to the egress
       port's fd; flood / mirror replicas the same way from the side outputs; ARP copies trapped to
       the slow path go to `on_punt`; frames for ports without a netdev (the uplink when none is
       attached) are counted as `no_netdev`;
    -> tunnel ports: the side pass's 50-B outer header is prepended and the frame leaves on the
       tunnel's underlay port; terminated tunnel traffic (reason `recirc`) is re-injected, inner
       frame only, as received on the tunnel port, in the next cycle (P4 do_recirculate).

Two engines run the pipeline under this loop:
  engine="batch" (default)  DataPlane.run per cycle: header slots uploaded, fused kernel, side kernel
  engine="ring"             the persistent ring kernel with its slots in pinned host memory
                            (RingPath host_slots=True): the loop writes header slots + in-meta
                            straight into the ring (bursts padded to whole 64-packet chunks with
                            filler slots that count nowhere), publishes, waits for the completion
                            flags, reads egress slots + meta from the same pinned buffers and runs
                            the side kernel over the ring's side list.  No launch per burst, no
                            copies: the resident kernel reads and writes the host slots over PCIe.
                            Table commits keep working (flow updates by epoch flip, anything else
                            drains and relaunches the ring between bursts); a ring that outlives its
                            device deadline is relaunched.

Every cycle records its stage times (rx / pipeline / side / tx / batch) and, on the GPU, the
kernel's sampled per-packet latencies into `dp.latency` (utils/latency.py), which the data-plane
metrics collector exports as `dpu_packet_latency_seconds{stage=...}` histograms.

Frames are whole Ethernet frames without FCS (TAP, IFF_NO_PI).  MAC learning, flooding, VLAN
tags, SNAT etc. are the pipeline's; this loop only moves bytes.
"""
from __future__ import annotations

import errno
import fcntl
import logging
import os
import select
import struct
import threading
import time

import numpy as np

from ..ops import packets as P

log = logging.getLogger("dpu.netio")

TUNSETIFF = 0x400454CA
IFF_TAP, IFF_NO_PI = 0x0002, 0x1000


class TapPort:
    """A TAP netdev whose fd the data plane owns (non-blocking)."""

    def __init__(self, name: str, mac: str | None = None, nl=None):
        if len(name) > 15:
            raise ValueError("interface names are at most 15 characters")
        self.name = name
        self.fd = os.open("/dev/net/tun", os.O_RDWR | os.O_NONBLOCK)
        try:
            fcntl.ioctl(self.fd, TUNSETIFF, struct.pack("16sH", name.encode(), IFF_TAP | IFF_NO_PI))
        except OSError:
            os.close(self.fd)
            raise
        if mac and nl is not None:
            nl.link_set_hw_addr(name, mac)
        self.rx = self.tx = self.tx_err = 0

    def read(self) -> bytes | None:
        try:
            f = os.read(self.fd, 1 << 16)
        except BlockingIOError:
            return None
        except OSError as e:
            if e.errno in (errno.EAGAIN, errno.EIO):  # EIO: the netdev is down
                return None
            raise
        self.rx += 1
        return f

    def write(self, frame: bytes) -> bool:
        try:
            os.write(self.fd, frame)
            self.tx += 1
            return True
        except OSError:  # down / no carrier: the frame is lost, as on a wire
            self.tx_err += 1
            return False

    def close(self) -> None:
        if self.fd >= 0:
            os.close(self.fd)
            self.fd = -1


class LivePath:
    def __init__(self, dp, ports: dict, burst: int = 256, on_punt=None, engine: str = "batch",
                 ring_capacity: int = 4096):
        if engine not in ("batch", "ring"):
            raise ValueError("engine is 'batch' or 'ring'")
        if engine == "ring" and not dp.gpu:
            raise ValueError("the ring engine needs a GPU data plane")
        self.engine = engine
        self.ring_capacity = int(ring_capacity)
        self.ring = None
        if engine == "ring" and burst > self.ring_capacity:
            raise ValueError("burst must fit the ring")
        self.dp = dp
        self.ports = dict(ports)          # data-plane port -> TapPort (anything with read/write/fd)
        self.burst = burst
        self.on_punt = on_punt            # f(frame: bytes, in_port: int, reason: int)
        self.stats = {"rx": 0, "tx": 0, "replicas": 0, "punt": 0, "drop": 0, "no_netdev": 0, "batches": 0}
        self._stop = threading.Event()
        self._t: threading.Thread | None = None
        self._lock = threading.Lock()     # port map changes vs the loop
        self.error: BaseException | None = None
        self.healthy = True
        self.restarts = 0
        self._recirc: list[tuple[bytes, int]] = []
        self.stats["recirc"] = 0
        # IPsec boundary (dataplane/ipsec.py, the GPU ESP engine): ESP arriving on these ports is
        # authenticated + decrypted before the header pipeline, frames leaving them pass the SPD
        # (protect -> ESP, bypass, drop) in one batch per cycle
        self.ipsec_ports: set[int] = set()
        self._esp_out: list[tuple[int, bytes]] = []
        self.stats.update(esp_in=0, esp_out=0, esp_drop=0)

    # ------------------------------------------------------------------ port map
    def add_port(self, idx: int, port) -> None:
        with self._lock:
            self.ports[idx] = port

    def remove_port(self, idx: int):
        with self._lock:
            return self.ports.pop(idx, None)

    # ------------------------------------------------------------------ one cycle
    def _gather(self, timeout: float) -> tuple[list[bytes], list[int]]:
        with self._lock:
            items = list(self.ports.items())
        if not items:
            time.sleep(timeout)
            return [], []
        p = select.poll()
        fd2port = {}
        for idx, port in items:
            p.register(port.fd, select.POLLIN)
            fd2port[port.fd] = (idx, port)
        frames, src = [], []
        if self._recirc:  # decapsulated frames re-enter first, without waiting
            frames, src = [f for f, _ in self._recirc], [q for _, q in self._recirc]
            self._recirc = []
            timeout = 0
        ready = p.poll(int(timeout * 1000))
        self._t_ready = time.perf_counter()   # frames are waiting: the batch's clock starts here
        for fd, _ev in ready:
            idx, port = fd2port[fd]
            while len(frames) < self.burst:
                f = port.read()
                if f is None:
                    break
                if 14 <= len(f) <= P.MAX_FRAME:
                    frames.append(f)
                    src.append(idx)
        return frames, src

    def _send(self, port_idx: int, frame: bytes) -> None:
        a = self.dp.ports.a
        if 0 <= port_idx < len(a) and a[port_idx]["flags"] & (1 << 14):  # tunnel port: its underlay
            tab = self.dp.tunnels6 if a[port_idx]["flags"] & (1 << 18) else self.dp.tunnels
            port_idx = int(tab.a[int(a[port_idx]["lag"])]["out_port"])
        if port_idx in self.ipsec_ports:
            self._esp_out.append((port_idx, frame))   # encrypted as one batch at the end of the cycle
            return
        self._write(port_idx, frame)

    def _write(self, port_idx: int, frame: bytes) -> None:
        port = self.ports.get(port_idx)
        if port is None:
            self.stats["no_netdev"] += 1
        elif port.write(frame):
            self.stats["tx"] += 1

    def _esp_inbound(self, frames: list, src: list) -> tuple[list, list]:
        """Decrypt the ESP frames of the batch that arrived on IPsec ports (one kernel launch);
        no SA -> slow path, authentication / replay failure -> dropped."""
        idx = [i for i, (f, p) in enumerate(zip(frames, src))
               if p in self.ipsec_ports and len(f) >= 34 and f[12:14] == b"\x08\x00" and f[23] == 50]
        if not idx:
            return frames, src
        dec, st = self.dp.ipsec.decrypt([frames[i] for i in idx])
        keep = np.ones(len(frames), bool)
        frames = list(frames)
        for k, i in enumerate(idx):
            if dec[k] is not None:
                frames[i] = dec[k]
                self.stats["esp_in"] += 1
            else:
                keep[i] = False
                if int(st[k]) == 4 and self.on_punt:       # no SA: the IPsec control plane's business
                    self.on_punt(bytes(frames[i]), src[i], 5)
                    self.stats["punt"] += 1
                else:
                    self.stats["esp_drop"] += 1
        return [f for f, k in zip(frames, keep) if k], [p for p, k in zip(src, keep) if k]

    def _esp_flush(self) -> None:
        if not self._esp_out:
            return
        out, self._esp_out = self._esp_out, []
        enc, _ = self.dp.ipsec.encrypt([f for _, f in out])
        for (port_idx, _), f in zip(out, enc):
            if f is None:
                self.stats["esp_drop"] += 1
            else:
                self.stats["esp_out"] += 1
                self._write(port_idx, f)

    def poll_once(self, timeout: float = 0.05) -> int:
        from ..utils.faults import FAULTS

        FAULTS.check("livepath.poll")
        self._t_ready = time.perf_counter()
        frames, src = self._gather(timeout)
        if self.ipsec_ports and frames:
            frames, src = self._esp_inbound(frames, src)
        n = len(frames)
        if not n:
            return 0
        t_start = self._t_ready
        t_rx = time.perf_counter()
        lens = np.array([len(f) for f in frames], np.uint32)
        slots = np.zeros((n, 64), np.uint8)
        for i, f in enumerate(frames):
            h = f[:64]
            slots[i, : len(h)] = np.frombuffer(h, np.uint8)
        im = P.inmeta(np.array(src, np.uint32), lens)
        if self.engine == "ring":
            out, meta, side, t_pipe = self._run_ring(slots, im)
            t_side = time.perf_counter()
            return self._deliver(frames, src, lens, out, meta, side, t_start, t_rx, t_pipe, t_side)
        if self.dp.gpu:
            import torch

            r = self.dp.run(torch.from_numpy(slots).to(self.dp.tdev), torch.from_numpy(im.view(np.int32)).to(self.dp.tdev))
            out = r.out.cpu().numpy()
            meta = r.meta.cpu().numpy().view(np.uint32)
            t_pipe = time.perf_counter()
            self.dp.fold_device_latency(r)
        else:
            r = self.dp.run(slots, im)
            out, meta = r.out, r.meta
            t_pipe = time.perf_counter()
        side = self.dp.side_result() if self.dp.side_active() else {"n_rep": 0}
        t_side = time.perf_counter()
        return self._deliver(frames, src, lens, out, meta, side, t_start, t_rx, t_pipe, t_side)

    def _run_ring(self, slots: np.ndarray, im: np.ndarray):
        """One burst through the persistent ring (host slots): returns out, meta, side, t_pipe."""
        if self.ring is None:
            self._ring_init()
        ring, n, c = self.ring, len(slots), self.ring_capacity
        n_pad = (n + 63) & ~63
        with ring.lock:
            if ring.ensure_alive():
                self.stats["ring_relaunch"] += 1
            pos = int(ring.eng.published) % c
            idx = (pos + np.arange(n_pad)) % c
            self._rin[idx[:n]] = slots
            self._rim[idx[:n]] = im
            self._rim[idx[n:]] = 0xFFFFFFFF          # filler slots (ring.h kRingPadMeta)
            ring.reset_side()
            end = ring.publish(n_pad)
            ring.wait(end, 5.0)
            out = self._rout[idx[:n]].copy()
            meta = self._rmeta[idx[:n]].copy()
            t_pipe = time.perf_counter()
            side = {"n_rep": 0}
            if self.dp.side_active():
                side = ring.side_pass()
                if side.get("n_learn"):
                    ring.eng.bump_epoch()             # learned MACs: the next chunks drop cached lines
                if side.get("n_rep"):                 # ring slot -> burst index
                    side["rep_src"] = (side["rep_src"].astype(np.int64) - pos) % c
                if side.get("xhdr") is not None:
                    side["xhdr"] = side["xhdr"][idx[:n]]
        return out, meta, side, t_pipe

    def _ring_init(self) -> None:
        """Launch the resident kernel (commits the data plane: call from the thread that owns
        table changes, i.e. start(), not the loop thread)."""
        from .ring import RingPath

        self.ring = RingPath(self.dp, capacity=self.ring_capacity, host_slots=True, coop=True, side=True,
                             deadline_s=3600.0)
        self.ring.start()
        self._rin, self._rim, self._rout, self._rmeta = self.ring.host_arrays()
        self.stats["ring_relaunch"] = 0

    def _deliver(self, frames, src, lens, out, meta, side, t_start, t_rx, t_pipe, t_side) -> int:
        n = len(frames)
        lat = self.dp.latency
        self.stats["rx"] += n
        self.stats["batches"] += 1
        port, olen, reason = P.meta_fields(meta)
        xh = side.get("xhdr")
        for i in range(n):
            if reason[i] == 13:  # tunnel terminated: the inner frame re-enters on the tunnel port
                self._recirc.append((frames[i][int(lens[i]) - int(olen[i]):], int(port[i])))
                self.stats["recirc"] += 1
                continue
            if reason[i] == 14:  # IPv6-underlay tunnel to the local VTEP: the VNI lookup needs the whole frame
                r6 = self.dp.resolve_recirc6(frames[i][: int(lens[i])])
                if r6 is not None:
                    self._recirc.append((r6[1], r6[0]))
                    self.stats["recirc"] += 1
                else:
                    self.stats["punt"] += 1
                    if self.on_punt:
                        self.on_punt(bytes(frames[i][: int(lens[i])]), src[i], 5)
                continue
            if reason[i]:
                self.stats["drop"] += 1
                continue
            rec = xh[i] if (xh is not None and P.meta_xhdr(meta[i:i + 1])[0]) else None
            self._send(int(port[i]), P.assemble(out[i], int(meta[i]), np.frombuffer(frames[i], np.uint8), int(lens[i]), rec))
        for k in range(side.get("n_rep", 0)):
            s = int(side["rep_src"][k])
            m = int(side["rep_meta"][k])
            rp, _, rr = P.meta_fields(np.array([m], np.uint32))
            fr = P.assemble(side["rep_hdr"][k], m, np.frombuffer(frames[s], np.uint8), int(lens[s]))
            if int(rr[0]):
                self.stats["punt"] += 1
                if self.on_punt:
                    self.on_punt(fr, src[s], int(rr[0]))
            else:
                self.stats["replicas"] += 1
                self._send(int(rp[0]), fr)
        self._esp_flush()
        t_end = time.perf_counter()
        lat.observe("rx", t_rx - t_start)
        lat.observe("pipeline", t_pipe - t_rx)
        lat.observe("side", t_side - t_pipe)
        lat.observe("tx", t_end - t_side)
        lat.observe("batch", t_end - t_start)
        return n

    # ------------------------------------------------------------------ thread
    def _run(self) -> None:
        """The loop survives its own failures: an exception marks the path unhealthy (the VSP
        reports its vports unhealthy to the device plugin), the engine state is rebuilt (a ring
        that failed is relaunched) and forwarding resumes after a backoff; the first successful
        cycle marks it healthy again."""
        backoff = 0.05
        while not self._stop.is_set():
            try:
                self.poll_once(0.02)
                if not self.healthy:
                    self.healthy = True
                    backoff = 0.05
                    log.warning("live path recovered (restart %d)", self.restarts)
            except BaseException as e:  # noqa: BLE001 - surfaced through .error / .healthy
                self.error = e
                self.healthy = False
                self.restarts += 1
                log.exception("live path cycle failed; restarting")
                if self.ring is not None:
                    try:
                        self.ring.close()
                    except Exception:  # noqa: BLE001
                        pass
                    self.ring = None      # relaunched by the next ring cycle
                self._recirc = []
                self._stop.wait(backoff)
                backoff = min(backoff * 2, 2.0)

    def start(self) -> "LivePath":
        if self.engine == "ring" and self.ring is None:
            self._ring_init()
        self._t = threading.Thread(target=self._run, daemon=True, name="dpu-livepath")
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=5)
        if self.ring is not None:
            self.ring.close()
            self.ring = None
