"""Low-latency data path: a persistent HIP kernel polling an ingress ring (csrc/nfdp/ring.hip).

The batch engine (`DataPlane.run`) launches one kernel per batch, so a packet's latency includes
the launch and the wait for the whole batch.  `RingPath` keeps a kernel resident on the CUs:
64-packet chunks are processed as soon as the producer publishes them, and completion flags come
back through pinned host memory, so a pod-to-pod hop costs a few µs instead of a launch.  This is
the GPU form of the always-on datapath the reference configures but never runs itself (the
Intel FXP / OvS-DPDK PMD loop, and the Octeon agent's 1 ms poll loop,
octep_cp_agent/main.c:307-311).

Usage::

    ring = RingPath(dp, capacity=1 << 16)
    ring.stage(frames, inmeta)          # fill ring slots (a NIC would DMA into them)
    ring.start()
    end = ring.publish(4096)            # hand 4096 packets to the resident kernel
    ring.wait(end)
    lat_us, elapsed = ring.probe(batches=2000, batch=64, inflight=1)
    ring.stop()                         # drains every published chunk, then the grid exits
    out, meta = ring.results()

While a ring runs, do NOT synchronize the whole device (torch.cuda.synchronize(), a blocking
copy on the default stream): that waits for the resident kernel.

Table updates while rings run (`DataPlane.commit()`): flow inserts / erases / action changes are
applied without stopping the rings — the flow table is double buffered on the device, the commit
writes the copy no wave reads and flips the epoch carried by the published word; the next commit
first waits for the flip's grace period (every chunk published before it completed; ring.h).
Changes to the LDS-staged tables (ports, chains, ACL, ...) drain, stop and relaunch the rings.
"""
from __future__ import annotations

import ctypes
import threading

import numpy as np

from .engine import DataPlane


class RingPath:
    def __init__(self, dp: DataPlane, capacity: int = 1 << 16, wgs_per_cu: int = 1, deadline_s: float = 120.0,
                 knobs: int = 0, coop: bool = True, host_slots: bool = False, side: bool = False, queues: int = 1,
                 cus: int = 0):
        """coop=True: a workgroup's 4 waves share each chunk (ACL rule tiles split 4 ways) —
        lowest latency.  coop=False: every wave takes its own chunks — highest throughput.
        host_slots=True: the ring slots live in pinned host memory and the resident kernel reads /
        writes the frames over PCIe itself (zero-copy host rings, e.g. pod vhost / AF_XDP).
        side=True: the kernel puts packets that need replicas / learn events / outer headers on
        the data plane's side list; `side_pass()` runs the side kernel over them.
        queues: independent rings served by the one resident grid (workgroup b serves queue
        b % queues): one per producer thread of the native I/O engine (ring.h).
        cus: CUs the resident grid takes (0: all).  Resident grids never yield their CUs, so rings
        sharing one GPU (two planes on one device) must split them, or the later grid never runs."""
        if not dp.gpu:
            raise RuntimeError("RingPath needs a GPU data plane")
        if capacity < 64 or capacity & (capacity - 1):
            raise ValueError("capacity must be a power of two >= 64")
        self.dp = dp
        self.capacity = int(capacity)
        self.deadline_s = float(deadline_s)
        self.knobs = int(knobs) & 0x60  # diagnostic knobs (ring.hip kRingTrace / kRingNoCounters), attribution only
        self.coop = bool(coop)
        self.host_slots = bool(host_slots)
        if queues > 1 and side:
            raise ValueError("the side list indexes one queue's slots: side=True needs queues=1")
        self.queues = int(queues)
        self.cus = int(cus) if cus else int(dp.num_cus)
        if not 1 <= self.cus <= int(dp.num_cus):
            raise ValueError(f"cus must be in [1, {int(dp.num_cus)}]")
        self.eng = dp.nf.RingEngine(self.capacity, self.cus, int(wgs_per_cu), self.coop, self.host_slots,
                                    self.queues)
        self._staged = 0
        self.side = bool(side)
        if self.side and self.capacity > dp.cap_rep:
            raise ValueError(f"a side-list ring holds at most {dp.cap_rep} slots")
        self._side = None
        # a burst (publish -> wait -> read) and a stop / relaunch for a table commit exclude
        # each other: DataPlane.commit() may run on another thread (the VSP's RPCs)
        self.lock = threading.RLock()
        self.launches = 0            # grid launches (start / resume after a drain)
        rings = getattr(dp, "_rings", None)
        if rings is None:
            dp._rings = rings = []
        rings.append(self)

    # ------------------------------------------------------------------ staging
    def stage(self, frames, inmeta) -> int:
        """Copy frames into the ring slots, repeated cyclically to fill all of them (a replayed
        trace).  Must be called while the ring is stopped."""
        if self.eng.running:
            raise RuntimeError("stage() while the ring runs")
        torch = _torch()
        f = frames if isinstance(frames, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frames))
        m = inmeta if isinstance(inmeta, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(inmeta).view(np.int32))
        f = f.to(self.dp.tdev).reshape(-1, 64).contiguous()
        m = m.to(self.dp.tdev).view(torch.int32).reshape(-1).contiguous()
        n = int(f.shape[0])
        if n == 0 or m.numel() != n:
            raise ValueError("frames / inmeta size mismatch")
        reps = (self.capacity + n - 1) // n
        f = f.repeat(reps, 1)[: self.capacity].contiguous()
        m = m.repeat(reps)[: self.capacity].contiguous()
        torch.cuda.current_stream(self.dp.tdev).synchronize()
        nf = self.dp.nf
        nf.memcpy(self.eng.dev_in(), f.data_ptr(), self.capacity * 64)
        nf.memcpy(self.eng.dev_inmeta(), m.data_ptr(), self.capacity * 4)
        self._staged = n
        return n

    # ------------------------------------------------------------------ session
    def _args(self) -> dict:
        dp = self.dp
        a = {"flow_ctr": dp._ptr("flow_ctr"), "port_ctr": dp._ptr("port_ctr"), "drop_ctr": dp._ptr("drop_ctr"),
             "acl_wfrag": dp._ptr("acl_wfrag"), "acl_cinit": dp._ptr("acl_cinit"), "acl_tiles": dp._acl_tiles,
             "toep_frag": dp._ptr("toep_frag"), "toep_tab": dp._ptr("toep_tab"),
             "flags": (0 if dp.count_flows else 4) | self.knobs}
        if self.side:
            self._side = dp._side_buffers(self.capacity)
            a["side"] = self._side
        return a

    @property
    def running(self) -> bool:
        return bool(self.eng.running)

    def _tables(self) -> dict:
        t = self.dp.tables_ptrs()
        t["flows"], t["flows_alt"] = self.dp.flow_copy_ptrs()   # copies by epoch parity
        # the kernel instance depends on it (ring.hip V6): a live table flip keeps it
        self.v6 = bool(t["flow6_on"] or t["n_acl6"])
        return t

    def start(self) -> None:
        self.dp.enable_flow_flip()   # commits; second flow-table copy for live updates
        self.dp.commit()
        _torch().cuda.current_stream(self.dp.tdev).synchronize()  # tables are in HBM before launch
        self.eng.set_epoch(self.dp._flow_active)
        self.eng.start(self._tables(), self._args(), self.dp.hash_mode, self.dp.acl_mode,
                       self.cus, self.deadline_s)
        self.eng.set_ctrl_regions(self.dp.ctrl_regions())
        self.launches += 1

    def stop(self, timeout_s: float = 30.0) -> None:
        with self.lock:
            self.eng.stop(timeout_s)

    def resume(self) -> None:
        """Relaunch over the current device tables (DataPlane.commit stops, updates, resumes)."""
        with self.lock:
            _torch().cuda.current_stream(self.dp.tdev).synchronize()
            self.eng.set_epoch(self.dp._flow_active)
            self.eng.start(self._tables(), self._args(), self.dp.hash_mode, self.dp.acl_mode,
                           self.cus, self.deadline_s)
            self.eng.set_ctrl_regions(self.dp.ctrl_regions())
            self.launches += 1

    def ensure_alive(self) -> bool:
        """Relaunch a ring whose grid left on its own (device deadline); True if it was relaunched."""
        with self.lock:
            if self.eng.running and not self.eng.alive():
                self.eng.stop(5.0)
                self.resume()
                return True
        return False

    # ------------------------------------------------------------------ live I/O (host slots)
    def host_arrays(self) -> tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """numpy views of the pinned slot buffers (host_slots rings): in [C,64] u8, inmeta [C] u32,
        out [C,64] u8, meta [C] u32.  The producer writes `in` / `inmeta` before publishing."""
        c = self.capacity
        pin, pim, pout, pmeta = self.eng.host_view()

        def view(ptr, n, dt):
            return np.ctypeslib.as_array((ctypes.c_uint8 * (n * np.dtype(dt).itemsize)).from_address(ptr)).view(dt)

        return (view(pin, c * 64, np.uint8).reshape(c, 64), view(pim, c, np.uint32),
                view(pout, c * 64, np.uint8).reshape(c, 64), view(pmeta, c, np.uint32))

    def reset_side(self) -> None:
        """Empty the side list before a burst (the ring must be idle: every published chunk done)."""
        if self._side is not None:
            self.dp._dev["side_cnt"][:] = 0
            _torch().cuda.current_stream(self.dp.tdev).synchronize()

    def side_pass(self) -> dict:
        """Side kernel over what the ring put on the side list since reset_side() (replicas,
        learn events applied to the device MAC table, tunnel outer headers); rep_src are ring
        slot indices.  Call once the burst's chunks completed."""
        if self._side is None:
            return {"n_rep": 0}
        dp = self.dp
        s = _torch().cuda.current_stream(dp.tdev).cuda_stream
        dp.nf.launch_side(dp.tables_ptrs(), self.eng.dev_in(), self.eng.dev_inmeta(), self.eng.dev_out(),
                          self.eng.dev_meta(), self._side, dp._ptr("port_ctr"), dp._ptr("drop_ctr"), s,
                          self.capacity, True)
        dp._apply_learn(s)
        return dp.side_result()

    def publish(self, n: int) -> int:
        return int(self.eng.publish(int(n)))

    def completed(self) -> int:
        return int(self.eng.completed())

    def wait(self, end: int, timeout_s: float = 10.0) -> None:
        if not self.eng.wait(int(end), float(timeout_s)):
            raise TimeoutError(f"ring: packets below {end} not completed within {timeout_s} s")

    def probe(self, batches: int, batch: int = 64, inflight: int = 1) -> tuple[np.ndarray, float]:
        """Closed-loop publish -> completion latencies (µs, host clock) and total elapsed seconds."""
        lat, el = self.eng.probe(int(batches), int(batch), int(inflight))
        return np.asarray(lat), float(el)

    # ------------------------------------------------------------------ results
    def results(self) -> tuple[np.ndarray, np.ndarray]:
        """Egress slots and metadata of the whole ring (read after stop())."""
        if self.eng.running:
            raise RuntimeError("results() while the ring runs (stop it first)")
        out = np.empty((self.capacity, 64), np.uint8)
        meta = np.empty(self.capacity, np.uint32)
        self.dp.nf.memcpy(out.ctypes.data, self.eng.dev_out(), out.nbytes)
        self.dp.nf.memcpy(meta.ctypes.data, self.eng.dev_meta(), meta.nbytes)
        return out, meta

    def peek(self, start: int = 0, n: int | None = None) -> tuple[np.ndarray, np.ndarray]:
        """Egress slots / metadata of ring slots [start, start + n) while the ring may run: only
        slots of completed chunks that no later publish reused hold meaningful data."""
        n = self.capacity - start if n is None else n
        if start < 0 or n < 0 or start + n > self.capacity:
            raise ValueError("peek range outside the ring")
        out = np.empty((n, 64), np.uint8)
        meta = np.empty(n, np.uint32)
        self.dp.nf.memcpy_nb(out.ctypes.data, self.eng.dev_out() + 64 * start, out.nbytes)
        self.dp.nf.memcpy_nb(meta.ctypes.data, self.eng.dev_meta() + 4 * start, meta.nbytes)
        return out, meta

    def service_ticks(self, phases: bool = False) -> np.ndarray:
        """Per-chunk device service time (chunk visible -> flag written), 10 ns ticks.  With
        phases=True: [chunks, 8] stage stamps (filled when the ring runs with the trace knob)."""
        if self.eng.running:
            raise RuntimeError("service_ticks() while the ring runs")
        t = np.empty((self.capacity // 64, 8), np.uint32)
        self.dp.nf.memcpy(t.ctypes.data, self.eng.dev_svc(), t.nbytes)
        return t if phases else t[:, 7].copy()

    def close(self) -> None:
        if self.eng.running:
            self.eng.stop(30.0)
        rings = getattr(self.dp, "_rings", [])
        if self in rings:
            rings.remove(self)


def _torch():
    import torch

    return torch

