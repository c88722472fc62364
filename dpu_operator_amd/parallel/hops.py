"""SFC hop pipeline across GPUs, device-resident: split chains with peer-store hand-offs over xGMI.

A chain whose hops are placed on different GPU planes (``ChainTable`` hops such as ``"ttl@1"``,
kHopXfer in csrc/nfdp/nfdp.h) runs hop by hop across the node's GPUs:

1. the entry plane's fused kernel (its XFER instance) classifies the batch and runs the hops up to
   the hand-off; a handed-off frame leaves its header slot (as the hops so far rewrote it), a meta
   word REMOTE | plane and a 32-B HopState record (ingress port + length, Toeplitz hash, ACL rule,
   resume hop, the flow's action);
2. ``hop_pack_kernel`` on the entry GPU gathers the frames for plane t and stores them - slot,
   record, source index - straight into plane t's inbox in that GPU's HBM (peer stores over xGMI
   with peer access enabled; the same kernel when both planes share a device), then a one-thread
   publish step writes the inbox count and resets the fill counter;
3. plane t's stream waits for the entry stream's event and ``resume_kernel`` runs the rest of the
   chain over the inbox (count read on the device: no host round trip anywhere), counting tx and
   drops on plane t; a frame its chain hands on again is packed from plane t's results the same
   way (depth = the most hand-offs any chain has).

Nothing passes through host memory and the host never waits: a step is launches and events only.
The frames stay on the GPU where their chain ends (that GPU's ports egress them); ``results()``
scatters every frame's final slot and meta back into arrival order for checks (a test / bench
helper, host synchronising).  ``MultiDataPlane.run`` (dataplane/multi.py) is the host-array API
over the same kernels' semantics; both match the one-plane chain bit for bit
(tests/test_hop_pipeline.py on the oracle, tests/test_hop_pipeline_gpu.py on the GPU).

Reference: the Marvell VSP chains NFs port to port (/root/reference/internal/daemon/
vendor-specific-plugins/marvell/main.go:490-563); BASELINE config 4 is SFC hops across devices.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

REMOTE = 10


@dataclass
class _Inbox:
    src: int            # index into self.stages (the buffer the frames come from)
    plane: int          # the plane that resumes them
    count: object       # [1] int32 on the plane's device
    hdr: object         # [cap, 64] uint8
    state: object       # [cap, 8] int32
    idx: object         # [cap] int32 (index in the source buffer)
    fill: object        # [1] int32 on the SOURCE device
    out: object         # resume results [cap, 64] / [cap] / [cap, 8]
    meta: object
    nxt: object
    last: object = None  # event after the latest resume over this inbox (the next pack waits for it)


class HopPipeline:
    def __init__(self, planes, batch: int, entry: int = 0, streams=None):
        """streams: per plane, the torch.cuda.Stream its kernels run on (None: the device's current
        stream at each step).  Consecutive steps reuse the inboxes: a step's pack into an inbox
        waits for the previous step's resume over it, whatever streams the planes use."""
        import torch

        self.torch = torch
        self.streams = list(streams) if streams is not None else None
        self.planes = planes
        self.batch = batch
        self.entry = entry
        nf = planes[0].nf
        self.nf = nf
        targets = sorted(planes[0].chains.xfer_planes())
        if not targets:
            raise ValueError("no split chain: nothing hands a frame to another plane")
        if max(targets) >= len(planes):
            raise ValueError(f"chains hand frames to plane {max(targets)}, only {len(planes)} planes")
        devs = [p.tdev for p in planes]
        for a in devs:
            for b in devs:
                if a != b and not nf.enable_peer_access(a.index, b.index):
                    raise RuntimeError(f"{a} cannot store into {b}'s memory (no peer access)")
        # hand-off depth: the most kHopXfer ops in any chain
        ch = planes[0].chains
        a = ch.a[: ch.n]
        depth = max(int(sum(int(c) >= 0x10 for c in r["hop"][: int(r["nhops"])])) for r in a)
        self.depth = depth
        p0 = planes[entry]
        self.out0, self.meta0, self.lat0 = p0.alloc_batch(batch)
        self.hop0 = None
        # stage 0 = the entry plane's batch; every inbox is a further stage (its resume results)
        self.stages = [("entry", entry)]
        self.inboxes: list[_Inbox] = []
        frontier = [0]
        for _ in range(depth):
            nxt_frontier = []
            for si in frontier:
                src_plane = self.stages[si][1]
                for t in targets:
                    d = devs[t]
                    ib = _Inbox(
                        src=si, plane=t,
                        count=torch.zeros(1, dtype=torch.int32, device=d),
                        hdr=torch.empty((batch, 64), dtype=torch.uint8, device=d),
                        state=torch.empty((batch, 8), dtype=torch.int32, device=d),
                        idx=torch.empty(batch, dtype=torch.int32, device=d),
                        fill=torch.zeros(1, dtype=torch.int32, device=devs[src_plane]),
                        out=torch.empty((batch, 64), dtype=torch.uint8, device=d),
                        meta=torch.empty(batch, dtype=torch.int32, device=d),
                        nxt=torch.zeros((batch, 8), dtype=torch.int32, device=d))
                    self.inboxes.append(ib)
                    self.stages.append(("inbox", t, len(self.inboxes) - 1))
                    nxt_frontier.append(len(self.stages) - 1)
            frontier = nxt_frontier

    def _stage_buffers(self, si: int):
        """(out, meta, hop_state, n_dev pointer) of stage si."""
        if si == 0:
            return self.out0, self.meta0, self.hop0, 0
        ib = self.inboxes[self.stages[si][2]]
        return ib.out, ib.meta, ib.nxt, ib.count.data_ptr()

    def _stream(self, plane: int):
        if self.streams is not None and self.streams[plane] is not None:
            return self.streams[plane]
        return self.torch.cuda.current_stream(self.planes[plane].tdev)

    def step(self, pkts, inmeta, timing: dict | None = None) -> None:
        """One batch through the split chains (launches and events only; no host wait).  `timing`:
        a dict that receives CUDA events {fused, handoff, resume} boundaries (for the bench)."""
        torch = self.torch
        p0 = self.planes[self.entry]
        s0 = self._stream(self.entry)
        ev = (lambda: torch.cuda.Event(enable_timing=True)) if timing is not None else None
        if timing is not None:
            timing["t0"] = ev()
            timing["t0"].record(s0)
        # (the entry buffers are rewritten on s0: the previous step's packs read them on s0 too;
        # s0 current while run() allocates, so its per-batch buffers belong to that stream)
        with torch.cuda.stream(s0):
            r = p0.run(pkts, inmeta, out=self.out0, meta=self.meta0, lat=self.lat0)
        self.hop0 = r.extra["hop_state"]
        if timing is not None:
            timing["fused"] = ev()
            timing["fused"].record(s0)
        n = int(pkts.shape[0])
        done: dict[int, object] = {0: None}
        for k, ib in enumerate(self.inboxes):
            src_plane = self.stages[ib.src][1]
            ss = self._stream(src_plane)
            if ib.src in done and done[ib.src] is not None:
                ss.wait_event(done[ib.src])
            if ib.last is not None:   # the previous step's resume still reads this inbox
                ss.wait_event(ib.last)
            out, meta, hop, n_dev = self._stage_buffers(ib.src)
            self.nf.launch_hop_pack(out.data_ptr(), meta.data_ptr(), hop.data_ptr(), n if ib.src == 0 else self.batch,
                                    n_dev, ib.plane, ib.fill.data_ptr(), ib.count.data_ptr(), ib.hdr.data_ptr(),
                                    ib.state.data_ptr(), ib.idx.data_ptr(), self.batch, ss.cuda_stream)
            e = torch.cuda.Event(enable_timing=timing is not None)
            e.record(ss)
            if timing is not None and "handoff" not in timing:
                timing["handoff"] = e
            q = self.planes[ib.plane]
            sq = self._stream(ib.plane)
            sq.wait_event(e)
            self.nf.launch_resume(q.tables_ptrs(), ib.count.data_ptr(), ib.hdr.data_ptr(), ib.state.data_ptr(),
                                  ib.idx.data_ptr(), self.batch, ib.out.data_ptr(), ib.meta.data_ptr(),
                                  ib.nxt.data_ptr(), q._ptr("port_ctr"), q._ptr("drop_ctr"), 0, q.num_cus,
                                  sq.cuda_stream)
            e2 = torch.cuda.Event(enable_timing=timing is not None)
            e2.record(sq)
            done[k + 1] = e2
            ib.last = e2
            if timing is not None:
                timing["resume"] = e2

    def synchronize(self) -> None:
        for i, p in enumerate(self.planes):
            self._stream(i).synchronize()
            self.torch.cuda.synchronize(p.tdev)

    def results(self, n: int) -> tuple[np.ndarray, np.ndarray]:
        """Every frame's final slot and meta in arrival order (host; synchronises)."""
        self.synchronize()
        out = self.out0[:n].cpu().numpy().copy()
        meta = self.meta0[:n].cpu().numpy().view(np.uint32).copy()
        origin = {0: np.arange(n, dtype=np.int64)}   # stage -> original index of each buffer row
        for k, ib in enumerate(self.inboxes):
            c = int(ib.count.item())
            src_origin = origin.get(ib.src)
            if src_origin is None or c == 0:
                origin[k + 1] = np.zeros(0, np.int64)
                continue
            idx = ib.idx[:c].cpu().numpy().astype(np.int64)
            orig = src_origin[idx]
            origin[k + 1] = np.full(self.batch, -1, np.int64)
            origin[k + 1][:c] = orig
            out[orig] = ib.out[:c].cpu().numpy()
            meta[orig] = ib.meta[:c].cpu().numpy().view(np.uint32)
        return out, meta
