"""Replicated-table multi-GPU data plane: one process per GPU, ONE all-to-all per chunk.

MI355X-first alternative to flow sharding (parallel/sharded.py).  With 288 GB of HBM3E per GPU
the whole state (1M flows = 64 MB of cuckoo buckets, ports/chains/MAC/ACL in KBs) is replicated on
every GPU, so a GPU classifies, looks up and runs the chain for its own ingress traffic with the
full-speed fused kernel — no descriptor/verdict round trip.  Only frames whose egress port lives
on another GPU cross xGMI: the fused kernel's REMOTE variant writes them straight into the
destination GPU's fixed-capacity segment (block-aggregated slot reservation), and a single
`all_to_all_single` per chunk delivers them; the receiving GPU's egress kernel does tx counting
and latency stamps.  Per step the batch is cut into chunks and pipelined:

    compute stream:  fused(k) | wait a2a(k-1) | egress(k-1) | fused(k+1) | ...
    RCCL stream:               a2a(k) ........ (overlaps egress(k-1) + fused(k+1))

Table updates are broadcast (every rank applies the same control-plane writes); per-flow
counters are per-GPU partials and are summed at harvest (all_reduce).  The CPU twin of the fused
REMOTE kernel lets the same class run on gloo processes for tests.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from ..dataplane.engine import DataPlane


class _Slot:
    """Exchange buffers of one in-flight chunk (reused every RING chunks)."""

    def __init__(self, dev, world: int, cap: int, pseg: int):
        u8 = dict(dtype=torch.uint8, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        self.send = torch.zeros(world * pseg, **u8)
        self.recv = torch.zeros(world * pseg, **u8)
        self.pcnt = torch.zeros(world, **i32)
        self.lat2 = torch.zeros((world * cap + 15) // 16, **i32)


class _Done:
    """Completed-work handle of a synchronous (host-staged) exchange."""

    def wait(self) -> None:
        pass


class ReplicatedDataPlane:
    RING = 3

    def __init__(self, dp: DataPlane, rank: int, world: int, batch: int, chunks: int = 4, slack: float = 1.08,
                 group=None, record_rx: bool = False):
        if world < 2:
            raise ValueError("ReplicatedDataPlane needs world >= 2 (use DataPlane.run for one GPU)")
        self.dp, self.nf = dp, dp.nf
        self.rank, self.world, self.group = rank, world, group
        self.chunks = max(1, chunks)
        self.chunk = int(math.ceil(batch / self.chunks / 16)) * 16  # latency samples index 1/16
        self.batch = batch
        self.gpu = dp.gpu
        self.dev = dp.tdev if self.gpu else torch.device("cpu")
        per = self.chunk / world
        self.cap = int(math.ceil(per * slack + 6 * math.sqrt(per) + 256))
        self.pseg = self.nf.pkt_seg_bytes(self.cap)
        self.slots = [_Slot(self.dev, world, self.cap, self.pseg) for _ in range(min(self.RING, self.chunks))]
        # whole-batch results (chunks write their own ranges)
        self.out = torch.zeros((batch, 64), dtype=torch.uint8, device=self.dev)
        self.out_meta_t = torch.zeros(batch, dtype=torch.int32, device=self.dev)
        self.lat = torch.zeros((batch + 15) // 16, dtype=torch.int32, device=self.dev)
        self.n = 0
        self.record_rx = record_rx
        self.rx_log: list[np.ndarray] = []
        self.t0 = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self.hash_mode = dp.hash_mode if dp.hash_mode != 0 else 1
        self.acl_mode = dp.acl_mode
        # gloo with device buffers (the 1-GPU rehearsal of the N-GPU path: every rank on one card):
        # the exchange is staged through host memory.  RCCL exchanges device buffers directly.
        self.host_staged = self.gpu and dist.is_initialized() and dist.get_backend(group) == "gloo"

    @staticmethod
    def _p(t) -> int:
        return int(t.data_ptr())

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream if self.gpu else 0

    def _geom(self) -> dict:
        return {"nranks": self.world, "rank": self.rank, "cap_desc": 0, "cap_pkt": self.cap}

    def _fused(self, s: _Slot, lo: int, hi: int, pkts: torch.Tensor, inmeta: torch.Tensor) -> None:
        dp, p = self.dp, self._p
        n = hi - lo
        s.pcnt.zero_()
        d = dict(self._geom(), pkts=p(pkts[lo:hi]), inmeta=p(inmeta[lo:hi]), out=p(self.out[lo:hi]),
                 out_meta=p(self.out_meta_t[lo:hi]), n=n,
                 flow_ctr=dp._ptr("flow_ctr") if dp.count_flows else 0, port_ctr=dp._ptr("port_ctr"),
                 drop_ctr=dp._ptr("drop_ctr"), t0=p(self.t0) if self.gpu else 0,
                 lat=p(self.lat[lo // 16:]) if self.gpu else 0,
                 acl_wfrag=dp._ptr("acl_wfrag"), acl_cinit=dp._ptr("acl_cinit"), acl_tiles=dp._acl_tiles,
                 toep_frag=dp._ptr("toep_frag"), toep_tab=dp._ptr("toep_tab"), send_pkt=p(s.send), pcnt=p(s.pcnt),
                 flags=0)
        self.nf.fused_remote(dp.tables_ptrs(), d, self.gpu, self.hash_mode, self.acl_mode, dp.num_cus, self._stream())

    def _egress(self, s: _Slot) -> None:
        p = self._p
        eg = dict(self._geom(), recv_pkt=p(s.recv), port_ctr=self.dp._ptr("port_ctr"),
                  t0=p(self.t0) if self.gpu else 0, lat=p(s.lat2) if self.gpu else 0)
        self.nf.shard_egress(eg, self.gpu, self.dp.num_cus, self._stream())

    def exchange(self, s: _Slot):
        """Start the all-to-all of one chunk's segments; returns a handle with wait()."""
        if not self.host_staged:
            return dist.all_to_all_single(s.recv, s.send, group=self.group, async_op=True)
        recv = torch.empty(s.recv.shape, dtype=s.recv.dtype)
        dist.all_to_all_single(recv, s.send.cpu(), group=self.group)
        s.recv.copy_(recv)
        return _Done()

    def step(self, pkts: torch.Tensor, inmeta: torch.Tensor) -> None:
        n = int(pkts.shape[0])
        if n > self.batch:
            raise ValueError("batch larger than the engine was sized for")
        if pkts.device != self.dev or inmeta.device != self.dev:
            raise ValueError("batch must live on the engine device")
        if self.gpu:
            self.nf.launch_stamp(self._p(self.t0), self._stream())
        self.n = n
        self.rx_log = []
        C = (n + self.chunk - 1) // self.chunk
        works = {}
        for k in range(C + 1):
            if k < C:
                s = self.slots[k % len(self.slots)]
                lo, hi = k * self.chunk, min(n, (k + 1) * self.chunk)
                self._fused(s, lo, hi, pkts, inmeta)
                works[k] = self.exchange(s)
            c = k - 1
            if c >= 0:
                works.pop(c).wait()
                s = self.slots[c % len(self.slots)]
                self._egress(s)
                if self.record_rx:
                    self.rx_log.append(s.recv.cpu().numpy().copy())

    # ---------------------------------------------------------------- results
    def out_meta(self) -> np.ndarray:
        return self.out_meta_t.cpu().numpy().view(np.uint32)[: self.n]

    def outputs(self) -> np.ndarray:
        return self.out.cpu().numpy()[: self.n]

    def received(self) -> tuple[np.ndarray, np.ndarray]:
        """Frames received from peers: every chunk of the last step with record_rx=True, else the
        last chunk of each ring slot.  -> (slots [m,64], metas [m])."""
        moff = self.nf.pkt_meta_off(self.cap)
        outs, metas = [], []
        raws = self.rx_log if self.record_rx else [s.recv.cpu().numpy() for s in self.slots]
        for raw in raws:
            for r in range(self.world):
                if r == self.rank:
                    continue
                seg = raw[r * self.pseg:(r + 1) * self.pseg]
                c = int(seg[:4].view(np.uint32)[0])
                outs.append(seg[64:64 + 64 * c].reshape(c, 64))
                metas.append(seg[moff:moff + 4 * c].view(np.uint32))
        if not outs:
            return np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32)
        return np.concatenate(outs), np.concatenate(metas)

    def latency_samples_us(self) -> np.ndarray:
        xs = []
        for t in [self.lat] + [s.lat2 for s in self.slots]:
            a = t.cpu().numpy().view(np.uint32)
            xs.append(a[a > 0])
        return np.concatenate(xs).astype(np.float64) * 0.01

    def harvest_flow_counters(self) -> np.ndarray:
        """Sum the per-GPU per-flow partials across ranks -> [slots, 2] (pkts, bytes) on every rank."""
        self.dp.harvest()
        t = torch.from_numpy(self.dp.flow_totals.view(np.int64).copy())
        if self.gpu and not self.host_staged:
            t = t.to(self.dev)
        dist.all_reduce(t, group=self.group)
        return t.cpu().numpy().view(np.uint64)


def simulate_replicated_step(engines: list[ReplicatedDataPlane], batches: list) -> None:
    """One replicated step for N ranks inside ONE process (all engines on one device, the
    all-to-all done with local copies): exercises the multi-rank kernels on a single GPU."""
    for e, (pk, im) in zip(engines, batches):
        n = int(pk.shape[0])
        if n > e.chunk:
            raise ValueError("simulate_replicated_step runs one chunk per rank")
        e.n = n
        if e.gpu:
            e.nf.launch_stamp(e._p(e.t0), e._stream())
        e._fused(e.slots[0], 0, n, pk, im)
    seg = engines[0].pseg
    for r, er in enumerate(engines):
        for s_, es in enumerate(engines):
            er.slots[0].recv[s_ * seg:(s_ + 1) * seg].copy_(es.slots[0].send[r * seg:(r + 1) * seg])
    for e in engines:
        e._egress(e.slots[0])
        if e.record_rx:
            e.rx_log = [e.slots[0].recv.cpu().numpy().copy()]
