"""Flow-sharded multi-GPU data plane: one process per GPU, RCCL all-to-all over xGMI.

The flow table is hash-partitioned across ranks (owner = top bits of the Toeplitz hash, the same
bits an RSS indirection table would use).  Every rank keeps the full (small) port / chain / MAC /
ACL tables.  A step moves, per packet, a 32-B descriptor to the flow owner and a 16-B verdict
back; the 64-B payload crosses xGMI at most once, to the GPU that owns the destination pod.
All exchange segments have static capacity, so each collective is a fixed-size
``all_to_all_single`` (one xGMI link per peer, no ring) and the step never round-trips to the host.

The same code runs on CPU processes with the gloo backend: the stage functions then call the
scalar C++ twins (``shard_cpu.cpp``), which is how the distributed path is tested without GPUs.
Reference analogue: the reference has no data-plane parallelism; its scaling axis is one
dpu-daemon per node (``internal/controller/bindata/daemon/99.daemonset.yaml:20-21``) — see
SURVEY.md §2.7.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from ..dataplane.engine import DataPlane


def shard_filter(rank: int, world: int):
    """flow_filter for scenario.build_sfc: keep the flows this rank owns."""
    from ..native import nfdp

    nf = nfdp()

    def f(keys: np.ndarray, hashes: np.ndarray) -> np.ndarray:
        owner = ((hashes.astype(np.uint64) * np.uint64(world)) >> np.uint64(32)).astype(np.int64)
        return owner == rank

    return f


class ShardedDataPlane:
    def __init__(self, dp: DataPlane, rank: int, world: int, batch: int, slack: float = 1.08,
                 group=None, hash_mode: int | None = None, acl_mode: int | None = None):
        self.dp = dp
        self.nf = dp.nf
        self.rank, self.world, self.batch = rank, world, batch
        self.group = group
        self.gpu = dp.gpu
        self.dev = dp.tdev if self.gpu else torch.device("cpu")
        per = batch / world
        # capacity: mean + slack + a few sigma of the multinomial fill
        self.cap_desc = int(math.ceil(per * slack + 6 * math.sqrt(per) + 256))
        self.cap_pkt = self.cap_desc
        self.dseg = self.nf.desc_seg_bytes(self.cap_desc)
        self.vseg = self.nf.verdict_seg_bytes(self.cap_desc)
        self.pseg = self.nf.pkt_seg_bytes(self.cap_pkt)
        self.hash_mode = dp.hash_mode if hash_mode is None else hash_mode
        if self.hash_mode == 0:
            self.hash_mode = 1  # scalar Toeplitz is a test-only variant of the fused kernel
        self.acl_mode = dp.acl_mode if acl_mode is None else acl_mode
        u8 = dict(dtype=torch.uint8, device=self.dev)
        i32 = dict(dtype=torch.int32, device=self.dev)
        self.send_desc = torch.zeros(world * self.dseg, **u8)
        self.recv_desc = torch.zeros(world * self.dseg, **u8)
        self.send_verdict = torch.zeros(world * self.vseg, **u8)
        self.recv_verdict = torch.zeros(world * self.vseg, **u8)
        self.send_pkt = torch.zeros(world * self.pseg, **u8)
        self.recv_pkt = torch.zeros(world * self.pseg, **u8)
        self.cnt = torch.zeros(world, **i32)
        self.pcnt = torch.zeros(world, **i32)
        self.ref = torch.zeros(batch, **i32)
        self.aux = torch.zeros(batch, **i32)
        self.out = torch.zeros((batch, 64), **u8)
        self.out_meta = torch.zeros(batch, **i32)
        self.lat = torch.zeros((batch + 15) // 16, **i32)
        self.lat2 = torch.zeros((world * self.cap_pkt + 15) // 16, **i32)
        self.t0 = torch.zeros(1, dtype=torch.int64, device=self.dev)  # this engine's batch-release stamp

    @staticmethod
    def _p(t) -> int:
        if isinstance(t, np.ndarray):
            return int(t.ctypes.data)
        return int(t.data_ptr())

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream if self.gpu else 0

    def _a2a(self, out: torch.Tensor, inp: torch.Tensor) -> None:
        dist.all_to_all_single(out, inp, group=self.group)

    def _geom(self) -> dict:
        return {"nranks": self.world, "rank": self.rank, "cap_desc": self.cap_desc, "cap_pkt": self.cap_pkt}

    def phase_ingress(self, pkts: torch.Tensor, inmeta: torch.Tensor, n: int | None = None) -> None:
        n = int(pkts.shape[0]) if n is None else n
        if n > self.batch:
            raise ValueError("batch larger than the engine was sized for")
        if pkts.device != self.dev or inmeta.device != self.dev:
            raise ValueError("batch must live on the engine device")
        self._cur = (pkts, inmeta, n)
        dp, nf, p, s = self.dp, self.nf, self._p, self._stream()
        self.cnt.zero_()
        self.pcnt.zero_()
        if self.gpu:
            nf.launch_stamp(p(self.t0), s)
        ing = dict(self._geom(), pkts=p(pkts), inmeta=p(inmeta), n=n, send_desc=p(self.send_desc), cnt=p(self.cnt),
                   ref=p(self.ref), aux=p(self.aux), acl_wfrag=dp._ptr("acl_wfrag"), acl_cinit=dp._ptr("acl_cinit"),
                   acl_tiles=dp._acl_tiles, toep_frag=dp._ptr("toep_frag"), toep_tab=dp._ptr("toep_tab"))
        nf.shard_ingress(dp.tables_ptrs(), ing, self.gpu, self.hash_mode, self.acl_mode, dp.num_cus, s)

    def phase_owner(self) -> None:
        dp, p = self.dp, self._p
        own = dict(self._geom(), recv_desc=p(self.recv_desc), send_verdict=p(self.send_verdict),
                   flow_ctr=dp._ptr("flow_ctr"), toep_tab=dp._ptr("toep_tab"))
        self.nf.shard_owner(dp.tables_ptrs(), own, self.gpu, dp.num_cus, self._stream())

    def phase_apply(self) -> None:
        dp, p = self.dp, self._p
        pkts, inmeta, n = self._cur
        app = dict(self._geom(), pkts=p(pkts), inmeta=p(inmeta), n=n, ref=p(self.ref), aux=p(self.aux),
                   recv_verdict=p(self.recv_verdict), out=p(self.out), out_meta=p(self.out_meta),
                   send_pkt=p(self.send_pkt), pcnt=p(self.pcnt), port_ctr=dp._ptr("port_ctr"),
                   drop_ctr=dp._ptr("drop_ctr"), t0=p(self.t0), lat=p(self.lat))
        self.nf.shard_apply(dp.tables_ptrs(), app, self.gpu, dp.num_cus, self._stream())

    def phase_egress(self) -> None:
        dp, p = self.dp, self._p
        eg = dict(self._geom(), recv_pkt=p(self.recv_pkt), port_ctr=dp._ptr("port_ctr"), t0=p(self.t0),
                  lat=p(self.lat2))
        self.nf.shard_egress(eg, self.gpu, dp.num_cus, self._stream())

    def step(self, pkts: torch.Tensor, inmeta: torch.Tensor, n: int | None = None) -> None:
        """One batch through the sharded SFC pipeline (3 fixed-size all-to-alls)."""
        self.phase_ingress(pkts, inmeta, n)
        self._a2a(self.recv_desc, self.send_desc)
        self.phase_owner()
        self._a2a(self.recv_verdict, self.send_verdict)
        self.phase_apply()
        self._a2a(self.recv_pkt, self.send_pkt)
        self.phase_egress()

    # ---------------------------------------------------------------- results
    def received(self) -> tuple[np.ndarray, np.ndarray]:
        """Packets received from peers in the last step: (slots [m,64], metas [m])."""
        raw = self.recv_pkt.cpu().numpy()
        slots, metas = [], []
        moff = self.nf.pkt_meta_off(self.cap_pkt)
        for s in range(self.world):
            if s == self.rank:
                continue
            seg = raw[s * self.pseg:(s + 1) * self.pseg]
            c = int(seg[:4].view(np.uint32)[0])
            slots.append(seg[64:64 + 64 * c].reshape(c, 64))
            metas.append(seg[moff:moff + 4 * c].view(np.uint32))
        if not slots:
            return np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32)
        return np.concatenate(slots), np.concatenate(metas)

    def latency_samples_us(self) -> np.ndarray:
        a = self.lat.cpu().numpy().view(np.uint32)
        b = self.lat2.cpu().numpy().view(np.uint32)
        x = np.concatenate([a[a > 0], b[b > 0]]).astype(np.float64)
        return x * 0.01  # 100 MHz ticks -> us


def _local_a2a(engines, send_attr: str, recv_attr: str, seg: int) -> None:
    """all_to_all_single emulated in one process: recv[r][s] = send[s][r]."""
    for r, er in enumerate(engines):
        recv = getattr(er, recv_attr)
        for s_, es in enumerate(engines):
            recv[s_ * seg:(s_ + 1) * seg].copy_(getattr(es, send_attr)[r * seg:(r + 1) * seg])


def simulate_step(engines: list, batches: list) -> None:
    """Run one sharded step for N ranks inside ONE process (all on one device): used to test the
    multi-rank GPU kernels on a single GPU, where RCCL cannot host two ranks on one device."""
    for e, (pk, im) in zip(engines, batches):
        e.phase_ingress(pk, im)
    _local_a2a(engines, "send_desc", "recv_desc", engines[0].dseg)
    for e in engines:
        e.phase_owner()
    _local_a2a(engines, "send_verdict", "recv_verdict", engines[0].vseg)
    for e in engines:
        e.phase_apply()
    _local_a2a(engines, "send_pkt", "recv_pkt", engines[0].pseg)
    for e in engines:
        e.phase_egress()


class PipelinedShardedDataPlane:
    """Chunked, software-pipelined sharded step: the batch is cut into `chunks` pieces and the
    stages of different chunks overlap, so the xGMI all-to-alls (RCCL stream) run while the
    compute stream processes other chunks.  Issue order per iteration k (chunk indices):

        egress(k-3) | apply(k-2) -> a2a_pkt(k-2) | owner(k-1) -> a2a_verdict(k-1) |
        ingress(k) -> a2a_desc(k)

    each consumer waits only on its own collective (Work.wait() = a stream-side wait), and a ring
    of 4 buffer sets is enough because a chunk's buffers are last touched 3 iterations after its
    ingress.
    """

    RING = 4

    def __init__(self, dp: DataPlane, rank: int, world: int, batch: int, chunks: int = 4, group=None, **kw):
        self.chunks = max(1, chunks)
        self.chunk = int(math.ceil(batch / self.chunks))
        self.rank, self.world, self.batch, self.group = rank, world, batch, group
        self.slots = [ShardedDataPlane(dp, rank, world, self.chunk, group=group, **kw)
                      for _ in range(min(self.RING, self.chunks))]

    def _slot(self, c: int) -> ShardedDataPlane:
        return self.slots[c % len(self.slots)]

    def _a2a(self, c: int, kind: str):
        e = self._slot(c)
        send, recv = {"d": (e.send_desc, e.recv_desc), "v": (e.send_verdict, e.recv_verdict),
                      "p": (e.send_pkt, e.recv_pkt)}[kind]
        return dist.all_to_all_single(recv, send, group=self.group, async_op=True)

    def step(self, pkts: torch.Tensor, inmeta: torch.Tensor) -> None:
        n = int(pkts.shape[0])
        C = min(self.chunks, (n + self.chunk - 1) // self.chunk)
        if len(self.slots) < min(self.RING, C):
            raise RuntimeError("ring too small")
        works = {}
        for k in range(C + 3):
            c = k - 3
            if 0 <= c < C:
                works.pop((c, "p")).wait()
                self._slot(c).phase_egress()
            c = k - 2
            if 0 <= c < C:
                works.pop((c, "v")).wait()
                self._slot(c).phase_apply()
                works[(c, "p")] = self._a2a(c, "p")
            c = k - 1
            if 0 <= c < C:
                works.pop((c, "d")).wait()
                self._slot(c).phase_owner()
                works[(c, "v")] = self._a2a(c, "v")
            c = k
            if c < C:
                lo, hi = c * self.chunk, min(n, (c + 1) * self.chunk)
                self._slot(c).phase_ingress(pkts[lo:hi], inmeta[lo:hi])
                works[(c, "d")] = self._a2a(c, "d")

    def out_meta(self) -> np.ndarray:
        return np.concatenate([e.out_meta.cpu().numpy().view(np.uint32)[: e._cur[2]] for e in self.slots])

    def latency_samples_us(self) -> np.ndarray:
        return np.concatenate([e.latency_samples_us() for e in self.slots])
