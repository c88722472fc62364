"""Flow-affine (RSS) sharded multi-GPU data plane: one process per GPU, flows owned by hash.

The MI355X-first answer to "1M-flow table sharded across 8 GPUs" (BASELINE config 4).  Flow f
belongs to GPU owner_of(toeplitz(f), N) - the same Toeplitz hash a NIC's RSS uses to pick a
queue - and only that GPU holds its table entry and counters.  The I/O layer steers each packet
to its owner's ring, exactly as host RSS steers to a queue; the owner runs the WHOLE chain (ACL,
SNAT, L2 steer) with the 1-GPU fused kernel and egresses the frame itself: pod rings live in host
memory, which every GPU can write, so no frame has to reach a "pod's GPU" first.

Packets the I/O layer could not steer (a producer without the hash, a reconfigured key) are
caught inside the fused kernel right after classification: the REMOTE variant in flow-owner mode
(steer = 1) writes the packet's INPUT header slot + ingress meta into the owner's exchange
segment instead of probing; one all-to-all per step delivers the segments (RCCL over xGMI); the
owner gathers them into a dense batch (device-side count, no host round trip) and runs the fused
kernel on it.  The exchange of step k overlaps the next step's kernel:

    compute stream:  fused(k) | wait a2a(k-1) | gather(k-1) + fused_rx(k-1) | fused(k+1) | ...
    RCCL stream:               a2a(k) ...................................... (overlaps)

Cross-GPU bytes per packet: 68 B (header slot + meta) for misdirected packets only; the payload
never moves.  Exchange segments are sized from the expected misdirected count (overflow ->
reason `overflow`, counted).  The CPU twins (oracle + gather) run the same class on gloo ranks.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.distributed as dist

from ..dataplane.engine import DataPlane


def flow_owner(keys: np.ndarray, world: int, rss_key: bytes) -> np.ndarray:
    """Owner GPU of each flow key (nfdp.h owner_of over the Toeplitz hash)."""
    from ..native import nfdp

    h = nfdp().toeplitz(np.ascontiguousarray(keys, np.uint32), rss_key).astype(np.uint64)
    return ((h * np.uint64(world)) >> np.uint64(32)).astype(np.int64)


class _Slot:
    def __init__(self, dev, world: int, pseg: int):
        self.send = torch.zeros(world * pseg, dtype=torch.uint8, device=dev)
        self.recv = torch.zeros(world * pseg, dtype=torch.uint8, device=dev)
        self.pcnt = torch.zeros(world, dtype=torch.int32, device=dev)
        self.t0 = torch.zeros(1, dtype=torch.int64, device=dev)


class _Done:
    def wait(self) -> None:
        pass


class RssShardedDataPlane:
    def __init__(self, dp: DataPlane, rank: int, world: int, batch: int, remote_frac: float = 0.01,
                 group=None):
        if world < 2:
            raise ValueError("RssShardedDataPlane needs world >= 2 (use DataPlane.run for one GPU)")
        self.dp, self.nf = dp, dp.nf
        self.rank, self.world, self.group = rank, world, group
        self.batch = batch
        self.gpu = dp.gpu
        self.dev = dp.tdev if self.gpu else torch.device("cpu")
        per = batch * max(remote_frac, 0.0) / (world - 1)
        self.cap = int(math.ceil((per * 1.25 + 6 * math.sqrt(per) + 64) / 64)) * 64
        self.pseg = self.nf.pkt_seg_bytes(self.cap)
        self.slots = [_Slot(self.dev, world, self.pseg) for _ in range(2)]
        u8, i32 = dict(dtype=torch.uint8, device=self.dev), dict(dtype=torch.int32, device=self.dev)
        self.out = torch.zeros((batch, 64), **u8)
        self.out_meta_t = torch.zeros(batch, **i32)
        self.lat = torch.zeros((batch + 15) // 16, **i32)
        nr = world * self.cap                       # received packets of one step (upper bound)
        self.rx_pkts = torch.zeros((nr, 64), **u8)
        self.rx_inmeta = torch.zeros(nr, **i32)
        self.rx_out = torch.zeros((nr, 64), **u8)
        self.rx_meta = torch.zeros(nr, **i32)
        self.rx_lat = torch.zeros((nr + 15) // 16, **i32)
        self.rx_n = torch.zeros(1, **i32)
        self.n = 0
        self.k = 0
        self.pending = None
        self.hash_mode = dp.hash_mode if dp.hash_mode != 0 else 1
        self.acl_mode = dp.acl_mode
        self.host_staged = self.gpu and dist.is_initialized() and dist.get_backend(group) == "gloo"

    @staticmethod
    def _p(t) -> int:
        return int(t.data_ptr())

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream if self.gpu else 0

    def _remote(self, s: _Slot, pkts: torch.Tensor, inmeta: torch.Tensor, n: int) -> None:
        dp, p = self.dp, self._p
        s.pcnt.zero_()
        d = dict(nranks=self.world, rank=self.rank, cap_desc=0, cap_pkt=self.cap, steer=1,
                 pkts=p(pkts), inmeta=p(inmeta), out=p(self.out), out_meta=p(self.out_meta_t), n=n,
                 flow_ctr=dp._ptr("flow_ctr") if dp.count_flows else 0, port_ctr=dp._ptr("port_ctr"),
                 drop_ctr=dp._ptr("drop_ctr"), t0=p(s.t0) if self.gpu else 0, lat=p(self.lat) if self.gpu else 0,
                 acl_wfrag=dp._ptr("acl_wfrag"), acl_cinit=dp._ptr("acl_cinit"), acl_tiles=dp._acl_tiles,
                 toep_frag=dp._ptr("toep_frag"), toep_tab=dp._ptr("toep_tab"), send_pkt=p(s.send), pcnt=p(s.pcnt),
                 flags=0)
        self.nf.fused_remote(dp.tables_ptrs(), d, self.gpu, self.hash_mode, self.acl_mode, dp.num_cus, self._stream())

    def _receive(self, s: _Slot) -> None:
        """Gather what peers sent (device-side count) and run the whole pipeline on it."""
        p = self._p
        nr = self.world * self.cap
        if self.gpu:
            self.nf.gather(p(s.recv), self.world, self.rank, self.cap, p(self.rx_pkts), p(self.rx_inmeta),
                           p(self.rx_n), True, self._stream())
            self.dp.launch(p(self.rx_pkts), p(self.rx_inmeta), nr, p(self.rx_out), p(self.rx_meta),
                           lat=p(self.rx_lat), t0=p(s.t0), stream=self._stream(), n_dev=p(self.rx_n))
        else:
            m = self.nf.gather(p(s.recv), self.world, self.rank, self.cap, p(self.rx_pkts), p(self.rx_inmeta),
                               p(self.rx_n), False, 0)
            r = self.dp.run(self.rx_pkts.numpy()[:m], self.rx_inmeta.numpy().view(np.uint32)[:m])
            self.rx_out.numpy()[:m] = r.out
            self.rx_meta.numpy().view(np.uint32)[:m] = r.meta

    def exchange(self, s: _Slot):
        if not self.host_staged:
            return dist.all_to_all_single(s.recv, s.send, group=self.group, async_op=True)
        recv = torch.empty(s.recv.shape, dtype=s.recv.dtype)
        dist.all_to_all_single(recv, s.send.cpu(), group=self.group)
        s.recv.copy_(recv)
        return _Done()

    def step(self, pkts: torch.Tensor, inmeta: torch.Tensor) -> None:
        """Process one ingress batch; the packets other GPUs sent for this GPU's flows in the
        previous step are processed here too (call flush() after the last step)."""
        n = int(pkts.shape[0])
        if n > self.batch:
            raise ValueError("batch larger than the engine was sized for")
        if pkts.device != self.dev or inmeta.device != self.dev:
            raise ValueError("batch must live on the engine device")
        s = self.slots[self.k & 1]
        if self.gpu:
            self.nf.launch_stamp(self._p(s.t0), self._stream())
        self.n = n
        self._remote(s, pkts, inmeta, n)
        work = self.exchange(s)
        self.flush()
        self.pending = (s, work)
        self.k += 1

    def flush(self) -> None:
        if self.pending is not None:
            s, work = self.pending
            self.pending = None
            work.wait()
            self._receive(s)

    # ---------------------------------------------------------------- results
    def out_meta(self) -> np.ndarray:
        return self.out_meta_t.cpu().numpy().view(np.uint32)[: self.n]

    def outputs(self) -> np.ndarray:
        return self.out.cpu().numpy()[: self.n]

    def received(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Last processed receive batch: (input slots, egress slots, egress metas)."""
        m = int(self.rx_n.cpu().numpy()[0])
        return (self.rx_pkts.cpu().numpy()[:m], self.rx_out.cpu().numpy()[:m],
                self.rx_meta.cpu().numpy().view(np.uint32)[:m])

    def latency_samples_us(self) -> np.ndarray:
        xs = []
        for t in (self.lat, self.rx_lat):
            a = t.cpu().numpy().view(np.uint32)
            xs.append(a[a > 0])
        return np.concatenate(xs).astype(np.float64) * 0.01

    def harvest_flow_counters(self) -> np.ndarray:
        """Per-flow counters live on the owner only: the shard's [slots, 2] (pkts, bytes)."""
        self.dp.harvest()
        return self.dp.flow_totals


def rss_traffic(sc, n: int, rank: int, world: int, owner: np.ndarray, remote_frac: float, seed: int,
                n_pods: int | None = None):
    """A rank's ingress batch under host RSS: packets of the flows this GPU owns, plus
    `remote_frac` of packets the producer could not steer (flows other GPUs own)."""
    from ..dataplane import scenario as S

    rng = np.random.default_rng(seed)
    mine = np.where(owner == rank)[0]
    others = np.where(owner != rank)[0]
    n_rem = int(round(n * remote_frac)) if len(others) else 0
    pk, im = S.traffic(sc, n - n_rem, seed=seed, flows=mine)
    if n_rem:
        pk2, im2 = S.traffic(sc, n_rem, seed=seed + 1, flows=others)
        pk, im = np.concatenate([pk, pk2]), np.concatenate([im, im2])
        perm = rng.permutation(n)
        pk, im = pk[perm], im[perm]
    return pk, im
