"""Flow-affine (RSS) sharded multi-GPU data plane: one process per GPU, flows owned by hash.

The MI355X-first answer to "1M-flow table sharded across 8 GPUs" (BASELINE config 4).  Flow f
belongs to GPU owner_of(toeplitz(f), N) - the same Toeplitz hash a NIC's RSS uses to pick a
queue - and only that GPU holds its table entry and counters.  The I/O layer steers each packet
to its owner's ring, exactly as host RSS steers to a queue; the owner runs the WHOLE chain (ACL,
SNAT, L2 steer) with the 1-GPU fused kernel and egresses the frame itself: pod rings live in host
memory, which every GPU can write, so no frame has to reach a "pod's GPU" first.

Packets the I/O layer could not steer (a producer without the hash, a reconfigured key) are
caught inside the fused kernel right after classification: the LIST instance of the 1-GPU kernel
puts them on a per-workgroup steer list (no probe, no chain, no counters) and steer_kernel copies
their INPUT header slot + ingress meta into the owner's exchange segment (sized for the whole
batch).  The exchange is count-first and loss-free: an all-to-all of the per-peer counts, then a
grouped send/recv of exactly those bytes (RCCL P2P over xGMI); the owner gathers them into a
dense batch and runs the fused kernel on it.  The exchange of step k overlaps the next step's
kernel:

    compute stream:  fused(k) + steer(k) | fused(k+1) + steer(k+1) | ...
    comm stream:          counts(k), send/recv(k) ....... (overlaps)
    rx stream:                        gather(k) + fused_rx(k)  (overlaps fused(k+1))

(The rx pass of step k used to run on the compute stream between fused(k) and fused(k+1): its
launches and its workgroups' table staging cost a fixed ~27-46 us per step, rss_probe r3 s11.
On its own stream it overlaps the next step's kernel; the slot events order the reuse of the
exchange slots and of the receive buffers.)

The host never waits for the GPU in steady state: the send/recv sizes of a step must be known on
the host (RCCL P2P), so the counts come back through pinned memory, but step k's counts are read
only at step k + `lag` (default 2), long after they landed - the host runs up to `lag` steps ahead
of the device.  `lag + 1` exchange slots rotate.

Cross-GPU bytes per packet: 68 B (header slot + meta) for misdirected packets only; the payload
never moves.  The CPU twins (oracle REMOTE steer + gather) run the same class on gloo ranks.
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
    def __init__(self, dev, world: int, pseg: int, batch: int, gpu: bool, list_len: int = 0, cnt_blocks: int = 1):
        self.send = torch.zeros(world * pseg, dtype=torch.uint8, device=dev)
        self.recv = torch.zeros(world * pseg, dtype=torch.uint8, device=dev)
        self.pcnt = torch.zeros(world, dtype=torch.int32, device=dev)    # packets this rank sends to each peer
        self.rcnt = torch.zeros(world, dtype=torch.int32, device=dev)    # packets each peer sends this rank
        self.t0 = torch.zeros(1, dtype=torch.int64, device=dev)
        # steer list (GPU): a region per fused workgroup; {grid, region size, count per workgroup}
        self.list = torch.zeros(max(list_len, 1), dtype=torch.int32, device=dev)
        self.list_cnt = torch.zeros(2 + cnt_blocks, dtype=torch.int32, device=dev)
        self.ev = torch.cuda.Event() if gpu else None     # local step (kernel + steer) done
        self.cev = torch.cuda.Event() if gpu else None    # exchange done
        self.rev = torch.cuda.Event() if gpu else None    # rx pass over this slot's receive segments done
        self.used = False                                 # the events were recorded (slot in use before)


class RssShardedDataPlane:
    """Count-first, loss-free flow-owner exchange.

    Per step on rank r: the 1-GPU fused kernel in steer-list mode (LIST instances: packets of other
    GPUs' flows are listed, not processed; the hot instance is untouched) + steer_kernel copying
    the listed input slots into per-owner segments sized for the WHOLE batch, so nothing can
    overflow whatever the misdirected fraction.  The exchange then moves exactly what was written:
    the per-peer counts first (one all-to-all of N ints), then one grouped send/recv of the slot
    and meta bytes each peer actually has (NCCL P2P over xGMI: each peer on its own link), on a
    communication stream that overlaps the next step's kernel.  The host learns the counts while
    the GPU runs that next kernel, so the count round trip costs no GPU time.
    """

    def __init__(self, dp: DataPlane, rank: int, world: int, batch: int, remote_frac: float = 0.01,
                 group=None, lag: int = 2):
        if world < 2:
            raise ValueError("RssShardedDataPlane needs world >= 2 (use DataPlane.run for one GPU)")
        self.dp, self.nf = dp, dp.nf
        self.rank, self.world, self.group = rank, world, group
        self.batch = batch
        self.remote_frac = remote_frac      # informational: the exchange is sized by counts, not by this
        self.gpu = dp.gpu
        self.dev = dp.tdev if self.gpu else torch.device("cpu")
        self.cap = max(int(batch), 64)      # a segment holds the whole batch: loss-free at any fraction
        self.pseg = int(self.nf.pkt_seg_bytes(self.cap))
        self.moff = int(self.nf.pkt_meta_off(self.cap))
        self.hash_mode = dp.hash_mode if dp.hash_mode != 0 else 1
        self.acl_mode = dp.acl_mode
        # LIST instances exist for the LDS / MFMA hash with the MFMA / no ACL; others use REMOTE steer
        self.use_list = self.gpu and self.hash_mode in (1, 2) and self.acl_mode in (1, 2)
        nl = int(self.nf.steer_list_len(batch, int(dp.num_cus))) if self.use_list else 0
        self.lag = max(int(lag), 1)
        self.nslots = self.lag + 1
        self.slots = [_Slot(self.dev, world, self.pseg, batch, self.gpu, nl, 4 * int(dp.num_cus) if self.use_list else 1)
                      for _ in range(self.nslots)]
        for i, sl in enumerate(self.slots):
            sl.idx = i
            sl.hev = torch.cuda.Event() if self.gpu else None   # counts are in host memory
        u8, i32 = dict(dtype=torch.uint8, device=self.dev), dict(dtype=torch.int32, device=self.dev)
        self.out = torch.zeros((batch, 64), **u8)
        self.out_meta_t = torch.zeros(batch, **i32)
        self.lat = torch.zeros((batch + 15) // 16, **i32)
        nr = world * self.cap if not self.gpu else max(int(batch * min(1.0, max(remote_frac, 0.0)) * 4) + 4096, 65536)
        self.rx_cap = min(nr, world * self.cap)
        self.rx_pkts = torch.zeros((self.rx_cap, 64), **u8)
        self.rx_inmeta = torch.zeros(self.rx_cap, **i32)
        self.rx_out = torch.zeros((self.rx_cap, 64), **u8)
        self.rx_meta = torch.zeros(self.rx_cap, **i32)
        self.rx_lat = torch.zeros((self.rx_cap + 15) // 16, **i32)
        self.rx_n = torch.zeros(1, **i32)
        self.n = 0
        self.k = 0
        self.pending: list = []             # slots whose counts are in flight, oldest first
        self.host_staged = self.gpu and dist.is_initialized() and dist.get_backend(group) == "gloo"
        self.comm = torch.cuda.Stream(self.dev) if self.gpu and not self.host_staged else None
        self.rx_stream = torch.cuda.Stream(self.dev) if self.comm is not None else None
        hc = torch.zeros((self.nslots, 2, world), dtype=torch.int32)
        self.hcnt = hc.pin_memory() if self.gpu else hc
        self.stats = {"sent": 0, "received": 0, "steps": 0, "max_peer": 0}

    @staticmethod
    def _p(t) -> int:
        return int(t.data_ptr())

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.dev).cuda_stream if self.gpu else 0

    def _local(self, s: _Slot, pkts: torch.Tensor, inmeta: torch.Tensor, n: int) -> None:
        """This rank's share: its own flows through the whole pipeline, other GPUs' packets into
        their owners' segments (count in pcnt)."""
        dp, p = self.dp, self._p
        if self.comm is not None and s.used:
            # this slot's previous exchange still reads its send segments / counts
            torch.cuda.current_stream(self.dev).wait_event(s.cev)
        s.pcnt.zero_()
        if self.use_list:
            s.list_cnt.zero_()
            st = self._stream()
            self.nf.launch_fused(dp.tables_ptrs(), p(pkts), p(inmeta), p(self.out), p(self.out_meta_t), n,
                                 dp._ptr("flow_ctr"), dp._ptr("port_ctr"), dp._ptr("drop_ctr"), p(s.t0), p(self.lat),
                                 dp._ptr("acl_wfrag"), dp._ptr("acl_cinit"), dp._acl_tiles, dp._ptr("toep_frag"),
                                 dp._ptr("toep_tab"), self.hash_mode, self.acl_mode, dp.num_cus, st,
                                 0 if dp.count_flows else 4, None, 0, p(s.list), p(s.list_cnt), self.world, self.rank,
                                 s.list.numel())
            self.nf.launch_steer(p(pkts), p(inmeta), p(s.list), p(s.list_cnt), s.list.numel(), s.list_cnt.numel(),
                                 p(s.send), p(s.pcnt), self.world, self.cap, st)
        else:
            d = dict(nranks=self.world, rank=self.rank, cap_desc=0, cap_pkt=self.cap, steer=1,
                     pkts=p(pkts), inmeta=p(inmeta), out=p(self.out), out_meta=p(self.out_meta_t), n=n,
                     flow_ctr=dp._ptr("flow_ctr") if dp.count_flows else 0, port_ctr=dp._ptr("port_ctr"),
                     drop_ctr=dp._ptr("drop_ctr"), t0=p(s.t0) if self.gpu else 0, lat=p(self.lat) if self.gpu else 0,
                     acl_wfrag=dp._ptr("acl_wfrag"), acl_cinit=dp._ptr("acl_cinit"), acl_tiles=dp._acl_tiles,
                     toep_frag=dp._ptr("toep_frag"), toep_tab=dp._ptr("toep_tab"), send_pkt=p(s.send),
                     pcnt=p(s.pcnt), flags=0)
            self.nf.fused_remote(dp.tables_ptrs(), d, self.gpu, self.hash_mode, self.acl_mode, dp.num_cus,
                                 self._stream())
        if self.gpu:
            s.ev.record(torch.cuda.current_stream(self.dev))

    def _views(self, buf: torch.Tensor, j: int, c: int) -> tuple[torch.Tensor, torch.Tensor]:
        b = j * self.pseg
        return buf[b + 64: b + 64 + 64 * c], buf[b + self.moff: b + self.moff + 4 * c]

    def _p2p(self, send: torch.Tensor, recv: torch.Tensor, sc, rc) -> list:
        ops = []
        for j in range(self.world):
            if j == self.rank:
                continue
            if sc[j]:
                a, m = self._views(send, j, int(sc[j]))
                ops += [dist.P2POp(dist.isend, a, j, self.group, 0), dist.P2POp(dist.isend, m, j, self.group, 1)]
            if rc[j]:
                a, m = self._views(recv, j, int(rc[j]))
                ops += [dist.P2POp(dist.irecv, a, j, self.group, 0), dist.P2POp(dist.irecv, m, j, self.group, 1)]
        return dist.batch_isend_irecv(ops) if ops else []

    def _counts(self, s: _Slot) -> None:
        """Enqueue the count all-to-all of a slot (comm stream, after its local step); the counts
        land in pinned host memory without the host waiting for them."""
        if self.comm is None:
            return
        w, cs = self.world, self.comm
        hc = self.hcnt[s.idx]
        with torch.cuda.stream(cs):
            cs.wait_event(s.ev)
            if s.used:
                cs.wait_event(s.rev)          # the previous rx pass over s.recv is done
            dist.all_to_all_single(s.rcnt, s.pcnt, group=self.group)
            hc[0].copy_(s.pcnt, non_blocking=True)
            hc[1].copy_(s.rcnt, non_blocking=True)
            # the gather kernel reads each receive segment's count from its header
            s.recv.view(w, self.pseg)[:, :4].view(torch.int32)[:, 0].copy_(s.rcnt)
            s.hev.record(cs)

    def _transfer(self, s: _Slot):
        """The grouped send/recv of exactly the bytes each peer has (counts read on the host)."""
        w = self.world
        if self.comm is not None:
            cs = self.comm
            s.hev.synchronize()                   # normally long done: the counts of `lag` steps ago
            hc = self.hcnt[s.idx]
            sc, rc = hc[0].numpy().copy(), hc[1].numpy().copy()
            with torch.cuda.stream(cs):
                for wk in self._p2p(s.send, s.recv, sc, rc):
                    wk.wait()                     # makes the comm stream wait for the transfers
                s.cev.record(cs)
        else:
            # gloo (CPU ranks, or a GPU rehearsal staged through the host)
            pc = s.pcnt.cpu()
            rcv = torch.zeros_like(pc)
            dist.all_to_all_single(rcv, pc, group=self.group)
            sc, rc = pc.numpy(), rcv.numpy()
            send = s.send.cpu() if self.gpu else s.send
            recv = torch.zeros_like(send) if self.gpu else s.recv
            for wk in self._p2p(send, recv, sc, rc):
                wk.wait()
            recv.view(w, self.pseg)[:, :4].view(torch.int32)[:, 0].copy_(rcv)
            if self.gpu:
                s.recv.copy_(recv)
            s.rcnt.copy_(rcv)
            self.hcnt[s.idx][1].copy_(rcv)
        self.stats["sent"] += int(sum(sc))
        self.stats["received"] += int(sum(rc))
        self.stats["max_peer"] = max(self.stats["max_peer"], int(max(sc)) if len(sc) else 0)
        return s

    def exchange(self, s: _Slot):
        """Counts first, then exactly the bytes each peer has (no fixed-capacity segments on the
        wire, no overflow).  Standalone form (the exchange probe): waits for the counts now."""
        self._counts(s)
        return self._transfer(s)

    def _receive(self, s: _Slot) -> None:
        """Gather what peers sent (device-side count) and run the whole pipeline on it."""
        p = self._p
        nr = int(self.rx_cap)
        if self.gpu:
            rs = self.rx_stream
            if rs is not None:
                rs.wait_event(s.cev)
            total = int(self.hcnt[s.idx][1].sum())
            if total > nr:                        # more than the receive buffers hold: grow them
                self._grow_rx(total)
                nr = int(self.rx_cap)
            st = rs.cuda_stream if rs is not None else self._stream()
            self.nf.gather(p(s.recv), self.world, self.rank, self.cap, p(self.rx_pkts), p(self.rx_inmeta),
                           p(self.rx_n), True, st)
            self.dp.launch(p(self.rx_pkts), p(self.rx_inmeta), nr, p(self.rx_out), p(self.rx_meta),
                           lat=p(self.rx_lat), t0=p(s.t0), stream=st, n_dev=p(self.rx_n))
            if rs is not None:
                s.rev.record(rs)
            s.used = True
        else:
            m = self.nf.gather(p(s.recv), self.world, self.rank, self.cap, p(self.rx_pkts), p(self.rx_inmeta),
                               p(self.rx_n), False, 0)
            r = self.dp.run(self.rx_pkts.numpy()[:m], self.rx_inmeta.numpy().view(np.uint32)[:m])
            self.rx_out.numpy()[:m] = r.out
            self.rx_meta.numpy().view(np.uint32)[:m] = r.meta

    def _grow_rx(self, n: int) -> None:
        if self.rx_stream is not None:
            self.rx_stream.synchronize()          # the old buffers may still be in use there
        n = min(int(n * 1.25) + 4096, self.world * self.cap)
        u8, i32 = dict(dtype=torch.uint8, device=self.dev), dict(dtype=torch.int32, device=self.dev)
        self.rx_cap = n
        self.rx_pkts = torch.zeros((n, 64), **u8)
        self.rx_inmeta = torch.zeros(n, **i32)
        self.rx_out = torch.zeros((n, 64), **u8)
        self.rx_meta = torch.zeros(n, **i32)
        self.rx_lat = torch.zeros((n + 15) // 16, **i32)

    def step(self, pkts: torch.Tensor, inmeta: torch.Tensor) -> None:
        """Process one ingress batch; packets other GPUs sent for this GPU's flows `lag` steps ago
        are exchanged and processed here too (call flush() after the last step)."""
        n = int(pkts.shape[0])
        if n > self.batch:
            raise ValueError("batch larger than the engine was sized for")
        if pkts.device != self.dev or inmeta.device != self.dev:
            raise ValueError("batch must live on the engine device")
        s = self.slots[self.k % self.nslots]
        if self.gpu:
            self.nf.launch_stamp(self._p(s.t0), self._stream())
        self.n = n
        self._local(s, pkts, inmeta, n)
        # exchanges of earlier steps first (one order of collectives on every rank), then this
        # step's counts; the host waits only for counts `lag` steps old
        while len(self.pending) >= self.lag:
            self._receive(self._transfer(self.pending.pop(0)))
        self._counts(s)
        self.pending.append(s)
        self.k += 1
        self.stats["steps"] += 1

    def flush(self) -> None:
        while self.pending:
            self._receive(self._transfer(self.pending.pop(0)))

    # ---------------------------------------------------------------- results
    def sync(self) -> None:
        """Wait for every stream of this engine (compute, exchange, rx)."""
        if self.gpu:
            torch.cuda.current_stream(self.dev).synchronize()
            for st in (self.comm, self.rx_stream):
                if st is not None:
                    st.synchronize()

    def out_meta(self) -> np.ndarray:
        return self.out_meta_t.cpu().numpy().view(np.uint32)[: self.n]

    def outputs(self) -> np.ndarray:
        return self.out.cpu().numpy()[: self.n]

    def received(self) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Last processed receive batch: (input slots, egress slots, egress metas)."""
        self.sync()
        m = int(self.rx_n.cpu().numpy()[0])
        return (self.rx_pkts.cpu().numpy()[:m], self.rx_out.cpu().numpy()[:m],
                self.rx_meta.cpu().numpy().view(np.uint32)[:m])

    def latency_samples_us(self) -> np.ndarray:
        self.sync()
        xs = []
        for t in (self.lat, self.rx_lat):
            a = t.cpu().numpy().view(np.uint32)
            xs.append(a[a > 0])
        return np.concatenate(xs).astype(np.float64) * 0.01

    def harvest_flow_counters(self) -> np.ndarray:
        """Per-flow counters live on the owner only: the shard's [slots, 2] (pkts, bytes)."""
        self.sync()
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
