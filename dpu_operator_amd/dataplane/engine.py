"""Single-device data-plane runtime.

``DataPlane`` owns the host table models, mirrors them into device memory (HBM tensors on a
GPU, numpy arrays for the CPU oracle) and runs packet batches through the fused HIP kernel
(`fused_kernel<HASH, ACL>` in csrc/nfdp/kernels.hip) or the bit-exact C++ oracle.

Table updates are applied between batches on the same HIP stream, so a batch always sees one
consistent table version (the reference serialises the same updates through `p4rt-ctl` calls;
here they are batched bucket-row writes).  Per-flow counters are packed (pkts << 40 | bytes)
and harvested (read + reset) before any update batch that moves entries.
"""
from __future__ import annotations

import contextlib
import threading

import os
import time
from dataclasses import dataclass, field

import numpy as np

from ..native import nfdp as _nfdp_mod
from ..utils.faults import FAULTS
from ..utils.latency import LatencyStats
from ..utils.trace import TRACER
from . import tables as T

HASH_MODES = {"scalar": 0, "lds": 1, "mfma": 2}
ACL_MODES = {"scalar": 0, "mfma": 1, "off": 2}


def _torch():
    import torch

    return torch


def unpack_ctr(x: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    x = np.asarray(x).astype(np.uint64)
    return x >> np.uint64(40), x & np.uint64((1 << 40) - 1)


@dataclass
class BatchResult:
    out: object          # [n,64] uint8 (torch or numpy)
    meta: object         # [n] uint32 (torch int32 view or numpy)
    n: int
    extra: dict = field(default_factory=dict)


class DataPlane:
    def __init__(
        self,
        device: str = "cuda",
        flow_buckets: int = 1 << 16,
        mac_slots: int = 1 << 14,
        chains: int = 4096,
        hash_mode: str = "mfma",
        acl_mode: str = "mfma",
        num_cus: int | None = None,
        rss_key: bytes = T.RSS_KEY,
    ):
        self._commit_lock = threading.RLock()   # commits vs the live path's maintenance restarts
        self.nf = _nfdp_mod()
        self.device = device
        self.gpu = device != "cpu"
        self.ports = T.PortTable()
        self.chains = T.ChainTable(chains)
        self.macs = T.MacTable(mac_slots)
        self.lag = T.LagTable()
        self.flood = T.FloodTable()
        self.routes = T.RouteTable()
        self.routes6 = T.Route6Table()
        self.nexthops = T.NextHopTable()
        self.ecmp = T.EcmpTable()
        self.tunnels = T.TunnelTable()
        self.terms = T.TermTable()
        self.vmmac = T.VmMacTable()
        self.tunnels6 = T.Tunnel6Table()
        self.vtep6 = T.Vtep6()
        self.terms6 = T.Term6Table()     # host side: finished by resolve_recirc6 on the whole frame
        self._ipsec = None               # ESP engine (dataplane/ipsec.py), created on first use
        self.acl = T.AclTable()
        self.flows = T.FlowTable(flow_buckets, rss_key)
        # IPv6 flows: folded FlowKey -> the 8 raw address words of its side entry (TablesView
        # flow6_on: the device flow buffer carries the side array after the buckets)
        self.flows6: dict[tuple, np.ndarray] = {}
        self._flow6_on = False
        self._flow6_full = False
        self.rss_key = rss_key
        self.hash_mode = HASH_MODES[hash_mode]
        self.acl_mode = ACL_MODES[acl_mode]
        self._dev: dict[str, object] = {}
        self._versions: dict[str, int] = {}
        self._acl_tiles = 1
        self.count_flows = True  # per-flow packed counters (one 64-bit atomic per packet)
        self.MAX_LAUNCH = 1 << 24
        self.flow_totals = np.zeros((self.flows.nbuckets * 4, 2), np.uint64)
        self.latency = LatencyStats()   # packet-path latency histograms (utils/latency.py)
        self._gen = 0                   # bumped whenever a device buffer address changes
        self._flow_active = 0           # flow-table copy in use (double buffered under running rings)
        self._flow_lag = np.zeros(0, np.int64)
        self.flip_stats = {"flips": 0, "grace_s": 0.0, "update_s": 0.0, "buckets": 0}
        # side outputs (flood / mirror / ARP replicas, learn events) and MAC learning state
        self.cap_rep, self.cap_learn = 1 << 16, 1 << 14
        self.stamp = 0                 # batch counter: the learned entries' last-seen stamp
        self._learned_on_device = False
        if self.gpu:
            torch = _torch()
            if not torch.cuda.is_available():
                raise RuntimeError("DataPlane(device='cuda') but no GPU is visible")
            self.tdev = torch.device(device)
            if self.tdev.index is None:
                self.tdev = torch.device("cuda", torch.cuda.current_device())
            props = torch.cuda.get_device_properties(self.tdev)
            self.num_cus = num_cus or props.multi_processor_count
            arch = getattr(props, "gcnArchName", "")
            if arch and not arch.startswith("gfx950"):
                raise RuntimeError(f"this data plane is built for gfx950 only (device is {arch})")
        else:
            self.num_cus = num_cus or 256
        self._alloc_counters()

    # ------------------------------------------------------------------ buffers
    def _buf(self, name: str, arr: np.ndarray):
        """Upload/replace a host array as a device buffer (torch uint8 view on GPU)."""
        self._gen += 1  # device addresses change: captured graphs must be re-captured
        arr = np.ascontiguousarray(arr)
        if self.gpu:
            torch = _torch()
            t = torch.from_numpy(arr.view(np.uint8).reshape(-1).copy()).to(self.tdev, non_blocking=False)
            self._dev[name] = t
        else:
            self._dev[name] = arr.copy()
        return self._dev[name]

    def _zeros(self, name: str, n: int, dtype=np.uint64):
        self._gen += 1
        if self.gpu:
            torch = _torch()
            tdt = {np.uint64: torch.int64, np.uint32: torch.int32, np.uint8: torch.uint8}[dtype]
            self._dev[name] = torch.zeros(n, dtype=tdt, device=self.tdev)
        else:
            self._dev[name] = np.zeros(n, dtype)
        return self._dev[name]

    def _ptr(self, name: str) -> int:
        b = self._dev.get(name)
        if b is None:
            return 0
        return int(b.data_ptr()) if self.gpu else int(b.ctypes.data)

    def _alloc_counters(self) -> None:
        self._zeros("flow_ctr", self.flows.nbuckets * 4)
        self._zeros("port_ctr", T.MAX_PORTS * 2)
        self._zeros("drop_ctr", 16)
        self._zeros("t0", 1)

    # ------------------------------------------------------------------ commit
    def commit(self, full: bool = False, _hooks: bool = True) -> dict:
        """Push host table changes to the device.  Returns what was sent.

        With resident ring kernels (dataplane/ring.py) running, a commit is applied under them
        without a stall whenever it can be: flow changes go to the idle copy of the
        double-buffered flow table, any other table to new buffers staged as each coop ring's idle
        table set; then ONE epoch change switches both (`_live_prepare` / `_live_flip`).  The
        native I/O engines feeding this plane only hold publication across that switch (no
        drain), so every burst sees either the old or the new tables.  Anything else (non-coop
        rings, a first IPv6 upload, `full`) pauses the engines, drains and stops the rings,
        updates the tables and relaunches them (their small tables are staged in LDS at launch).
        `_hooks=False`: the caller (MultiDataPlane) runs the engine hooks once for all planes."""
        FAULTS.check("dataplane.commit")
        with self._commit_lock:
            return self._commit_locked(full, _hooks)

    def _commit_locked(self, full: bool, _hooks: bool) -> dict:
        hooks = list(getattr(self, "_io_hooks", ())) if _hooks else []
        rings = self._running_rings()
        plan = self._live_plan(rings, full)
        if plan is not None:
            with TRACER.span("dataplane.commit_live", plan=plan):
                prep = self._live_prepare(rings, plan)
                live_switch(self, [(self, rings, prep)], hooks)
            return prep["sent"]
        # native I/O engines (dataplane/native_io.py) feeding this data plane: nothing in flight
        # while tables move, then they re-read the new tables
        for h in hooks:
            h.pre_commit(self)
        try:
            for r in rings:
                r.stop()
            with TRACER.span("dataplane.commit", full=full):
                sent = self._commit(full)
            if rings:
                _torch().cuda.current_stream(self.tdev).synchronize()
                for r in rings:
                    r.resume()
            return sent
        finally:
            for h in hooks:
                h.post_commit(self)

    def _running_rings(self) -> list:
        return [r for r in getattr(self, "_rings", []) if r.running]

    def _live_plan(self, rings, full: bool) -> str | None:
        """How a commit can be applied under running rings: "flows" (flow buckets only), "tables"
        (any table: coop rings with the double-buffered flow table), or None (drain + relaunch)."""
        if not rings or full:
            return None
        if self._only_flows_pending():
            return "flows"
        if (all(getattr(r, "coop", False) for r in rings) and "flows_b" in self._dev and not self._flow6_full
                and all(getattr(r, "v6", False) == self._v6_keys() for r in rings)):
            return "tables"
        return None

    def _models(self):
        return (("ports", self.ports), ("chains", self.chains), ("macs", self.macs), ("lag", self.lag),
                ("flood", self.flood), ("nexthops", self.nexthops), ("ecmp", self.ecmp),
                ("tunnels", self.tunnels), ("terms", self.terms), ("vmmac", self.vmmac),
                ("tunnels6", self.tunnels6), ("terms6", self.terms6),
                ("vtep6", self.vtep6))   # vtep6: a kernarg fold, listed for the version tracking

    def _only_flows_pending(self) -> bool:
        """True when the device is current in everything but (possibly) flow buckets."""
        if "flows" not in self._dev or "rss_key" not in self._dev or "acl_value" not in self._dev:
            return False
        if self._flow6_full:   # the flow buffer grows its IPv6 side array: a full upload
            return False
        if any(self._versions.get(n) != m.version or n not in self._dev for n, m in self._models()):
            return False
        if len(self.routes) and (self._versions.get("routes") != self.routes.version or "lpm24" not in self._dev):
            return False
        if len(self.routes6) and (self._versions.get("routes6") != self.routes6.version or "lpm6" not in self._dev):
            return False
        return self._versions.get("acl") == self.acl.version

    # ------------------------------------------------------------------ IPv6 flows
    def _v6_keys(self) -> bool:
        """IPv6 flows / rules in the tables (after the pending commit): IPv6-capable kernels."""
        return bool(self._flow6_on or self.acl.rules6)

    def add_flow6(self, src, dst, sport: int = 0, dport: int = 0, proto: int = 17, zone: int = 0,
                  action=None) -> int:
        """Install an IPv6 5-tuple flow (pushed by the next commit).  The table holds its folded
        key (tables.flow_key6); the side entry of its slot holds the addresses, which the data
        plane compares on every hit (nfdp.h flow6_verify), so lookups are exact.  Two 5-tuples
        with one folded key cannot both be installed (ValueError)."""
        key, addrs = T.flow_key6(src, dst, sport, dport, proto, zone)
        k = tuple(int(x) for x in key)
        old = self.flows6.get(k)
        if old is not None and not np.array_equal(old, addrs):
            raise ValueError("IPv6 flow key collision: the folded key belongs to another 5-tuple")
        slot = self.flows.insert(key, action if action is not None else T.flow_action()[0])
        self.flows6[k] = addrs
        if not self._flow6_on:
            self._flow6_on = True
            self._flow6_full = True
        return slot

    def remove_flow6(self, src, dst, sport: int = 0, dport: int = 0, proto: int = 17, zone: int = 0) -> bool:
        key, addrs = T.flow_key6(src, dst, sport, dport, proto, zone)
        k = tuple(int(x) for x in key)
        old = self.flows6.get(k)
        if old is None or not np.array_equal(old, addrs):
            return False     # not installed, or the folded key belongs to another 5-tuple
        del self.flows6[k]
        return self.flows.erase(key)

    def _side6_rows(self, buckets: np.ndarray, slots: np.ndarray | None = None) -> np.ndarray:
        """IPv6 side rows (uint32 [len(buckets), 32]: 4 slots x {src6, dst6}) of these buckets."""
        sl = (slots if slots is not None else self.flows.t.slots()).reshape(-1, 32)[buckets].reshape(-1, 4, 8)
        out = np.zeros((len(buckets), 4, 8), np.uint32)
        meta = sl[:, :, 3]
        for b, j in zip(*np.nonzero((meta & np.uint32(T.KEY_V6 | T.SLOT_USED)) == np.uint32(T.KEY_V6 | T.SLOT_USED))):
            k = (int(sl[b, j, 0]), int(sl[b, j, 1]), int(sl[b, j, 2]), int(meta[b, j]) & ~T.SLOT_USED)
            a = self.flows6.get(k)
            if a is not None:
                out[b, j] = a
        return out.reshape(-1, 32)

    def _flow_image(self) -> np.ndarray:
        """The device flow buffer: the buckets, then (IPv6 flows on) their side rows."""
        slots = self.flows.t.slots()
        if not self._flow6_on:
            return slots
        side = self._side6_rows(np.arange(self.flows.nbuckets), slots)
        return np.concatenate([slots.reshape(-1), side.reshape(-1)])

    # ------------------------------------------------------------------ live flow updates
    # Double-buffered flow table: copy 0 = "flows", copy 1 = "flows_b"; tables_ptrs() and the
    # batch path use copy `_flow_active`, a ring kernel the copy its chunk's epoch names.  An
    # update writes the inactive copy (the rows changed by this commit plus those the copy missed
    # at the previous flip), flips, and the next update first waits for the flip's grace period.
    def enable_flow_flip(self) -> None:
        if not self.gpu or "flows_b" in self._dev:
            return
        self.commit()
        self._dev["flows_b"] = self._dev["flows"].clone()
        self._flow_lag = np.zeros(0, np.int64)

    def _flows_key(self, copy: int) -> str:
        return "flows_b" if copy else "flows"

    def flow_copy_ptrs(self) -> tuple[int, int]:
        return self._ptr("flows"), self._ptr("flows_b") or self._ptr("flows")

    def _live_prepare(self, rings, plan: str) -> dict:
        """Everything of a live commit but the switch: the previous flip's grace period waited
        out, the idle flow-table copy brought up to date, and ("tables") every other changed
        table uploaded into NEW device buffers (the running grid still reads the old ones) and
        staged as each ring's idle table set.  The old buffers live until the next grace period
        is over (the next live commit waits for it, then lets them go)."""
        t0 = time.perf_counter()
        for r in rings:
            if not r.eng.wait_grace(10.0):
                raise TimeoutError("ring: grace period of the previous flip did not end")
        t1 = time.perf_counter()
        sent: dict = {}
        ft = self.flows.t
        dirty = ft.take_dirty()
        moves = ft.take_moves()
        flow = bool(len(dirty))
        if flow:
            if "flows_b" not in self._dev:
                raise RuntimeError("live flow updates need enable_flow_flip() before the rings start")
            if moves:
                self.harvest()  # counters of moved slots are attributed before the move
            rows = np.union1d(dirty, self._flow_lag)
            self._push_buckets(rows, self._flows_key(self._flow_active ^ 1))
            sent["flow_buckets"] = int(len(dirty))
            self.flip_stats["buckets"] += int(len(rows))
        tset = plan == "tables"
        if tset:
            self._retired = dict(self._dev)             # the running set's buffers stay alive
            sent.update(self._commit(False))
        _torch().cuda.current_stream(self.tdev).synchronize()   # uploads complete before any wave can see them
        if tset:
            tables = self.tables_ptrs()
            tables["flows"], tables["flows_alt"] = self.flow_copy_ptrs()
            args = {"acl_wfrag": self._ptr("acl_wfrag"), "acl_cinit": self._ptr("acl_cinit"),
                    "acl_tiles": self._acl_tiles, "toep_frag": self._ptr("toep_frag"), "toep_tab": self._ptr("toep_tab")}
            regions = self.ctrl_regions()
            for r in rings:
                with r.lock:
                    r.eng.stage_tables(tables, args, 1 - int(r.eng.table_set))
                    r.eng.set_ctrl_regions(regions)
            sent["table_flip"] = True
        self.flip_stats["grace_s"] += t1 - t0
        return {"sent": sent, "flow": flow, "set": tset, "dirty": dirty, "t0": t0, "t1": t1}

    # ------------------------------------------------------------------ device control mailbox
    CTRL_TABLES = ("ports", "chains", "acl_permit", "macs")

    def ctrl_regions(self) -> list[tuple[int, int]]:
        """Device buffers a running ring's control mailbox may write: the small tables of the
        current table set (flow tables are excluded: they change only through the epoch flip)."""
        out = []
        for name in self.CTRL_TABLES:
            b = self._dev.get(name)
            if b is not None and self.gpu:
                out.append((int(b.data_ptr()), int(b.numel() * b.element_size())))
        return out

    def ctrl_ports(self, ports, timeout_s: float = 1.0) -> bool:
        """Push the host's entries of `ports` to the running coop rings through their control
        mailbox (ring.h RingCtrlRing): the resident grid writes them into its port table and every
        workgroup restages its LDS port copies.  A ctrl-net link / RX-state / MTU change this way
        costs no commit, no epoch change and no hold (a few microseconds of the poller wave).  The
        host model keeps the change; the next commit uploads it with everything else.  Returns
        False, having done nothing, when no coop ring runs (then commit() is the way)."""
        with self._commit_lock:   # (a live path's maintenance restart does not replace the rings meanwhile)
            return self._ctrl_ports_locked(ports, timeout_s)

    def _ctrl_ports_locked(self, ports, timeout_s: float) -> bool:
        rings = [r for r in self._running_rings() if getattr(r, "coop", False)]
        if not rings or not self.gpu or "ports" not in self._dev:
            return False
        base = int(self._dev["ports"].data_ptr())
        size = self.ports.a.dtype.itemsize
        writes = [(base + int(p) * size, self.ports.a[int(p)].tobytes()) for p in ports]
        t0 = time.perf_counter()
        for r in rings:
            seq = 0
            for dst, data in writes:
                seq = r.eng.post_write(dst, data, timeout_s)
            if not r.eng.wait_ctrl(seq, timeout_s):
                raise TimeoutError(f"ring: control mailbox write not applied (posted {r.eng.ctrl_posted}, "
                                   f"done {r.eng.ctrl_done}, alive {r.eng.alive()})")
        self.flip_stats["ctrl_last_s"] = time.perf_counter() - t0   # post -> applied by every grid
        for h in getattr(self, "_io_hooks", ()):
            if hasattr(h, "refresh"):
                h.refresh(self)   # the native engine's side-pass snapshot follows
        self.flip_stats["ctrl_writes"] = self.flip_stats.get("ctrl_writes", 0) + len(writes)
        return True

    def _live_flip(self, rings, prep: dict) -> None:
        """The switch: one epoch change per ring (flow copy and / or table set together)."""
        if not (prep["flow"] or prep["set"]):
            return
        for r in rings:
            r.eng.change_epoch(prep["flow"], prep["set"])
        self._after_flip(prep)

    def _after_flip(self, prep: dict) -> None:
        """Host bookkeeping of a switch that happened (the rings' epochs changed)."""
        if not (prep["flow"] or prep["set"]):
            return
        if prep["flow"]:
            self._flow_active ^= 1
            self._flow_lag = prep["dirty"]          # rows the now idle copy missed
            self.flip_stats["flips"] += 1
            prep["sent"]["flip"] = self._flow_active
        self._gen += 1
        now = time.perf_counter()
        if prep["set"]:
            self.flip_stats["table_flips"] = self.flip_stats.get("table_flips", 0) + 1
            self.flip_stats["table_update_s"] = self.flip_stats.get("table_update_s", 0.0) + now - prep["t0"]
        self.flip_stats["update_s"] += now - prep["t1"]

    def _commit(self, full: bool) -> dict:
        sent = {}
        if self._learned_on_device and (full or self._versions.get("macs") != self.macs.version):
            self.pull_learned()  # the host re-uploads the MAC table: keep what the GPU learned
        for name, model in self._models():
            if full or self._versions.get(name) != model.version or name not in self._dev:
                self._buf(name, model.a)
                self._versions[name] = model.version
                sent[name] = model.a.nbytes
        if len(self.routes) and (full or self._versions.get("routes") != self.routes.version or "lpm24" not in self._dev):
            t24, t8 = self.routes.build()   # DIR-24-8: 64 MB tbl24 + tbl8 groups
            self._buf("lpm24", t24)
            self._buf("lpm8", t8)
            self._n_lpm8 = len(t8) // 256
            self._versions["routes"] = self.routes.version
            sent["routes"] = len(self.routes)
        if len(self.routes6) and (full or self._versions.get("routes6") != self.routes6.version or "lpm6" not in self._dev):
            tab, lens, nl = self.routes6.build()
            self._buf("lpm6", tab)
            self._buf("lpm6_lens", lens)
            self._lpm6 = (len(tab) - 1, int(nl))
            self._versions["routes6"] = self.routes6.version
            sent["routes6"] = len(self.routes6)
        if full or "rss_key" not in self._dev:
            key = np.frombuffer(self.rss_key, np.uint8)
            self._buf("rss_key", key)
            self._buf("toep_frag", self.nf.build_toeplitz_frags(self.rss_key))
            self._buf("toep_tab", self.nf.build_toeplitz_table(self.rss_key))
        if full or self._versions.get("acl") != self.acl.version or "acl_value" not in self._dev:
            val, msk, per, n = self.acl.arrays()
            self._buf("acl_value", val)
            self._buf("acl_mask", msk)
            self._buf("acl_permit", per)
            w, c, tiles = self.nf.build_acl_frags(val[: max(n, 1)] if n else np.zeros((0, 4), np.uint32),
                                                  msk[: max(n, 1)] if n else np.zeros((0, 4), np.uint32))
            self._buf("acl_wfrag", w)
            self._buf("acl_cinit", c)
            self._acl_tiles = int(tiles)
            self._n_acl = n
            # IPv6 rules: their verdicts follow the IPv4 ones (one rule index space), MFMA tiles
            # for v6_kernel, value / mask for the scalar paths
            v6, m6, p6, n6 = self.acl.arrays6()
            self._n_acl6 = n6
            if n6:
                self._buf("acl_permit", np.concatenate([per[: max(n, 1)] if n else np.zeros(0, np.uint8), p6[:n6]]))
                self._buf("acl6_value", v6[:n6])
                self._buf("acl6_mask", m6[:n6])
                w6, c6, t6 = self.nf.build_acl6_frags(v6[:n6], m6[:n6])
                self._buf("acl6_wfrag", w6)
                self._buf("acl6_cinit", c6)
                self._acl6_tiles = int(t6)
            self._versions["acl"] = self.acl.version
            sent["acl"] = n
        ft = self.flows.t
        if full or "flows" not in self._dev or self._flow6_full:
            self.harvest()
            img = self._flow_image()
            self._buf("flows", img)
            if "flows_b" in self._dev:   # both copies current: nothing lags
                self._buf("flows_b", img)
                self._flow_lag = np.zeros(0, np.int64)
            ft.clear_dirty()
            ft.take_moves()
            self._flow6_full = False
            sent["flows_full"] = len(self.flows)
        else:
            dirty = ft.take_dirty()
            moves = ft.take_moves()
            if len(dirty):
                if moves:
                    self.harvest()  # counters of moved slots are attributed before the move
                sent["flow_buckets"] = int(len(dirty))
                self._push_buckets(np.union1d(dirty, self._flow_lag) if "flows_b" in self._dev else dirty, "flows")
                if "flows_b" in self._dev:
                    self._push_buckets(np.union1d(dirty, self._flow_lag), "flows_b")
                    self._flow_lag = np.zeros(0, np.int64)
        return sent

    def _push_buckets(self, dirty: np.ndarray, dst: str = "flows") -> None:
        ft = self.flows.t
        slots = ft.slots()
        rows = slots.reshape(-1, 32)[dirty]   # whole 128-B buckets
        idx, mask = dirty.astype(np.uint32), ft.mask
        if self._flow6_on:
            # the side rows of the same buckets follow (rows nbuckets + b of the 2x buffer)
            nb = self.flows.nbuckets
            rows = np.concatenate([rows, self._side6_rows(dirty, slots)])
            idx = np.concatenate([idx, idx + np.uint32(nb)])
            mask = 2 * nb - 1
        if self.gpu:
            torch = _torch()
            up = {k: torch.from_numpy(np.ascontiguousarray(v).view(np.uint8).reshape(-1).copy()).to(self.tdev)
                  for k, v in (("idx", idx), ("rows", rows))}
            s = torch.cuda.current_stream(self.tdev).cuda_stream
            self.nf.launch_bucket_update(up["idx"].data_ptr(), len(idx), up["rows"].data_ptr(), self._ptr(dst),
                                         mask, s)
            self._keepalive = up
        else:
            self._dev[dst].view(np.uint32).reshape(-1, 32)[idx] = rows

    def tables_ptrs(self) -> dict:
        return {
            "ports": self._ptr("ports"), "chains": self._ptr("chains"), "n_chains": int(self.chains.n),
            "flows": self._ptr(self._flows_key(self._flow_active)),
            "bucket_mask": int(self.flows.t.mask), "macs": self._ptr("macs"), "mac_mask": int(self.macs.mask),
            "rss_key": self._ptr("rss_key"), "acl_value": self._ptr("acl_value"), "acl_mask": self._ptr("acl_mask"),
            "acl_permit": self._ptr("acl_permit"), "n_acl": int(getattr(self, "_n_acl", 0)),
            "acl_default_permit": 1 if self.acl.default_permit else 0,
            "lag_members": self._ptr("lag"), "n_lag_groups": int(self.lag.n),
            "flood": self._ptr("flood") if self.flood.n else 0, "n_flood": int(self.flood.n),
            "lpm24": self._ptr("lpm24") if len(self.routes) else 0, "lpm8": self._ptr("lpm8") if len(self.routes) else 0,
            "n_lpm8": int(getattr(self, "_n_lpm8", 0)),
            "nexthops": self._ptr("nexthops"), "n_nexthops": int(self.nexthops.n),
            "ecmp": self._ptr("ecmp"), "n_ecmp": int(self.ecmp.n),
            "tunnels": self._ptr("tunnels") if self.tunnels.n else 0, "n_tunnels": int(self.tunnels.n),
            "terms": self._ptr("terms") if self.terms.n else 0, "term_mask": int(self.terms.mask),
            "vmmac": self._ptr("vmmac") if self.vmmac.n else 0, "vmmac_mask": int(self.vmmac.mask),
            "lpm6": self._ptr("lpm6") if len(self.routes6) else 0,
            "lpm6_mask": int(getattr(self, "_lpm6", (0, 0))[0]),
            "lpm6_lens": self._ptr("lpm6_lens") if len(self.routes6) else 0,
            "n_lpm6_lens": int(getattr(self, "_lpm6", (0, 0))[1]),
            "tunnels6": self._ptr("tunnels6") if self.tunnels6.n else 0, "n_tunnels6": int(self.tunnels6.n),
            "vtep6_fold": int(self.nf.vtep6_fold(*(int(x) for x in self.vtep6.a))) if self.vtep6.active else 0,
            "vtep6": [int(x) for x in self.vtep6.a],
            "terms6": self._ptr("terms6") if len(self.terms6) else 0, "term6_mask": int(self.terms6.mask),
            "flow6_on": 1 if self._flow6_on and not self._flow6_full else 0,
            "n_acl6": int(getattr(self, "_n_acl6", 0)),
            "acl6_value": self._ptr("acl6_value") if getattr(self, "_n_acl6", 0) else 0,
            "acl6_mask": self._ptr("acl6_mask") if getattr(self, "_n_acl6", 0) else 0,
            "acl6_wfrag": self._ptr("acl6_wfrag") if getattr(self, "_n_acl6", 0) else 0,
            "acl6_cinit": self._ptr("acl6_cinit") if getattr(self, "_n_acl6", 0) else 0,
            "acl6_tiles": int(getattr(self, "_acl6_tiles", 0)) if getattr(self, "_n_acl6", 0) else 0,
        }

    def pairs_possible(self) -> bool:
        """Wide header pairs (128-B slots of VTEP-port frames: single-pass tunnel termination) can
        be in a batch: some port is a VTEP."""
        return bool(np.any(self.ports.a["flags"] & np.uint32(T.PORT_VTEP)))

    # ------------------------------------------------------------------ side outputs / learning
    SIDE_FLAGS = T.PORT_LEARN | T.PORT_ARP_TRAP | T.PORT_MIRROR | T.PORT_TUNNEL

    def side_active(self) -> bool:
        """Replicas / learn events can occur: a flood group or a learning / ARP-trap / mirror port."""
        return self.flood.n > 0 or bool(np.any(self.ports.a["flags"] & np.uint32(self.SIDE_FLAGS)))

    XHDR_WORDS = 32   # nfdp.h kXhdrBytes / 4: one packet's outer-header record

    def _tunnels_on(self) -> bool:
        return bool(self.tunnels.n or self.tunnels6.n)

    def _side_buffers(self, n: int = 0) -> dict:
        w = self.XHDR_WORDS
        if self._tunnels_on() and (self._dev.get("side_xhdr") is None or len(self._dev["side_xhdr"]) < n * w):
            self._zeros("side_xhdr", max(n, 1024) * w, np.uint32)   # outer-header record per packet
        if "side_cnt" not in self._dev:
            self._zeros("side_hdr", self.cap_rep * 16, np.uint32)
            self._zeros("side_meta", self.cap_rep, np.uint32)
            self._zeros("side_src", self.cap_rep, np.uint32)
            self._zeros("side_learn", self.cap_learn * 4, np.uint32)
            self._zeros("side_list", self.cap_rep, np.uint32)
            self._zeros("side_cnt", 8, np.uint32)
        # with tunnel ports every packet of a batch can need its outer-header record: the side list
        # holds the whole batch then (replicas keep their own cap)
        if len(self._dev["side_list"]) < n + 4 * self.num_cus * 512:
            # every packet of a batch can need the side pass (tunnel encap, learning ports); the
            # fused kernel's per-workgroup regions round each workgroup's share up to a block
            self._zeros("side_list", n + 4 * self.num_cus * 512, np.uint32)
        if "side_blk" not in self._dev:
            self._zeros("side_blk", 4 * self.num_cus, np.uint32)   # region counts (<= 4 workgroups / CU)
        self._dev["side_cnt"][:] = 0
        return {"rep_hdr": self._ptr("side_hdr"), "rep_meta": self._ptr("side_meta"), "rep_src": self._ptr("side_src"),
                "cap_rep": self.cap_rep, "learn": self._ptr("side_learn"), "cap_learn": self.cap_learn,
                "cnt": self._ptr("side_cnt"), "list": self._ptr("side_list"), "cap_list": int(len(self._dev["side_list"])),
                "blk_cnt": self._ptr("side_blk"), "blk_max": 4 * int(self.num_cus),
                "xhdr": self._ptr("side_xhdr") if self._tunnels_on() else 0}

    def _apply_learn(self, stream=None) -> None:
        """Apply this batch's learn events to the device MAC table (GPU: mac_learn_kernel on the
        batch's stream, no host sync; CPU: the sequential twin)."""
        self.stamp += 1
        if self.gpu:
            s = stream if stream is not None else _torch().cuda.current_stream(self.tdev).cuda_stream
            cnt = self._ptr("side_cnt")
            self.nf.launch_mac_learn(self._ptr("macs"), int(self.macs.mask), self._ptr("side_learn"), cnt + 4,
                                     self.cap_learn, self.stamp, cnt + 16, s)
        else:
            c = self._dev["side_cnt"]
            n = int(min(c[1], self.cap_learn))
            if n:
                c[4] += self.nf.mac_learn_cpu(self._ptr("macs"), int(self.macs.mask), self._ptr("side_learn"), n,
                                              self.stamp)
        self._learned_on_device = True

    def side_result(self) -> dict:
        """Replicas and learn counts of the last batch (synchronises on a GPU)."""
        if "side_cnt" not in self._dev:
            return {"n_rep": 0, "n_learn": 0}
        g = (lambda k: self._dev[k].cpu().numpy().view(np.uint32)) if self.gpu else (lambda k: self._dev[k])
        c = g("side_cnt")
        n = int(min(c[0], self.cap_rep))
        return {"n_rep": n, "rep_hdr": g("side_hdr").reshape(-1, 64 // 4)[:n].view(np.uint8).reshape(n, 64).copy(),
                "rep_meta": g("side_meta")[:n].copy(), "rep_src": g("side_src")[:n].copy(),
                "n_learn": int(c[1]), "rep_dropped": int(c[2]), "learn_dropped": int(c[3]),
                "learn_unplaced": int(c[4]), "n_side": int(c[5]), "side_dropped": int(c[6]),
                "xhdr": (g("side_xhdr").reshape(-1, self.XHDR_WORDS).view(np.uint8).reshape(-1, 4 * self.XHDR_WORDS)
                         if self._tunnels_on() else None)}

    @property
    def ipsec(self):
        """The IPsec ESP engine of this data plane (SA database, SPD, inbound SA table, kernels)."""
        if self._ipsec is None:
            from .ipsec import IpsecEngine

            self._ipsec = IpsecEngine(device=str(self.tdev) if self.gpu else "cpu", num_cus=self.num_cus)
        return self._ipsec

    def resolve_recirc6(self, frame: bytes) -> tuple[int, bytes] | None:
        """Finish the termination of a frame the kernel marked recirc6 (IPv6-underlay VXLAN /
        GENEVE to the local VTEP): (tunnel port, inner frame) from ipv6_tunnel_term_table on the
        whole frame (its VNI lies past the header slot), or None when no tunnel matches (the frame
        then goes to the slow path)."""
        fr = bytes(frame)
        off = 4 if fr[12:14] == b"\x81\x00" else 0
        if not self.vtep6.active or fr[38 + off:54 + off] != self.vtep6.a.tobytes():   # the kernel compared a fold
            return None
        r = self.terms6.lookup(fr)
        if r is None:
            return None
        port, off = r
        return port, bytes(frame[off:])

    def pull_learned(self) -> int:
        """Fold the entries the data plane learned into the host MAC model (native I/O engines
        feeding this plane first apply every learn event they have queued)."""
        if "macs" not in self._dev:
            return 0
        for h in getattr(self, "_io_hooks", ()):
            fl = getattr(h, "flush_learning", None)
            if fl is not None:
                fl()
        raw = self._dev["macs"]
        arr = (raw.cpu().numpy() if self.gpu else raw).view(T.MAC_DTYPE)
        n = self.macs.merge_learned(arr)
        self._learned_on_device = False
        return n

    def age_macs(self, max_age: int) -> int:
        """Host aging of learned MAC entries (older than `max_age` batches); commits the table."""
        self.pull_learned()
        n = self.macs.age(self.stamp, max_age)
        if n:
            self.commit()
        return n

    # ------------------------------------------------------------------ run
    def alloc_batch(self, n: int):
        """Output buffers for a batch of n packets."""
        if self.gpu:
            torch = _torch()
            out = torch.empty((n, 64), dtype=torch.uint8, device=self.tdev)
            meta = torch.empty(n, dtype=torch.int32, device=self.tdev)
            lat = torch.zeros((n + 15) // 16, dtype=torch.int32, device=self.tdev)
        else:
            out = np.zeros((n, 64), np.uint8)
            meta = np.zeros(n, np.uint32)
            lat = None
        return out, meta, lat

    def run(self, pkts, inmeta, out=None, meta=None, lat=None, stamp: bool = True, stream=None,
            flags: int = 0) -> BatchResult:
        """Process one batch.  GPU: pkts/inmeta torch tensors on the device ([n,64] uint8 / [n]
        int32); CPU: numpy arrays (runs the C++ oracle)."""
        n = int(pkts.shape[0])
        if TRACER.enabled:
            with TRACER.span("dataplane.run", n=n, gpu=self.gpu):
                return self._run(pkts, inmeta, out, meta, lat, stamp, stream, flags)
        return self._run(pkts, inmeta, out, meta, lat, stamp, stream, flags)

    def _run(self, pkts, inmeta, out, meta, lat, stamp, stream, flags) -> BatchResult:
        n = int(pkts.shape[0])
        if out is None:
            out, meta, lat = self.alloc_batch(n)
        tp = self.tables_ptrs()
        if self.gpu:
            torch = _torch()
            if pkts.device != self.tdev or inmeta.device != self.tdev:
                raise ValueError("batch must live on the data-plane device")
            if pkts.dtype != torch.uint8 or pkts.dim() != 2 or pkts.shape[1] != 64 or not pkts.is_contiguous():
                raise ValueError("pkts must be contiguous [n,64] uint8")
            if inmeta.numel() != n or out.shape[0] < n or meta.numel() < n:
                raise ValueError("batch buffer size mismatch")
            s = stream if stream is not None else torch.cuda.current_stream(self.tdev).cuda_stream
            if not self.count_flows:
                flags |= 4  # the kernel always gets the counter table; bit 2 makes it add 0
            pairs = self.pairs_possible()
            # batch-release stamp for the latency samples: by default each workgroup of the fused
            # kernel counts from its own start (t0 pointer null: a resident grid's workgroups all
            # begin at the launch), so no stamp kernel runs in front of every batch - nor in a
            # captured graph, whose every replay stamps anew; a stamp kernel still marks the
            # release before a pair pass
            t0_ptr = self._ptr("t0")
            if stamp and pairs:
                self.nf.launch_stamp(t0_ptr, s)
            elif stamp:
                t0_ptr = 0
            if pairs:
                # wide header pairs resolved in place over the whole batch first (kernels.hip pair_kernel)
                self.nf.launch_pairs(tp, pkts.data_ptr(), inmeta.data_ptr(), n, self._ptr("port_ctr"),
                                     not (flags & 1), s)
            side = self._side_buffers(n) if self.side_active() else None
            # split chains (a hop placed on another GPU): the XFER instances leave each handed-off
            # frame's HopState record here (MultiDataPlane / parallel.hops resume them there)
            hop = torch.empty((n, 8), dtype=torch.int32, device=self.tdev) if self.chains.split() else None
            # IPv6 tables: v6_kernel's folded keys, one 16-B row per slot for the fused V6 instances
            # (parked in the out slots instead, the V6 instance's key read touches 4x the lines)
            k6 = torch.empty((n, 4), dtype=torch.int32, device=self.tdev) if (tp.get("n_acl6") or tp.get("flow6_on")) else None
            # one launch covers < 2^25 slots (32-bit buffer views); bigger batches are split
            for lo in range(0, n, self.MAX_LAUNCH):
                m = min(self.MAX_LAUNCH, n - lo)
                self.nf.launch_fused(
                    tp, pkts.data_ptr() + 64 * lo, inmeta.data_ptr() + 4 * lo, out.data_ptr() + 64 * lo,
                    meta.data_ptr() + 4 * lo, m,
                    self._ptr("flow_ctr"), self._ptr("port_ctr"), self._ptr("drop_ctr"),
                    t0_ptr,
                    lat.data_ptr() + 4 * (lo // 16) if lat is not None else 0,
                    self._ptr("acl_wfrag"), self._ptr("acl_cinit"), self._acl_tiles,
                    self._ptr("toep_frag"), self._ptr("toep_tab"),
                    self.hash_mode, self.acl_mode, self.num_cus, s, flags, side,
                    hop_state=hop.data_ptr() + 32 * lo if hop is not None else 0,
                    v6_keys=k6.data_ptr() + 16 * lo if k6 is not None else 0,
                )
            if pairs:   # continuation slots: kCont metas carrying their pair's strip / valid bytes
                self.nf.launch_pair_fix(inmeta.data_ptr(), meta.data_ptr(), n, self._ptr("drop_ctr"), not (flags & 1), s)
            if side is not None:
                self._apply_learn(s)
            ex = {"lat": lat}
            if hop is not None:
                ex["hop_state"] = hop
            return BatchResult(out, meta, n, ex)
        pk = np.ascontiguousarray(pkts, np.uint8)
        im = np.ascontiguousarray(inmeta, np.uint32)
        hashes = np.zeros(n, np.uint32)
        acl = np.zeros(n, np.int32)
        side = self._side_buffers(n) if self.side_active() else None
        hop = np.zeros((n, 8), np.uint32) if self.chains.split() else None
        self.nf.oracle_run(tp, pk.ctypes.data, im.ctypes.data, n, out.ctypes.data, meta.ctypes.data,
                           self._ptr("flow_ctr"), self._ptr("port_ctr"), self._ptr("drop_ctr"),
                           hashes.ctypes.data, acl.ctypes.data, side, hop_state=hop.ctypes.data if hop is not None else 0)
        if side is not None:
            self._apply_learn()
        ex = {"hash": hashes, "acl": acl}
        if hop is not None:
            ex["hop_state"] = hop
        return BatchResult(out, meta, n, ex)

    def resume(self, hdr, state, stream=None, flags: int = 0) -> BatchResult:
        """The rest of split chains on this plane (the SFC hop pipeline across GPUs): `hdr` are
        handed-over header slots ([n,64] uint8), `state` their HopState records ([n,8] 32-bit), as
        another plane's run() left them (BatchResult.extra["hop_state"] rows of the frames whose meta
        says REMOTE with this plane as port).  Tx and drops are counted here; a frame its chain hands
        on again gets its record in extra["hop_state"].  GPU: tensors on this device (copy them over
        first: that copy is the xGMI hop); CPU: numpy (the oracle)."""
        n = int(hdr.shape[0])
        tp = self.tables_ptrs()
        if self.gpu:
            torch = _torch()
            if hdr.device != self.tdev or state.device != self.tdev:
                raise ValueError("resume: hand-off must live on the data-plane device")
            if hdr.dtype != torch.uint8 or tuple(hdr.shape) != (n, 64) or not hdr.is_contiguous():
                raise ValueError("hdr must be contiguous [n,64] uint8")
            if tuple(state.shape) != (n, 8) or state.element_size() != 4 or not state.is_contiguous():
                raise ValueError("state must be contiguous [n,8] 32-bit")
            out = torch.empty((n, 64), dtype=torch.uint8, device=self.tdev)
            meta = torch.empty(n, dtype=torch.int32, device=self.tdev)
            nxt = torch.zeros((n, 8), dtype=torch.int32, device=self.tdev)
            if n:
                cnt = torch.tensor([n], dtype=torch.int32, device=self.tdev)
                s = stream if stream is not None else torch.cuda.current_stream(self.tdev).cuda_stream
                self.nf.launch_resume(tp, cnt.data_ptr(), hdr.data_ptr(), state.data_ptr(), 0, n, out.data_ptr(),
                                      meta.data_ptr(), nxt.data_ptr(), self._ptr("port_ctr"), self._ptr("drop_ctr"),
                                      flags, self.num_cus, s)
            return BatchResult(out, meta, n, {"hop_state": nxt})
        hdr = np.ascontiguousarray(hdr, np.uint8).reshape(n, 64)
        state = np.ascontiguousarray(np.asarray(state).view(np.uint32)).reshape(n, 8)
        out = np.zeros((n, 64), np.uint8)
        meta = np.zeros(n, np.uint32)
        nxt = np.zeros((n, 8), np.uint32)
        if n:
            self.nf.oracle_resume(tp, hdr.ctypes.data, state.ctypes.data, n, out.ctypes.data, meta.ctypes.data,
                                  nxt.ctypes.data, self._ptr("port_ctr"), self._ptr("drop_ctr"))
        return BatchResult(out, meta, n, {"hop_state": nxt})

    def capture(self, n: int) -> "GraphedRun":
        """A batch of n slots as a captured HIP graph (see GraphedRun)."""
        return GraphedRun(self, n)

    def launch(self, pkts: int, inmeta: int, n: int, out: int, meta: int, lat: int = 0, t0: int | None = None,
               stream: int | None = None, n_dev: int = 0, flags: int = 0) -> None:
        """Pointer-level fused launch on the GPU (no batch checks): `n_dev` (optional) is a device
        word holding the real packet count (<= n), for batches whose size only the GPU knows."""
        if not self.gpu:
            raise RuntimeError("launch() is the GPU path; use run() for the oracle")
        s = stream if stream is not None else _torch().cuda.current_stream(self.tdev).cuda_stream
        if not self.count_flows:
            flags |= 4
        self.nf.launch_fused(
            self.tables_ptrs(), pkts, inmeta, out, meta, n,
            self._ptr("flow_ctr"), self._ptr("port_ctr"), self._ptr("drop_ctr"),
            self._ptr("t0") if t0 is None else t0, lat,
            self._ptr("acl_wfrag"), self._ptr("acl_cinit"), self._acl_tiles,
            self._ptr("toep_frag"), self._ptr("toep_tab"),
            self.hash_mode, self.acl_mode, self.num_cus, s, flags, None, n_dev,
        )

    # ------------------------------------------------------------------ counters
    def harvest(self) -> None:
        """Read-and-reset the packed per-flow counters into 64-bit host totals."""
        if "flow_ctr" not in self._dev:
            return
        n = self.flows.nbuckets * 4
        if self.gpu:
            torch = _torch()
            tmp = torch.empty(n, dtype=torch.int64, device=self.tdev)
            s = torch.cuda.current_stream(self.tdev).cuda_stream
            self.nf.launch_harvest(self._ptr("flow_ctr"), tmp.data_ptr(), n, s)
            raw = tmp.cpu().numpy().view(np.uint64)
        else:
            raw = self._dev["flow_ctr"].copy()
            self._dev["flow_ctr"][:] = 0
        pk, by = unpack_ctr(raw)
        self.flow_totals[:, 0] += pk
        self.flow_totals[:, 1] += by

    def flow_counters(self, key) -> tuple[int, int]:
        self.harvest()
        s = self.flows.find(key)
        if s < 0:
            return 0, 0
        return int(self.flow_totals[s, 0]), int(self.flow_totals[s, 1])

    def port_counters(self) -> np.ndarray:
        """[MAX_PORTS, 4] = rx_pkts, rx_bytes, tx_pkts, tx_bytes."""
        raw = self._dev["port_ctr"]
        raw = raw.cpu().numpy().view(np.uint64) if self.gpu else raw
        rx_p, rx_b = unpack_ctr(raw[0::2])
        tx_p, tx_b = unpack_ctr(raw[1::2])
        out = np.stack([rx_p, rx_b, tx_p, tx_b], axis=1)
        # side-pass output of native I/O engines (replicas they emitted on the host)
        for h in getattr(self, "_ctr_hooks", ()):
            sp = np.asarray(h.side_port_counters(), np.uint64).reshape(-1, 2)
            n = min(len(sp), len(out))
            out[:n, 2] += sp[:n, 0]
            out[:n, 3] += sp[:n, 1]
        return out

    def drop_counters(self) -> dict:
        raw = self._dev["drop_ctr"]
        raw = (raw.cpu().numpy().view(np.uint64) if self.gpu else raw).copy()
        for h in getattr(self, "_ctr_hooks", ()):
            d = np.asarray(h.side_drop_counters(), np.uint64)
            raw[: len(d)] += d[: len(raw)]
        return {T.REASONS.get(i, str(i)): int(v) for i, v in enumerate(raw) if v}

    def side_tables_host(self) -> dict:
        """Host copies of the tables the native engine's CPU side pass reads (iox SideTables):
        ports, MAC table, LAG groups, flood rows, tunnels, RSS key."""
        return {"ports": self.ports.a, "macs": self.macs.a, "mac_mask": int(self.macs.mask),
                "lag": self.lag.a, "n_lag_groups": int(self.lag.n), "flood": self.flood.a, "n_flood": int(self.flood.n),
                "tunnels": self.tunnels.a, "n_tunnels": int(self.tunnels.n), "tunnels6": self.tunnels6.a,
                "n_tunnels6": int(self.tunnels6.n), "rss": bytes(self.rss_key), "v6": bool(self._v6_keys())}

    TICK_S = 1e-8  # s_memrealtime: 100 MHz

    def fold_device_latency(self, res: "BatchResult") -> int:
        """Fold a GPU batch's sampled per-packet latencies (ticks since the batch's t0 stamp, one
        sample per 16 packets) into the `device` histogram; returns the number of samples."""
        lat = res.extra.get("lat") if self.gpu else None
        if lat is None:
            return 0
        ticks = lat[: (res.n + 15) // 16].cpu().numpy().view(np.uint32)
        ticks = ticks[ticks > 0]
        self.latency.observe_many("device", ticks.astype(np.float64) * self.TICK_S)
        return int(ticks.size)

    def reset_counters(self) -> None:
        self._alloc_counters()
        self.flow_totals[:] = 0


class GraphedRun:
    """`DataPlane.run` over fixed device buffers, captured once as a HIP graph
    (torch.cuda.CUDAGraph is hipGraph on ROCm): a replay is ONE graph launch for the fused kernel
    (whose workgroups stamp their own start for the latency samples) and, when side outputs are
    active, the side and learn kernels, instead of several host launches - what a launch-bound loop
    of small batches pays for.

        g = dp.capture(64)
        r = g(pkts, inmeta)          # copies into the captured input buffers, replays

    The graph holds the tables' device addresses: a commit that reallocates a buffer (or flips the
    flow-table copy) bumps the data plane's generation and the next call re-captures.  Replays
    reuse the capture's MAC-learning stamp (aging counts graph replays as one batch)."""

    def __init__(self, dp: DataPlane, n: int):
        if not dp.gpu:
            raise RuntimeError("graphs are a GPU feature")
        torch = _torch()
        self.dp, self.n = dp, int(n)
        self.pkts = torch.zeros((self.n, 64), dtype=torch.uint8, device=dp.tdev)
        self.inmeta = torch.zeros(self.n, dtype=torch.int32, device=dp.tdev)
        self.out, self.meta, self.lat = dp.alloc_batch(self.n)
        self.captures = 0
        self._capture()

    def _capture(self) -> None:
        torch = _torch()
        dp = self.dp
        dp.commit()
        s = torch.cuda.Stream(dp.tdev)
        s.wait_stream(torch.cuda.current_stream(dp.tdev))
        with torch.cuda.stream(s):       # warm-up: one-time kernel attributes, side buffers
            for _ in range(2):
                dp.run(self.pkts, self.inmeta, self.out, self.meta, self.lat)
        torch.cuda.current_stream(dp.tdev).wait_stream(s)
        torch.cuda.synchronize(dp.tdev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            dp.run(self.pkts, self.inmeta, self.out, self.meta, self.lat)
        self.gen = dp._gen
        self.captures += 1

    def __call__(self, pkts=None, inmeta=None) -> BatchResult:
        if self.dp._gen != self.gen:
            self._capture()
        if pkts is not None:
            self.pkts.copy_(pkts, non_blocking=True)
            self.inmeta.copy_(inmeta.view(self.inmeta.dtype) if inmeta.dtype != self.inmeta.dtype else inmeta,
                              non_blocking=True)
        self.graph.replay()
        return BatchResult(self.out, self.meta, self.n, {"lat": self.lat})


@contextlib.contextmanager
def commit_guard(planes):
    """Hold every plane's commit lock (a fixed order: no inversion between two holders): no
    commit runs while a live path rebuilds the rings its commits would flip."""
    locks = [p._commit_lock for p in sorted({id(p): p for p in planes}.values(), key=id) if hasattr(p, "_commit_lock")]
    for lk in locks:
        lk.acquire()
    try:
        yield
    finally:
        for lk in reversed(locks):
            lk.release()


def live_switch(dp, items, hooks) -> None:
    """The switch of a live commit over one or several planes: items = [(plane, running rings,
    its _live_prepare result)].  Behind a single native I/O engine the whole switch is one native
    call (hold, every ring's epoch change, the engine's new side tables / lists, release: the
    hold lasts microseconds and never waits for Python); otherwise the hooks hold, the epochs
    change, the hooks release."""
    flips = [(r, pr) for _p, rs, pr in items if (pr["flow"] or pr["set"]) for r in rs]
    if len(hooks) == 1 and hasattr(hooks[0], "switch"):
        hooks[0].switch(dp, [r.eng for r, _ in flips], [bool(pr["flow"]) for _, pr in flips],
                        [bool(pr["set"]) for _, pr in flips])
    else:
        for h in hooks:
            h.hold(dp)
        try:
            for r, pr in flips:
                r.eng.change_epoch(pr["flow"], pr["set"])
        finally:
            for h in hooks:
                h.release(dp)
    for p, _rs, pr in items:
        p._after_flip(pr)
