"""All of a node's GPUs behind one data plane: small tables replicated, flows sharded by RSS owner.

The reference runs ONE data-plane owner per node covering every port (the dpu-daemon DaemonSet,
internal/controller/bindata/daemon/99.daemonset.yaml:20-21, with its VFs requested in
dpudevicehandler.go:89).  On an MI355X node that owner is eight GPUs.  ``MultiDataPlane`` gives
the VSP the same table API as a single ``DataPlane`` while spreading the work:

* every small table model (ports, chains, MAC, LAG, flood, FIB, nexthops, ECMP, tunnels, ACL, ...)
  is ONE host object shared by all planes; a commit uploads it to every GPU (replicated: each GPU
  runs the whole chain for the flows it owns);
* the flow table is sharded: flow f lives only on GPU ``owner_of(toeplitz(f), N)`` (its counters
  too), the same owner the native I/O engine computes on ingress (csrc/nfdp/iox.cpp
  `owner_of_frame`), so a packet always meets its flow entry;
* MAC learning happens on whichever GPU saw the frame; ``pull_learned`` folds every GPU's learned
  entries into the shared model and the next commit replicates them;
* counters: port / drop counters are summed over the GPUs, flow counters come from the owner.

The planes are ordinary ``DataPlane`` objects on ``cuda:0 .. cuda:N-1`` (or CPU oracle planes in
tests).  One process drives them: the live path needs no GPU-to-GPU traffic because the host
steers every frame to its owner's ring (pod rings are host memory every GPU can reach).

``placement="port"`` is the other split — the SFC hop pipeline across GPUs.  Every port (a pod's
VF, so one hop of a service function chain) is placed on one GPU (``place_port``; default
port % N) and every frame runs on its ingress port's GPU: a chain A -> B -> C whose hops sit on
GPUs 0, 1, 2 is processed hop by hop on 0, then 1, then 2, as the frames pass through the NF pods.
The flow table is then replicated (each hop's GPU meets every flow; 288 GB per GPU holds it many
times over), and a flow's counters are the sum of its counts on every GPU that carried it.  It
trades the flow split's memory and insert cost for port affinity: one GPU serves a pod's ingress
whatever its flows, so per-port order and per-port tables stay on one device.
"""
from __future__ import annotations

import numpy as np

from .engine import BatchResult, DataPlane, live_switch

# table models shared by all planes (one host object, replicated to every device)
SHARED_MODELS = ("ports", "chains", "macs", "lag", "flood", "routes", "routes6", "nexthops", "ecmp", "tunnels",
                 "terms", "vmmac", "tunnels6", "vtep6", "terms6", "acl")


class ShardedFlows:
    """The flow-table API of one DataPlane (insert_many / erase_many / find / len) over the
    per-GPU shards: every key goes to (and is looked up on) its owner only."""

    def __init__(self, planes: list[DataPlane]):
        self.planes = planes
        self.rss_key = planes[0].flows.rss_key

    def owner(self, keys: np.ndarray) -> np.ndarray:
        from ..native import nfdp

        keys = np.ascontiguousarray(np.asarray(keys, np.uint32).reshape(-1, 4))
        h = nfdp().toeplitz(keys, self.rss_key).astype(np.uint64)
        return ((h * np.uint64(len(self.planes))) >> np.uint64(32)).astype(np.int64)

    def __len__(self) -> int:
        return sum(len(p.flows) for p in self.planes)

    @property
    def nbuckets(self) -> int:
        return self.planes[0].flows.nbuckets

    def insert_many(self, keys: np.ndarray, actions: np.ndarray) -> np.ndarray:
        keys = np.ascontiguousarray(keys, np.uint32).reshape(-1, 4)
        actions = np.ascontiguousarray(actions, np.uint32).reshape(-1, 4)
        own = self.owner(keys)
        slots = np.full(len(keys), -1, np.int64)
        for g, p in enumerate(self.planes):
            sel = np.nonzero(own == g)[0]
            if len(sel):
                slots[sel] = p.flows.insert_many(keys[sel], actions[sel])
        return slots

    def insert(self, key, action) -> int:
        return int(self.insert_many(np.asarray([key], np.uint32), np.asarray([action], np.uint32))[0])

    def erase_many(self, keys: np.ndarray) -> int:
        keys = np.ascontiguousarray(keys, np.uint32).reshape(-1, 4)
        own = self.owner(keys)
        return sum(p.flows.erase_many(keys[own == g]) for g, p in enumerate(self.planes) if (own == g).any())

    def erase(self, key) -> bool:
        return self.erase_many(np.asarray([key], np.uint32)) == 1

    def find(self, key) -> int:
        g = int(self.owner(np.asarray([key], np.uint32))[0])
        return self.planes[g].flows.find(key)


class ReplicatedFlows:
    """The flow-table API over planes that all hold every flow (port placement): inserts and
    erases go to every plane (identical tables: the same slot everywhere), lookups to plane 0."""

    def __init__(self, planes: list[DataPlane]):
        self.planes = planes
        self.rss_key = planes[0].flows.rss_key

    def __len__(self) -> int:
        return len(self.planes[0].flows)

    @property
    def nbuckets(self) -> int:
        return self.planes[0].flows.nbuckets

    def insert_many(self, keys: np.ndarray, actions: np.ndarray) -> np.ndarray:
        slots = [p.flows.insert_many(keys, actions) for p in self.planes]
        if any(not np.array_equal(slots[0], s) for s in slots[1:]):
            raise RuntimeError("replicated flow tables diverged")
        return slots[0]

    def insert(self, key, action) -> int:
        return int(self.insert_many(np.asarray([key], np.uint32), np.asarray([action], np.uint32))[0])

    def erase_many(self, keys: np.ndarray) -> int:
        return [p.flows.erase_many(keys) for p in self.planes][0]

    def erase(self, key) -> bool:
        return self.erase_many(np.asarray([key], np.uint32)) == 1

    def find(self, key) -> int:
        return self.planes[0].flows.find(key)


class MultiDataPlane:
    def __init__(self, devices: list[str], placement: str = "flow", **kw):
        """placement: "flow" (flows sharded by RSS owner, each frame on its flow's GPU) or "port"
        (each frame on its ingress port's GPU, flows replicated: the SFC hop pipeline)."""
        if not devices:
            raise ValueError("at least one device")
        if placement not in ("flow", "port"):
            raise ValueError("placement: 'flow' or 'port'")
        self.planes = [DataPlane(device=d, **kw) for d in devices]
        p0 = self.planes[0]
        for dp in self.planes[1:]:
            for name in SHARED_MODELS:
                setattr(dp, name, getattr(p0, name))
        self.n = len(self.planes)
        self.placement = placement
        self.port_owner = None
        if placement == "port":
            from ..native import nfdp

            self.flows = ReplicatedFlows(self.planes)
            self.port_owner = np.arange(int(nfdp().MAX_PORTS) + 2, dtype=np.int64) % self.n
            for dp in self.planes:
                dp._port_owner = self.port_owner   # (the native engine steers by it: NativeLivePath)
        else:
            self.flows = ShardedFlows(self.planes)

    # table models, modes, device facts: plane 0's (shared objects)
    def __getattr__(self, name):
        if name in ("planes", "flows", "n", "placement", "port_owner"):
            raise AttributeError(name)
        return getattr(self.planes[0], name)

    def place_port(self, port: int, gpu: int) -> None:
        """Port placement: frames entering on `port` run on GPU `gpu` (takes effect for a
        running native engine at the next commit)."""
        if self.port_owner is None:
            raise RuntimeError("place_port needs placement='port'")
        if not 0 <= gpu < self.n:
            raise ValueError(f"gpu in [0, {self.n})")
        self.port_owner[int(port)] = int(gpu)
        self.ports.version += 1   # the next commit re-applies the engine's steering

    @property
    def gpu(self) -> bool:
        return self.planes[0].gpu

    # ------------------------------------------------------------------ commit / learning
    def ctrl_ports(self, ports, timeout_s: float = 1.0) -> bool:
        """Every plane's rings take the port entries through their control mailbox
        (DataPlane.ctrl_ports); False, with nothing done, unless every plane can."""
        from .engine import commit_guard

        with commit_guard(self.planes):   # (rings are not replaced meanwhile)
            if not all(any(getattr(r, "coop", False) for r in p._running_rings()) for p in self.planes):
                return False
            return all(p.ctrl_ports(ports, timeout_s) for p in self.planes)

    def commit(self, full: bool = False) -> dict:
        """Every plane's commit as one update for the engines that feed them.

        Live (every GPU's rings can take it without a relaunch): all planes prepare first (idle
        flow copies written, new table sets staged), then the engines hold publication once, every
        GPU switches epoch, and they release - so no burst sees GPU g on new tables and GPU h on
        old ones.  Otherwise the engines pause once around all planes' commits (not once per
        plane), and resume when every plane has its new tables."""
        from .engine import commit_guard

        with commit_guard(self.planes):
            return self._commit_all(full)

    def _commit_all(self, full: bool) -> dict:
        # learned MACs of every GPU reach the shared model before it is re-uploaded anywhere
        if any(getattr(p, "_learned_on_device", False) for p in self.planes):
            mv = self.planes[0].macs.version
            if any(p._versions.get("macs") != mv for p in self.planes) or full:
                self.pull_learned()
        hooks = []
        for p in self.planes:
            for h in getattr(p, "_io_hooks", ()):
                if h not in hooks:
                    hooks.append(h)
        rings = [p._running_rings() for p in self.planes]
        plans = [p._live_plan(r, full) for p, r in zip(self.planes, rings)]
        sent = {}
        if all(pl is not None for pl in plans):
            preps = [p._live_prepare(r, pl) for p, r, pl in zip(self.planes, rings, plans)]
            live_switch(self, list(zip(self.planes, rings, preps)), hooks)
            for g, pr in enumerate(preps):
                for k, v in pr["sent"].items():
                    sent[f"{k}@{g}"] = v
            return sent
        for h in hooks:
            h.pre_commit(self)
        try:
            for g, p in enumerate(self.planes):
                for k, v in p.commit(full, _hooks=False).items():
                    sent[f"{k}@{g}"] = v
        finally:
            for h in hooks:
                h.post_commit(self)
        return sent

    def pull_learned(self) -> int:
        return sum(p.pull_learned() for p in self.planes)

    def harvest(self) -> None:
        for p in self.planes:
            p.harvest()

    # ------------------------------------------------------------------ counters
    def port_counters(self) -> np.ndarray:
        return sum(p.port_counters() for p in self.planes)

    def drop_counters(self) -> dict:
        out: dict[str, int] = {}
        for p in self.planes:
            for k, v in p.drop_counters().items():
                out[k] = out.get(k, 0) + v
        return out

    def flow_counters(self, key) -> tuple[int, int]:
        if self.placement == "port":   # every GPU a hop of the flow ran on counted its share
            c = [p.flow_counters(key) for p in self.planes]
            return sum(x[0] for x in c), sum(x[1] for x in c)
        g = int(self.flows.owner(np.asarray([key], np.uint32))[0])
        return self.planes[g].flow_counters(key)

    @property
    def flow_totals(self) -> np.ndarray:
        """Per-slot [packets, bytes] (harvested).  Port placement: summed over the planes
        (replicated flows have the same slot on every plane); flow placement: plane 0's."""
        if self.placement == "port":
            return sum(p.flow_totals for p in self.planes)
        return self.planes[0].flow_totals

    def reset_counters(self) -> None:
        for p in self.planes:
            p.reset_counters()

    # ------------------------------------------------------------------ batches
    def owners(self, pkts: np.ndarray, inmeta: np.ndarray) -> np.ndarray:
        """Owner GPU of each packet, exactly as the native I/O engine steers it on ingress."""
        from ..native import nfdp

        if self.placement == "port":
            return self.port_owner[np.asarray(inmeta, np.uint32) & 0xFFFF] % self.n

        return np.asarray(nfdp().owner_of_frames(np.ascontiguousarray(pkts, np.uint8),
                                                 np.ascontiguousarray(inmeta, np.uint32),
                                                 np.ascontiguousarray(self.ports.a), bytes(self.flows.rss_key),
                                                 self.n, self._v6_keys()), np.int64)

    def _v6_keys(self) -> bool:
        return any(p._v6_keys() for p in self.planes)

    # ------------------------------------------------------------------ IPv6 flows
    def add_flow6(self, src, dst, sport: int = 0, dport: int = 0, proto: int = 17, zone: int = 0, action=None) -> int:
        """An IPv6 flow on its owner GPU (the Toeplitz owner of its folded key: where owners()
        and the native engine steer its frames)."""
        from . import tables as T2

        if self.placement == "port":
            slots = [p.add_flow6(src, dst, sport, dport, proto, zone, action) for p in self.planes]
            return slots[0]
        key, _ = T2.flow_key6(src, dst, sport, dport, proto, zone)
        g = int(self.flows.owner(key[None, :])[0])
        return self.planes[g].add_flow6(src, dst, sport, dport, proto, zone, action)

    def remove_flow6(self, src, dst, sport: int = 0, dport: int = 0, proto: int = 17, zone: int = 0) -> bool:
        from . import tables as T2

        if self.placement == "port":
            return [p.remove_flow6(src, dst, sport, dport, proto, zone) for p in self.planes][0]
        key, _ = T2.flow_key6(src, dst, sport, dport, proto, zone)
        g = int(self.flows.owner(key[None, :])[0])
        return self.planes[g].remove_flow6(src, dst, sport, dport, proto, zone)

    def run(self, pkts, inmeta, **kw) -> BatchResult:
        """A batch split by owner, each part through its GPU, results back in arrival order
        (host arrays in and out; the multi-GPU live path is the native engine's job).

        Split chains (a hop placed on another GPU, ``"ttl@1"``): a frame whose chain hands it over
        comes out of its first GPU with meta REMOTE (port = the GPU plane) and a HopState record;
        its header slot and record go device-to-device to that plane (the xGMI hop), which runs the
        rest of the chain (DataPlane.resume), as often as the chain hands it on."""
        if self.gpu:
            import torch

            pk = pkts.cpu().numpy() if isinstance(pkts, torch.Tensor) else np.asarray(pkts)
            im = inmeta.cpu().numpy().view(np.uint32) if isinstance(inmeta, torch.Tensor) else np.asarray(inmeta)
        else:
            pk, im = np.asarray(pkts), np.asarray(inmeta, np.uint32)
        n = len(pk)
        own = self.owners(pk, im)
        out = np.zeros((n, 64), np.uint8)
        meta = np.zeros(n, np.uint32)
        pend = []   # (global indices, header slots, HopState records) handed to another plane
        for g, p in enumerate(self.planes):
            sel = np.nonzero(own == g)[0]
            if not len(sel):
                continue
            if p.gpu:
                import torch

                r = p.run(torch.from_numpy(pk[sel].copy()).to(p.tdev), torch.from_numpy(im[sel].view(np.int32).copy()).to(p.tdev))
                torch.cuda.synchronize(p.tdev)
                out[sel] = r.out.cpu().numpy()
                meta[sel] = r.meta.cpu().numpy().view(np.uint32)
            else:
                r = p.run(pk[sel], im[sel])
                out[sel], meta[sel] = r.out, r.meta
            if "hop_state" in r.extra:
                pend += self._handoffs(sel, meta[sel], r.out, r.extra["hop_state"])
        hops = 0
        while pend:
            hops += 1
            if hops > 7:   # (a chain has at most 7 hops: a record cannot come round again)
                raise RuntimeError("split chain handed over more often than it has hops")
            nxt = []
            for gidx, tgt, hdr, st in pend:
                if tgt >= self.n:   # a hop placed on a GPU this node does not have: dropped
                    meta[gidx] = _drop_meta(T_BADPORT)
                    continue
                q = self.planes[tgt]
                if q.gpu:
                    import torch

                    rr = q.resume(hdr.to(q.tdev), st.to(q.tdev))   # device to device: the xGMI hop
                    torch.cuda.synchronize(q.tdev)
                    out[gidx] = rr.out.cpu().numpy()
                    meta[gidx] = rr.meta.cpu().numpy().view(np.uint32)
                else:
                    rr = q.resume(hdr, st)
                    out[gidx], meta[gidx] = rr.out, rr.meta
                nxt += self._handoffs(gidx, meta[gidx], rr.out, rr.extra["hop_state"])
            pend = nxt
        return BatchResult(out, meta, n, {"owner": own, "handoff_rounds": hops})

    @staticmethod
    def _handoffs(gidx: np.ndarray, meta: np.ndarray, out, hop_state) -> list:
        """The frames of one plane's results that its chains hand to another plane, grouped by
        target: [(global indices, target plane, header slots, HopState records)] (slots and records
        stay where they are: device tensors on a GPU plane)."""
        reason = (meta >> 26) & 0xF
        h = np.nonzero(reason == T_REMOTE)[0]
        if not len(h):
            return []
        tgt = meta[h] & 0xFFF
        res = []
        for t in np.unique(tgt):
            li = h[tgt == t]
            if not isinstance(out, np.ndarray):   # a GPU plane's tensors
                import torch

                ix = torch.from_numpy(li.astype(np.int64)).to(out.device)
                res.append((gidx[li], int(t), out.index_select(0, ix).contiguous(), hop_state.index_select(0, ix).contiguous()))
            else:
                res.append((gidx[li], int(t), np.ascontiguousarray(out[li]), np.ascontiguousarray(hop_state[li])))
        return res


T_BADPORT, T_REMOTE = 1, 10


def _drop_meta(reason: int) -> int:
    return 0xFFF | (reason << 26)


def visible_devices() -> list[str]:
    """Every MI355X this process can see (cuda:0 .. cuda:N-1), or ['cpu'] without one."""
    try:
        import torch

        n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:  # noqa: BLE001
        n = 0
    return [f"cuda:{i}" for i in range(n)] or ["cpu"]
