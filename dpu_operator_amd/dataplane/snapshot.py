"""Data-plane checkpoint / restore.

Saves every host table model of a DataPlane (ports, chains, MAC, ACL rules, LAG, flows with their
actions, per-flow counter totals, RSS key) into one .npz written without pickling, and restores it
into a fresh DataPlane (CPU or GPU) followed by a full commit — a restarted VSP resumes forwarding
with identical behaviour and counters.  Flow entries are re-inserted (bucket positions may differ;
lookups are equivalent), counters follow their flow key.
"""
from __future__ import annotations

import os

import numpy as np

from . import tables as T

_USED = 0x100  # kSlotUsed marker in key.meta byte 1 (nfdp.h)


def _flows(dp) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    if getattr(dp, "placement", "flow") == "port":   # replicated flows: one copy, counts summed
        parts = [_flows(p) for p in dp.planes]
        return parts[0][0], parts[0][1], sum(x[2] for x in parts)
    if hasattr(dp, "planes"):       # MultiDataPlane: every GPU's shard
        parts = [_flows(p) for p in dp.planes]
        return tuple(np.concatenate([x[i] for x in parts]) for i in range(3))
    slots = dp.flows.t.slots()
    occ = (slots[:, 3] & _USED) != 0
    keys = slots[occ, 0:4].copy()
    keys[:, 3] &= ~np.uint32(_USED)
    dp.harvest()
    return keys, slots[occ, 4:8].copy(), dp.flow_totals[occ].copy()


def save(dp, path: str) -> dict:
    keys, acts, totals = _flows(dp)
    val, msk, per, n = dp.acl.arrays()
    tmp = path + ".tmp.npz"
    np.savez(tmp, ports=dp.ports.a, chains=dp.chains.a, n_chains=np.int64(dp.chains.n), macs=dp.macs.a,
             acl_value=val[:n], acl_mask=msk[:n], acl_permit=per[:n], acl_default=np.int64(dp.acl.default_permit),
             lag=dp.lag.a, n_lag=np.int64(dp.lag.n), flow_keys=keys, flow_actions=acts, flow_totals=totals,
             rss_key=np.frombuffer(dp.rss_key, np.uint8), flow_buckets=np.int64(dp.flows.nbuckets))
    os.replace(tmp, path)
    return {"flows": len(keys), "acl": int(n)}


def load(dp, path: str) -> dict:
    with np.load(path, allow_pickle=False) as z:
        if bytes(z["rss_key"]) != dp.rss_key:
            raise ValueError("snapshot was taken with a different RSS key")
        if z["ports"].dtype != T.PORT_DTYPE or z["macs"].dtype != T.MAC_DTYPE:
            raise ValueError("snapshot table layout does not match this build")
        dp.ports.a[:] = z["ports"]
        dp.ports.version += 1
        dp.chains.a[: len(z["chains"])] = z["chains"]
        dp.chains.n = int(z["n_chains"])
        dp.chains.version += 1
        if len(z["macs"]) != len(dp.macs.a):
            raise ValueError("MAC table size differs from the snapshot")
        dp.macs.a[:] = z["macs"]
        dp.macs.version += 1
        dp.acl.rules = [T.AclRule(v.copy(), m.copy(), bool(p)) for v, m, p in
                        zip(z["acl_value"], z["acl_mask"], z["acl_permit"])]
        dp.acl.default_permit = bool(z["acl_default"])
        dp.acl.version += 1
        dp.lag.a[: len(z["lag"])] = z["lag"]
        dp.lag.n = int(z["n_lag"])
        dp.lag.version += 1
        keys, acts, totals = z["flow_keys"], z["flow_actions"], z["flow_totals"]
        if len(keys):
            slots = np.asarray(dp.flows.insert_many(keys, acts), np.int64)
            if np.any(slots < 0):
                raise RuntimeError("flow table too small for the snapshot")
            if getattr(dp, "placement", "flow") == "port":   # a flow's count: on the first plane
                dp.planes[0].flow_totals[slots] = totals
            elif hasattr(dp, "planes"):   # counters follow their flow to its owner GPU
                own = dp.flows.owner(keys)
                for g, p in enumerate(dp.planes):
                    p.flow_totals[slots[own == g]] = totals[own == g]
            else:
                dp.flow_totals[slots] = totals
    dp.commit(full=True)
    return {"flows": int(len(keys)), "acl": len(dp.acl.rules)}
