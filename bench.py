#!/usr/bin/env python3
"""Headline benchmark: Mpps (+ p50 pod-to-pod latency) of a 1M-flow service-function chain.

Metric / config from BASELINE.json: "Mpps + p50 pod-to-pod µs latency, 1M-flow SFC at 1/2/4/8
MI355X".  One step = one batch of B 64-byte packets PER GPU (weak scaling) pushed through the
whole chain:

    pod VF ingress (VLAN-isolated, spoof-checked)  ->  ACL (TCAM, 256 ternary rules, MFMA)  ->
    SNAT (per-flow state, 1M-flow exact-match table)  ->  L2 steer + egress VLAN tag  ->  pod VF

N = 1: one fused HIP kernel.  N > 1 (one process per GPU, torchrun), default `--mode rss`
(parallel/rss.py): flow-affine sharding - GPU k owns the flows whose Toeplitz hash maps to it
(`--flows` per GPU shard, N x 1M in total: weak scaling), the I/O layer steers packets to their
owner as host RSS does, and the owner runs the whole chain and egresses itself (pod rings are
host memory every GPU can write).  `--remote-frac` (default 1 %) of every batch is traffic the
producer could NOT steer: the fused kernel sends those packets' header slots to their owner,
one all-to-all per step (RCCL over xGMI) overlapped with the next step's kernel, and the owner
processes them.  `--mode replicated` (every GPU holds all flows, frames to pods on other GPUs
cross xGMI) and `--mode sharded` (descriptor / verdict / packet all-to-alls) are kept.

Data: synthetic (random-init 1M-flow table, random 5-tuples); inputs rotate over 4 pre-generated
batches so no step re-reads a cached one.  Latency: per-packet time from the batch release stamp
(s_memrealtime at the start of the step) to the packet's egress, sampled 1/16, p50 over the timed
steps' last batch — the latency AT the headline throughput.  The low-latency path is measured
separately (1 GPU, after the timed region): the persistent ring kernel (csrc/nfdp/ring.hip) with
64-packet chunks published one at a time, host-clock publish -> completion-flag round trip
(`p50_latency_us_ring`), plus the throughput-mode ring's Mpps with 32 x 4096 packets in flight.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import dpu_operator_amd  # noqa: E402,F401

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

BASELINE_METRIC = "Mpps + p50 pod-to-pod µs latency, 1M-flow SFC at 1/2/4/8 MI355X"
_T0 = time.time()


def _log(msg: str) -> None:
    """Progress on stderr (the JSON line stays the only stdout line): a long bench is never silent."""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


# RSS exchange protocol facts the multi-GPU tests check against (tests/test_multigpu.py,
# tests/test_rss_cpu.py): per step, one all-to-all of the per-peer counts, then one grouped
# send/recv of exactly those packets
RSS_A2A_PER_STEP = 2
RSS_EXCHANGE_KEYS = ("a2a_ms", "a2a_per_step", "protocol", "remote_frac", "max_packets_per_peer", "overflow_drops",
                     "xgmi_bytes_out_per_gpu_per_step", "xgmi_gbps_out_per_gpu", "host_lag_steps", "note")


def rss_exchange_info(a2a_s: float, sent_per_step: float, max_peer: int, remote_frac: float, lag: int) -> dict:
    """The `exchange` block of an RSS run: one exchange's time, bytes a GPU sends per step (68 B
    per misdirected packet: header slot + meta) and the xGMI rate that implies."""
    peer_bytes = int(sent_per_step * 68)
    return {"a2a_ms": round(a2a_s * 1e3, 4), "a2a_per_step": RSS_A2A_PER_STEP,
            "protocol": "count-first: counts all-to-all, then grouped send/recv of exactly those packets",
            "remote_frac": remote_frac, "max_packets_per_peer": int(max_peer), "overflow_drops": 0,
            "xgmi_bytes_out_per_gpu_per_step": peer_bytes,
            "xgmi_gbps_out_per_gpu": round(peer_bytes / max(a2a_s, 1e-9) / 1e9, 3),
            "host_lag_steps": int(lag),
            "note": "overlapped with later steps' kernels in the timed region; counts read lag steps late"}


# The exchange-bound variant of an N > 1 RSS run (`unsteered` block): the same pipeline with traffic
# no producer steered - every packet arrives at a random GPU, so (N-1)/N of each batch crosses
# xGMI to its flow's owner.  The headline steers like a NIC's RSS (1 % misdirected) and so mostly
# measures N independent GPUs; this block measures the all-to-all exchange.
RSS_UNSTEERED_KEYS = ("mpps", "mpps_per_gpu", "ms_per_step", "steps", "remote_frac", "sent_per_gpu_per_step",
                      "xgmi_bytes_out_per_gpu_per_step", "xgmi_gbps_out_per_gpu", "forwarded_fraction", "note")


def rss_unsteered_info(elapsed_s: float, steps: int, world: int, batch: int, sent_per_step: float,
                       fwd: float) -> dict:
    step_s = elapsed_s / max(steps, 1)
    peer_bytes = int(sent_per_step * 68)
    return {"mpps": round(world * batch / step_s / 1e6, 2), "mpps_per_gpu": round(batch / step_s / 1e6, 2),
            "ms_per_step": round(step_s * 1e3, 4), "steps": int(steps), "remote_frac": round((world - 1) / world, 4),
            "sent_per_gpu_per_step": int(sent_per_step), "xgmi_bytes_out_per_gpu_per_step": peer_bytes,
            "xgmi_gbps_out_per_gpu": round(peer_bytes / max(step_s, 1e-9) / 1e9, 2),
            "forwarded_fraction": round(fwd, 6),
            "note": "unsteered traffic: (N-1)/N of every batch exchanged with its owner over xGMI each step "
                    "(count-first all-to-all), timed like the headline (barrier + sync, max over ranks)"}


def _unsteered(a, dp, sc, owner, rank, world, dev, cdev, torch, dist, P, RssShardedDataPlane, rss_traffic) -> dict:
    """The exchange-bound variant of an N > 1 RSS run (rss_unsteered_info)."""
    rf = (world - 1) / world
    ub = []
    for r in range(min(a.rotate, 2)):
        pk, im = rss_traffic(sc, a.batch, rank, world, owner, rf, seed=7000 + 1000 * rank + r)
        ub.append((torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev)))
        del pk, im
    eng_u = RssShardedDataPlane(dp, rank, world, a.batch, remote_frac=rf)
    nu = max(1, min(a.steps, 10))
    for k in range(2):
        eng_u.step(*ub[k % len(ub)])
    eng_u.flush()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    s0 = eng_u.stats["sent"]
    tu = time.perf_counter()
    for k in range(nu):
        eng_u.step(*ub[k % len(ub)])
    eng_u.flush()
    torch.cuda.synchronize()
    dist.barrier()
    el_u = time.perf_counter() - tu
    tt = torch.tensor([el_u], dtype=torch.float64, device=cdev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el_u = float(tt.item())
    _, _, ru = P.meta_fields(eng_u.out_meta())
    fu = torch.tensor([float(np.mean((ru == 0) | (ru == 10)))], dtype=torch.float64, device=cdev)
    dist.all_reduce(fu, op=dist.ReduceOp.SUM)
    res = rss_unsteered_info(el_u, nu, world, a.batch, (eng_u.stats["sent"] - s0) / nu, float(fu.item()) / world)
    del eng_u, ub
    torch.cuda.empty_cache()
    return res


SCALE_KEYS = ("world_size", "backend", "rccl_version", "device_count", "local_devices", "per_rank_ms_per_step",
              "step_skew", "peer_access")


def scale_info(dist, torch, elapsed_s: float, steps: int, cdev) -> dict:
    """What the N > 1 run actually ran on (every rank calls it; a collective): the process group's
    size and backend, the RCCL version torch carries, the GPUs this node shows, every rank's own
    timed-loop ms per step (the headline takes the max) and the peer-access matrix of the local
    GPUs (the hop pipeline's peer stores need it).  Works under gloo on the CPU as well."""
    world = dist.get_world_size()
    mine = torch.tensor([elapsed_s / max(steps, 1) * 1e3], dtype=torch.float64, device=cdev)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    per = [round(float(x.item()), 4) for x in allr]
    try:
        v = torch.cuda.nccl.version() if torch.cuda.is_available() else None
        rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else (str(v) if v is not None else None)
    except Exception:  # noqa: BLE001 - no RCCL in this build
        rccl = None
    n = torch.cuda.device_count() if torch.cuda.is_available() else 0
    peer = [[bool(i == j or torch.cuda.can_device_access_peer(i, j)) for j in range(n)] for i in range(n)]
    return {"world_size": world, "backend": str(dist.get_backend()), "rccl_version": rccl, "device_count": n,
            "local_devices": n, "per_rank_ms_per_step": per,
            "step_skew": round(max(per) / max(min(per), 1e-9), 4), "peer_access": peer}


def measure_hops(a, devices: str) -> dict:
    """SFC hop pipeline across GPUs (BASELINE config 4): the headline chain split after nat - acl +
    nat on one data plane, l2fwd + egress on another - with the product's in-HBM hand-off
    (parallel/hops.py: XFER fused instance -> hop_pack_kernel storing slot + 32-B record into the
    other plane's inbox -> resume_kernel).  1 GPU: both planes on cuda:0 (a rehearsal: the stages run
    back to back on one GPU).  N > 1: rank 0 puts them on cuda:0 and cuda:1, so the hand-off's
    peer stores cross xGMI.  Run as a child process (tools/hop_bench.py) so nothing on that path
    can take the headline with it; `per_hop_us` splits a 64K batch's latency."""
    import subprocess

    cmd = [sys.executable, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "hop_bench.py"),
           "--devices", devices, "--batch", str(a.batch), "--flows", str(a.flows), "--acl", str(a.acl),
           "--pods", str(a.pods_per_gpu), "--steps", str(max(3, a.variant_steps)), "--hash", a.hash]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    except subprocess.TimeoutExpired:
        return {"error": "timed out (600 s)"}
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"exit {r.returncode}: {(r.stderr or r.stdout)[-300:]}"}
    return json.loads(lines[-1])


def _live_split(a, dev: str, planes: str) -> dict:
    """The live split-chain run (tools/live_bench.py --split) as a child process under a time limit:
    a stalled hand-off path must not take the headline with it."""
    import subprocess

    cmd = [sys.executable, "-u", os.path.join(REPO, "tools", "live_bench.py"), "--device", dev,
           "--pods", str(a.pods_per_gpu), "--flows", str(a.flows), "--duration", "0.5",
           "--threads", str(a.live_gen_threads), "--tx-workers", str(a.live_workers), "--queues", str(a.live_queues),
           "--split", "acl,nat,l2fwd@1"] + (["--planes", planes] if planes else [])
    try:
        r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=120)
    except subprocess.TimeoutExpired:
        return {"error": "timed out (120 s)"}
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    if r.returncode != 0 or not line:
        return {"error": f"exit {r.returncode}: {(r.stderr or r.stdout)[-300:]}"}
    return json.loads(line[-1])


def _live_veth(dev: str) -> dict:
    """veth pods -> native engine -> GPU ring (the deployed default), measured in-process with
    CAP_NET_ADMIN, else in `unshare -Urnm` (a user namespace of our own), else skipped."""
    import shutil
    import subprocess
    import tempfile

    from dpu_operator_amd.testutils import netns as NS

    cmd = [sys.executable, "-u", os.path.join(REPO, "tools", "live_bench.py"), "--veth", "pipeline", "--device", dev,
           "--pods", "4", "--threads", "2", "--queues", "2", "--tx-workers", "1", "--duration", "0.5"]
    try:
        if NS.privileged():
            argv, env = cmd, dict(os.environ)
        else:
            ok = shutil.which("unshare") and subprocess.run(["unshare", "-Urnm", "true"], capture_output=True,
                                                              timeout=20).returncode == 0
            if not ok:
                return {"skipped": "no CAP_NET_ADMIN / CAP_NET_RAW and no user namespaces on this box "
                                   "(veth pods cannot be created); see tests/test_deployed_node.py"}
            argv = ["unshare", "-Urnm"] + cmd
            env = dict(os.environ, DPU_NETNS_DIR=tempfile.mkdtemp(prefix="dpns", dir="/tmp"))
        r = subprocess.run(argv, env=env, cwd=REPO, capture_output=True, text=True, timeout=240)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        return json.loads(line[-1]) if line else {"error": (r.stderr or "no output")[-300:]}
    except Exception as ex:  # noqa: BLE001 - the headline must still be reported
        return {"error": str(ex)[:200]}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 22, help="packets per GPU per step")
    ap.add_argument("--flows", type=int, default=1 << 20)
    ap.add_argument("--acl", type=int, default=256, help="ACL (TCAM) rules evaluated per packet")
    ap.add_argument("--pods-per-gpu", type=int, default=8)
    ap.add_argument("--hash", default="lds", choices=["lds", "mfma"])
    ap.add_argument("--acl-mode", default="mfma", choices=["mfma", "scalar"])
    ap.add_argument("--rotate", type=int, default=4)
    ap.add_argument("--no-lowlat", action="store_true", help="skip the small-batch latency probe")
    ap.add_argument("--no-variants", action="store_true", help="skip the mixed / ACL1024 / IMIX measurements")
    ap.add_argument("--no-hops", action="store_true", help="skip the SFC hop pipeline across GPUs (tools/hop_bench.py)")
    ap.add_argument("--no-live", action="store_true", help="skip the live pod-to-pod (native I/O engine) block")
    ap.add_argument("--no-unsteered", action="store_true", help="N > 1 rss: skip the exchange-bound (unsteered) variant")
    ap.add_argument("--live-workers", type=int, default=0,
                    help="native I/O engine delivery threads per queue (0: run to completion, the rx thread delivers)")
    ap.add_argument("--live-queues", type=int, default=6, help="native I/O engine rx queues (threads)")
    ap.add_argument("--live-gen-threads", type=int, default=8, help="pod traffic generator threads (one per pod)")
    ap.add_argument("--live-trials", type=int, default=3, help="saturated live trials of 1 s (median reported)")
    ap.add_argument("--live-gpu-egress", action="store_true",
                    help="live block: the ring grid writes frames into the pods' rings itself (GPU-direct egress)")
    ap.add_argument("--variant-steps", type=int, default=30)
    ap.add_argument("--chunks", type=int, default=4, help="pipeline chunks per step (N > 1)")
    ap.add_argument("--mode", default="rss", choices=["rss", "replicated", "sharded"],
                    help="multi-GPU strategy for N > 1")
    ap.add_argument("--remote-frac", type=float, default=0.01,
                    help="rss: fraction of each batch the producer could not steer to its owner GPU")
    ap.add_argument("--io", default="device", choices=["device", "host"],
                    help="device: batches resident in HBM (DPU wire side); host: pinned host slots, SDMA up/down "
                         "around every kernel (1 GPU)")
    ap.add_argument("--force-sharded", action="store_true",
                    help="use the sharded multi-GPU pipeline even at N = 1 (measures its compute cost)")
    ap.add_argument("--rehearse", action="store_true",
                    help="correctness rehearsal of the N-GPU path on a 1-GPU box: every rank on cuda:0, gloo "
                         "with host-staged exchanges (RCCL refuses two ranks on one device); not a measurement")
    return ap.parse_args()


def _time_fused(dp, batches, steps, torch):
    out, meta, lat = dp.alloc_batch(int(batches[0][0].shape[0]))
    for k in range(3):
        dp.run(*batches[k % len(batches)], out, meta, lat)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        dp.run(*batches[k % len(batches)], out, meta, lat)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, meta


def _time_fresh(dp, batches, steps, torch):
    """Like _time_fused for batches the pipeline rewrites in place (pair_kernel terminates wide
    header pairs in the slots, so a replayed batch would skip the decap): every step runs on its
    own fresh copy, all made before the timed loop (steps x 256 MB of HBM), and the loop is timed
    like _time_fused (launches queued back to back).  Returns (seconds, last meta)."""
    work = [(batches[k % len(batches)][0].clone(), batches[k % len(batches)][1].clone()) for k in range(steps + 3)]
    out, meta, lat = dp.alloc_batch(int(batches[0][0].shape[0]))
    for k in range(3):
        dp.run(*work[k], out, meta, lat)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        dp.run(*work[3 + k], out, meta, lat)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    del work
    return el, meta


def measure_variants(a, dp, sc, dev, torch, S, P) -> dict:
    """Mixed traffic, L3-routed SFC, 1024-rule ACL and IMIX sizes on the headline's data plane (1 GPU)."""
    res = {"steps": a.variant_steps}
    n = a.batch
    # IMIX (7 x 64, 4 x 576, 1 x 1500): same flows, frame lengths from the mix
    imix = []
    for r in range(2):
        pk, im = S.traffic(sc, n, seed=7000 + r)
        sizes = S.imix_sizes(n, S.IMIX_SIMPLE, seed=r)
        pk, im = S.with_sizes(pk, im, sizes)
        imix.append((torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev), int(sizes.sum())))
    el, meta = _time_fused(dp, [(b[0], b[1]) for b in imix], a.variant_steps, torch)
    byts = sum(imix[k % 2][2] for k in range(a.variant_steps))
    fwd = float(np.mean(P.meta_fields(meta.cpu().numpy().view(np.uint32))[2] == 0))
    res["imix"] = {"mpps": round(n * a.variant_steps / el / 1e6, 1), "gbps": round(byts * 8 / el / 1e9, 1),
                   "mix": "7x64,4x576,1x1500", "forwarded_fraction": round(fwd, 4),
                   "note": "header slots through the kernel; payload stays in place (header-split I/O)"}
    del imix
    _log("variant: mixed")
    # mixed: 5 % flow miss, 2 % ACL deny, 0.1 % malformed
    deny = S.install_deny_flows(dp, sc, k=4096)
    dp.commit()
    mixed = []
    for r in range(2):
        pk, im = S.traffic_mixed(sc, deny, n, seed=8000 + r)
        mixed.append((torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev)))
    el, meta = _time_fused(dp, mixed, a.variant_steps, torch)
    rs = P.meta_fields(meta.cpu().numpy().view(np.uint32))[2]
    res["mixed_mpps"] = round(n * a.variant_steps / el / 1e6, 1)
    res["mixed_dispositions"] = {k: round(float(np.mean(rs == v)), 4) for k, v in
                                 (("ok", 0), ("acl_deny", 4), ("no_route", 5), ("malformed", 9))}
    _log("variant: L3-routed SFC")
    # L3-routed SFC: acl -> nat -> route (pod /32s through 8-way ECMP, 100K background prefixes
    # in the DIR-24-8 FIB), same flows and traffic as the headline
    info = S.install_l3_routes(dp, sc)
    dp.commit()
    pk, im = S.traffic(sc, n, seed=9101)
    b = [(torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev))]
    el, meta = _time_fused(dp, b, a.variant_steps, torch)
    res["l3_mpps"] = round(n * a.variant_steps / el / 1e6, 1)
    res["l3_forwarded_fraction"] = round(float(np.mean(P.meta_fields(meta.cpu().numpy().view(np.uint32))[2] == 0)), 4)
    res["l3_fib"] = info
    dp.chains.set(sc.chain_id, ["acl", "nat", "l2fwd"])
    dp.commit()
    del b
    _log("variant: ACL1024 on the headline traffic")
    # ACL1024 on the headline traffic
    acl_headline = list(dp.acl.rules)
    S.add_acl_rules(dp, 1024)
    dp.commit()
    pk, im = S.traffic(sc, n, seed=9001)
    b = [(torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev))]
    el, meta = _time_fused(dp, b, a.variant_steps, torch)
    res["acl1024_mpps"] = round(n * a.variant_steps / el / 1e6, 1)
    res["acl1024_forwarded_fraction"] = round(float(np.mean(P.meta_fields(meta.cpu().numpy().view(np.uint32))[2] == 0)), 4)
    _log("variant: ClassBench-style ACL")
    # ClassBench-style ACL: 1024 5-tuple rules, nested prefixes, port ranges, wildcard protocols
    info = S.install_acl_wild(dp, 1024)
    dp.commit()
    el, meta = _time_fused(dp, b, a.variant_steps, torch)
    res["acl_wild_mpps"] = round(n * a.variant_steps / el / 1e6, 1)
    res["acl_wild"] = {"rules": info["rules"], "ternary_entries": info["entries"], "rule_tiles": int(dp._acl_tiles),
                       "forwarded_fraction": round(float(np.mean(P.meta_fields(meta.cpu().numpy().view(np.uint32))[2] == 0)), 4)}
    # back to the headline's 256 rules: the dual-stack variant is the headline plus IPv6 (through
    # r4 s13 it ran with the 1024-rule variant's 1280 IPv4 rules left in place)
    dp.acl.rules = acl_headline
    dp.acl.version += 1
    dp.commit()
    del mixed, b
    _log("variant: dual stack")
    # dual stack: half the batch IPv6 (64K IPv6 flows of the same pods, 64 IPv6 ACL rules: the
    # v6_kernel pre-pass + the IPv6-capable fused instance), half the headline's IPv4 traffic.
    # Last: it turns the data plane's IPv6 features on.
    info6 = S.install_ipv6(dp, sc, 1 << 16, 64)
    dp.commit()
    b = []
    for r in range(2):
        pk4, im4 = S.traffic(sc, n - n // 2, seed=9200 + r)
        pk6, im6 = S.traffic_ipv6(sc, info6, n // 2, seed=9300 + r)
        perm = np.random.default_rng(r).permutation(n)
        pk, im = np.concatenate([pk4, pk6])[perm], np.concatenate([im4, im6])[perm]
        b.append((torch.from_numpy(np.ascontiguousarray(pk)).to(dev),
                  torch.from_numpy(np.ascontiguousarray(im).view(np.int32)).to(dev)))
    el, meta = _time_fused(dp, b, a.variant_steps, torch)
    res["ipv6_mpps"] = round(n * a.variant_steps / el / 1e6, 1)
    rs6 = P.meta_fields(meta.cpu().numpy().view(np.uint32))[2]
    res["ipv6_dispositions"] = {int(k): int(v) for k, v in zip(*np.unique(rs6, return_counts=True))}
    res["ipv6"] = {"ipv6_fraction": 0.5, "ipv6_flows": info6["flows"], "ipv6_acl_rules": info6["rules"],
                   "ipv4_acl_rules": len(dp.acl.rules),
                   "forwarded_fraction": round(float(np.mean(P.meta_fields(meta.cpu().numpy().view(np.uint32))[2] == 0)), 4),
                   "frames": "64-B IPv4 + 66-B tagged IPv6/UDP (the smallest)"}
    del b
    _log("variant: overlay")
    # overlay: the headline's traffic VXLAN-encapsulated on an underlay VTEP port (64-B inner frames,
    # 114-B outer): single-pass termination of wide header pairs (pair_kernel -> fused ->
    # pair_fix), the SFC on the inner frame.  n / 2 frames = n slots per step.
    ports = S.install_vxlan(dp, sc)
    dp.commit()
    b = []
    for r in range(2):
        pk, im, _ = S.traffic_vxlan(sc, ports, n // 2, seed=9400 + r)
        b.append((torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev)))
    el, meta = _time_fresh(dp, b, a.variant_steps, torch)
    rsx = P.meta_fields(meta.cpu().numpy().view(np.uint32))[2]
    res["vxlan_mpps"] = round((n // 2) * a.variant_steps / el / 1e6, 1)
    res["vxlan"] = {"frames_per_step": n // 2, "slots_per_step": n, "inner": "64-B frames of the headline's flows",
                    "forwarded_fraction": round(float(np.mean(rsx[0::2] == 0)), 4),
                    "note": "Mpps of encapsulated frames; each is a 128-B wide header pair (two slots); "
                            "a fresh copy of the batch per step, made before the timed loop (the pair pass "
                            "rewrites heads in place)"}
    dp.ports.clear(ports["vtep"])
    dp.commit()
    del b
    _log("variant: overlay egress")
    # overlay egress: every pod VF a VXLAN tunnel port, so every forwarded packet also gets its
    # outer-header record from the side pass (the headline's traffic, 4M packets per step)
    eg = S.install_vxlan_egress(dp, sc)
    dp.commit()
    pk, im = S.traffic(sc, n, seed=9500)
    b = [(torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev))]
    el, meta = _time_fused(dp, b, a.variant_steps, torch)
    m = meta.cpu().numpy().view(np.uint32)
    res["vxlan_egress_mpps"] = round(n * a.variant_steps / el / 1e6, 1)
    res["vxlan_egress"] = {"forwarded_fraction": round(float(np.mean(P.meta_fields(m)[2] == 0)), 4),
                           "encapsulated_fraction": round(float(np.mean(P.meta_xhdr(m))), 4),
                           "note": "fused kernel + side pass (50-B outer-header record per packet)"}
    for p_ in sc.pod_port:
        dp.ports.a[int(p_)]["flags"] &= ~np.uint32(S.T.PORT_TUNNEL)
    dp.ports.clear(eg["underlay"])
    dp.ports.version += 1
    dp.commit()
    del b
    _log("variant: BASELINE config 5")
    # BASELINE config 5: the rule set the Intel IPU VSP programs (8 host VFs: AddHostVfP4Rules x 8,
    # AddPeerToPeerP4Rules O(n^2), one NF: AddNFP4Rules; Init's phy-port / LAG / primary-network
    # rules) through the P4Runtime compile onto a fresh data plane, then VF->VF, VF->NF, NF->wire
    # and VF->OvS traffic of a 1M-5-tuple pool (dataplane/p4_scenario.py)
    from dpu_operator_amd.dataplane import p4_scenario as Q
    from dpu_operator_amd.dataplane.engine import DataPlane

    d4 = DataPlane(device=str(dev), flow_buckets=1 << 10, hash_mode=a.hash, acl_mode=a.acl_mode)
    q = Q.build(d4)
    pk, im, exp, kind = Q.traffic(q, 1 << 20, seed=9600)
    reps = max(1, n // (1 << 20))
    b = [(torch.from_numpy(np.tile(pk, (reps, 1))).to(dev), torch.from_numpy(np.tile(im, reps).view(np.int32)).to(dev))]
    el, meta = _time_fused(d4, b, a.variant_steps, torch)
    port, _, rs = P.meta_fields(meta.cpu().numpy().view(np.uint32))
    exp_t = np.tile(exp, reps)
    res["p4_ipu_mpps"] = round(int(b[0][0].shape[0]) * a.variant_steps / el / 1e6, 1)
    res["p4_ipu"] = {"host_vfs": len(q.vf_macs), "nf": 1, "p4_entries": q.n_entries, "tables": q.rules,
                     "batch": int(b[0][0].shape[0]), "mix": {k: w for k, w in Q.MIX},
                     "forwarded_fraction": round(float(np.mean(rs == 0)), 4),
                     "expected_port_fraction": round(float(np.mean(port == exp_t)), 4),
                     "note": "entries compiled from the Intel VSP's p4rt-ctl strings; 64-B frames, fused kernel"}
    del b, d4
    torch.cuda.empty_cache()
    return res


def main() -> None:
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus > 1 must be launched with torch.distributed.run (one process per GPU)")
    if a.rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    cdev = torch.device("cpu") if a.rehearse else dev  # where the small stats collectives run
    sharded = world > 1 or a.force_sharded
    if sharded:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if a.rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.ops import packets as P
    from dpu_operator_amd.parallel.replicated import ReplicatedDataPlane
    from dpu_operator_amd.parallel.rss import RssShardedDataPlane, flow_owner, rss_traffic
    from dpu_operator_amd.parallel.sharded import PipelinedShardedDataPlane, ShardedDataPlane, shard_filter

    replicated = sharded and world > 1 and a.mode == "replicated" and not a.force_sharded
    rss = sharded and world > 1 and a.mode == "rss" and not a.force_sharded
    t_setup = time.time()
    total_flows = a.flows * world if rss else a.flows  # rss: --flows per GPU shard (weak scaling)
    flows_here = a.flows if (replicated or rss or world == 1) else a.flows / world
    buckets = 1 << max(10, int(math.ceil(math.log2(flows_here / 2))))  # <= 50% load, 4 slots/bucket
    dp = DataPlane(device=str(dev), flow_buckets=buckets, hash_mode=a.hash, acl_mode=a.acl_mode)
    n_pods = a.pods_per_gpu * world
    pod_gpu = np.arange(n_pods) // a.pods_per_gpu
    sc = S.build_sfc(dp, n_pods=n_pods, n_flows=total_flows, n_acl=a.acl, seed=0, pod_gpu=pod_gpu,
                     flow_filter=shard_filter(rank, world) if (world > 1 and not replicated) else None)
    dp.commit(full=True)
    my_pods = np.where(pod_gpu == rank)[0]
    owner = flow_owner(sc.keys, world, dp.flows.rss_key) if rss else None
    batches = []
    for r in range(a.rotate):
        if rss:
            pk, im = rss_traffic(sc, a.batch, rank, world, owner, a.remote_frac, seed=1000 * rank + r + 1)
        else:
            pk, im = S.traffic(sc, a.batch, seed=1000 * rank + r + 1, src_pods=my_pods)
        batches.append((torch.from_numpy(pk).to(dev), torch.from_numpy(im.view(np.int32)).to(dev)))
        del pk, im
    drain = None
    if not sharded and a.io == "host":
        from dpu_operator_amd.dataplane.pktio import HostPath

        hp = HostPath(dp, a.batch, depth=3)
        for s in range(hp.depth):  # the NIC side fills the pinned slots; synthetic frames here
            pk, im = batches[s % a.rotate]
            hp.load(s, pk.cpu().numpy(), im.cpu().numpy())
        batch_ms = []

        def step(k):
            s = k % hp.depth
            if k >= hp.depth:
                hp.wait(s)
                batch_ms.append(hp.timings_ms(s)["total"])
            hp.submit(s, a.batch)

        def drain():
            for s in range(hp.depth):
                hp.wait(s)

        def results():
            _, m = hp.results(0)
            return np.array(m), np.array(batch_ms[-64:]) * 1e3
    elif not sharded:
        out, meta, lat = dp.alloc_batch(a.batch)

        def step(k):
            pk, im = batches[k % a.rotate]
            dp.run(pk, im, out, meta, lat)

        def results():
            return meta.cpu().numpy().view(np.uint32), lat.cpu().numpy().view(np.uint32).astype(np.float64) * 0.01
    elif rss:
        eng = RssShardedDataPlane(dp, rank, world, a.batch, remote_frac=a.remote_frac)

        def step(k):
            pk, im = batches[k % a.rotate]
            eng.step(pk, im)

        def drain():
            eng.flush()

        def results():
            return eng.out_meta(), eng.latency_samples_us()
    elif replicated:
        eng = ReplicatedDataPlane(dp, rank, world, a.batch, chunks=a.chunks)

        def step(k):
            pk, im = batches[k % a.rotate]
            eng.step(pk, im)

        def results():
            return eng.out_meta(), eng.latency_samples_us()
    else:
        eng = PipelinedShardedDataPlane(dp, rank, world, a.batch, chunks=a.chunks)

        def step(k):
            pk, im = batches[k % a.rotate]
            eng.step(pk, im)

        def results():
            return eng.out_meta(), eng.latency_samples_us()

    setup_s = time.time() - t_setup
    _log(f"setup done ({setup_s:.1f} s), warmup + timed steps")
    for k in range(a.warmup):
        step(k)
    if drain:
        drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(a.warmup + k)
    if drain:
        drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    scale = None
    if world > 1:
        scale = scale_info(dist, torch, elapsed, a.steps, cdev)
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    _log(f"timed region: {elapsed * 1e3 / a.steps:.4f} ms / step")
    meta_np, lat_us = results()
    _, _, reasons = P.meta_fields(meta_np)
    fwd_local = float(np.mean((reasons == 0) | (reasons == 10)))  # 10: handed to its owner / egress GPU
    p50 = float(np.median(lat_us)) if len(lat_us) else float("nan")
    p99 = float(np.percentile(lat_us, 99)) if len(lat_us) else float("nan")
    if world > 1:
        st = torch.tensor([p50, p99, fwd_local], dtype=torch.float64, device=cdev)
        g = [torch.zeros_like(st) for _ in range(world)]
        dist.all_gather(g, st)
        arr = torch.stack(g).cpu().numpy()
        p50, p99, fwd_local = float(np.median(arr[:, 0])), float(np.max(arr[:, 1])), float(np.mean(arr[:, 2]))

    # exchange alone (outside the timed region, N > 1 replicated): the step's all-to-alls with no
    # compute around them -> achieved xGMI bandwidth per GPU and the exchange floor of a step
    xchg = None
    if rss:
        # the timed steps' traffic: packets this GPU handed to their owners (68 B each on xGMI)
        sent_per_step = eng.stats["sent"] / max(eng.stats["steps"], 1)
        max_peer = eng.stats["max_peer"]
        s0 = eng.slots[eng.k % eng.nslots]   # (flushed: no slot is in flight)

        def xone():
            eng.exchange(s0)
            if eng.comm is not None:
                eng.comm.synchronize()

        for _ in range(3):
            xone()
        torch.cuda.synchronize()
        dist.barrier()
        reps = 20
        t1 = time.perf_counter()
        for _ in range(reps):
            xone()
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        tt = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        xchg = rss_exchange_info(el / reps, sent_per_step, max_peer, a.remote_frac, eng.lag)
    if replicated:
        s0 = eng.slots[0]
        for _ in range(3):
            eng.exchange(s0).wait()
        torch.cuda.synchronize()
        dist.barrier()
        reps = 10
        t1 = time.perf_counter()
        for _ in range(reps):
            eng.exchange(s0).wait()
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        tt = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
        n_chunks = (a.batch + eng.chunk - 1) // eng.chunk
        peer_bytes = (world - 1) * eng.pseg  # what one GPU sends over its links per all-to-all
        xchg = {"a2a_ms": round(el / reps * 1e3, 4), "a2a_per_step": n_chunks,
                "exchange_ms_per_step": round(el / reps * n_chunks * 1e3, 4),
                "xgmi_bytes_out_per_gpu_per_step": peer_bytes * n_chunks,
                "xgmi_gbps_out_per_gpu": round(peer_bytes / (el / reps) / 1e9, 1)}

    # exchange-bound variant (outside the timed region, N > 1 RSS): unsteered traffic, (N-1)/N of
    # every batch crosses xGMI to its owner
    unsteered = None
    if rss and not a.no_unsteered:
        try:
            unsteered = _unsteered(a, dp, sc, owner, rank, world, dev, cdev, torch, dist, P, RssShardedDataPlane,
                                   rss_traffic)
        except Exception as ex:  # noqa: BLE001 - the headline must still be reported (every rank gets here)
            unsteered = {"error": str(ex)[:200]}

    # small-batch latency probe (outside the timed region): 64K packets per step, fused/sharded alike
    p50_small = None
    if not a.no_lowlat and a.io == "device":
        nsm = 1 << 16
        pk, im = batches[0][0][:nsm].contiguous(), batches[0][1][:nsm].contiguous()
        if not sharded:
            o2, m2, l2 = dp.alloc_batch(nsm)
            for _ in range(20):   # (latency from a stamp kernel before the launch, as through r5)
                dp.nf.launch_stamp(dp._ptr("t0"), torch.cuda.current_stream().cuda_stream)
                dp.run(pk, im, o2, m2, l2, stamp=False)
            torch.cuda.synchronize()
            ls = l2.cpu().numpy().view(np.uint32).astype(np.float64) * 0.01
        elif rss:
            eng_s = RssShardedDataPlane(dp, rank, world, nsm, remote_frac=a.remote_frac)
            for _ in range(20):
                eng_s.step(pk, im)
            eng_s.flush()
            torch.cuda.synchronize()
            ls = eng_s.latency_samples_us()
        elif replicated:
            eng_s = ReplicatedDataPlane(dp, rank, world, nsm, chunks=1)
            for _ in range(20):
                eng_s.step(pk, im)
            torch.cuda.synchronize()
            ls = eng_s.latency_samples_us()
        else:
            eng_s = ShardedDataPlane(dp, rank, world, nsm)
            for _ in range(20):
                eng_s.step(pk, im)
            torch.cuda.synchronize()
            ls = eng_s.latency_samples_us()
        p50_small = float(np.median(ls)) if len(ls) else None
        if world > 1:
            t = torch.tensor([p50_small or 0.0], dtype=torch.float64, device=cdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            p50_small = float(t.item())

    # host round trip of a small batch (outside the timed region, 1 GPU): submit -> results ready
    # on the host clock, with per-batch launches vs one replay of the captured HIP graph
    _log("small-batch probes")
    rtt = None
    if not a.no_lowlat and world == 1 and a.io == "device" and not sharded:
        nb = 256
        pk, im = batches[0][0][:nb].contiguous(), batches[0][1][:nb].contiguous()
        o3, m3, l3 = dp.alloc_batch(nb)
        gr = dp.capture(nb)

        def _rtt(fn, reps=300):
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t) * 1e6)
            return float(np.median(ts))

        rtt = {"batch": nb, "launch_p50_us": round(_rtt(lambda: dp.run(pk, im, o3, m3, l3)), 2),
               "graph_p50_us": round(_rtt(lambda: gr()), 2)}
        del gr

    # low-latency path (outside the timed region): persistent ring kernel, host publishes 64-packet
    # chunks and times publish -> completion flag on its own clock (dataplane/ring.py)
    _log("ring kernel probes")
    ring = None
    if not a.no_lowlat and world == 1 and a.io == "device":
        from dpu_operator_amd.dataplane.ring import RingPath

        try:
            # latency: cooperative ring (a workgroup's 4 waves share each chunk), one chunk in flight
            rp = RingPath(dp, capacity=1 << 16, deadline_s=60.0, coop=True)
            rp.stage(batches[0][0][: 1 << 16], batches[0][1][: 1 << 16])
            rp.start()
            lat1, _ = rp.probe(batches=4000, batch=64, inflight=1)
            rp.stop()
            rp.close()
            # loaded: throughput ring (every wave takes its own chunks), 32 x 4096 packets in flight.
            # One trial is a few ms of GPU work, so a single host-thread stall (the host both
            # publishes and reaps) can halve it: 5 trials of 10000 batches, the median reported.
            # 64 chunks of 4096 in flight (tools/ring_ab.py, r6: 4,622 Mpps median against 2,869 at 32
            # in flight - the host thread's publish -> reap loop needs that much depth to cover the
            # grid's completion latency; the r4/r5 swings were this depth at 32 plus box drift)
            rq = RingPath(dp, capacity=1 << 18, wgs_per_cu=2, deadline_s=120.0, coop=False)
            rq.stage(batches[0][0][: 1 << 18], batches[0][1][: 1 << 18])
            rq.start()
            rq.probe(batches=500, batch=4096, inflight=64)  # warm-up
            trials, lat2 = [], []
            for _ in range(5):
                lt, el2 = rq.probe(batches=10000, batch=4096, inflight=64)
                trials.append(10000 * 4096 / el2 / 1e6)
                lat2.append(lt[200:])
            rq.stop()
            rq.close()
            lat1 = lat1[400:]
            lat2 = np.concatenate(lat2)
            ring = {"p50_us": round(float(np.median(lat1)), 2), "p99_us": round(float(np.percentile(lat1, 99)), 2),
                    "loaded_mpps": round(float(np.median(trials)), 1),
                    "loaded_mpps_trials": [round(x, 1) for x in trials],
                    "loaded_p50_us": round(float(np.median(lat2)), 2),
                    "loaded_p99_us": round(float(np.percentile(lat2, 99)), 2)}
        except Exception as ex:  # the headline number must still be reported
            ring = {"error": str(ex)[:200]}

    # realistic variants (1 GPU, after the timed region, same kernel and table): the headline is the
    # best case (every packet forwarded), so also report a mix with flow misses / ACL denies /
    # malformed frames, a 1024-rule ACL, and IMIX frame sizes (header path; payload stays in place)
    _log("variants")
    variants = None
    if world == 1 and a.io == "device" and not a.no_variants:
        variants = measure_variants(a, dp, sc, dev, torch, S, P)

    # SFC hop pipeline across GPUs (after the timed region): the headline chain split over two
    # data planes with the in-HBM hand-off between them - both on cuda:0 at N = 1, cuda:0 -> cuda:1
    # over xGMI at N > 1 (rank 0 measures while the other ranks wait at the barrier)
    _log("hop pipeline")
    hops = None
    if a.io == "device" and not a.no_variants and not a.no_hops:
        if world > 1:
            dist.barrier()
        if rank == 0:
            peer = world > 1 and not a.rehearse and torch.cuda.device_count() > 1
            hops = measure_hops(a, "cuda:0,cuda:1" if peer else "cuda:0,cuda:0")
        if world > 1:
            dist.barrier()

    # live pod -> pod path (1 GPU, after the timed region): shared-memory pod vports, the native C++
    # I/O engine (csrc/nfdp/iox) and the persistent ring kernel; C++ pod generator / sinks measure
    # delivered Mpps and one-way latency on one clock (tools/live_bench.py)
    _log("live block")
    live = live_veth = None
    if world == 1 and a.io == "device" and not a.no_live:
        try:
            import importlib.util

            spec = importlib.util.spec_from_file_location(
                "live_bench", os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "live_bench.py"))
            lb = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(lb)
            from dpu_operator_amd.utils import cpuquota

            gde = bool(a.live_gpu_egress)
            # the CPU time the box really grants (a CFS quota the process cannot read: 256 CPUs
            # listed, 16 granted on the GPU box) - the live path is host-CPU work: pods + engine
            share = cpuquota.cpu_share()
            _log(f"live: cpu share {share.get('cpus')}; main run")
            live = lb.run(device=str(dev), n_pods=a.pods_per_gpu, flows=a.flows, n_acl=a.acl, duration=1.0,
                          threads=a.live_gen_threads, tx_workers=a.live_workers, queues=a.live_queues,
                          hash_mode=a.hash, gpu_egress=gde, trials=a.live_trials)
            live["gpu_egress"] = gde
            # the other egress mode for comparison (GPU-direct egress or host egress), same threads,
            # saturated rate only
            alt = dict(threads=a.live_gen_threads, tx_workers=a.live_workers, queues=a.live_queues, gpu_egress=not gde)
            _log(f"live: {live.get('mpps')} Mpps; other egress")
            hp = lb.run(device=str(dev), n_pods=a.pods_per_gpu, flows=a.flows, n_acl=a.acl, duration=0.5,
                        hash_mode=a.hash, saturated_only=True, **alt)
            live["other_egress"] = {**alt, "mpps": hp.get("mpps"), "p50_us": hp.get("p50_us"), "error": hp.get("error")}
            # the engine's queue curve: saturated pod -> pod Mpps at 1 / 2 / 4 / 6 / 8 rx queues, the
            # same pods, pipeline and delivery mode, each point with the CPUs it used: pods and
            # engine share the box's CPU grant, so past the grant more queues cannot help
            curve = []
            for q in (1, 2, 4, 6, 8):
                _log(f"live: queue curve {q}")
                r = lb.run(device=str(dev), n_pods=a.pods_per_gpu, flows=a.flows, n_acl=a.acl, duration=0.5,
                           threads=a.live_gen_threads, tx_workers=a.live_workers, queues=q, hash_mode=a.hash,
                           saturated_only=True, gpu_egress=gde)
                curve.append({"queues": q, "mpps": r.get("mpps"), "p50_us": r.get("p50_us"),
                              "cpus_used": (r.get("cpu") or {}).get("process_cpus_used"), "error": r.get("error")})
            live["queue_curve"] = curve
            # SFC hops across GPUs in the live path: the headline chain split after nat (acl, nat on
            # the plane the frame entered, l2fwd on plane 1; ring.h XferEntry), two ring planes (the
            # two GPUs when there are two, else both on this one: a rehearsal of the xGMI path)
            import torch as _t

            two = _t.cuda.device_count() > 1
            _log("live: split chain")
            sp = _live_split(a, str(dev), "cuda:0,cuda:1" if two else "")
            live["split_chain"] = {k: sp.get(k) for k in ("split", "planes", "xfer_active", "mpps", "p50_us", "idle_p50_us",
                                                          "idle_p99_us", "half_p50_us", "half_p99_us", "error")}
            if sp.get("idle_p50_us") and live.get("idle_p50_us"):
                live["split_chain"]["hop_handoff_us"] = round(sp["idle_p50_us"] - live["idle_p50_us"], 2)
            live["host_cpus"] = len(os.sched_getaffinity(0))
            live["cpu_share"] = share
            live["threads_busy"] = a.live_gen_threads + a.live_queues * (1 + a.live_workers)
        except Exception as ex:  # the headline number must still be reported
            live = {"error": str(ex)[:200]}
        # kernel-netdev (veth) pods in front of the same GPU ring (tools/live_bench.py run_veth
        # "pipeline", the deployed default vport): needs CAP_NET_ADMIN / CAP_NET_RAW, or user
        # namespaces to get them; reported as skipped (with the reason) where the box has neither
        if live is not None:
            _log("live: veth")
            live_veth = _live_veth(str(dev))
    _log("done")

    total_pkts = world * a.batch * a.steps
    mpps = total_pkts / elapsed / 1e6
    if rank == 0:
        line = {
            "metric": BASELINE_METRIC,
            "value": round(mpps, 2),
            "unit": "Mpps",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8 packets / FP4 (e2m1) MFMA ACL classify",
            "data": "synthetic (random 1M-flow table, random pod->pod 5-tuples, 64B frames)",
            "config": {
                "model": f"1M-flow SFC: acl({a.acl} TCAM rules)->snat->l2fwd, 64B frames, {a.pods_per_gpu} pods/GPU",
                "global_batch": world * a.batch,
                "seq_len": 64,
                "parallelism": "fused-1gpu" if not sharded else
                (f"rss flow-shard x{world} ({a.flows} flows/GPU, {total_flows} total), owner-local chain + egress, "
                 f"{a.remote_frac:.1%} misdirected headers -> owner: 1x all-to-all/step (RCCL/xGMI), overlapped"
                 if rss else
                 f"replicated tables x{world}, fused kernel + 1x all-to-all of cross-GPU frames (RCCL/xGMI), "
                 f"{a.chunks}-chunk overlap" if replicated else
                 f"flow-shard x{world} + 3x all-to-all (RCCL/xGMI), {a.chunks}-chunk overlap"),
                "io": a.io if not sharded else "device",
            },
            "p50_latency_us": round(p50, 2),
            "latency_origin": "4M batch: each fused-kernel workgroup's start (r6; no stamp kernel per batch); "
                              "64K batch: a stamp kernel launched before the batch (as through r5)",
            "p99_latency_us": round(p99, 2),
            "p50_latency_us_64k_batch": None if p50_small is None else round(p50_small, 2),
            "small_batch_host_rtt": rtt,
            # persistent ring kernel: 64-packet chunks, host-clock publish -> completion RTT
            "p50_latency_us_ring": None if not ring or "p50_us" not in ring else ring["p50_us"],
            "ring": ring,
            "exchange": xchg,
            "unsteered": unsteered,
            "forwarded_fraction": round(fwd_local, 6),
            "value_mixed": None if not variants else variants["mixed_mpps"],
            "value_acl1024": None if not variants else variants["acl1024_mpps"],
            "value_acl_wild": None if not variants else variants["acl_wild_mpps"],
            "value_l3": None if not variants else variants["l3_mpps"],
            "value_ipv6": None if not variants else variants["ipv6_mpps"],
            "value_vxlan": None if not variants else variants["vxlan_mpps"],
            "value_vxlan_egress": None if not variants else variants["vxlan_egress_mpps"],
            "value_p4_ipu": None if not variants else variants.get("p4_ipu_mpps"),
            "imix": None if not variants else variants["imix"],
            "variants": variants,
            # split chain over two data planes (one GPU): pipeline Mpps and per-hop latency
            "hop_pipeline": hops,
            # live pod -> pod through the native I/O engine + ring kernel (memif vports, 64-B frames)
            "live": live,
            "live_veth": live_veth,
            "p50_latency_us_pod": None if not live or "idle_p50_us" not in live else live["idle_p50_us"],
            "flows": total_flows,
            "batch_per_gpu": a.batch,
            "hash": a.hash,
            "acl_mode": a.acl_mode,
            "setup_s": round(setup_s, 1),
            "baseline_note": "reference publishes no numbers (BASELINE.md); 200GbE line rate at 64B = 297.6 Mpps",
        }
        if scale is not None:
            line["scale"] = scale   # what the N > 1 run ran on (SCALE_KEYS)
        if a.rehearse:
            line["rehearsal"] = "all ranks on cuda:0, gloo host-staged exchange: correctness only, not a measurement"
        print(json.dumps(line), flush=True)
    if sharded:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
