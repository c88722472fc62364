"""GPU tests: every HIP kernel variant must be bit-exact with the C++ oracle."""
import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    return torch


def _build(device, hash_mode="mfma", acl_mode="mfma", n_flows=1 << 14, n_acl=200, seed=0, buckets=1 << 13, **kw):
    dp = DataPlane(device=device, flow_buckets=buckets, hash_mode=hash_mode, acl_mode=acl_mode)
    sc = S.build_sfc(dp, n_pods=16, n_flows=n_flows, n_acl=n_acl, seed=seed, **kw)
    # rules that really match traffic, at random priorities before the final permit
    rng = np.random.default_rng(seed + 7)
    final = dp.acl.rules.pop()
    for _ in range(24):
        k = sc.keys[rng.integers(0, len(sc.keys))]
        m = (rng.integers(0, 2**32, 4, dtype=np.uint64) & rng.integers(0, 2**32, 4, dtype=np.uint64)).astype(np.uint32)
        dp.acl.rules.insert(int(rng.integers(0, len(dp.acl.rules) + 1)), type(final)(k & m, m, bool(rng.integers(0, 2))))
    dp.acl.rules.append(final)
    dp.acl.version += 1
    dp.commit(full=True)
    return dp, sc


def _traffic(sc, n=1 << 15, seed=3):
    pk, im = S.traffic(sc, n, seed=seed)
    im[5] = (im[5] & 0xFFFF) | (10 << 16)   # malformed
    pk[7, 15] ^= 1                           # wrong vlan
    pk[9, 11] ^= 1                           # spoofed
    return pk, im


@pytest.fixture(scope="module")
def oracle():
    cpu, sc = _build("cpu")
    pk, im = _traffic(sc)
    return cpu, sc, pk, im, cpu.run(pk, im)


@pytest.mark.parametrize("hash_mode", ["scalar", "lds", "mfma"])
@pytest.mark.parametrize("acl_mode", ["scalar", "mfma"])
def test_fused_variants_bit_exact(oracle, hash_mode, acl_mode):
    torch = _torch()
    cpu, sc, pk, im, rc = oracle
    g, _ = _build("cuda", hash_mode, acl_mode)
    r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    reasons = P.meta_fields(rc.meta)[2]
    assert (reasons == 4).sum() > 0 and (reasons == 0).sum() > len(reasons) // 2  # ACL hits exercised


def test_counters_match_oracle():
    torch = _torch()
    g, sc = _build("cuda")
    c, _ = _build("cpu")
    pk, im = _traffic(sc)
    for _ in range(3):
        g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
        c.run(pk, im)
    torch.cuda.synchronize()
    assert np.array_equal(g.port_counters(), c.port_counters())
    assert g.drop_counters() == c.drop_counters()
    g.harvest()
    c.harvest()
    assert np.array_equal(g.flow_totals, c.flow_totals)


def test_incremental_flow_updates_on_device():
    """Bucket-row pushes (bucket_update_kernel) keep HBM identical to the host table."""
    torch = _torch()
    g, sc = _build("cuda", n_flows=4000, buckets=1 << 11)
    c, _ = _build("cpu", n_flows=4000, buckets=1 << 11)
    rng = np.random.default_rng(11)
    # erase some flows, re-point others, add new ones
    for dp in (g, c):
        for i in range(0, 4000, 7):
            dp.flows.erase(sc.keys[i])
        a = sc.actions[1::5].copy()
        a[:, 0] = (a[:, 0] & 0xFFFF) | (np.uint32(sc.pod_port[0]) << 16)
        dp.flows.insert_many(sc.keys[1::5], a)
        dp.commit()
    pk, im = S.traffic(sc, 8192, seed=4)
    r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    rc = c.run(pk, im)
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(g._dev["flows"].cpu().numpy(), g.flows.t.slots().view(np.uint8).reshape(-1))


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_kernels_simulated_ranks(world):
    """All N ranks' stage kernels on one GPU, exchange emulated by copies; outcome per packet
    must equal the single-table oracle and remote packets must be delivered bit-exact."""
    torch = _torch()
    from dpu_operator_amd.parallel.sharded import ShardedDataPlane, shard_filter, simulate_step

    n_pods = 4 * world
    pod_gpu = np.arange(n_pods) // 4
    engines, batches, refs = [], [], []
    oracle_dp = DataPlane("cpu", flow_buckets=1 << 14)
    sc0 = S.build_sfc(oracle_dp, n_pods=n_pods, n_flows=20000, n_acl=64, pod_gpu=pod_gpu)
    oracle_dp.commit()
    for r in range(world):
        dp = DataPlane("cuda", flow_buckets=1 << 13)
        sc = S.build_sfc(dp, n_pods=n_pods, n_flows=20000, n_acl=64, pod_gpu=pod_gpu, flow_filter=shard_filter(r, world))
        dp.commit(full=True)
        pk, im = S.traffic(sc, 6000, seed=20 + r, src_pods=np.where(pod_gpu == r)[0])
        engines.append(ShardedDataPlane(dp, r, world, 6000))
        batches.append((torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda()))
        refs.append(oracle_dp.run(pk, im))
    simulate_step(engines, batches)
    torch.cuda.synchronize()
    delivered = set()
    for e in engines:
        rx, _ = e.received()
        delivered |= {rx[i].tobytes() for i in range(len(rx))}
    for r, (e, rc) in enumerate(zip(engines, refs)):
        meta = e.out_meta.cpu().numpy().view(np.uint32)
        rs = P.meta_fields(meta)[2]
        rrs = P.meta_fields(rc.meta)[2]
        assert ((rs == 10) | (rs == rrs)).all()
        loc = rs == 0
        assert np.array_equal(e.out.cpu().numpy()[loc], rc.out[loc])
        rem = np.where(rs == 10)[0]
        assert len(rem) > 0
        assert all(rc.out[i].tobytes() in delivered for i in rem)


def _p4_plane(device):
    """Ports programmed through the P4 compile (K2-K9) and an OvS bridge, plus SFC flows."""
    from dpu_operator_amd.dataplane.ovs import OvsSwitch
    from dpu_operator_amd.dataplane.p4rt import P4Runtime
    from dpu_operator_amd.dataplane.p4server import InProcessP4rtClient, Rule, program_rules
    from dpu_operator_amd.vsp import intel_ipu as ipu

    dp, sc = _build(device, n_flows=1 << 12)
    rt = P4Runtime(dp, lag_ports={0: 4093})
    c = InProcessP4rtClient({"br0": rt})
    vfs = [f"00:{0x40 + i:02x}:00:00:00:01" for i in range(6)]
    accs = [f"00:{0x60 + i:02x}:00:00:00:02" for i in range(6)]
    rules = []
    for v, a in zip(vfs, accs):
        rules += ipu.host_vf_rules(v, a)
    rules += ipu.peer_to_peer_rules(vfs)
    rules += [Rule("add-entry", "br0", "linux_networking_control.tx_lag_table",
                   f"user_meta.cmeta.lag_group_id=0/255,hash={h}/7,priority=1,"
                   f"action=linux_networking_control.set_egress_port(0,{h % 3})") for h in range(8)]
    rules += [Rule("add-entry", "br0", "linux_networking_control.tx_acc_vsi",
                   "vmeta.common.vsi=101,zero_padding=0,action=linux_networking_control.l2_fwd_and_bypass_bridge(4093)")]
    rules += ipu.primary_network_rules("00:70:00:00:00:04", "00:71:00:00:00:01")
    rules += ipu.vf_vlan_rules("00:72:00:00:00:01", 9, port_mux_vsi=115)
    assert program_rules(c, rules) == []
    br = OvsSwitch(dp).add_br("br-gpu")
    for i, n in enumerate(("a", "b", "nin", "nout")):
        br.add_port(n, 3000 + i, mac=f"02:cc:00:00:00:{i:02x}")
    br.add_flow("priority=10,in_port=a,actions=output:nin")
    br.add_flow("priority=100,in_port=nout,dl_dst=02:cc:00:00:00:00,actions=in_port")
    dp.commit(full=True)
    return dp, sc, vfs


def _p4_traffic(sc, vfs, n=1 << 14, seed=11):
    rng = np.random.default_rng(seed)
    pk, im = S.traffic(sc, n, seed=seed)
    src_ports = np.array([0x40 + 16 + i for i in range(6)] + [101 + 16, 4000, 0x72 + 16, 115 + 16, 3000, 3003])
    dst_macs = [bytes.fromhex(m.replace(":", "")) for m in vfs] + [bytes.fromhex("007100000001"),
                                                                   bytes.fromhex("02cc00000000"), bytes(6)]
    sel = rng.integers(0, len(src_ports), n)
    dm = rng.integers(0, len(dst_macs), n)
    for i in range(0, n, 2):  # half of the batch exercises the P4/OvS ports
        pk[i, 0:6] = np.frombuffer(dst_macs[dm[i]], np.uint8)
        im[i] = (im[i] & 0xFFFF0000) | src_ports[sel[i]]
    return pk, im


def test_p4_ovs_features_bit_exact():
    """LAG (hash-selected member), mirror flag, VSI-keyed loopback, ingress VLAN push, OvS
    hairpin: the GPU kernel must agree with the oracle bit for bit."""
    torch = _torch()
    cpu, sc, vfs = _p4_plane("cpu")
    gpu, _, _ = _p4_plane("cuda")
    pk, im = _p4_traffic(sc, vfs)
    rc = cpu.run(pk, im)
    rg = gpu.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    mg = rg.meta.cpu().numpy().view(np.uint32)
    assert np.array_equal(mg, rc.meta)
    assert np.array_equal(rg.out.cpu().numpy(), rc.out)
    op = P.meta_fields(rc.meta)[0]
    # K9: real mirror copies (side pass), same set on both
    sc_, sg = cpu.side_result(), gpu.side_result()
    assert sc_["n_rep"] > 0
    key = lambda r: sorted(zip(r["rep_src"].tolist(), r["rep_meta"].tolist(), map(bytes, r["rep_hdr"])))
    assert key(sc_) == key(sg)
    assert len({4000, 4001, 4002} & set(op.tolist())) == 3   # LAG spread over three members


def _replicated_engines(device, world=4, batch=1 << 14):
    from dpu_operator_amd.parallel.replicated import ReplicatedDataPlane

    n_pods = 4 * world
    pod_gpu = np.arange(n_pods) // 4
    engines, batches = [], []
    for r in range(world):
        dp = DataPlane(device=device, flow_buckets=1 << 13, hash_mode="lds", acl_mode="mfma")
        sc = S.build_sfc(dp, n_pods=n_pods, n_flows=1 << 14, n_acl=64, pod_gpu=pod_gpu, seed=5)
        dp.commit(full=True)
        pk, im = S.traffic(sc, batch, seed=50 + r, src_pods=np.where(pod_gpu == r)[0])
        engines.append(ReplicatedDataPlane(dp, r, world, batch, chunks=1, record_rx=True))
        batches.append((pk, im))
    return engines, batches


def test_replicated_remote_kernel_matches_cpu_twin():
    """Fused REMOTE kernel (replicated tables, per-GPU egress segments) vs its CPU twin, 4 ranks
    simulated on one GPU: same per-packet verdicts, same local frames, the same set of frames
    delivered to every rank, same counters."""
    torch = _torch()
    from dpu_operator_amd.parallel.replicated import simulate_replicated_step

    ge, gb = _replicated_engines("cuda")
    ce, cb = _replicated_engines("cpu")
    simulate_replicated_step(ge, [(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
                                  for pk, im in gb])
    simulate_replicated_step(ce, [(torch.from_numpy(pk), torch.from_numpy(im.view(np.int32))) for pk, im in cb])
    torch.cuda.synchronize()
    n_remote = 0
    for g, c in zip(ge, ce):
        mg, mc = g.out_meta(), c.out_meta()
        assert np.array_equal(mg, mc)
        local = P.meta_fields(mc)[2] == 0
        assert np.array_equal(g.outputs()[local], c.outputs()[local])
        rg, rmg = g.received()
        rc, rmc = c.received()
        n_remote += len(rc)
        key = lambda a, m: sorted(x.tobytes() + int(y).to_bytes(4, "little") for x, y in zip(a, m))
        assert key(rg, rmg) == key(rc, rmc)
        assert np.array_equal(g.dp.port_counters(), c.dp.port_counters())
        assert g.dp.drop_counters() == c.dp.drop_counters()
    assert n_remote > (1 << 14)  # 3/4 of the traffic crossed "GPUs"


def test_snapshot_restore_cpu_to_gpu(tmp_path):
    """A CPU-side checkpoint restores onto the GPU tables and forwards bit-identically."""
    from dpu_operator_amd.dataplane import snapshot

    torch = _torch()
    c, sc = _build("cpu", n_flows=3000, buckets=1 << 11)
    path = str(tmp_path / "dp.npz")
    snapshot.save(c, path)
    g = DataPlane(device="cuda", flow_buckets=1 << 11, hash_mode="mfma", acl_mode="mfma")
    snapshot.load(g, path)
    pk, im = S.traffic(sc, 8192, seed=9)
    r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    rc = c.run(pk, im)
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)


def test_host_path_pipeline_matches_oracle():
    """Pinned host slots -> SDMA -> fused kernel -> SDMA: three batches in flight, bit-exact."""
    from dpu_operator_amd.dataplane.pktio import HostPath

    _torch()
    g, sc = _build("cuda", n_flows=4000, buckets=1 << 11)
    c, _ = _build("cpu", n_flows=4000, buckets=1 << 11)
    hp = HostPath(g, capacity=8192, depth=3)
    batches = [S.traffic(sc, 8192 - 1000 * k, seed=20 + k) for k in range(3)]
    for s, (pk, im) in enumerate(batches):
        hp.load(s, pk, im)
        hp.submit(s, len(pk))
    for s, (pk, im) in enumerate(batches):
        out, meta = hp.results(s)
        rc = c.run(pk, im)
        assert np.array_equal(meta, rc.meta) and np.array_equal(out, rc.out)
    t = hp.timings_ms(0)
    assert t["total"] >= t["kernel"] > 0


@pytest.mark.parametrize("mode,n", [("rss", 2), ("rss", 4), ("replicated", 2)])
def test_bench_multirank_rehearsal_on_one_gpu(mode, n):
    """The N-GPU bench path end to end (torchrun, one process per rank; rss: flow-shard tables,
    owner-steering REMOTE kernel, exchange, gather + fused kernel on what arrived; replicated:
    fused REMOTE kernel, exchange, egress kernel; stats collectives) with the ranks sharing cuda:0
    over gloo (RCCL refuses two ranks on one device).  Every packet must be forwarded."""
    import json
    import os
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(n), "--steps", "2",
           "--warmup", "1", "--batch", str(1 << 16), "--flows", str(1 << 16), "--rehearse", "--mode", mode,
           "--remote-frac", "0.05", "--no-variants"]
    r = subprocess.run(cmd, cwd=repo, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, "\n".join(ln for ln in r.stderr.splitlines() if ln.startswith("[rank0]"))[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == n and line["forwarded_fraction"] == 1.0
    assert line["config"]["global_batch"] == n << 16
    assert line["exchange"]["a2a_per_step"] >= 1 and line["exchange"]["xgmi_bytes_out_per_gpu_per_step"] > 0
    if mode == "rss":   # the exchange-bound variant: (N-1)/N of every batch to its owner, all forwarded
        import bench

        u = line["unsteered"]
        assert set(u) == set(bench.RSS_UNSTEERED_KEYS) and u["remote_frac"] == round((n - 1) / n, 4)
        assert u["sent_per_gpu_per_step"] > 0 and u["forwarded_fraction"] == 1.0


@pytest.mark.gpu
def test_batch_larger_than_one_launch():
    """A batch of 2^24 + 64K packets (1.1 GB of header slots): DataPlane.run splits it into
    launches of <= 2^24 slots (32-bit buffer views); every slot and every counter matches the
    oracle."""
    import torch

    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane

    g = DataPlane(device="cuda", flow_buckets=1 << 12)
    c = DataPlane(device="cpu", flow_buckets=1 << 12)
    for dp in (g, c):
        sc = S.build_sfc(dp, n_pods=8, n_flows=4096, n_acl=64, seed=0)
        dp.commit(full=True)
    pk1, im1 = S.traffic(sc, 1 << 20, seed=3)
    n = (1 << 24) + (1 << 16)
    reps = n // len(pk1) + 1
    pk = np.tile(pk1, (reps, 1))[:n]
    im = np.tile(im1, reps)[:n]
    assert g.MAX_LAUNCH < n
    r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    rc = c.run(pk, im)
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert np.array_equal(g.port_counters(), c.port_counters())


@pytest.mark.gpu
def test_graphed_run_matches_oracle_and_recaptures_after_commit():
    """DataPlane.capture(n): the fused (+ side + learn) launches of a batch replayed as one
    HIP graph.  Replays over new inputs match the oracle; a commit that reallocates a table makes
    the next call re-capture (the graph holds device addresses)."""
    import torch

    from dpu_operator_amd.dataplane import scenario as S
    from dpu_operator_amd.dataplane.engine import DataPlane

    g = DataPlane(device="cuda", flow_buckets=1 << 12)
    c = DataPlane(device="cpu", flow_buckets=1 << 12)
    for dp in (g, c):
        sc = S.build_sfc(dp, n_pods=8, n_flows=4096, n_acl=64, seed=0)
        dp.commit(full=True)
    gr = g.capture(4096)
    for seed in (1, 2):
        pk, im = S.traffic(sc, 4096, seed=seed)
        r = gr(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
        torch.cuda.synchronize()
        rc = c.run(pk, im)
        assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
        assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert gr.captures == 1
    for dp in (g, c):                      # a new ACL rule (before the final permit): buffers reallocated
        final = dp.acl.rules.pop()
        dp.acl.add(permit=False, dst="10.128.0.3/32")
        dp.acl.rules.append(final)
        dp.acl.version += 1
        dp.commit()
    pk, im = S.traffic(sc, 4096, seed=3)
    r = gr(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    rc = c.run(pk, im)
    assert gr.captures == 2
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert (P.meta_fields(rc.meta)[2] == 4).any()     # the new deny rule fired


@pytest.mark.gpu
@pytest.mark.parametrize("world,frac", [(2, 0.3), (4, 0.75)])
def test_rss_steer_list_matches_cpu_twin(world, frac):
    """Flow-owner steering by list (the 1-GPU kernel's LIST instance + steer_kernel) against the
    CPU twin of REMOTE steering: every meta equal, every locally processed slot equal, and each
    owner's segment holds the same (slot, ingress meta) multiset - count-first, nothing dropped."""
    import torch

    from dpu_operator_amd.parallel.rss import RssShardedDataPlane, flow_owner, rss_traffic
    from dpu_operator_amd.parallel.sharded import shard_filter

    engs = {}
    for dev in ("cuda", "cpu"):
        dp = DataPlane(device=dev, flow_buckets=1 << 13, hash_mode="lds")
        sc = S.build_sfc(dp, n_pods=8, n_flows=20000, n_acl=64, flow_filter=shard_filter(0, world))
        dp.commit(full=True)
        owner = flow_owner(sc.keys, world, dp.flows.rss_key)
        pk, im = rss_traffic(sc, 8192, 0, world, owner, frac, seed=7)
        eng = RssShardedDataPlane(dp, 0, world, 8192, remote_frac=frac)
        tpk, tim = torch.from_numpy(pk), torch.from_numpy(im.view(np.int32))
        if dev == "cuda":
            tpk, tim = tpk.cuda(), tim.cuda()
        s = eng.slots[0]
        eng._local(s, tpk, tim, len(pk))
        if dev == "cuda":
            torch.cuda.synchronize()
        engs[dev] = (eng, s)
    (g, gs), (c, cs) = engs["cuda"], engs["cpu"]
    assert g.use_list
    mg, mc = g.out_meta_t.cpu().numpy().view(np.uint32), c.out_meta_t.numpy().view(np.uint32)
    assert np.array_equal(mg, mc)
    loc = P.meta_fields(mc)[2] != 10
    assert np.array_equal(g.out.cpu().numpy()[loc], c.out.numpy()[loc])
    assert "overflow" not in g.dp.drop_counters()
    cg, cc = gs.pcnt.cpu().numpy(), cs.pcnt.numpy()
    assert np.array_equal(cg, cc) and cg.sum() == (~loc).sum() > 0
    for j in range(1, world):
        def seg(eng, sl):
            buf = sl.send.cpu().numpy()
            n = int(sl.pcnt.cpu().numpy()[j])
            b = j * eng.pseg
            slots = buf[b + 64: b + 64 + 64 * n].reshape(n, 64)
            metas = buf[b + eng.moff: b + eng.moff + 4 * n].view(np.uint32)
            return sorted(zip(map(bytes, slots), metas.tolist()))
        assert seg(g, gs) == seg(c, cs)


@pytest.mark.parametrize("hash_mode,acl_mode", [("lds", "mfma"), ("mfma", "mfma"), ("lds", "scalar")])
def test_acl_wild_bit_exact(hash_mode, acl_mode):
    """ClassBench-style 1024-rule ACL (> 3000 ternary entries: tiles beyond the LDS-staged 64,
    the early-fetch instance) is bit-exact with the oracle, which is itself checked against an
    independent first-match model (test_dataplane_oracle.py)."""
    torch = _torch()
    res = {}
    for dev in ("cuda", "cpu"):
        dp, sc = _build(dev, hash_mode if dev == "cuda" else "mfma", acl_mode if dev == "cuda" else "mfma")
        S.install_acl_wild(dp, 1024)
        dp.commit()
        pk, im = _traffic(sc)
        if dev == "cuda":
            r = dp.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
            torch.cuda.synchronize()
            res[dev] = (r.meta.cpu().numpy().view(np.uint32), r.out.cpu().numpy())
            assert dp._acl_tiles > 64
        else:
            r = dp.run(pk, im)
            res[dev] = (r.meta, r.out)
    assert np.array_equal(res["cuda"][0], res["cpu"][0])
    assert np.array_equal(res["cuda"][1], res["cpu"][1])
