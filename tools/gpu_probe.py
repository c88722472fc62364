"""First-contact GPU probe: correctness of every kernel variant vs the C++ oracle + quick timing.

Run on the GPU box:  python tools/gpu_probe.py
"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.ops import packets as P  # noqa: E402


def build(device, n_flows, n_acl, hash_mode="mfma", acl_mode="mfma", buckets=None, seed=0):
    buckets = buckets or max(1 << 10, 1 << int(np.ceil(np.log2(n_flows / 4))))
    dp = DataPlane(device=device, flow_buckets=buckets, hash_mode=hash_mode, acl_mode=acl_mode)
    sc = S.build_sfc(dp, n_pods=16, n_flows=n_flows, n_acl=n_acl, seed=seed)
    # extra ACL rules that DO match some traffic, at random priorities (inserted before the
    # final permit): value = a real flow key, random ternary mask
    rng = np.random.default_rng(seed + 7)
    rules = dp.acl.rules
    final = rules.pop()
    for _ in range(min(32, 1023 - len(rules))):
        k = sc.keys[rng.integers(0, len(sc.keys))]
        m = rng.integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32) & rng.integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32)
        m[3] &= np.uint32(0xFFFF00FF)
        pos = int(rng.integers(0, len(rules) + 1))
        dp.acl.rules.insert(pos, type(final)(k & m, m, bool(rng.integers(0, 2))))
    rules.append(final)
    dp.acl.version += 1
    dp.commit(full=True)
    return dp, sc


def main():
    dev = "cuda"
    props = torch.cuda.get_device_properties(0)
    print("device", props.name, getattr(props, "gcnArchName", "?"), "CUs", props.multi_processor_count, flush=True)
    n_flows, n_acl, n = 1 << 16, 200, 1 << 17
    cpu, sc = build("cpu", n_flows, n_acl)
    pk, im = S.traffic(sc, n, seed=3)
    # some malformed / wrong-vlan / spoofed packets
    im[5] = (im[5] & 0xFFFF) | (10 << 16)
    pk[7, 15] ^= 0x1
    pk[9, 11] ^= 0x1
    rc = cpu.run(pk, im)
    _, _, rs = P.meta_fields(rc.meta)
    print("oracle reasons", dict(zip(*np.unique(rs, return_counts=True))), "acl hits",
          np.bincount(np.clip(rc.extra["acl"], -1, 2000) + 1)[:1], flush=True)
    ok_all = True
    for hm in ("scalar", "lds", "mfma"):
        for am in ("scalar", "mfma", "off"):
            g, _ = build(dev, n_flows, n_acl, hm, am)
            tp = torch.from_numpy(pk).to(dev)
            ti = torch.from_numpy(im.view(np.int32)).to(dev)
            r = g.run(tp, ti)
            torch.cuda.synchronize()
            out = r.out.cpu().numpy()
            meta = r.meta.cpu().numpy().view(np.uint32)
            if am == "off":
                # ACL off: compare only packets whose oracle ACL rule was default/permit path
                same = (meta == rc.meta) & np.all(out == rc.out, axis=1)
                print(f"hash={hm:6s} acl={am:6s} agree={same.mean():.4f} (acl off; mismatches expected on acl_deny)", flush=True)
                continue
            bad = np.where((meta != rc.meta) | np.any(out != rc.out, axis=1))[0]
            pc_ok = np.array_equal(g.port_counters(), cpu.port_counters() if False else g.port_counters())
            print(f"hash={hm:6s} acl={am:6s} mismatches={len(bad)}", flush=True)
            if len(bad):
                ok_all = False
                i = bad[0]
                print("  first", i, hex(meta[i]), hex(rc.meta[i]), "acl", rc.extra["acl"][i])
    # counters: compare GPU (mfma/mfma) vs oracle
    g, _ = build(dev, n_flows, n_acl)
    cpu2, _ = build("cpu", n_flows, n_acl)
    tp = torch.from_numpy(pk).to(dev)
    ti = torch.from_numpy(im.view(np.int32)).to(dev)
    g.run(tp, ti)
    cpu2.run(pk, im)
    torch.cuda.synchronize()
    pcg, pcc = g.port_counters(), cpu2.port_counters()
    print("port counters equal:", np.array_equal(pcg, pcc), "drops", g.drop_counters(), cpu2.drop_counters(), flush=True)
    g.harvest(); cpu2.harvest()
    print("flow counters equal:", np.array_equal(g.flow_totals, cpu2.flow_totals), flush=True)
    print("ALL_OK" if ok_all else "MISMATCH", flush=True)

    # ---- timing at scale: 1M flows, 4M-packet batch ----
    for (hm, am, nacl) in (("mfma", "mfma", 256), ("lds", "mfma", 256), ("lds", "scalar", 256), ("lds", "off", 0),
                           ("mfma", "mfma", 1024), ("lds", "scalar", 1024), ("mfma", "off", 0)):
        t0 = time.time()
        g = DataPlane(device=dev, flow_buckets=1 << 19, hash_mode=hm, acl_mode=am)
        sc = S.build_sfc(g, n_pods=16, n_flows=1 << 20, n_acl=nacl, seed=1)
        g.commit(full=True)
        nb = 1 << 22
        pk, im = S.traffic(sc, nb, seed=5)
        tp = torch.from_numpy(pk).to(dev)
        ti = torch.from_numpy(im.view(np.int32)).to(dev)
        out, meta, lat = g.alloc_batch(nb)
        for _ in range(3):
            g.run(tp, ti, out, meta, lat)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        iters = 20
        ev0.record()
        for _ in range(iters):
            g.run(tp, ti, out, meta, lat)
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / iters
        _, _, rs = P.meta_fields(meta.cpu().numpy().view(np.uint32))
        l = lat.cpu().numpy().astype(np.float64) * 10.0 / 1000.0
        print(f"[time] hash={hm} acl={am} R={nacl}: {ms:.3f} ms / {nb} pkts = {nb / ms / 1e3:.1f} Mpps; "
              f"fwd={np.mean(rs == 0):.4f} p50 lat={np.median(l):.1f}us setup={time.time() - t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
