"""Variable-length frames and L2 side outputs.

* Frames of any length up to 9600 B: the data plane reads and writes a 64-B header slot; the
  payload stays in place and the frame that leaves is ohdr[:hl] ++ in_frame[to:len]
  (nfdp.h out_tail).  Checked independently of the C++ oracle: the assembled egress frames are
  recomputed field by field in numpy and their IPv4 / UDP checksums verified over the WHOLE
  frame (SNAT's RFC 1624 incremental updates must hold for 9000-B payloads).
* Port MTU -> too_big, oversized length -> malformed.
* OvS NORMAL semantics on a bridge: broadcast / unknown-unicast flooding with per-member egress
  tagging (replicas), MAC learning (learn events + the lock-free learn kernel), ARP copies to the
  slow path (P4 always_trap_arp_table), K9 mirror copies.
The GPU tests compare the HIP kernels against the oracle bit for bit (replicas as sets: the GPU
appends them with atomics).
"""
import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P


def _torch():
    import torch

    return torch


def _sfc(device, **kw):
    dp = DataPlane(device=device, flow_buckets=1 << 12, **kw)
    sc = S.build_sfc(dp, n_pods=8, n_flows=4096, n_acl=32, seed=0)
    dp.commit(full=True)
    return dp, sc


def _imix(sc, n=1024, seed=5):
    sizes = S.imix_sizes(n, S.IMIX_JUMBO, seed)
    return S.traffic_frames(sc, n, sizes, seed=seed)


def _untag(fr: bytes) -> bytes:
    return fr[:12] + fr[16:] if fr[12:14] == b"\x81\x00" else fr


def _check_sfc_egress(sc, frames, lens, out, meta):
    """Independent model of acl -> snat -> l2fwd on whole frames."""
    port, olen, reason = P.meta_fields(meta)
    assert (reason == 0).all(), np.unique(reason, return_counts=True)
    idx = {tuple(sc.keys[i]): i for i in range(len(sc.keys))}
    by_len: dict[int, list] = {}
    for i in range(len(meta)):
        o = P.assemble(out[i], int(meta[i]), frames[i], int(lens[i]))
        assert len(o) == int(lens[i])  # tag popped at ingress, pushed at egress
        fin = bytes(frames[i, : lens[i]])
        key = T.flow_key(int.from_bytes(fin[30:34], "big"), int.from_bytes(fin[34:38], "big"),
                         int.from_bytes(fin[38:40], "big"), int.from_bytes(fin[40:42], "big"), 17, sc.bridge)[0]
        f = idx[tuple(key)]
        d = int(sc.flow_dst_pod[f])
        assert int(port[i]) == int(sc.pod_port[d])
        assert o[0:6] == S.pod_mac(d) and o[6:12] == S.pod_mac(d)           # l2fwd MAC rewrite
        assert o[12:14] == b"\x81\x00" and (int.from_bytes(o[14:16], "big") & 0xFFF) == d % 4094 + 2
        act = sc.actions[f]
        u = _untag(o)
        assert u[26:30] == int(act[1]).to_bytes(4, "little")                   # SNAT address (raw LE word)
        assert u[34:36] == (int(act[2]) & 0xFFFF).to_bytes(2, "little")        # SNAT port
        assert u[42:] == _untag(fin)[42:]                                       # payload untouched
        by_len.setdefault(len(u), []).append(np.frombuffer(u, np.uint8))
    for L, rows in by_len.items():
        a = np.stack(rows)
        assert P.check_csums(a, np.full(len(a), L)).all(), f"bad checksum at length {L}"


def test_imix_frames_oracle_model():
    dp, sc = _sfc("cpu")
    slots, im, frames, lens = _imix(sc)
    assert set(np.unique(lens)) == {64, 576, 1500, 9000}
    r = dp.run(slots, im)
    _check_sfc_egress(sc, frames, lens, r.out, r.meta)
    pc = dp.port_counters()
    assert int(pc[:, 1].sum()) == int(lens.sum()) and int(pc[:, 3].sum()) == int(lens.sum())


def test_mtu_and_oversize():
    dp, sc = _sfc("cpu")
    slots, im, frames, lens = _imix(sc)
    for p in sc.pod_port:
        dp.ports.set_mtu(int(p), 1500)
    dp.commit()
    r = dp.run(slots, im)
    _, _, rs = P.meta_fields(r.meta)
    assert (rs[lens == 9000] == 6).all()            # too_big: L3 8982 > 1500
    assert (rs[lens != 9000] == 0).all()            # 1500-B (L3 1482) fits
    im2 = im.copy()
    im2[:4] = (im2[:4] & 0xFFFF) | (9601 << 16)
    assert (P.meta_fields(dp.run(slots, im2).meta)[2][:4] == 9).all()  # malformed


A, B, C = "02:00:00:00:0a:01", "02:00:00:00:0b:01", "02:00:00:00:0c:01"
BR = 5


def _bridge(device):
    """4 ports on bridge 5, OvS NORMAL style: learning, ARP copies to the slow path, flooding.
    Port 3 tags its egress with vid 7; port 2 mirrors what it sends to port 3."""
    dp = DataPlane(device=device, flow_buckets=1 << 10, mac_slots=1 << 10)
    for p in range(4):
        fl = T.PORT_VALID | T.PORT_LEARN | T.PORT_ARP_TRAP | (T.PORT_TAG_EGRESS if p == 3 else 0)
        dp.ports.set(p, flags=fl, vlan=7 if p == 3 else 0, bridge_id=BR)
    dp.flood.set_members(BR, [0, 1, 2, 3])
    dp.ports.set_mirror(2, 3)
    dp.commit(full=True)
    return dp


def _l2_trace():
    arp, al = P.craft_arp(1, smac=A, sender_ip=0x0A000001, target_ip=0x0A000002)           # from port 0
    uni, ul = P.craft(1, dmac=A, smac=B, src_ip=0x0A000002, dst_ip=0x0A000001, sport=1, dport=2)  # port 2 -> A
    unk, kl = P.craft(1, dmac="02:00:00:00:0f:0f", smac=C, src_ip=0x0A000003, dst_ip=0x0A000009,
                      sport=3, dport=4)                                                   # port 1, unknown dst
    return [(arp, al, 0), (uni, ul, 2), (unk, kl, 1)]


def _run_l2(dp, to_dev=None):
    res = []
    for fr, ln, port in _l2_trace():
        slots = P.header_slots(fr, ln)
        im = P.inmeta(np.array([port]), ln)
        if to_dev:
            torch = _torch()
            r = dp.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
            torch.cuda.synchronize()
            out, meta = r.out.cpu().numpy(), r.meta.cpu().numpy().view(np.uint32)
        else:
            r = dp.run(slots, im)
            out, meta = r.out, r.meta
        res.append((out.copy(), meta.copy(), dp.side_result()))
    return res


def _reps(sr):
    return sorted((int(s), int(m), bytes(h)) for s, m, h in zip(sr["rep_src"], sr["rep_meta"], sr["rep_hdr"]))


def test_flood_learn_arp_mirror_oracle():
    dp = _bridge("cpu")
    (o1, m1, s1), (o2, m2, s2), (o3, m3, s3) = _run_l2(dp)
    # 1. broadcast ARP from port 0: carried to port 1, replicas to 2 and 3 (tagged), ARP copy punted
    p1, l1, r1 = P.meta_fields(m1)
    assert (int(p1[0]), int(r1[0]), int(l1[0])) == (1, 0, 60)
    reps = {(int(pp), int(rr), int(ll)) for pp, ll, rr in zip(*P.meta_fields(s1["rep_meta"]))}
    assert reps == {(2, 0, 60), (3, 0, 64), (T.PORT_PUNT, 12, 60)}
    tagged = [h for h, m in zip(s1["rep_hdr"], s1["rep_meta"]) if P.meta_fields(np.array([m]))[0][0] == 3][0]
    assert bytes(tagged[12:16]) == b"\x81\x00\x00\x07" and bytes(tagged[16:18]) == b"\x08\x06"
    assert s1["n_learn"] == 1 and dp.drop_counters().get("arp_trap") == 1
    # the data plane learned A -> port 0 (lock-free learn kernel / its CPU twin)
    dp.pull_learned()
    assert (BR, A, 0) in dp.macs.learned()
    # 2. unicast to A from port 2: straight to port 0, plus the K9 mirror copy to port 3 (tagged)
    p2, _, r2 = P.meta_fields(m2)
    assert (int(p2[0]), int(r2[0])) == (0, 0)
    assert {int(x) for x in P.meta_fields(s2["rep_meta"])[0]} == {3}
    # 3. unknown unicast from port 1: flooded to 0 (carried), 2 and 3 (replicas)
    p3, _, r3 = P.meta_fields(m3)
    assert (int(p3[0]), int(r3[0])) == (0, 0)
    assert sorted(int(x) for x in P.meta_fields(s3["rep_meta"])[0]) == [2, 3]
    assert {(b, m) for b, m, _ in dp.macs.learned()} >= {(BR, A), (BR, B), (BR, C)}


def _big_bridge(device, n=64):
    """n ports on one bridge, more than one 16-entry flood row: the group is a chain of rows."""
    dp = DataPlane(device=device, flow_buckets=1 << 10, mac_slots=1 << 10)
    for p in range(n):
        dp.ports.set(p, flags=T.PORT_VALID | T.PORT_LEARN | T.PORT_ARP_TRAP, bridge_id=BR)
    dp.flood.set_members(BR, list(range(n)))
    dp.commit(full=True)
    return dp


def _broadcast_from(dp, port, to_dev=False):
    arp, al = P.craft_arp(1, smac=A, sender_ip=0x0A000001, target_ip=0x0A000002)
    slots, im = P.header_slots(arp, al), P.inmeta(np.array([port]), al)
    if to_dev:
        torch = _torch()
        r = dp.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
        torch.cuda.synchronize()
        return r.out.cpu().numpy(), r.meta.cpu().numpy().view(np.uint32), dp.side_result()
    r = dp.run(slots, im)
    return r.out, r.meta, dp.side_result()


def test_flood_groups_beyond_one_row_oracle():
    """64 VFs on one bridge: a broadcast ARP reaches all 63 peers (primary copy + 62 replicas),
    plus the ARP slow-path copy; membership changes recycle the overflow rows."""
    dp = _big_bridge("cpu")
    assert dp.flood.members(BR) == list(range(64)) and len(dp.flood.a) > 4096
    for src in (0, 17, 63):
        _, m, sr = _broadcast_from(dp, src)
        p0, _, r0 = P.meta_fields(m)
        got = [int(p0[0])] + [int(x) for x, rr in zip(*P.meta_fields(sr["rep_meta"])[::2]) if rr == 0]
        assert int(r0[0]) == 0 and sorted(got) == [q for q in range(64) if q != src]
        assert (P.meta_fields(sr["rep_meta"])[2] == 12).sum() == 1       # one ARP copy punted
    rows = len(dp.flood._free)
    dp.flood.set_members(BR, list(range(40)))
    dp.flood.set_members(BR, list(range(64)))
    assert len(dp.flood._free) == rows                                   # rows reused, not leaked
    dp.flood.remove_member(BR, 5)
    assert 5 not in dp.flood.members(BR) and len(dp.flood.members(BR)) == 63


def test_mac_aging():
    dp = _bridge("cpu")
    _run_l2(dp)
    dp.pull_learned()
    assert len(dp.macs.learned()) == 3
    for _ in range(5):
        dp.run(np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32))
    assert dp.age_macs(max_age=3) == 3 and dp.macs.learned() == []


def test_station_move_relearns():
    dp = _bridge("cpu")
    _run_l2(dp)
    fr, ln = P.craft(1, dmac=B, smac=A, src_ip=1, dst_ip=2, sport=1, dport=2)
    dp.run(P.header_slots(fr, ln), P.inmeta(np.array([3]), ln))   # A moved to port 3
    dp.pull_learned()
    assert (BR, A, 3) in dp.macs.learned()


@pytest.mark.gpu
def test_imix_frames_gpu_bit_exact():
    torch = _torch()
    cpu, sc = _sfc("cpu")
    g, _ = _sfc("cuda", hash_mode="lds")
    slots, im, frames, lens = _imix(sc, n=4096)
    rc = cpu.run(slots, im)
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    _check_sfc_egress(sc, frames, lens, r.out.cpu().numpy(), r.meta.cpu().numpy().view(np.uint32))
    assert np.array_equal(g.port_counters(), cpu.port_counters())


def _port_states(dp, sc):
    """Agent-driven port states (cpagent.PortStateSync): pod 0 link down, pod 1 RX off, pod 2 MTU 576."""
    pods = [int(p) for p in sc.pod_port]
    dp.ports.set_link(pods[0], False)
    dp.ports.set_rx(pods[1], False)
    dp.ports.set_mtu(pods[2], 576)
    dp.commit()
    return pods


def test_port_states_oracle():
    dp, sc = _sfc("cpu")
    pods = _port_states(dp, sc)
    slots, im, frames, lens = _imix(sc)
    r = dp.run(slots, im)
    port, _, rs = P.meta_fields(r.meta)
    inp = im & 0xFFFF
    assert (rs[inp == pods[0]] == 1).all()                          # bad_port: a down link sends nothing
    assert (rs[inp == pods[1]] == 0).any()                          # RX off still transmits
    fwd = rs == 0
    assert not np.isin(port[fwd], pods[:2]).any()                   # nothing delivered to either
    to2 = (port == pods[2]) & fwd
    assert to2.any() and (lens[to2] - 14 <= 576).all()


@pytest.mark.gpu
def test_port_states_gpu_bit_exact():
    torch = _torch()
    cpu, sc = _sfc("cpu")
    g, _ = _sfc("cuda")
    _port_states(cpu, sc)
    _port_states(g, sc)
    slots, im, _, _ = _imix(sc, n=4096)
    rc = cpu.run(slots, im)
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(r.meta.cpu().numpy().view(np.uint32), rc.meta)
    assert np.array_equal(r.out.cpu().numpy(), rc.out)
    assert cpu.drop_counters() == g.drop_counters()


@pytest.mark.gpu
def test_flood_learn_arp_mirror_gpu_bit_exact():
    cpu, gpu = _bridge("cpu"), _bridge("cuda")
    rc, rg = _run_l2(cpu), _run_l2(gpu, to_dev=True)
    for (oc, mc, sc_), (og, mg, sg) in zip(rc, rg):
        assert np.array_equal(mc, mg) and np.array_equal(oc, og)
        assert _reps(sc_) == _reps(sg) and sc_["n_learn"] == sg["n_learn"]
    cpu.pull_learned()
    gpu.pull_learned()
    assert sorted(cpu.macs.learned()) == sorted(gpu.macs.learned())
    assert np.array_equal(cpu.port_counters(), gpu.port_counters())
    assert cpu.drop_counters() == gpu.drop_counters()


@pytest.mark.gpu
def test_flood_groups_beyond_one_row_gpu_bit_exact():
    cpu, gpu = _big_bridge("cpu"), _big_bridge("cuda")
    for src in (0, 40):
        oc, mc, sc_ = _broadcast_from(cpu, src)
        og, mg, sg = _broadcast_from(gpu, src, to_dev=True)
        assert np.array_equal(mc, mg) and np.array_equal(oc, og)
        assert _reps(sc_) == _reps(sg) and sg["n_rep"] == 63          # 62 replicas + the ARP copy


@pytest.mark.gpu
def test_learn_kernel_concurrent_inserts():
    """Thousands of learn events (many duplicates, colliding probe chains) applied by the
    lock-free GPU learn kernel end in the same key -> port map as the sequential twin."""
    torch = _torch()
    rng = np.random.default_rng(3)
    n, slots = 6000, 1 << 13
    macs = rng.integers(0, 1500, n)  # ~1500 distinct stations, each seen ~4 times
    ev = np.zeros((n, 4), np.uint32)
    ev[:, 0] = (macs.astype(np.uint32) << 8) | 0x02
    ev[:, 1] = 0x1234 | (9 << 16)
    ev[:, 2] = (macs % 50).astype(np.uint32)
    nf = DataPlane(device="cpu").nf
    host = np.zeros(slots, T.MAC_DTYPE)
    assert nf.mac_learn_cpu(host.ctypes.data, slots - 1, ev.ctypes.data, n, 1) == 0
    dev = torch.zeros(slots * 16, dtype=torch.uint8, device="cuda")
    evd = torch.from_numpy(ev.view(np.uint8).reshape(-1).copy()).cuda()
    cnt = torch.tensor([n, 0], dtype=torch.int32, device="cuda")
    nf.launch_mac_learn(dev.data_ptr(), slots - 1, evd.data_ptr(), cnt.data_ptr(), n, 1, cnt.data_ptr() + 4,
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert int(cnt[1]) == 0
    g = dev.cpu().numpy().view(T.MAC_DTYPE)

    def entries(a):
        a = a[a["valid"] == T.MAC_LEARNED]
        return sorted(zip(a["mac_lo"].tolist(), a["bridge_id"].tolist(), a["out_port"].tolist()))

    assert entries(g) == entries(host) and len(entries(host)) == len(np.unique(macs))
