"""An independent model of the bench's headline pipeline, checked byte for byte against the C++ oracle and the GPU.

The GPU tests hold the HIP kernels to the oracle bit-exactly, but the oracle shares the per-packet
stages (pipeline.h / nfdp.h) with the kernels, so a semantic bug in a shared stage would pass them.
This model shares nothing with that code: it is written from the scenario's definition
(dataplane/scenario.py: pod VFs tagged vlan = pod + 2 and spoof-checked, chain ACL -> SNAT -> L2
steer, egress tag = the destination VF's vlan) and the frame formats alone.  Flow lookup is a
Python dict over the installed 5-tuples, the ACL a first-match scan of the configured rules over
the key words read straight from the frame bytes, checksums are recomputed from scratch (no
incremental update).  Traffic is the bench's mixed trace (flow misses, ACL denies, malformed
lengths) so every disposition of the headline path is exercised.

The cuda variant holds the HIP kernels (MFMA Toeplitz hash, FP4-MFMA ACL, wave-cooperative probe)
to the same model directly.
"""
import numpy as np
import pytest

from dpu_operator_amd.dataplane import scenario as S
from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P

OK, SPOOF, VLAN, DENY, NOROUTE, MALFORMED = 0, 3, 2, 4, 5, 9


def _csum(b: bytes) -> int:
    if len(b) & 1:
        b += b"\0"
    c = sum(int.from_bytes(b[k:k + 2], "big") for k in range(0, len(b), 2))
    while c >> 16:
        c = (c & 0xFFFF) + (c >> 16)
    return ~c & 0xFFFF


def _model(frame: bytes, in_port: int, ln: int, sc, flows: dict, acl, default_permit: bool):
    """-> (reason, out_port, out_frame or None) for one tagged frame of the scenario."""
    if ln < 64 or ln > len(frame):
        return MALFORMED, None, None
    pod = in_port - int(sc.pod_port[0])
    if frame[6:12] != S.pod_mac(pod):
        return SPOOF, None, None
    if int.from_bytes(frame[14:16], "big") & 0xFFF != pod + 2:
        return VLAN, None, None
    # untagged view: Ethernet (14) + IPv4 (20) + UDP
    u = bytearray(frame[:12] + frame[16:ln])
    src, dst = bytes(u[26:30]), bytes(u[30:34])
    sport, dport = int.from_bytes(u[34:36], "big"), int.from_bytes(u[36:38], "big")
    act = flows.get((src, dst, sport, dport))
    if act is None:
        return NOROUTE, T.PORT_PUNT, None      # no flow, GW MAC unknown on the bridge: slow path
    # ACL over the 128-bit key: the frame's address / port bytes as little-endian words + proto |
    # zone, with the port-class bits (meta bit 10: sport >= 1024, bit 11: dport >= 1024)
    pcls = (0x400 if sport >= 1024 else 0) | (0x800 if dport >= 1024 else 0)
    words = np.array([int.from_bytes(src, "little"), int.from_bytes(dst, "little"),
                      int.from_bytes(bytes(u[34:38]), "little"), u[23] | (sc.bridge << 16) | pcls], np.uint64)
    permit = default_permit
    for value, mask, rule_permit in acl:
        if ((words & mask) == value).all():
            permit = rule_permit
            break
    if not permit:
        return DENY, None, None
    out_port, nat_ip, nat_port = act
    # SNAT, then both checksums recomputed over the whole header / datagram
    u[26:30] = nat_ip.to_bytes(4, "big")
    u[34:36] = nat_port.to_bytes(2, "big")
    u[24:26] = b"\0\0"
    u[24:26] = _csum(bytes(u[14:34])).to_bytes(2, "big")
    if u[40:42] != b"\0\0":
        ulen = int.from_bytes(u[38:40], "big")
        pseudo = bytes(u[26:34]) + bytes([0, 17]) + ulen.to_bytes(2, "big")
        u[40:42] = b"\0\0"
        c = _csum(pseudo + bytes(u[34:34 + ulen]))
        u[40:42] = (c or 0xFFFF).to_bytes(2, "big")
    # L2 steer to the destination pod's VF: its MAC as both ends, its vlan tag on egress
    dpod = out_port - int(sc.pod_port[0])
    u[0:6] = S.pod_mac(dpod)
    u[6:12] = S.pod_mac(dpod)
    out = bytes(u[:12]) + b"\x81\x00" + (dpod + 2).to_bytes(2, "big") + bytes(u[12:])
    return OK, out_port, out


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_headline_pipeline_matches_independent_model(device):
    """device=cpu: the C++ oracle; device=cuda: the HIP kernels themselves (MFMA hash + FP4 ACL)."""
    dp = DataPlane(device=device, flow_buckets=1 << 14, hash_mode="mfma", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=20000, n_acl=256, seed=0)
    deny = S.install_deny_flows(dp, sc, k=512)
    dp.commit(full=True)
    pk, im = S.traffic_mixed(sc, deny, 6000, seed=7)
    if device == "cuda":
        import torch

        r = dp.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
        torch.cuda.synchronize()
        meta, out = r.meta.cpu().numpy().view(np.uint32), r.out.cpu().numpy()
    else:
        r = dp.run(pk, im)
        meta, out = r.meta, r.out
    port, olen, reason = P.meta_fields(meta)

    flows = {}
    for k in range(len(sc.keys)):
        s, d = S.POD_NET + int(sc.flow_src_pod[k]), S.POD_NET + int(sc.flow_dst_pod[k])
        flows[(s.to_bytes(4, "big"), d.to_bytes(4, "big"), int(sc.flow_sport[k]), int(sc.flow_dport[k]))] = (
            int(sc.pod_port[sc.flow_dst_pod[k]]), S.NAT_NET + (k % 250) + 1, 1024 + (k % 60000))
    for j in range(len(deny["src"])):
        flows[((S.POD_NET + int(deny["src"][j])).to_bytes(4, "big"), int(deny["dst_ip"][j]).to_bytes(4, "big"),
               int(deny["sport"][j]), int(deny["dport"][j]))] = (0, 0, 0)
    acl = [(r_.value.astype(np.uint64), r_.mask.astype(np.uint64), r_.permit) for r_ in dp.acl.rules]

    seen = {}
    for i in range(len(pk)):
        ln = int(im[i]) >> 16
        want_reason, want_port, want = _model(bytes(pk[i]), int(im[i]) & 0xFFFF, ln, sc, flows, acl,
                                              dp.acl.default_permit)
        seen[want_reason] = seen.get(want_reason, 0) + 1
        assert int(reason[i]) == want_reason, (i, int(reason[i]), want_reason)
        if want_port is not None:
            assert int(port[i]) == want_port, i
        if want is not None:
            assert int(olen[i]) == len(want)
            assert bytes(out[i][: len(want)]) == want, i
    # every disposition of the mixed trace occurred
    assert seen.get(OK, 0) > 5000 and seen.get(NOROUTE, 0) > 100 and seen.get(DENY, 0) > 50
    assert seen.get(MALFORMED, 0) >= 1


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_imix_frames_match_independent_model(device):
    """Header-split IMIX frames (64 / 576 / 1500 / 9000 B): the data plane sees only the 64-B
    header slot; the frame that leaves = egress header slot ++ the payload left in place
    (P.assemble).  The model works on the whole frame and must give the same bytes."""
    dp = DataPlane(device=device, flow_buckets=1 << 14, hash_mode="mfma", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=20000, n_acl=256, seed=0)
    dp.commit(full=True)
    sizes = S.imix_sizes(800, S.IMIX_JUMBO, seed=3)
    slots, im, frames, lens = S.traffic_frames(sc, len(sizes), sizes, seed=4)
    if device == "cuda":
        import torch

        r = dp.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
        torch.cuda.synchronize()
        meta, out = r.meta.cpu().numpy().view(np.uint32), r.out.cpu().numpy()
    else:
        r = dp.run(slots, im)
        meta, out = r.meta, r.out
    flows = {}
    for k in range(len(sc.keys)):
        s, d = S.POD_NET + int(sc.flow_src_pod[k]), S.POD_NET + int(sc.flow_dst_pod[k])
        flows[(s.to_bytes(4, "big"), d.to_bytes(4, "big"), int(sc.flow_sport[k]), int(sc.flow_dport[k]))] = (
            int(sc.pod_port[sc.flow_dst_pod[k]]), S.NAT_NET + (k % 250) + 1, 1024 + (k % 60000))
    acl = [(r_.value.astype(np.uint64), r_.mask.astype(np.uint64), r_.permit) for r_ in dp.acl.rules]
    big = 0
    for i in range(len(sizes)):
        ln = int(lens[i])
        want_reason, want_port, want = _model(bytes(frames[i][:ln]), int(im[i]) & 0xFFFF, ln, sc, flows, acl,
                                              dp.acl.default_permit)
        assert want_reason == OK
        got = P.assemble(out[i], int(meta[i]), frames[i], ln)
        assert got == want, (i, ln)
        big += ln > 64
    assert big > 200


def _flow_dict(sc, nat_ip, nat_port, deny, live_mask=None):
    flows = {}
    for k in range(len(sc.keys)):
        if live_mask is not None and not live_mask[k]:
            continue
        s, d = S.POD_NET + int(sc.flow_src_pod[k]), S.POD_NET + int(sc.flow_dst_pod[k])
        flows[(s.to_bytes(4, "big"), d.to_bytes(4, "big"), int(sc.flow_sport[k]), int(sc.flow_dport[k]))] = (
            int(sc.pod_port[sc.flow_dst_pod[k]]), int(nat_ip[k]), int(nat_port[k]))
    for j in range(len(deny["src"])):
        flows[((S.POD_NET + int(deny["src"][j])).to_bytes(4, "big"), int(deny["dst_ip"][j]).to_bytes(4, "big"),
               int(deny["sport"][j]), int(deny["dport"][j]))] = (0, 0, 0)
    return flows


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_live_table_flip_matches_independent_model(device):
    """The live path (native engine; on the GPU the persistent ring kernel) before and after a
    commit that puts a deny rule first, erases an eighth of the flows and re-points the NAT of
    another eighth: each phase's delivered frames equal the model's over that phase's tables.
    On the GPU the commit is a table-set flip under the running ring (no relaunch), so this holds
    the flip's results — not only the oracle's — to code that shares nothing with pipeline.h."""
    import ipaddress
    import shutil
    import tempfile
    import time
    from pathlib import Path

    from dpu_operator_amd.dataplane.native_io import MemifVport, NativeLivePath, memif_dir
    from dpu_operator_amd.native import nfdp

    nf = nfdp()
    dp = DataPlane(device=device, flow_buckets=1 << 14, hash_mode="mfma", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=6000, n_acl=256, seed=0)
    deny = S.install_deny_flows(dp, sc, k=256)
    dp.commit(full=True)
    d = Path(tempfile.mkdtemp(prefix="dpu-flipm-", dir=memif_dir()))
    pods = [int(p) for p in sc.pod_port]
    live = NativeLivePath(dp, {p: MemifVport(str(d / f"p{p}"), ring_size=4096) for p in pods}, burst=128,
                          ring_capacity=1024, queues=2).start()
    eps = {p: nf.MemifEndpoint(str(d / f"p{p}")) for p in pods}

    def phase(seed, flows):
        pk, im = S.traffic_mixed(sc, deny, 3000, seed=seed)
        acl = [(r_.value.astype(np.uint64), r_.mask.astype(np.uint64), r_.permit) for r_ in dp.acl.rules]
        want: dict[int, list[bytes]] = {}
        sent = {p: [] for p in pods}
        seen = {}
        for i in range(len(pk)):
            ln = min(int(im[i]) >> 16, 64)
            fr = bytes(pk[i][:ln])
            sent[int(im[i]) & 0xFFFF].append(fr)
            reason, port, out = _model(fr, int(im[i]) & 0xFFFF, ln, sc, flows, acl, dp.acl.default_permit)
            seen[reason] = seen.get(reason, 0) + 1
            if reason == OK:
                want.setdefault(port, []).append(out)
        for p, frs in sent.items():
            k, t_end = 0, time.monotonic() + 10
            while k < len(frs) and time.monotonic() < t_end:
                k += eps[p].send(frs[k:])
        got = {p: [] for p in pods}
        n_want = sum(map(len, want.values()))
        t_end = time.monotonic() + 15
        while sum(map(len, got.values())) < n_want and time.monotonic() < t_end:
            for p in pods:
                got[p] += eps[p].recv()
            time.sleep(0.002)
        time.sleep(0.05)
        for p in pods:
            got[p] += eps[p].recv()
        for p in pods:
            assert sorted(got[p]) == sorted(want.get(p, [])), (p, len(got[p]), len(want.get(p, [])), live.stats)
        return seen

    try:
        kk = np.arange(len(sc.keys))
        nat_ip, nat_port = S.NAT_NET + (kk % 250) + 1, 1024 + (kk % 60000)   # (build_sfc's, host order)
        seen_a = phase(31, _flow_dict(sc, nat_ip, nat_port, deny))
        assert seen_a.get(OK, 0) > 2000 and seen_a.get(DENY, 0) > 20
        # the commit: a deny rule first (everything to pod 1), flows k % 8 == 3 erased, the NAT of
        # flows k % 8 == 5 re-pointed
        dp.acl.add(permit=False, dst=f"{ipaddress.IPv4Address(S.POD_NET + 1)}/32")
        dp.acl.rules.insert(0, dp.acl.rules.pop())
        dp.acl.version += 1
        gone = kk % 8 == 3
        dp.flows.erase_many(sc.keys[gone])
        moved = kk % 8 == 5
        nat_ip, nat_port = nat_ip.copy(), nat_port.copy()
        nat_ip[moved] = S.NAT_NET + 251 + (kk[moved] % 3)
        nat_port[moved] = 40000 + (kk[moved] % 1000)
        acts = sc.actions[moved].copy()
        acts[:, 1:3] = T.flow_action(nat_ip=nat_ip[moved], nat_port=nat_port[moved])[:, 1:3]
        dp.flows.erase_many(sc.keys[moved])
        assert (np.asarray(dp.flows.insert_many(sc.keys[moved], acts)) >= 0).all()
        dp.commit()
        seen_b = phase(32, _flow_dict(sc, nat_ip, nat_port, deny, ~gone))
        assert seen_b.get(DENY, 0) > seen_a.get(DENY, 0) + 200      # the new first rule denies pod 1's traffic
        assert seen_b.get(NOROUTE, 0) > seen_a.get(NOROUTE, 0) + 200
        if device == "cuda":
            assert dp.flip_stats.get("table_flips", 0) >= 1 and live.restarts == 0, dp.flip_stats
    finally:
        live.stop()
        shutil.rmtree(d, ignore_errors=True)
