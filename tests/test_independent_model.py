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
