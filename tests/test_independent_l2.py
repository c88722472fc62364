"""Independent models of the side features: flooding (groups longer than one 16-entry row),
MAC learning, the K9 mirror copy, the ARP slow-path copy (always_trap_arp_table) and VXLAN /
GENEVE encapsulation (these were checked only against the C++ oracle, which
shares pipeline.h with the kernels).

The models share no code with pipeline.h / nfdp.h: the bridge is a Python dict of MAC -> port
that changes only between batches (the data plane applies learn events after the batch), the
flood order is the group's member list, egress tags / the mirror copy / the ARP copy are built
byte by byte, and the tunnel outer header is built from RFC 7348 / RFC 8926 with its IPv4
checksum summed from scratch and the entropy source port from a bit-by-bit Toeplitz over the
flow key written from the Microsoft RSS definition.  device=cuda holds the HIP kernels
(fused_kernel + side_kernel + mac_learn_kernel) to the same models directly."""
import ipaddress

import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P

BR = 5
NPORT = 20
TAG_PORT, TAG_VID = 3, 7
MIRROR_FROM, MIRROR_TO = 2, 19
PUNT, ARP_TRAP = T.PORT_PUNT, 12


def _mac(i: int) -> bytes:
    return bytes([0x02, 0x10, 0, 0, i >> 8, i & 0xFF])


def _mstr(b: bytes) -> str:
    return ":".join(f"{x:02x}" for x in b)


def _bridge(device):
    dp = DataPlane(device=device, flow_buckets=1 << 10, mac_slots=1 << 10)
    for p in range(NPORT):
        fl = T.PORT_VALID | T.PORT_LEARN | T.PORT_ARP_TRAP | (T.PORT_TAG_EGRESS if p == TAG_PORT else 0)
        dp.ports.set(p, flags=fl, vlan=TAG_VID if p == TAG_PORT else 0, bridge_id=BR)
    order = list(np.random.default_rng(3).permutation(NPORT))   # group order is not port order
    dp.flood.set_members(BR, order)
    dp.ports.set_mirror(MIRROR_FROM, MIRROR_TO)
    dp.macs.insert(BR, _mstr(_mac(900)), 11)                      # a static entry
    dp.commit(full=True)
    return dp, [int(x) for x in order]


def _trace(n, seed):
    """Hosts h (MAC _mac(h)) sit behind port h % NPORT; frames: broadcast ARP, unicast to a host,
    unicast to an unknown MAC, unicast to the static MAC."""
    rng = np.random.default_rng(seed)
    frames, ports = [], []
    for j in range(n):
        h = int(rng.integers(0, 60))
        port = h % NPORT
        kind = j % 4
        if kind == 0:
            fr, _ = P.craft_arp(1, smac=_mac(h), sender_ip=0x0A000000 + h, target_ip=0x0A0000FF)
            f = bytes(fr[0, :60])
        else:
            dst = {1: _mac(int(rng.integers(0, 60))), 2: _mac(500 + j), 3: _mac(900)}[kind]
            fr, ln = P.craft_full(1, dmac=np.frombuffer(dst, np.uint8), smac=np.frombuffer(_mac(h), np.uint8),
                                  src_ip=0x0A000000 + h, dst_ip=0x0A000100 + j, sport=1000 + j, dport=80,
                                  frame_len=int(rng.choice([60, 200, 1000])))
            f = bytes(fr[0, : int(ln[0])])
        frames.append(f)
        ports.append(port)
    return frames, ports


def _tag(f: bytes, vid: int) -> bytes:
    return f[:12] + b"\x81\x00" + vid.to_bytes(2, "big") + f[12:]


def _model_batch(frames, ports, table: dict, order):
    """-> primaries [(reason, port, out_len, out_bytes)], replicas multiset, learn events."""
    prim, reps, learn = [], [], []
    for f, p in zip(frames, ports):
        dst, src = f[0:6], f[6:12]
        if not (src[0] & 1) and table.get(src) != p:
            learn.append((src, p))
        if f[12:14] == b"\x08\x06":
            reps.append((PUNT, ARP_TRAP, len(f), f[:64]))
        out = table.get(dst)
        flood_rest = []
        if out is None:
            members = [m for m in order if m != p]
            out, flood_rest = members[0], members[1:]
        o = _tag(f, TAG_VID) if out == TAG_PORT else f
        prim.append((0, out, len(o), o[:64]))
        for m in flood_rest:
            r = _tag(f, TAG_VID) if m == TAG_PORT else f
            reps.append((m, 0, len(r), r[:64]))
        if p == MIRROR_FROM:
            reps.append((MIRROR_TO, 0, len(o), o[:64]))
    return prim, sorted(reps), learn


def _run(dp, frames, ports, device):
    arena = np.zeros((len(frames), 1600), np.uint8)
    lens = np.array([len(f) for f in frames], np.uint32)
    for i, f in enumerate(frames):
        arena[i, : len(f)] = np.frombuffer(f, np.uint8)
    slots, im = P.header_slots(arena, lens), P.inmeta(np.array(ports), lens)
    if device == "cuda":
        import torch

        r = dp.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
        torch.cuda.synchronize()
        out, meta = r.out.cpu().numpy(), r.meta.cpu().numpy().view(np.uint32)
    else:
        r = dp.run(slots, im)
        out, meta = r.out, r.meta
    return out, meta, dp.side_result()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_flood_learn_mirror_arp_match_independent_model(device):
    dp, order = _bridge(device)
    table = {_mac(900): 11}
    for batch in range(3):
        frames, ports = _trace(400, seed=batch)
        out, meta, side = _run(dp, frames, ports, device)
        prim, reps, learn = _model_batch(frames, ports, table, order)
        port, olen, reason = P.meta_fields(meta)
        for i, (wr, wp, wl, wo) in enumerate(prim):
            assert (int(reason[i]), int(port[i]), int(olen[i])) == (wr, wp, wl), (batch, i)
            assert bytes(out[i][: min(wl, 64)]) == wo[: min(wl, 64)], (batch, i)
        rp, rl, rr = P.meta_fields(side["rep_meta"])
        got = sorted((int(a), int(b), int(c), bytes(h[: min(int(c), 64)]))
                     for a, b, c, h in zip(rp, rr, rl, side["rep_hdr"]))
        want = sorted((a, b, c, h[: min(c, 64)]) for a, b, c, h in reps)
        assert got == want, batch
        assert side["n_learn"] == len(learn) and side["rep_dropped"] == 0
        # learning takes effect for the next batch (static entries win)
        for src, p in learn:
            table[src] = p
        dp.pull_learned()
        learned = {(b, m, p) for b, m, p in dp.macs.learned()}
        assert learned == {(BR, _mstr(s), p) for s, p in table.items() if s != _mac(900)}
    assert dp.drop_counters().get("arp_trap", 0) == sum(1 for _ in range(3) for j in range(400) if j % 4 == 0)


# ---- VXLAN / GENEVE encapsulation ----
LOCAL_VTEP, REMOTE_VTEP = "192.0.2.1", "192.0.2.2"
POD_MAC, REMOTE_MAC = "02:00:00:00:aa:01", "02:00:00:00:bb:01"
VNI = 5000


def _toeplitz(key: bytes, data: bytes) -> int:
    """Microsoft RSS Toeplitz, bit by bit: for every set input bit (MSB first), XOR in the 32-bit
    window of the key starting at that bit."""
    kint = int.from_bytes(key, "big")
    kbits = len(key) * 8
    h = 0
    for i in range(len(data) * 8):
        if (data[i // 8] >> (7 - i % 8)) & 1:
            h ^= (kint >> (kbits - 32 - i)) & 0xFFFFFFFF
    return h


def _overlay(device, kind):
    dp = DataPlane(device=device, flow_buckets=1 << 10)
    dp.ports.set(1, flags=T.PORT_VALID, bridge_id=3, mac=POD_MAC)
    dp.ports.set(20, flags=T.PORT_VALID | T.PORT_TUNNEL, bridge_id=3)
    dp.ports.a[20]["lag"] = 0
    dp.ports.set(30, flags=T.PORT_VALID | T.PORT_VTEP, mac="02:00:00:00:0e:01")
    dp.tunnels.set(0, src=LOCAL_VTEP, dst=REMOTE_VTEP, vni=VNI, out_port=30, smac="02:00:00:00:0e:01",
                   dmac="02:00:00:00:0e:02", kind=kind)
    dp.macs.insert(3, REMOTE_MAC, 20)
    dp.ports.version += 1
    dp.commit(full=True)
    return dp


def _outer(inner: bytes, kind, rss_key: bytes) -> bytes:
    """The 50 outer bytes the tunnel port puts in front of `inner` (an IPv4 / UDP frame from the pod)."""
    u = inner
    key = u[26:30] + u[30:34] + u[34:38] + bytes([u[23], 0]) + (3).to_bytes(2, "little")   # src, dst, ports, proto | zone
    sport = 0xC000 | (_toeplitz(rss_key, key) & 0x3FFF)
    eth = bytes.fromhex("02000000 0e02".replace(" ", "")) + bytes.fromhex("020000000e01") + b"\x08\x00"
    total = 20 + 8 + 8 + len(inner)
    ip = bytearray(b"\x45\x00" + total.to_bytes(2, "big") + b"\x00\x00\x40\x00\x40\x11\x00\x00"
                   + ipaddress.IPv4Address(LOCAL_VTEP).packed + ipaddress.IPv4Address(REMOTE_VTEP).packed)
    c = sum(int.from_bytes(ip[k:k + 2], "big") for k in range(0, 20, 2))
    while c >> 16:
        c = (c & 0xFFFF) + (c >> 16)
    ip[10:12] = (~c & 0xFFFF).to_bytes(2, "big")
    udp = sport.to_bytes(2, "big") + (4789 if kind == T.TUN_VXLAN else 6081).to_bytes(2, "big") \
        + (8 + 8 + len(inner)).to_bytes(2, "big") + b"\x00\x00"
    if kind == T.TUN_VXLAN:
        hdr = b"\x08\x00\x00\x00" + VNI.to_bytes(3, "big") + b"\x00"
    else:
        hdr = b"\x00\x00\x65\x58" + VNI.to_bytes(3, "big") + b"\x00"
    return eth + bytes(ip) + udp + hdr


@pytest.mark.parametrize("kind", [T.TUN_VXLAN, T.TUN_GENEVE])
@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_tunnel_encap_matches_independent_model(device, kind):
    dp = _overlay(device, kind)
    rng = np.random.default_rng(5)
    n = 64
    frames = []
    for j in range(n):
        fr, ln = P.craft_full(1, dmac=REMOTE_MAC, smac=POD_MAC, src_ip=0x0A000001 + j, dst_ip=0x0A000200 + (j * 7) % 50,
                              sport=int(rng.integers(1024, 65535)), dport=int(rng.integers(1, 65535)),
                              proto=int(rng.choice([6, 17])), frame_len=int(rng.choice([60, 300, 1400])))
        frames.append(bytes(fr[0, : int(ln[0])]))
    out, meta, side = _run(dp, frames, [1] * n, device)
    port, olen, reason = P.meta_fields(meta)
    arena = np.zeros((n, 1500), np.uint8)
    for i, f in enumerate(frames):
        arena[i, : len(f)] = np.frombuffer(f, np.uint8)
    for i, f in enumerate(frames):
        assert (int(reason[i]), int(port[i]), int(olen[i])) == (0, 20, len(f) + 50), i
        got = P.assemble(out[i], int(meta[i]), arena[i], len(f), side["xhdr"][i])
        assert got == _outer(f, kind, dp.rss_key) + f, i
