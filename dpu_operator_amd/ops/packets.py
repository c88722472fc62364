"""Vectorized synthetic packet crafting / checking (numpy): header slots + full frames.

Used by tests, the benchmark and the traffic generator.  The data plane reads a 64-B header
slot per packet (``_nfdp.SLOT_BYTES``): the first min(len, 64) bytes of the frame, with the
whole frame's length in the ingress meta word.  The payload beyond the slot stays where the I/O
layer put it (``craft_full`` returns it).  A "64-byte packet" on the wire is a 60-byte frame plus
4-byte FCS, so an untagged 64-B packet occupies 60 B of its slot and a VLAN-tagged one 64 B.

Egress meta word (nfdp.h make_meta): port[11:0] (0xFFF none, 0xFFE punt) | len[25:12] |
reason[29:26] | xhdr[30].  The frame that leaves is ``xrec[:x] ++ ohdr[:hl] ++ in_frame[to:len]``
(``out_tail``/``assemble``; x = the outer-header bytes of a tunnel-encapsulated packet, 50 for an
IPv4 underlay, 70 for IPv6, read off its record's ethertype).
"""
from __future__ import annotations

import numpy as np

SLOT = 64
MAX_FRAME = 9600      # nfdp.h kMaxFrame
ENCAP_BYTES = 50      # nfdp.h kEncapBytes (outer Ethernet + IPv4 + UDP + VXLAN/GENEVE)
ENCAP6_BYTES = 70     # nfdp.h kEncap6Bytes (outer Ethernet + IPv6 + UDP + VXLAN/GENEVE)
ETH_IPV4 = 0x0800
ETH_VLAN = 0x8100
ETH_ARP = 0x0806


def mac_bytes(mac) -> np.ndarray:
    """'aa:bb:..' | int | bytes -> uint8[6]."""
    if isinstance(mac, str):
        return np.array([int(x, 16) for x in mac.split(":")], dtype=np.uint8)
    if isinstance(mac, (bytes, bytearray)):
        return np.frombuffer(bytes(mac), dtype=np.uint8).copy()
    if isinstance(mac, (int, np.integer)):
        return np.array([(int(mac) >> (8 * (5 - i))) & 0xFF for i in range(6)], dtype=np.uint8)
    return np.asarray(mac, dtype=np.uint8)


def mac_raw(mac) -> tuple[int, int]:
    """MAC -> (lo32, hi16) as the kernels hold it (little-endian load of the network bytes)."""
    b = mac_bytes(mac)
    return int(b[0]) | int(b[1]) << 8 | int(b[2]) << 16 | int(b[3]) << 24, int(b[4]) | int(b[5]) << 8


def mac_str(b) -> str:
    return ":".join(f"{int(x):02x}" for x in mac_bytes(b))


def ip_raw(ip_host_order) -> np.ndarray:
    """IPv4 as host-order int (e.g. 0x0A000001 = 10.0.0.1) -> raw LE-loaded network bytes."""
    x = np.asarray(ip_host_order, dtype=np.uint32)
    return ((x >> 24) & 0xFF) | ((x >> 8) & 0xFF00) | ((x << 8) & 0xFF0000) | ((x << 24) & 0xFF000000)


def port_raw(p) -> np.ndarray:
    p = np.asarray(p, dtype=np.uint32)
    return ((p >> 8) & 0xFF) | ((p & 0xFF) << 8)


def _put16(buf: np.ndarray, off, val) -> None:
    val = np.asarray(val, dtype=np.uint32)
    buf[:, off] = (val >> 8) & 0xFF
    buf[:, off + 1] = val & 0xFF


def _put32(buf: np.ndarray, off, val) -> None:
    val = np.asarray(val, dtype=np.uint32)
    for i in range(4):
        buf[:, off + i] = (val >> (8 * (3 - i))) & 0xFF


def _csum16(words: np.ndarray) -> np.ndarray:
    """One's complement of the one's-complement sum over axis 1 of big-endian 16-bit words."""
    s = words.astype(np.uint64).sum(axis=1)
    while True:
        hi = s >> 16
        if not np.any(hi):
            break
        s = (s & 0xFFFF) + hi
    return (~s.astype(np.uint32)) & 0xFFFF


def _be16_words(buf: np.ndarray, start: int, end: int) -> np.ndarray:
    seg = buf[:, start:end].astype(np.uint32)
    if (end - start) % 2:
        seg = np.concatenate([seg, np.zeros((seg.shape[0], 1), np.uint32)], axis=1)
    return (seg[:, 0::2] << 8) | seg[:, 1::2]


def craft(
    n: int,
    *,
    dmac,
    smac,
    src_ip,
    dst_ip,
    sport,
    dport,
    proto: int = 17,
    ttl: int = 64,
    vlan=None,
    frame_len: int = 60,
    payload_seed: int = 0,
) -> tuple[np.ndarray, np.ndarray]:
    """Craft n IPv4 UDP/TCP frames; returns their 64-B header slots.

    Per-packet arrays (length n) or scalars for every field.  ``dmac``/``smac`` are [n,6] or [6]
    uint8.  ``vlan``: None (untagged) or per-packet VID array (-1 = untagged).  ``frame_len`` is
    the untagged L2 length without FCS (42..9596).  Returns (slots uint8[n,64], lens uint32[n])
    with valid IPv4 and L4 checksums over the whole frame; ``craft_full`` also returns the frames.
    """
    frames, lens = craft_full(n, dmac=dmac, smac=smac, src_ip=src_ip, dst_ip=dst_ip, sport=sport, dport=dport,
                              proto=proto, ttl=ttl, vlan=vlan, frame_len=frame_len, payload_seed=payload_seed)
    return header_slots(frames, lens), lens


def craft_arp(n: int, *, smac, sender_ip, target_ip, op: int = 1, vlan=None, dmac="ff:ff:ff:ff:ff:ff"):
    """n ARP frames (request by default, broadcast), padded to 60 B (+4 with a tag).
    Returns (frames uint8[n, 64], lens)."""
    fr = np.zeros((n, 64), np.uint8)
    fr[:, 0:6] = mac_bytes(dmac)
    fr[:, 6:12] = np.broadcast_to(mac_bytes(smac) if np.ndim(smac) <= 1 else np.asarray(smac, np.uint8), (n, 6))
    _put16(fr, 12, np.full(n, ETH_ARP))
    _put16(fr, 14, np.full(n, 1))          # htype Ethernet
    _put16(fr, 16, np.full(n, ETH_IPV4))   # ptype IPv4
    fr[:, 18], fr[:, 19] = 6, 4
    _put16(fr, 20, np.full(n, op))
    fr[:, 22:28] = fr[:, 6:12]
    _put32(fr, 28, np.broadcast_to(np.asarray(sender_ip, np.uint32), (n,)))
    _put32(fr, 38, np.broadcast_to(np.asarray(target_ip, np.uint32), (n,)))
    lens = np.full(n, 60, np.uint32)
    if vlan is not None:
        t = fr.copy()
        fr[:, 12:14] = (0x81, 0x00)
        fr[:, 14] = (int(vlan) >> 8) & 0x0F
        fr[:, 15] = int(vlan) & 0xFF
        fr[:, 16:64] = t[:, 12:60]
        lens[:] = 64
    return fr, lens


def craft6_full(n: int, *, dmac, smac, src6, dst6, sport, dport, hop_limit=64, frame_len: int = 78,
                payload_seed: int = 0) -> tuple[np.ndarray, np.ndarray]:
    """n IPv6 / UDP frames (whole frames, untagged, no FCS) with a valid UDP checksum.
    `src6` / `dst6`: one address or a sequence of n (str or int); per-packet hop limits and
    ports allowed.  Returns (frames uint8[n, frame_len], lens)."""
    import ipaddress

    if frame_len < 62 or frame_len > MAX_FRAME - 4:
        raise ValueError("frame_len must hold Ethernet + IPv6 + UDP")

    def addrs(a):
        seq = a if isinstance(a, (list, tuple, np.ndarray)) else [a] * n
        return np.array([list(int(ipaddress.IPv6Address(x) if not isinstance(x, (int, np.integer)) else int(x))
                              .to_bytes(16, "big")) for x in seq], np.uint8)

    fr = np.zeros((n, frame_len), np.uint8)
    fr[:, 0:6] = np.broadcast_to(mac_bytes(dmac) if np.ndim(dmac) <= 1 else np.asarray(dmac, np.uint8), (n, 6))
    fr[:, 6:12] = np.broadcast_to(mac_bytes(smac) if np.ndim(smac) <= 1 else np.asarray(smac, np.uint8), (n, 6))
    _put16(fr, 12, np.full(n, 0x86DD))
    fr[:, 14] = 0x60
    plen = frame_len - 54
    _put16(fr, 18, np.full(n, plen))
    fr[:, 20] = 17
    fr[:, 21] = np.broadcast_to(np.asarray(hop_limit, np.uint8), (n,))
    fr[:, 22:38] = addrs(src6)
    fr[:, 38:54] = addrs(dst6)
    _put16(fr, 54, np.broadcast_to(np.asarray(sport, np.uint32), (n,)))
    _put16(fr, 56, np.broadcast_to(np.asarray(dport, np.uint32), (n,)))
    _put16(fr, 58, np.full(n, plen))
    rng = np.random.default_rng(payload_seed)
    fr[:, 62:] = rng.integers(0, 256, (n, frame_len - 62), dtype=np.uint8)
    # UDP checksum over the IPv6 pseudo-header (src, dst, length, next header) + UDP header + data
    seg = fr[:, 54:].copy()
    if seg.shape[1] & 1:
        seg = np.concatenate([seg, np.zeros((n, 1), np.uint8)], axis=1)
    words = (seg[:, 0::2].astype(np.uint64) << 8) | seg[:, 1::2]
    ps = fr[:, 22:54]
    pw = (ps[:, 0::2].astype(np.uint64) << 8) | ps[:, 1::2]
    c = words.sum(axis=1) + pw.sum(axis=1) + plen + 17
    while (c >> 16).any():
        c = (c & 0xFFFF) + (c >> 16)
    c = (~c) & 0xFFFF
    c[c == 0] = 0xFFFF
    _put16(fr, 60, c.astype(np.uint32))
    return fr, np.full(n, frame_len, np.uint32)


def header_slots(frames: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """[n, stride] frames -> [n, 64] header slots (first min(len, 64) bytes, zero padded)."""
    slots = np.zeros((frames.shape[0], SLOT), np.uint8)
    w = min(SLOT, frames.shape[1])
    slots[:, :w] = frames[:, :w]
    cols = np.arange(SLOT)[None, :]
    slots[cols >= np.asarray(lens, np.int64)[:, None]] = 0
    return slots


def craft_full(
    n: int,
    *,
    dmac,
    smac,
    src_ip,
    dst_ip,
    sport,
    dport,
    proto: int = 17,
    ttl: int = 64,
    vlan=None,
    frame_len: int = 60,
    payload_seed: int = 0,
) -> tuple[np.ndarray, np.ndarray]:
    """Like ``craft`` but returns the whole frames: (frames uint8[n, frame_len + 4], lens)."""
    if frame_len < 42 or frame_len > MAX_FRAME - 4:
        raise ValueError(f"frame_len must be in [42, {MAX_FRAME - 4}] (untagged, without FCS)")
    l3 = np.zeros((n, frame_len), np.uint8)
    dm = np.broadcast_to(mac_bytes(dmac) if np.ndim(dmac) <= 1 else np.asarray(dmac, np.uint8), (n, 6))
    sm = np.broadcast_to(mac_bytes(smac) if np.ndim(smac) <= 1 else np.asarray(smac, np.uint8), (n, 6))
    l3[:, 0:6] = dm
    l3[:, 6:12] = sm
    _put16(l3, 12, np.full(n, ETH_IPV4))
    l3[:, 14] = 0x45
    tot = frame_len - 14
    _put16(l3, 16, np.full(n, tot))
    _put16(l3, 18, np.arange(n, dtype=np.uint32) & 0xFFFF)
    _put16(l3, 20, np.full(n, 0x4000))
    l3[:, 22] = ttl
    l3[:, 23] = proto
    _put32(l3, 26, np.broadcast_to(np.asarray(src_ip, np.uint32), (n,)))
    _put32(l3, 30, np.broadcast_to(np.asarray(dst_ip, np.uint32), (n,)))
    _put16(l3, 34, np.broadcast_to(np.asarray(sport, np.uint32), (n,)))
    _put16(l3, 36, np.broadcast_to(np.asarray(dport, np.uint32), (n,)))
    rng = np.random.default_rng(payload_seed)
    if proto == 17:
        _put16(l3, 38, np.full(n, tot - 20))
        l3[:, 42:] = rng.integers(0, 256, (n, frame_len - 42), dtype=np.uint8)
    elif proto == 6:
        if frame_len < 54:
            raise ValueError("TCP needs frame_len >= 54")
        _put32(l3, 38, rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32))
        l3[:, 46] = 0x50
        l3[:, 47] = 0x18
        _put16(l3, 48, np.full(n, 8192))
        l3[:, 54:] = rng.integers(0, 256, (n, frame_len - 54), dtype=np.uint8)
    else:
        l3[:, 34:] = rng.integers(0, 256, (n, frame_len - 34), dtype=np.uint8)
    # IPv4 header checksum
    _put16(l3, 24, _csum16(_be16_words(l3, 14, 34)))
    if proto in (6, 17):
        set_l4_csum(l3, proto)
    frames = np.zeros((n, max(frame_len + 4, SLOT)), np.uint8)
    lens = np.full(n, frame_len, np.uint32)
    if vlan is None:
        frames[:, :frame_len] = l3
    else:
        vid = np.broadcast_to(np.asarray(vlan, np.int64), (n,))
        tagged = vid >= 0
        frames[~tagged, :frame_len] = l3[~tagged]
        t = np.where(tagged)[0]
        if len(t):
            frames[t, 0:12] = l3[t, 0:12]
            frames[t, 12] = 0x81
            frames[t, 13] = 0x00
            frames[t, 14] = (vid[t] >> 8) & 0x0F
            frames[t, 15] = vid[t] & 0xFF
            frames[t, 16 : frame_len + 4] = l3[t, 12:frame_len]
            lens[t] = frame_len + 4
    return frames, lens


def set_l4_csum(l3: np.ndarray, proto: int) -> None:
    """(Re)compute the UDP/TCP checksum of untagged frames in place."""
    tot = ((l3[:, 16].astype(np.uint32) << 8) | l3[:, 17]).astype(np.int64)
    L = int(tot[0]) - 20
    if not np.all(tot == tot[0]):
        raise ValueError("set_l4_csum expects a uniform IP total length")
    coff = 34 + (16 if proto == 6 else 6)
    l3[:, coff] = 0
    l3[:, coff + 1] = 0
    pseudo = np.concatenate(
        [
            _be16_words(l3, 26, 34),
            np.full((l3.shape[0], 1), proto, np.uint32),
            np.full((l3.shape[0], 1), L, np.uint32),
        ],
        axis=1,
    )
    words = np.concatenate([pseudo, _be16_words(l3, 34, 34 + L)], axis=1)
    c = _csum16(words)
    if proto == 17:
        c = np.where(c == 0, 0xFFFF, c)
    _put16(l3, coff, c)


def strip(slots: np.ndarray, lens: np.ndarray) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Return (untagged frames [n,64], untagged lens, vid or -1)."""
    et = (slots[:, 12].astype(np.uint32) << 8) | slots[:, 13]
    tagged = et == ETH_VLAN
    out = slots.copy()
    vid = np.full(len(slots), -1, np.int64)
    t = np.where(tagged)[0]
    out[t, 12:60] = slots[t, 16:64]
    out[t, 60:] = 0
    vid[t] = ((slots[t, 14].astype(np.int64) & 0x0F) << 8) | slots[t, 15]
    nl = lens.astype(np.int64) - np.where(tagged, 4, 0)
    return out, nl, vid


def check_csums(frames: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """Per-packet bool: IPv4 header + (UDP|TCP) checksum valid, for untagged frames."""
    ok = _csum16(_be16_words(frames, 14, 34)) == 0
    proto = frames[:, 23]
    tot = (frames[:, 16].astype(np.int64) << 8) | frames[:, 17]
    res = ok.copy()
    for p in (6, 17):
        idx = np.where(proto == p)[0]
        for L in np.unique(tot[idx]):
            sub = idx[tot[idx] == L]
            l4 = int(L) - 20
            pseudo = np.concatenate(
                [
                    _be16_words(frames[sub], 26, 34),
                    np.full((len(sub), 1), p, np.uint32),
                    np.full((len(sub), 1), l4, np.uint32),
                ],
                axis=1,
            )
            words = np.concatenate([pseudo, _be16_words(frames[sub], 34, 34 + l4)], axis=1)
            if p == 17:
                zero = (frames[sub, 40] == 0) & (frames[sub, 41] == 0)
                res[sub] &= zero | (_csum16(words) == 0)
            else:
                res[sub] &= _csum16(words) == 0
    return res


def inmeta(in_port, lens) -> np.ndarray:
    """Per-packet ingress metadata word: in_port | len << 16 (len = whole frame, <= 9600)."""
    return (np.asarray(in_port, np.uint32) & 0xFFFF) | (np.asarray(lens, np.uint32) << 16)


def make_meta(port, length, reason=0, xhdr=False) -> np.ndarray:
    """nfdp.h make_meta (vectorized)."""
    return ((np.asarray(port, np.uint32) & 0xFFF) | ((np.asarray(length, np.uint32) & 0x3FFF) << 12)
            | ((np.asarray(reason, np.uint32) & 0xF) << 26) | (np.asarray(xhdr, np.uint32) << 30)).astype(np.uint32)


def meta_fields(meta: np.ndarray) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Egress metadata -> (out_port, len, reason); port 0xFFF / 0xFFE read back as 0xFFFF / 0xFFFE."""
    m = np.asarray(meta, np.uint32)
    port = m & 0xFFF
    port = np.where(port >= 0xFFE, port | 0xF000, port)
    return port, (m >> 12) & 0x3FFF, (m >> 26) & 0xF


def meta_xhdr(meta: np.ndarray) -> np.ndarray:
    """Per-packet bool: prepend the packet's outer-header record (tunnel encap)."""
    return ((np.asarray(meta, np.uint32) >> 30) & 1).astype(bool)


def xhdr_len(rec) -> int:
    """Outer-header bytes of an outer-header record: 70 when it carries IPv6 (ethertype 0x86DD), else 50."""
    r = np.asarray(rec, np.uint8)
    return ENCAP6_BYTES if (int(r[12]) << 8 | int(r[13])) == 0x86DD else ENCAP_BYTES


def out_tail(in_len, olen, xlen=0, hv=SLOT):
    """nfdp.h out_tail: (hl, to) - valid header bytes of the out slot, tail offset in the input
    (`xlen`: outer-header bytes of an encapsulated packet, 0 otherwise; `hv`: valid bytes of the
    view the out slot was built from - less than 64 for an IPv6-underlay terminated frame)."""
    d = np.asarray(olen, np.int64) - np.asarray(xlen, np.int64) - np.asarray(in_len, np.int64)
    h = np.minimum(np.minimum(np.asarray(in_len, np.int64), np.asarray(hv, np.int64)) + d, SLOT)
    return h, h - d


def wide_slots(arena: np.ndarray, lens: np.ndarray, in_ports, wide_ports=()) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Header slots + in-meta of frames, with a wide header pair (nfdp.h kPortCont) for every frame
    longer than 64 B that arrives on a port in `wide_ports` (VTEP ports: single-pass tunnel
    termination).  Returns (slots [m,64], inmeta [m], head position of each frame)."""
    arena = np.asarray(arena, np.uint8)
    lens = np.asarray(lens, np.uint32)
    ports = np.broadcast_to(np.asarray(in_ports, np.uint32), lens.shape)
    wide = np.isin(ports, np.asarray(list(wide_ports), np.uint32)) & (lens > SLOT)
    pos = np.zeros(len(lens), np.int64)
    pos[1:] = np.cumsum(1 + wide.astype(np.int64))[:-1]
    m = int(len(lens) + wide.sum())
    slots = np.zeros((m, SLOT), np.uint8)
    im = np.zeros(m, np.uint32)
    cols = np.arange(SLOT)
    slots[pos] = np.where(cols[None, :] < lens[:, None], arena[:, :SLOT], 0)
    im[pos] = inmeta(ports, lens)
    w = np.nonzero(wide)[0]
    if len(w):
        second = arena[w, SLOT:2 * SLOT] if arena.shape[1] >= 2 * SLOT else np.pad(
            arena[w, SLOT:], ((0, 0), (0, 2 * SLOT - arena.shape[1])))
        slots[pos[w] + 1] = np.where(cols[None, :] + SLOT < lens[w, None], second, 0)
        im[pos[w] + 1] = np.uint32(0xFFFD) | (lens[w] << np.uint32(16))
    return slots, im, pos


def cont_info(meta) -> tuple[int, int]:
    """(strip, hv) of a continuation slot's egress meta (reason cont): the bytes the head's egress
    strips from its input frame and the valid bytes of the head's out slot."""
    port, ln, reason = meta_fields(np.array([meta], np.uint32))
    if int(reason[0]) != 15:
        raise ValueError("not a continuation meta")
    return int(port[0]) & 0xFF, int(ln[0])


def assemble(ohdr: np.ndarray, meta: int, in_frame: np.ndarray, in_len: int, xhdr_rec: np.ndarray | None = None,
             cont_meta: int | None = None) -> bytes:
    """The frame that leaves for one packet: [outer header] ++ ohdr[:hl] ++ in_frame[to:in_len].
    `cont_meta`: the egress meta of the packet's continuation slot when it arrived as a wide header
    pair (a terminated tunnel frame leaves without its outer `strip` bytes)."""
    _, olen, _ = meta_fields(np.array([meta], np.uint32))
    x = bool(meta_xhdr(np.array([meta], np.uint32))[0])
    if x and xhdr_rec is None:
        raise ValueError("meta says encapsulated but no outer-header record given")
    strip, hv = cont_info(cont_meta) if cont_meta is not None else (0, SLOT)
    in_frame = np.asarray(in_frame, np.uint8)[strip:]
    in_len = int(in_len) - strip
    xl = xhdr_len(xhdr_rec) if x else 0
    hl, to = out_tail(in_len, int(olen[0]), xl, hv)
    hl, to = int(hl), int(to)
    pre = bytes(np.asarray(xhdr_rec, np.uint8)[:xl]) if x else b""
    out = pre + bytes(np.asarray(ohdr, np.uint8)[:hl]) + bytes(np.asarray(in_frame, np.uint8)[to:in_len])
    if len(out) != int(olen[0]):
        raise ValueError(f"assembled {len(out)} bytes, meta says {int(olen[0])}")
    return out
