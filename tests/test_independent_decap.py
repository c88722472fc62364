"""Independent model of VXLAN / GENEVE tunnel termination (the reference's FXP
ipv4_tunnel_term_table / ipv6_tunnel_term_table + rx_*_tunnel_source_port, p4info.txt:342,510).

`terminate()` below is written from the wire formats (RFC 7348 VXLAN, RFC 8926 GENEVE, RFC 791 /
8200 outer headers) and shares nothing with csrc/nfdp/pipeline.h: it walks the WHOLE outer frame
and says whether it is terminated, onto which tunnel port, and which inner frame continues from
there.  The data plane's two termination paths are held to it:
  * single pass (frames > 64 B on a VTEP port arrive as wide header pairs: pair_kernel ->
    fused kernel -> pair_fix on the GPU, decap_pair in the oracle) - the head's egress must be the
    inner frame processed on the tunnel port;
  * 64-B slots (recirculation: kRecirc re-enters the inner frame, kRecirc6 goes through
    DataPlane.resolve_recirc6 on the whole frame).
Frames the model does NOT terminate must come out exactly as the same frame received as an
ordinary 64-B slot on the VTEP port.  Cases: IPv4 and IPv6 underlays, untagged and 802.1Q-tagged
outer frames, VXLAN and GENEVE, unknown VNI / source, another VTEP's address, IPv4 options and
fragments, a VXLAN header without its I flag, GENEVE with options / the OAM bit / a non-Ethernet
payload, and truncated frames."""
import ipaddress
import struct

import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.dataplane.engine import DataPlane
from dpu_operator_amd.ops import packets as P

LOCAL4, REMOTE4, OTHER4 = "192.0.2.1", "192.0.2.2", "192.0.2.7"
LOCAL6, REMOTE6, OTHER6 = "2001:db8:f::1", "2001:db8:f::2", "2001:db8:f::7"
VNI4, VNI6 = 5000, 7000
VTEP_PORT, TUN4, TUN6, POD = 30, 20, 21, 1
POD_MAC, REMOTE_MAC, VTEP_MAC = "02:00:00:00:0a:01", "02:00:00:00:bb:01", "02:00:00:00:0e:01"


# ---------------------------------------------------------------------------- the model
def terminate(frame: bytes, vtep4: str, terms4: dict, vtep6: str, terms6: dict):
    """(tunnel port, inner frame) if this outer frame is a VXLAN / GENEVE frame for the local VTEP
    with a termination entry for its (outer source, VNI); None otherwise."""
    off = 12
    etype = struct.unpack_from("!H", frame, off)[0] if len(frame) >= 14 else 0
    if etype == 0x8100:                       # one 802.1Q tag on the outer frame
        off += 4
        if len(frame) < off + 2:
            return None
        etype = struct.unpack_from("!H", frame, off)[0]
    l3 = off + 2
    if etype == 0x0800:
        if len(frame) < l3 + 20:
            return None
        ver_ihl, _tos, _tot, _ident, flags_frag, _ttl, proto = struct.unpack_from("!BBHHHBB", frame, l3)
        if ver_ihl != 0x45 or proto != 17:                      # IPv4, no options, UDP
            return None
        if flags_frag & 0x3FFF:                                 # a fragment (MF or offset): not a whole datagram
            return None
        src = ipaddress.IPv4Address(frame[l3 + 12:l3 + 16])
        dst = ipaddress.IPv4Address(frame[l3 + 16:l3 + 20])
        if dst != ipaddress.IPv4Address(vtep4):
            return None
        l4, table = l3 + 20, terms4
    elif etype == 0x86DD:
        if len(frame) < l3 + 40:
            return None
        if frame[l3] >> 4 != 6 or frame[l3 + 6] != 17:          # IPv6, next header UDP
            return None
        src = ipaddress.IPv6Address(frame[l3 + 8:l3 + 24])
        dst = ipaddress.IPv6Address(frame[l3 + 24:l3 + 40])
        if vtep6 is None or dst != ipaddress.IPv6Address(vtep6):
            return None
        l4, table = l3 + 40, terms6
    else:
        return None
    if len(frame) < l4 + 8 + 8 + 14:                            # UDP + tunnel header + an inner Ethernet header
        return None
    dport = struct.unpack_from("!H", frame, l4 + 2)[0]
    t = l4 + 8
    if dport == 4789:                                           # VXLAN: I flag, VNI
        if not frame[t] & 0x08:
            return None
    elif dport == 6081:                                         # GENEVE: version 0, no options, not OAM, Ethernet
        ver_optlen, flags, ptype = frame[t], frame[t + 1], struct.unpack_from("!H", frame, t + 2)[0]
        if ver_optlen >> 6 != 0 or ver_optlen & 0x3F or flags & 0x80 or ptype != 0x6558:
            return None
    else:
        return None
    vni = int.from_bytes(frame[t + 4:t + 7], "big")
    port = table.get((src, vni))
    if port is None:
        return None
    return port, frame[t + 8:]


# ---------------------------------------------------------------------------- frames
def _inner(n=3):
    out = []
    for k, sz in enumerate((60, 200, 1000)[:n]):
        f, ln = P.craft_full(1, dmac=POD_MAC, smac=REMOTE_MAC, src_ip=0x0A000002, dst_ip=0x0A000001, sport=1000 + k,
                             dport=80, frame_len=sz)
        out.append(bytes(f[0, : ln[0]]))
    return out


def _csum(b: bytes) -> int:
    s = sum(struct.unpack(f"!{len(b) // 2}H", b))
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def _outer(inner: bytes, v6: bool, kind: str = "vxlan", src=None, dst=None, vni=None, tag=False, flags_frag=0x4000,
           ihl=5, vx_flags=0x08, gn=(0, 0, 0x6558)) -> bytes:
    tunnel = (bytes([vx_flags, 0, 0, 0]) if kind == "vxlan" else bytes([gn[0], gn[1]]) + struct.pack("!H", gn[2]))
    tunnel += ((vni if vni is not None else (VNI6 if v6 else VNI4)) << 8).to_bytes(4, "big")
    udp_len = 8 + len(tunnel) + len(inner)
    udp = struct.pack("!HHHH", 0xC123, 4789 if kind == "vxlan" else 6081, udp_len, 0)
    if v6:
        ip = struct.pack("!IHBB", 6 << 28, udp_len, 17, 64) + ipaddress.IPv6Address(src or REMOTE6).packed + \
            ipaddress.IPv6Address(dst or LOCAL6).packed
        et = 0x86DD
    else:
        opts = b"\x01\x01\x01\x01" * (ihl - 5)
        hdr = struct.pack("!BBHHHBBH4s4s", (4 << 4) | ihl, 0, 20 + len(opts) + udp_len, 7, flags_frag, 64, 17, 0,
                          ipaddress.IPv4Address(src or REMOTE4).packed, ipaddress.IPv4Address(dst or LOCAL4).packed)
        hdr += opts
        ip = hdr[:10] + struct.pack("!H", _csum(hdr)) + hdr[12:]
        et = 0x0800
    eth = P.mac_bytes(VTEP_MAC).tobytes() + P.mac_bytes("02:00:00:00:0e:02").tobytes()
    if tag:
        eth += struct.pack("!HH", 0x8100, 0)       # priority tag (vid 0): passes the port's checks
    return eth + struct.pack("!H", et) + ip + udp + tunnel + inner


def _cases():
    """(name, outer frame, terminated by the model?)"""
    cases = []
    for v6 in (False, True):
        fam = "v6" if v6 else "v4"
        for kind in ("vxlan", "geneve"):
            for tag in (False, True):
                for k, inner in enumerate(_inner()):
                    cases.append((f"{fam}-{kind}-{'tag' if tag else 'untag'}-{k}", _outer(inner, v6, kind, tag=tag)))
        inner = _inner(2)[1]
        cases += [(f"{fam}-unknown-vni", _outer(inner, v6, vni=(VNI6 if v6 else VNI4) + 1)),
                  (f"{fam}-unknown-source", _outer(inner, v6, src=OTHER6 if v6 else OTHER4)),
                  (f"{fam}-other-vtep", _outer(inner, v6, dst=OTHER6 if v6 else OTHER4)),
                  (f"{fam}-vxlan-no-I-flag", _outer(inner, v6, vx_flags=0x00)),
                  (f"{fam}-geneve-options", _outer(inner, v6, "geneve", gn=(1, 0, 0x6558))),
                  (f"{fam}-geneve-oam", _outer(inner, v6, "geneve", gn=(0, 0x80, 0x6558))),
                  (f"{fam}-geneve-version1", _outer(inner, v6, "geneve", gn=(0x40, 0, 0x6558))),
                  (f"{fam}-geneve-ipv4-payload", _outer(inner, v6, "geneve", gn=(0, 0, 0x0800)))]
    inner = _inner(2)[1]
    cases += [("v4-first-fragment", _outer(inner, False, flags_frag=0x2000)),
              ("v4-later-fragment", _outer(inner, False, flags_frag=0x0010)),
              ("v4-options", _outer(inner, False, ihl=6))]
    return cases


def _plane(device="cpu"):
    dp = DataPlane(device=device, flow_buckets=1 << 10)
    dp.ports.set(POD, flags=T.PORT_VALID, bridge_id=3, mac=POD_MAC)
    for tp in (TUN4, TUN6):
        dp.ports.set(tp, flags=T.PORT_VALID, bridge_id=3)
    dp.ports.set(VTEP_PORT, flags=T.PORT_VALID | T.PORT_VTEP, mac=VTEP_MAC, bridge_id=9)
    dp.ports.a[VTEP_PORT]["ext"] = int(P.ip_raw(np.uint32(int(ipaddress.IPv4Address(LOCAL4)))))
    dp.terms.insert(REMOTE4, VNI4, TUN4)
    dp.vtep6.set(LOCAL6)
    dp.terms6.insert(REMOTE6, VNI6, TUN6)
    dp.macs.insert(3, POD_MAC, POD)
    dp.macs.insert(3, REMOTE_MAC, TUN4)
    dp.ports.version += 1
    dp.commit(full=True)
    return dp


TERMS4 = {(ipaddress.IPv4Address(REMOTE4), VNI4): TUN4}
TERMS6 = {(ipaddress.IPv6Address(REMOTE6), VNI6): TUN6}


def _arena(frames):
    ln = np.array([len(f) for f in frames], np.uint32)
    ar = np.zeros((len(frames), max(int(ln.max()), 128)), np.uint8)
    for i, f in enumerate(frames):
        ar[i, : len(f)] = np.frombuffer(f, np.uint8)
    return ar, ln


def _one(dp, frame: bytes, port: int):
    """(egress port, reason, assembled frame or b"") of one frame as an ordinary 64-B slot."""
    ar, ln = _arena([frame])
    r = dp.run(P.header_slots(ar, ln), P.inmeta(np.array([port]), ln))
    p, _, rs = P.meta_fields(r.meta)
    out = P.assemble(r.out[0], int(r.meta[0]), ar[0], int(ln[0])) if int(rs[0]) == 0 else b""
    return int(p[0]), int(rs[0]), out


def test_model_cases_cover_both_outcomes():
    verdicts = [terminate(f, LOCAL4, TERMS4, LOCAL6, TERMS6) is not None for _, f in _cases()]
    assert sum(verdicts) == 24 and len(verdicts) - sum(verdicts) == 19


def test_single_pass_termination_matches_the_model():
    """Wide header pairs (one pass, pipeline.h decap_pair on the oracle): every head egresses as the
    model's inner frame processed on the model's tunnel port; every frame the model leaves alone
    egresses as the same frame received as a 64-B slot on the VTEP port."""
    dp, ref = _plane(), _plane()
    cases = _cases()
    frames = [f for _, f in cases]
    ar, ln = _arena(frames)
    slots, im, pos = P.wide_slots(ar, ln, VTEP_PORT, wide_ports={VTEP_PORT})
    r = dp.run(slots, im)
    port, _, reason = P.meta_fields(r.meta)
    for i, (name, f) in enumerate(cases):
        h = int(pos[i])
        cont = int(r.meta[h + 1]) if len(f) > 64 else None
        got = (int(port[h]), int(reason[h]),
               P.assemble(r.out[h], int(r.meta[h]), ar[i], int(ln[i]), cont_meta=cont) if int(reason[h]) == 0 else b"")
        m = terminate(f, LOCAL4, TERMS4, LOCAL6, TERMS6)
        want = _one(ref, m[1], m[0]) if m is not None else _one(ref, f, VTEP_PORT)
        assert got == want, name


def test_slot_path_termination_matches_the_model():
    """64-B slots: a terminated IPv4-underlay frame says kRecirc with the model's tunnel port and
    inner length; an IPv6-underlay one says kRecirc6 and DataPlane.resolve_recirc6 returns the
    model's (port, inner frame); frames the model leaves alone are never recirculated."""
    dp = _plane()
    for name, f in _cases():
        m = terminate(f, LOCAL4, TERMS4, LOCAL6, TERMS6)
        p, rs, _ = _one(dp, f, VTEP_PORT)
        if m is None:
            assert rs not in (13,) or False, name
            if rs == 14:                             # recognised by the slot path, refused on the whole frame
                assert dp.resolve_recirc6(f) is None, name
            continue
        if ":" in name[:3] or name.startswith("v6"):
            assert rs == 14, name
            assert dp.resolve_recirc6(f) == (m[0], m[1]), name
        else:
            assert (rs, p) == (13, m[0]), name


@pytest.mark.gpu
def test_single_pass_termination_gpu_matches_the_model():
    """The GPU's pair_kernel -> fused kernel -> pair_fix against the model (not against the oracle)."""
    import torch

    g, ref = _plane("cuda"), _plane()
    cases = _cases()
    frames = [f for _, f in cases]
    ar, ln = _arena(frames)
    slots, im, pos = P.wide_slots(ar, ln, VTEP_PORT, wide_ports={VTEP_PORT})
    r = g.run(torch.from_numpy(slots).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
    torch.cuda.synchronize()
    meta = r.meta.cpu().numpy().view(np.uint32)
    out = r.out.cpu().numpy()
    port, _, reason = P.meta_fields(meta)
    for i, (name, f) in enumerate(cases):
        h = int(pos[i])
        cont = int(meta[h + 1]) if len(f) > 64 else None
        got = (int(port[h]), int(reason[h]),
               P.assemble(out[h], int(meta[h]), ar[i], int(ln[i]), cont_meta=cont) if int(reason[h]) == 0 else b"")
        m = terminate(f, LOCAL4, TERMS4, LOCAL6, TERMS6)
        want = _one(ref, m[1], m[0]) if m is not None else _one(ref, f, VTEP_PORT)
        assert got == want, name
