"""Tunnel outer headers (pipeline.h make_outer / make_outer6) against a byte-level Python model.

The native builders assemble the headers as little-endian dwords (r5: the byte array they used
before lived in scratch memory on the GPU); this checks them byte for byte, over random tunnel
entries, for both underlays, both encapsulations, a raw or a hash-derived UDP source port and
IPv6 flow labels.  The native code is the same on the CPU oracle and in side_kernel; the GPU twin
is covered by the overlay tests (tests/test_l3_tunnels.py, tests/test_overlay_sfc.py).
"""
import numpy as np
import pytest

from dpu_operator_amd.dataplane import tables as T
from dpu_operator_amd.native import nfdp


def _le(x: int, n: int) -> bytes:
    return int(x).to_bytes(n, "little")


def _be(x: int, n: int) -> bytes:
    return int(x).to_bytes(n, "big")


def _sport(e, h: int) -> bytes:
    return _le(e["sport"], 2) if int(e["sport"]) else _be(0xC000 | (h & 0x3FFF), 2)


def _l2(e, ethertype: int) -> bytes:
    return _le(e["dmac_lo"], 4) + _le(e["dmac_hi"], 2) + _le(e["smac_lo"], 4) + _le(e["smac_hi"], 2) + _be(ethertype, 2)


def _shim(e) -> bytes:
    vni = int(e["vni"]) & 0xFFFFFF
    if int(e["type"]) == T.TUN_GENEVE:
        return b"\x00\x00\x65\x58" + _be(vni, 3) + b"\x00"
    return b"\x08\x00\x00\x00" + _be(vni, 3) + b"\x00"


def model4(e, inner_len: int, h: int) -> bytes:
    ip = bytearray(b"\x45\x00" + _be(20 + 8 + 8 + inner_len, 2) + b"\x00\x00\x40\x00\x40\x11\x00\x00" +
                   _le(e["src_ip"], 4) + _le(e["dst_ip"], 4))
    c = sum(int.from_bytes(ip[i:i + 2], "big") for i in range(0, 20, 2))
    c = (c & 0xFFFF) + (c >> 16)
    c = (c & 0xFFFF) + (c >> 16)
    ip[10:12] = _be(~c & 0xFFFF, 2)
    udp = _sport(e, h) + _le(e["dport"], 2) + _be(8 + 8 + inner_len, 2) + b"\x00\x00"
    return _l2(e, 0x0800) + bytes(ip) + udp + _shim(e)


def model6(e, inner_len: int, h: int) -> bytes:
    tc = int(e["tc_flow"])
    fl = (tc & 0xFFFFF) or (h & 0xFFFFF)
    vtf = (6 << 28) | (((tc >> 20) & 0xFF) << 20) | fl
    hl = (int(e["hop_limit"]) & 0xFF) or 64
    ip = _be(vtf, 4) + _be(8 + 8 + inner_len, 2) + bytes([17, hl]) + \
        b"".join(_le(w, 4) for w in e["src"]) + b"".join(_le(w, 4) for w in e["dst"])
    udp = _sport(e, h) + _le(e["dport"], 2) + _be(8 + 8 + inner_len, 2) + b"\x00\x00"
    return _l2(e, 0x86DD) + ip + udp + _shim(e)


@pytest.mark.parametrize("v6", [False, True])
def test_outer_headers_match_byte_model(v6):
    nf = nfdp()
    rng = np.random.default_rng(11 + v6)
    dt = T.TUNNEL6_DTYPE if v6 else T.TUNNEL_DTYPE
    for k in range(400):
        e = np.zeros(1, dt)[0]
        for name in dt.names:
            if name == "type":
                e[name] = T.TUN_GENEVE if k % 2 else T.TUN_VXLAN
            elif name == "sport":
                e[name] = 0 if k % 3 == 0 else rng.integers(1, 1 << 16)
            elif name == "tc_flow":
                e[name] = 0 if k % 4 == 0 else rng.integers(0, 1 << 28)
            elif name == "hop_limit":
                e[name] = 0 if k % 5 == 0 else rng.integers(1, 256)
            else:
                info = dt.fields[name][0]
                hi = 1 << (8 * info.base.itemsize)
                e[name] = rng.integers(0, hi, size=info.shape, dtype=np.uint64) if info.shape else rng.integers(0, hi)
        inner_len = int(rng.integers(14, 1500))
        h = int(rng.integers(0, 1 << 32))
        got = nf.make_outer(e.tobytes(), inner_len, h)
        want = (model6 if v6 else model4)(e, inner_len, h)
        assert len(want) == (70 if v6 else 50)
        assert got == want, (k, got.hex(), want.hex())
