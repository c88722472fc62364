"""IPsec ESP engine (dataplane/ipsec.py, csrc/nfdp/ipsec.{h,hip}): AES-GCM ESP tunnel / transport
mode, SPD and inbound SA classification, anti-replay, the P4 IPsec tables.

Independent oracle: the system OpenSSL (libcrypto, through ctypes) computes AES-GCM over the same
nonce / AAD / padded payload the ESP frame must carry (RFC 4106: nonce = salt || explicit IV,
AAD = SPI || sequence number); frames are parsed field by field.  Known answer: H = AES-128(0^128)
under the zero key is 66e94bd4ef8a2c3b884cfa59ca342b2e.  The GPU test holds the HIP kernels to the
C++ oracle bit for bit."""
import ctypes
import ctypes.util
import ipaddress

import numpy as np
import pytest

from dpu_operator_amd.dataplane import ipsec as I
from dpu_operator_amd.ops import packets as P

KEY128, KEY256, SALT = bytes(range(16)), bytes(range(100, 132)), b"\xca\xfe\xba\xbe"


def _libcrypto():
    name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
    try:
        lc = ctypes.CDLL(name)
    except OSError:
        return None
    lc.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    lc.EVP_aes_128_gcm.restype = ctypes.c_void_p
    lc.EVP_aes_256_gcm.restype = ctypes.c_void_p
    return lc


LC = _libcrypto()


def gcm_ref(key: bytes, nonce: bytes, aad: bytes, pt: bytes) -> tuple[bytes, bytes]:
    if LC is None:
        pytest.skip("libcrypto not available for the AES-GCM oracle")
    ctx = ctypes.c_void_p(LC.EVP_CIPHER_CTX_new())
    cipher = LC.EVP_aes_128_gcm() if len(key) == 16 else LC.EVP_aes_256_gcm()
    assert LC.EVP_EncryptInit_ex(ctx, ctypes.c_void_p(cipher), None, None, None) == 1
    LC.EVP_CIPHER_CTX_ctrl(ctx, 0x9, len(nonce), None)          # EVP_CTRL_GCM_SET_IVLEN
    assert LC.EVP_EncryptInit_ex(ctx, None, None, key, nonce) == 1
    n = ctypes.c_int(0)
    LC.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad))
    out = ctypes.create_string_buffer(len(pt) + 32)
    LC.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt))
    LC.EVP_EncryptFinal_ex(ctx, ctypes.byref(out, n.value), ctypes.byref(ctypes.c_int(0)))
    tag = ctypes.create_string_buffer(16)
    LC.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, tag)                    # EVP_CTRL_GCM_GET_TAG
    LC.EVP_CIPHER_CTX_free(ctx)
    return out.raw[: len(pt)], tag.raw


def _frames(dsts, sizes, proto=17):
    out = []
    for d, sz in zip(dsts, sizes):
        fr, ln = P.craft_full(1, dmac="02:00:00:00:00:09", smac="02:00:00:00:00:08", src_ip=0x0A000001,
                              dst_ip=int(ipaddress.IPv4Address(d)), sport=1000 + sz, dport=53, proto=proto,
                              frame_len=sz, payload_seed=sz)
        out.append(bytes(fr[0, : ln[0]]))
    return out


def _engine(device="cpu", key=KEY128):
    e = I.IpsecEngine(device=device)
    e.add_sa(0, key=key, salt=SALT, spi=0x1001, mode=I.TUNNEL, src="192.0.2.1", dst="192.0.2.2",
             smac="02:00:00:00:0e:01", dmac="02:00:00:00:0e:02")
    e.add_sa(1, key=KEY256, salt=b"\x01\x02\x03\x04", spi=0x2002, mode=I.TRANSPORT)
    e.set_spd("10.0.0.2", 17, I.PROTECT, 0)
    e.set_spd("10.0.0.3", 17, I.PROTECT, 1)
    e.set_spd("10.0.0.5", 17, I.DROP)
    e.set_spd("10.0.0.6", 17, I.BYPASS)
    return e


def _csum_ok(h: bytes) -> bool:
    w = np.frombuffer(h[:20], ">u2").astype(np.uint32)
    c = int(w.sum())
    c = (c & 0xFFFF) + (c >> 16)
    return ((c & 0xFFFF) + (c >> 16)) & 0xFFFF == 0xFFFF


def test_known_answer_h_and_key_schedule():
    e = I.IpsecEngine()
    e.add_sa(0, key=bytes(16), salt=bytes(4), spi=1)
    w = e.sa[0].view(np.uint64)
    # htab[0x80] = H = E_K(0) as (hi, lo); EspSa: rk 240 B, 8 words, pad 12 B -> htab at byte 288
    hi, lo = int(w[(288 + 0x80 * 16) // 8]), int(w[(288 + 0x80 * 16) // 8 + 1])
    assert f"{hi:016x}{lo:016x}" == "66e94bd4ef8a2c3b884cfa59ca342b2e"


@pytest.mark.parametrize("key", [KEY128, KEY256])
def test_tunnel_mode_matches_openssl(key):
    e = _engine(key=key)
    sizes = [60, 61, 62, 63, 64, 100, 333, 1500, 9000]
    frames = _frames(["10.0.0.2"] * len(sizes), sizes)
    out, st = e.encrypt(frames)
    assert (st == I.DONE).all()
    for k, (f, o) in enumerate(zip(frames, out)):
        inner = f[14:]
        pad = (4 - ((len(inner) + 2) & 3)) & 3
        pt = inner + bytes(range(1, pad + 1)) + bytes([pad, 4])
        assert len(o) == 50 + len(pt) + 16
        assert o[0:6] == bytes.fromhex("02000000 0e02".replace(" ", "")) and o[12:14] == b"\x08\x00"
        assert o[14] == 0x45 and o[23] == 50 and _csum_ok(o[14:34]) and int.from_bytes(o[16:18], "big") == len(o) - 14
        assert o[26:30] == bytes([192, 0, 2, 1]) and o[30:34] == bytes([192, 0, 2, 2])
        assert int.from_bytes(o[34:38], "big") == 0x1001 and int.from_bytes(o[38:42], "big") == k + 1   # in order
        ct, tag = gcm_ref(key, SALT + o[42:50], o[34:42], pt)
        assert o[50: 50 + len(pt)] == ct and o[50 + len(pt):] == tag


def test_transport_mode_matches_openssl_and_round_trips():
    e = _engine()
    e.set_rx_sa("10.0.0.1", "10.0.0.3", 0x2002, 1)
    frames = _frames(["10.0.0.3"] * 4, [60, 200, 777, 1500])
    out, st = e.encrypt(frames)
    assert (st == I.DONE).all()
    for f, o in zip(frames, out):
        l4 = f[34:]
        pad = (4 - ((len(l4) + 2) & 3)) & 3
        pt = l4 + bytes(range(1, pad + 1)) + bytes([pad, 17])
        assert o[:14] == f[:14] and o[23] == 50 and _csum_ok(o[14:34]) and o[26:34] == f[26:34]
        ct, tag = gcm_ref(KEY256, b"\x01\x02\x03\x04" + o[42:50], o[34:42], pt)
        assert o[50:-16] == ct and o[-16:] == tag
    dec, st2 = e.decrypt(out)
    assert (st2 == I.DONE).all()
    assert all(d == f for d, f in zip(dec, frames))       # header, checksum and payload restored


def test_tunnel_round_trip_spd_actions_failures_and_replay():
    e = _engine()
    e.set_rx_sa("192.0.2.1", "192.0.2.2", 0x1001, 0)
    frames = _frames(["10.0.0.2", "10.0.0.4", "10.0.0.5", "10.0.0.6", "10.0.0.2"], [100, 100, 100, 100, 1400])
    out, st = e.encrypt(frames)
    assert list(st) == [I.DONE, I.BYPASSED, I.DROPPED, I.BYPASSED, I.DONE]
    assert out[1] == frames[1] and out[2] is None and out[3] == frames[3]
    dec, st2 = e.decrypt([out[0], out[4]])
    assert (st2 == I.DONE).all()
    for d, f in zip(dec, (frames[0], frames[4])):
        assert d[:12] == bytes.fromhex("020000000e02020000000e01") and d[12:] == f[12:]   # outer MACs, inner packet
    # replay: the same frames again are rejected by the window
    _, st3 = e.decrypt([out[0]])
    assert st3[0] == I.AUTH_FAIL and e.stats["replay"] == 1
    # tampered ciphertext / ICV, unknown SPI
    o2, _ = e.encrypt(_frames(["10.0.0.2"] * 3, [300, 300, 300]))
    bad_ct = bytearray(o2[0]); bad_ct[80] ^= 1
    bad_icv = bytearray(o2[1]); bad_icv[-1] ^= 0x80
    no_sa = bytearray(o2[2]); no_sa[37] ^= 1
    _, st4 = e.decrypt([bytes(bad_ct), bytes(bad_icv), bytes(no_sa)])
    assert list(st4) == [I.AUTH_FAIL, I.AUTH_FAIL, I.NO_SA]


def test_non_ipv4_bypasses_and_sequence_numbers_per_sa():
    e = _engine()
    fr6, ln6 = P.craft6_full(1, dmac="02:00:00:00:00:09", smac="02:00:00:00:00:08", src6="2001:db8::1",
                             dst6=["2001:db8::2"], sport=1, dport=2)
    frames = [bytes(fr6[0, : ln6[0]])] + _frames(["10.0.0.2", "10.0.0.3", "10.0.0.2", "10.0.0.3"], [80] * 4)
    out, st = e.encrypt(frames)
    assert list(st) == [I.BYPASSED, I.DONE, I.DONE, I.DONE, I.DONE]
    seqs = [int.from_bytes(o[38:42], "big") for o in out[1:]]
    assert seqs == [1, 1, 2, 2]                            # each SA counts its own packets, in order


def test_p4_ipsec_tables_compile_onto_the_engine():
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.dataplane.p4rt import P4Runtime

    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    rt = P4Runtime(dp)
    eng = dp.ipsec
    eng.add_sa(5, key=KEY128, salt=SALT, spi=0x55, mode=I.TRANSPORT)
    eng.add_sa(6, key=KEY128, salt=SALT, spi=0x66, mode=I.TRANSPORT)
    C = "linux_networking_control."
    rt.add_entry(C + "ipsec_spd", "hdrs.ipv4[vmeta.common.depth].dst_ip=10.0.0.2,hdrs.ipv4[vmeta.common.depth].protocol=17,"
                 "action=linux_networking_control.ipsec_protect_set_metadata(5)")
    rt.add_entry(C + "ipsec_tx_sa_classification_table", "hdrs.ipv4[vmeta.common.depth].dst_ip=10.0.0.2,"
                 "hdrs.ipv4[vmeta.common.depth].protocol=17,user_meta.cmeta.is_tunnel=1,"
                 "action=linux_networking_control.tx_ipsec_tunnel(192.0.2.9)")
    rt.add_entry(C + "ipsec_tunnel_table", "vmeta.common.saidx=5,bit16_zeros=0,action=linux_networking_control.set_ipsec_tunnel(3)")
    rt.add_entry(C + "ipsec_tunnel_encap_mod_table", "vmeta.common.mod_blob_ptr=3,"
                 "action=linux_networking_control.ipsec_tunnel_encap_mod(192.0.2.8,192.0.2.9,50)")
    rt.add_entry("MainControlDecrypt.ipsec_rx_sa_classification_table",
                 "hdrs.ipv4[vmeta.common.depth].src_ip=192.0.2.9,hdrs.ipv4[vmeta.common.depth].dst_ip=192.0.2.8,"
                 "hdrs.esp.spi=0x66,action=MainControlDecrypt.ipsec_decrypt(6)")
    rt.add_entry(C + "ipv4_ipsec_tunnel_term_table", "ipv4_src=192.0.2.9,ipv4_dst=192.0.2.8,"
                 "action=linux_networking_control.decap_ipsec_tunnel_hdr()")
    assert eng.sa_info[5]["mode"] == I.TUNNEL and eng.sa_info[5]["dst"] == "192.0.2.9"
    assert eng.sa_info[6]["mode"] == I.TUNNEL
    out, st = eng.encrypt(_frames(["10.0.0.2"], [200]))
    assert st[0] == I.DONE and out[0][26:34] == bytes([192, 0, 2, 8, 192, 0, 2, 9])
    from dpu_operator_amd.dataplane.p4rt import P4Error

    with pytest.raises(P4Error) as ei:
        rt.add_entry(C + "ipsec_tx_sa_classification_table", "hdrs.ipv4[vmeta.common.depth].dst_ip=10.0.0.7,"
                     "hdrs.ipv4[vmeta.common.depth].protocol=6,user_meta.cmeta.is_tunnel=1,"
                     "action=linux_networking_control.tx_ipsec_tunnel_v6(1,2,3)")
    assert ei.value.code == "UNIMPLEMENTED"
    # the refused write left nothing behind: the SPD still protects, sequence numbers keep
    # counting (never 0, never reused) and later writes compile
    assert eng.spd_rules and not rt.get_entries(C + "ipsec_tx_sa_classification_table")[1:]
    out2, st2 = eng.encrypt(_frames(["10.0.0.2"] * 3, [200, 300, 400]))
    assert (st2 == I.DONE).all()
    seqs = [int.from_bytes(o[38:42], "big") for o in out2]
    assert seqs == [2, 3, 4]
    rt.add_entry(C + "ipsec_spd", "hdrs.ipv4[vmeta.common.depth].dst_ip=10.0.0.9,hdrs.ipv4[vmeta.common.depth].protocol=17,"
                 "action=linux_networking_control.ipsec_bypass()")
    assert len(eng.spd_rules) == 2


def test_failed_compile_rolls_back_the_write():
    """A write whose compile fails is taken back out: the runtime is not stuck on it."""
    from dpu_operator_amd.dataplane.engine import DataPlane
    from dpu_operator_amd.dataplane.p4rt import P4Runtime

    dp = DataPlane(device="cpu", flow_buckets=1 << 10)
    rt = P4Runtime(dp)
    C = "linux_networking_control."
    calls = {"n": 0}
    real = rt._compile_ipsec

    def boom(d):
        calls["n"] += 1
        if calls["n"] == 2:
            raise RuntimeError("injected compile failure")
        return real(d)

    rt._compile_ipsec = boom
    rt.add_entry(C + "ipsec_spd", "hdrs.ipv4[vmeta.common.depth].dst_ip=10.0.0.2,hdrs.ipv4[vmeta.common.depth].protocol=17,"
                 "action=linux_networking_control.ipsec_bypass()")
    with pytest.raises(RuntimeError):
        rt.add_entry(C + "ipsec_spd", "hdrs.ipv4[vmeta.common.depth].dst_ip=10.0.0.3,hdrs.ipv4[vmeta.common.depth].protocol=17,"
                     "action=linux_networking_control.ipsec_bypass()")
    assert len(rt.get_entries(C + "ipsec_spd")) == 1
    rt.add_entry(C + "ipsec_spd", "hdrs.ipv4[vmeta.common.depth].dst_ip=10.0.0.4,hdrs.ipv4[vmeta.common.depth].protocol=17,"
                 "action=linux_networking_control.ipsec_bypass()")
    assert len(dp.ipsec.spd_rules) == 2


def test_sequence_space_exhaustion_stops_protecting_and_asks_for_a_rekey():
    """RFC 4303 3.3.3: the outbound counter never cycles.  Near 2^32 the last numbers go out,
    then the SA protects nothing more (drop, never IV reuse) and the control plane is asked to
    rekey; re-installing the same key keeps the counter, a new key restarts it."""
    e = _engine()
    asked = []
    e.on_rekey = asked.append
    e.next_seq[0] = I.SEQ_MAX - 1
    out, st = e.encrypt(_frames(["10.0.0.2"] * 4, [100] * 4))
    assert list(st) == [I.DONE, I.DONE, I.DROPPED, I.DROPPED]
    assert [int.from_bytes(o[38:42], "big") for o in out[:2]] == [I.SEQ_MAX - 1, I.SEQ_MAX]
    assert out[2] is None and out[3] is None and asked == [0] and e.stats["seq_exhausted"] == 2
    # same key material again (a restart): still exhausted, nothing is sent with a reused nonce
    e.add_sa(0, key=KEY128, salt=SALT, spi=0x1001, mode=I.TUNNEL, src="192.0.2.1", dst="192.0.2.2",
             smac="02:00:00:00:0e:01", dmac="02:00:00:00:0e:02")
    _, st2 = e.encrypt(_frames(["10.0.0.2"], [100]))
    assert st2[0] == I.DROPPED
    # a new key: counting restarts at 1
    e.add_sa(0, key=bytes(range(50, 66)), salt=SALT, spi=0x1003, mode=I.TUNNEL, src="192.0.2.1", dst="192.0.2.2")
    out3, st3 = e.encrypt(_frames(["10.0.0.2"], [100]))
    assert st3[0] == I.DONE and int.from_bytes(out3[0][38:42], "big") == 1


def test_packets_the_host_spd_does_not_protect_are_never_sent_with_seq_0():
    """Stale device SPD vs an emptied host rule set: the kernel sees seq 0 and drops."""
    e = _engine()
    e._device_tables()                 # device copy says PROTECT
    e.spd_rules.clear()                # host rules gone without a rebuild (the advisor's case)
    out, st = e.encrypt(_frames(["10.0.0.2"], [100]))
    assert st[0] == I.DROPPED and out[0] is None


@pytest.mark.gpu
def test_esp_gpu_bit_exact_and_round_trip():
    import torch

    c, g = _engine("cpu"), _engine("cuda")
    for e in (c, g):
        e.set_rx_sa("192.0.2.1", "192.0.2.2", 0x1001, 0)
    rng = np.random.default_rng(5)
    n = 3000
    dsts = [("10.0.0.2", "10.0.0.3", "10.0.0.4", "10.0.0.5")[k] for k in rng.integers(0, 4, n)]
    sizes = rng.integers(60, 1515, n)
    frames = _frames(dsts, sizes)
    oc, sc = c.encrypt(frames)
    og, sg = g.encrypt(frames)
    assert np.array_equal(sc, sg) and oc == og
    torch.cuda.synchronize()
    tun = [o for o, s, d in zip(oc, sc, dsts) if s == I.DONE and d == "10.0.0.2"]
    dc, s2 = c.decrypt(tun)
    dg, s3 = g.decrypt(tun)
    assert np.array_equal(s2, s3) and (s3 == I.DONE).all() and dc == dg
