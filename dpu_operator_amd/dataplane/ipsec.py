"""IPsec ESP engine of the data plane: AES-GCM (RFC 4106) tunnel and transport mode on MI355X.

The reference's IPU runs IPsec in its inline crypto engine; its P4 program only classifies
(``ipsec_spd``, ``ipsec_tx_sa_classification_table``, ``ipsec_tunnel_table``,
``ipsec_tunnel_encap_mod_table``, ``ipsec_rx_sa_classification_table``,
``ipv4_ipsec_tunnel_term_table``: fxp-net_linux-networking.p4info.txt).  Here the crypto itself is
a HIP kernel over whole frames at the port boundary (``csrc/nfdp/ipsec.{h,hip}``): outbound frames
leaving an IPsec port are looked up in the SPD and encapsulated, inbound ESP is classified by
(outer src, outer dst, SPI), authenticated and decrypted, then handed to the header pipeline.

Host duties: SA material (key schedule, GHASH tables: ``esp_build_sa``), per-SA outbound
sequence numbers allocated in batch order (so receivers' replay windows see them in order), and
the RFC 4303 anti-replay window on inbound (64 packets).  Frames are staged in fixed-stride
slots: cleartext at slot + 2, ESP at slot + 14, so every crypto word access is aligned.
"""
from __future__ import annotations

import ipaddress

import numpy as np

from ..native import nfdp as _nfdp_mod
from ..ops.packets import ip_raw, mac_raw
from .tables import fmix32

SPD_DTYPE = np.dtype([("dst_ip", "<u4"), ("proto", "u1"), ("action", "u1"), ("sa", "<u2"), ("pad", "<u4", (2,))])
RXSA_DTYPE = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("spi", "<u4"), ("sa", "<u2"), ("valid", "<u2")])
assert SPD_DTYPE.itemsize == 16 and RXSA_DTYPE.itemsize == 16

TUNNEL, TRANSPORT = 1, 2
PROTECT, BYPASS, DROP = 1, 2, 3
BYPASSED, DONE, DROPPED, AUTH_FAIL, NO_SA = 0, 1, 2, 3, 4
STATUS = {BYPASSED: "bypass", DONE: "done", DROPPED: "drop", AUTH_FAIL: "auth_fail", NO_SA: "no_sa"}
CLEAR_OFF, ESP_OFF = 2, 14
ESP_OVERHEAD = 50 + 16 + 3 + 2     # outer header + ICV + worst-case padding + trailer
REPLAY_WINDOW = 64
SEQ_MAX = 0xFFFFFFFF                # last outbound sequence number of an SA (no extended sequence numbers)


def _raw_ip(ip) -> int:
    return int(ip_raw(np.uint32(int(ipaddress.IPv4Address(ip)) if not isinstance(ip, (int, np.integer)) else int(ip))))


def _h32(x) -> int:
    with np.errstate(over="ignore"):
        return int(fmix32(np.uint32(int(x) & 0xFFFFFFFF)))


class IpsecEngine:
    """SA database + SPD + inbound SA classification, and the ESP kernels over frame batches."""

    def __init__(self, device: str = "cpu", max_sa: int = 1024, spd_slots: int = 1024, rx_slots: int = 1024,
                 num_cus: int = 256):
        self.nf = _nfdp_mod()
        self.device = device
        self.gpu = device != "cpu"
        self.num_cus = num_cus
        self.sa = np.zeros((max_sa, int(self.nf.ESP_SA_BYTES)), np.uint8)
        self.sa_info: dict[int, dict] = {}
        self.spd = np.zeros(spd_slots, SPD_DTYPE)
        self.rxsa = np.zeros(rx_slots, RXSA_DTYPE)
        self.spd_rules: dict[tuple[int, int], tuple[int, int]] = {}     # (dst raw, proto) -> (action, sa)
        self.rx_rules: dict[tuple[int, int, int], int] = {}            # (src raw, dst raw, spi) -> sa
        self.next_seq = np.ones(max_sa, np.uint64)                     # outbound: next sequence number
        self.replay: dict[int, list[int]] = {}                         # inbound: sa -> [top, bitmap]
        # SAs whose 32-bit outbound sequence space is used up: they protect nothing more (their
        # packets are dropped) until the control plane installs a new key (`on_rekey(sa)` asks)
        self.exhausted: set[int] = set()
        self.on_rekey = None
        self.version = 0
        self._dev: dict[str, object] = {}
        self._dev_version = -1
        self.stats = {k: 0 for k in ("enc", "dec", "bypass", "drop", "auth_fail", "no_sa", "replay", "seq_exhausted")}
        te0, sbox, rem = self.nf.esp_tables()
        self._tabs = (np.frombuffer(te0, np.uint32).copy(), np.frombuffer(sbox, np.uint8).copy(),
                      np.frombuffer(rem, np.uint64).copy())

    # ------------------------------------------------------------------ control plane
    def add_sa(self, idx: int, *, key: bytes, salt: bytes, spi: int, mode: int = TUNNEL, src=0, dst=0,
               smac="00:00:00:00:00:00", dmac="00:00:00:00:00:00") -> None:
        """SA `idx`: AES-GCM key (16 / 32 B), 4-B salt, SPI; tunnel outer addresses / MACs."""
        if not 0 <= idx < len(self.sa):
            raise ValueError("SA index out of range")
        slo, shi = mac_raw(smac)
        dlo, dhi = mac_raw(dmac)
        raw = self.nf.esp_build_sa(bytes(key), bytes(salt), spi & 0xFFFFFFFF, mode, _raw_ip(src), _raw_ip(dst),
                                   int(slo), int(shi), int(dlo), int(dhi))
        ident = (bytes(key), bytes(salt), spi & 0xFFFFFFFF)
        prev = self.sa_info.get(idx)
        self.sa[idx] = np.frombuffer(raw, np.uint8)
        self.sa_info[idx] = {"spi": spi, "mode": mode, "src": src, "dst": dst, "ident": ident}
        if prev is None or prev.get("ident") != ident:
            # a new key: its counters start over.  Re-installing the SAME key material (a restart,
            # a mode change) keeps them: resetting would reuse GCM nonces under that key.
            self.next_seq[idx] = 1
            self.replay.pop(idx, None)
            self.exhausted.discard(idx)
        self.version += 1

    def set_sa_mode(self, idx: int, mode: int, src=None, dst=None) -> None:
        """Change an SA's encapsulation (P4 tx SA classification / tunnel encap tables)."""
        info = self.sa_info.get(idx)
        if info is None:
            raise KeyError(f"no SA {idx}")
        w = self.sa[idx].view(np.uint32)
        # EspSa words: rk[0..59], nr 60, salt 61, spi 62, mode 63, src_ip 64, dst_ip 65
        w[63] = mode
        if src is not None:
            w[64] = _raw_ip(src)
        if dst is not None:
            w[65] = _raw_ip(dst)
        info.update(mode=mode, **({"src": src} if src is not None else {}), **({"dst": dst} if dst is not None else {}))
        self.version += 1

    def remove_sa(self, idx: int) -> None:
        self.sa[idx] = 0
        self.sa_info.pop(idx, None)
        self.version += 1

    def set_spd(self, dst, proto: int, action: int, sa: int = 0) -> None:
        self.spd_rules[(_raw_ip(dst), proto & 0xFF)] = (action, sa)
        self._rebuild_spd()

    def remove_spd(self, dst, proto: int) -> None:
        self.spd_rules.pop((_raw_ip(dst), proto & 0xFF), None)
        self._rebuild_spd()

    def set_rx_sa(self, src, dst, spi: int, sa: int) -> None:
        self.rx_rules[(_raw_ip(src), _raw_ip(dst), spi & 0xFFFFFFFF)] = sa
        self._rebuild_rx()

    def remove_rx_sa(self, src, dst, spi: int) -> None:
        self.rx_rules.pop((_raw_ip(src), _raw_ip(dst), spi & 0xFFFFFFFF), None)
        self._rebuild_rx()

    def _rebuild_spd(self) -> None:
        self.spd[:] = np.zeros((), SPD_DTYPE)
        m = len(self.spd) - 1
        for (d, p), (act, sa) in self.spd_rules.items():
            h = _h32(d ^ ((p * 0x9E3779B1) & 0xFFFFFFFF))
            for q in range(8):
                i = (h + q) & m
                if self.spd[i]["action"] == 0:
                    self.spd[i] = (d, p, act, sa, (0, 0))
                    break
            else:
                raise RuntimeError("SPD probe limit reached")
        self.version += 1

    def _rebuild_rx(self) -> None:
        self.rxsa[:] = np.zeros((), RXSA_DTYPE)
        m = len(self.rxsa) - 1
        for (s, d, spi), sa in self.rx_rules.items():
            h = _h32(s ^ ((d * 0x85EBCA6B) & 0xFFFFFFFF) ^ ((spi * 0xC2B2AE35) & 0xFFFFFFFF))
            for q in range(8):
                i = (h + q) & m
                if not self.rxsa[i]["valid"]:
                    self.rxsa[i] = (s, d, spi, sa, 1)
                    break
            else:
                raise RuntimeError("RX SA probe limit reached")
        self.version += 1

    # ------------------------------------------------------------------ staging
    @staticmethod
    def _stride(n: int) -> int:
        return (n + 15) & ~15

    def stage(self, frames, headroom: int, extra: int) -> tuple[np.ndarray, np.ndarray, int]:
        """Frames -> (arena [n, stride], lengths, stride) with the frame at slot + headroom."""
        lens = np.array([len(f) for f in frames], np.uint32)
        stride = self._stride(int(lens.max(initial=0)) + headroom + extra + 8)
        arena = np.zeros((len(frames), max(stride, 128)), np.uint8)
        for i, f in enumerate(frames):
            arena[i, headroom: headroom + len(f)] = np.frombuffer(bytes(f), np.uint8)
        return arena, lens, arena.shape[1]

    def assign_seq(self, arena: np.ndarray, lens: np.ndarray) -> np.ndarray:
        """Outbound sequence numbers: the packets the SPD protects with SA s get the next numbers
        of s in batch order (vectorised mirror of the kernel's SPD lookup)."""
        n = len(lens)
        seq = np.zeros(n, np.uint32)
        if not n or not self.spd_rules:
            return seq
        o = CLEAR_OFF
        ipv4 = (arena[:, o + 12] == 8) & (arena[:, o + 13] == 0) & ((arena[:, o + 14] >> 4) == 4) & (lens >= 34)
        dst = arena[:, o + 30: o + 34].copy().view("<u4").reshape(-1)
        proto = arena[:, o + 23]
        sa = np.full(n, -1, np.int64)
        for (d, p), (act, s) in self.spd_rules.items():
            if act == PROTECT:
                sa[ipv4 & (dst == d) & (proto == p)] = s
        for s in np.unique(sa[sa >= 0]):
            idx = np.nonzero(sa == s)[0]
            base = int(self.next_seq[s])
            # sequence numbers 1 .. 2^32 - 1, never cycled (RFC 4303 3.3.3); past the end a packet
            # gets 0, which the kernel drops
            ok = max(0, min(len(idx), SEQ_MAX + 1 - base))
            seq[idx[:ok]] = base + np.arange(ok, dtype=np.int64)
            self.next_seq[s] = base + ok
            if ok < len(idx):
                self.stats["seq_exhausted"] += len(idx) - ok
                if s not in self.exhausted:
                    self.exhausted.add(int(s))
                    if self.on_rekey is not None:
                        self.on_rekey(int(s))
        return seq

    def replace_rules(self, spd: dict, rx: dict, sa_modes=()) -> None:
        """Swap in a complete SPD / inbound-SA rule set at once (P4 compile): both device arrays
        are rebuilt from the new sets, and the SA modes applied, only after everything is known."""
        old_spd, old_rx = self.spd_rules, self.rx_rules
        self.spd_rules = {(_raw_ip(d), p & 0xFF): v for (d, p), v in spd.items()}
        self.rx_rules = {(_raw_ip(s), _raw_ip(d), spi & 0xFFFFFFFF): sa for (s, d, spi), sa in rx.items()}
        try:
            self._rebuild_spd()
            self._rebuild_rx()
        except Exception:
            self.spd_rules, self.rx_rules = old_spd, old_rx
            self._rebuild_spd()
            self._rebuild_rx()
            raise
        for sa, mode, src, dst in sa_modes:
            self.set_sa_mode(sa, mode, src=src, dst=dst)

    def _device_tables(self):
        if self._dev_version == self.version and self._dev:
            return self._dev
        if self.gpu:
            import torch

            up = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(self.device)  # noqa: E731
        else:
            up = lambda a: np.ascontiguousarray(a).copy()  # noqa: E731
        self._dev = {"sa": up(self.sa), "spd": up(self.spd), "rxsa": up(self.rxsa),
                     "te0": up(self._tabs[0]), "sbox": up(self._tabs[1]), "rem": up(self._tabs[2])}
        self._dev_version = self.version
        return self._dev

    def _ptr(self, x) -> int:
        return int(x.data_ptr()) if self.gpu else int(x.ctypes.data)

    # ------------------------------------------------------------------ batches
    def run_staged(self, enc: bool, arena, lens, stride: int, out_stride: int, seq=None, stream=None) -> dict:
        """Run the kernel (or the CPU oracle) over staged slots; device tensors or numpy arrays.
        Returns the output arena and per-packet lengths / status (and SA / seq inbound)."""
        n = int(lens.shape[0])
        t = self._device_tables()
        if self.gpu:
            import torch

            z = lambda *s, dt=torch.int32: torch.zeros(*s, dtype=dt, device=self.device)  # noqa: E731
            out = z(n, out_stride, dt=torch.uint8)
            out_len, status, out_sa, out_seq = z(n), z(n), z(n), z(n)
        else:
            out = np.zeros((n, out_stride), np.uint8)
            out_len, status, out_sa, out_seq = (np.zeros(n, np.uint32) for _ in range(4))
        d = {"in": self._ptr(arena), "in_stride": stride, "in_len": self._ptr(lens), "out": self._ptr(out),
             "out_stride": out_stride, "out_len": self._ptr(out_len), "status": self._ptr(status),
             "sa": self._ptr(t["sa"]), "n_sa": len(self.sa), "n": n,
             "spd": self._ptr(t["spd"]), "spd_mask": len(self.spd) - 1,
             "rxsa": self._ptr(t["rxsa"]), "rxsa_mask": len(self.rxsa) - 1,
             "out_sa": self._ptr(out_sa), "out_seq": self._ptr(out_seq)}
        if enc:
            d["seq"] = self._ptr(seq)
        if self.gpu:
            import torch

            s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
            self.nf.launch_esp(enc, d, self._ptr(t["te0"]), self._ptr(t["sbox"]), self._ptr(t["rem"]), self.num_cus, s)
        else:
            self.nf.esp_run_cpu(enc, d)
        return {"out": out, "len": out_len, "status": status, "sa": out_sa, "seq": out_seq}

    def encrypt(self, frames) -> tuple[list[bytes | None], np.ndarray]:
        """Outbound: per frame the ESP frame (protected), the frame itself (bypass) or None (drop)."""
        if not frames:
            return [], np.zeros(0, np.uint32)
        arena, lens, stride = self.stage(frames, CLEAR_OFF, 0)
        seq = self.assign_seq(arena, lens)
        out_stride = self._stride(int(lens.max()) + ESP_OFF + ESP_OVERHEAD + 8)
        r = self._run_host(True, arena, lens, stride, out_stride, seq)
        res = []
        for i, f in enumerate(frames):
            st = int(r["status"][i])
            if st == DONE:
                res.append(bytes(r["out"][i, ESP_OFF: ESP_OFF + int(r["len"][i])]))
                self.stats["enc"] += 1
            elif st == BYPASSED:
                res.append(bytes(f))
                self.stats["bypass"] += 1
            else:
                res.append(None)
                self.stats["drop"] += 1
        return res, r["status"]

    def decrypt(self, frames) -> tuple[list[bytes | None], np.ndarray]:
        """Inbound ESP: per frame the decrypted frame, or None (status says why: no SA -> slow
        path, auth failure / replay -> drop)."""
        if not frames:
            return [], np.zeros(0, np.uint32)
        arena, lens, stride = self.stage(frames, ESP_OFF, 0)
        out_stride = self._stride(int(lens.max()) + CLEAR_OFF + 8)
        r = self._run_host(False, arena, lens, stride, out_stride, None)
        res = []
        status = r["status"].copy()
        for i in range(len(frames)):
            st = int(status[i])
            if st == DONE and not self._replay_ok(int(r["sa"][i]), int(r["seq"][i])):
                status[i] = AUTH_FAIL
                self.stats["replay"] += 1
                res.append(None)
                continue
            if st == DONE:
                res.append(bytes(r["out"][i, CLEAR_OFF: CLEAR_OFF + int(r["len"][i])]))
                self.stats["dec"] += 1
            else:
                res.append(None)
                self.stats[{AUTH_FAIL: "auth_fail", NO_SA: "no_sa"}.get(st, "drop")] += 1
        return res, status

    def _run_host(self, enc, arena, lens, stride, out_stride, seq) -> dict:
        if self.gpu:
            import torch

            dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)  # noqa: E731
            r = self.run_staged(enc, dev(arena), dev(lens.view(np.int32)), stride, out_stride,
                                dev(seq.view(np.int32)) if seq is not None else None)
            torch.cuda.synchronize()
            return {k: (v.cpu().numpy().view(np.uint32) if v.dtype != torch.uint8 else v.cpu().numpy()) for k, v in r.items()}
        return self.run_staged(enc, arena, lens, stride, out_stride, seq)

    def _replay_ok(self, sa: int, seq: int) -> bool:
        """RFC 4303 3.4.3 sliding window (64), updated for authenticated packets only."""
        top, bits = self.replay.get(sa, [0, 0])
        if seq == 0:
            return False
        if seq > top:
            shift = seq - top
            bits = ((bits << shift) | 1) & ((1 << REPLAY_WINDOW) - 1) if shift < REPLAY_WINDOW else 1
            self.replay[sa] = [seq, bits]
            return True
        off = top - seq
        if off >= REPLAY_WINDOW or (bits >> off) & 1:
            return False
        self.replay[sa] = [top, bits | (1 << off)]
        return True
