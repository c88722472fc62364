"""ESP (AES-GCM) kernel throughput on one MI355X: device-resident frame batches, encrypt (tunnel
mode, SPD lookup + encap + AES-GCM) and decrypt (SA lookup + auth + decap) of the same batch.
One JSON line per frame size.  python tools/esp_bench.py [--sizes 64,512,1400] [--n 262144]
"""
import argparse
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import ipsec as I  # noqa: E402
from dpu_operator_amd.ops import packets as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,512,1400")
    ap.add_argument("--n", type=int, default=1 << 18)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--key-bits", type=int, default=128)
    a = ap.parse_args()
    props = torch.cuda.get_device_properties(0)
    e = I.IpsecEngine(device="cuda", num_cus=props.multi_processor_count)
    key = bytes(range(a.key_bits // 8))
    e.add_sa(0, key=key, salt=b"\x01\x02\x03\x04", spi=0x100, mode=I.TUNNEL, src="192.0.2.1", dst="192.0.2.2")
    e.set_spd("10.0.0.2", 17, I.PROTECT, 0)
    e.set_rx_sa("192.0.2.1", "192.0.2.2", 0x100, 0)
    for sz in [int(s) for s in a.sizes.split(",")]:
        fr, ln = P.craft_full(a.n, dmac="02:00:00:00:00:09", smac="02:00:00:00:00:08", src_ip=0x0A000001,
                              dst_ip=0x0A000002, sport=np.arange(a.n) % 60000 + 1, dport=53, frame_len=sz)
        L = int(ln[0])
        stride = (L + I.CLEAR_OFF + 8 + 15) & ~15
        arena = np.zeros((a.n, max(stride, 128)), np.uint8)
        arena[:, I.CLEAR_OFF: I.CLEAR_OFF + L] = fr[:, :L]
        seq = e.assign_seq(arena, ln.astype(np.uint32))
        d_in = torch.from_numpy(arena).cuda()
        d_len = torch.from_numpy(ln.astype(np.uint32).view(np.int32)).cuda()
        d_seq = torch.from_numpy(seq.view(np.int32)).cuda()
        ostride = (L + I.ESP_OFF + I.ESP_OVERHEAD + 8 + 15) & ~15
        r = e.run_staged(True, d_in, d_len, arena.shape[1], ostride, d_seq)
        torch.cuda.synchronize()
        ok_enc = bool((r["status"] == I.DONE).all().item())
        t0 = time.perf_counter()
        for _ in range(a.steps):
            r = e.run_staged(True, d_in, d_len, arena.shape[1], ostride, d_seq)
        torch.cuda.synchronize()
        t_enc = (time.perf_counter() - t0) / a.steps
        esp, esp_len = r["out"], r["len"]
        dstride = (int(esp_len.max().item()) + I.CLEAR_OFF + 8 + 15) & ~15
        r2 = e.run_staged(False, esp, esp_len, ostride, max(dstride, 128))
        torch.cuda.synchronize()
        ok_dec = bool((r2["status"] == I.DONE).all().item())
        same = bool(torch.equal(r2["out"][:, I.CLEAR_OFF + 14: I.CLEAR_OFF + L], d_in[:, I.CLEAR_OFF + 14: I.CLEAR_OFF + L]))
        t0 = time.perf_counter()
        for _ in range(a.steps):
            r2 = e.run_staged(False, esp, esp_len, ostride, max(dstride, 128))
        torch.cuda.synchronize()
        t_dec = (time.perf_counter() - t0) / a.steps
        print(json.dumps({"frame_bytes": L + 4, "packets": a.n, "key_bits": a.key_bits,
                          "encrypt_mpps": round(a.n / t_enc / 1e6, 1), "encrypt_gbps": round(a.n * L * 8 / t_enc / 1e9, 1),
                          "decrypt_mpps": round(a.n / t_dec / 1e6, 1), "decrypt_gbps": round(a.n * L * 8 / t_dec / 1e9, 1),
                          "encrypt_ms": round(t_enc * 1e3, 3), "decrypt_ms": round(t_dec * 1e3, 3),
                          "all_encrypted": ok_enc, "all_authenticated": ok_dec, "round_trip_equal": same}), flush=True)
        del d_in, r, r2, esp


if __name__ == "__main__":
    main()
