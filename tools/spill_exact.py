"""Bit-exactness of a build variant's fused kernel against the C++ oracle over many slots, with the
mismatches (if any) broken down by lane (slot % 64), dword and launch: the check for output
corruption that tracks register spills (docs/DATAPLANE.md "Register budget").

NFDP_EXT_DIR=variants/w5 python tools/spill_exact.py [--slots 4194304] [--seeds 3]
"""
import argparse
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=1 << 22)
    ap.add_argument("--seeds", type=int, default=3)
    a = ap.parse_args()
    out = {}
    for hm in ("lds", "mfma"):
        g = DataPlane(device="cuda", flow_buckets=1 << 14, hash_mode=hm)
        c = DataPlane(device="cpu", flow_buckets=1 << 14, hash_mode=hm)
        for dp in (g, c):
            sc = S.build_sfc(dp, n_pods=8, n_flows=16384, n_acl=256, seed=0)
            dp.commit(full=True)
        bad_slots, lanes, dwords, total = 0, np.zeros(64, np.int64), np.zeros(17, np.int64), 0
        for seed in range(a.seeds):
            pk, im = S.traffic(sc, a.slots, seed=100 + seed)
            r = g.run(torch.from_numpy(pk).cuda(), torch.from_numpy(im.view(np.int32)).cuda())
            torch.cuda.synchronize()
            go, gm = r.out.cpu().numpy(), r.meta.cpu().numpy().view(np.uint32)
            rc = c.run(pk, im)
            d = (go.view(np.uint32).reshape(-1, 16) != rc.out.view(np.uint32).reshape(-1, 16))
            dm = gm != rc.meta
            bad = d.any(1) | dm
            bad_slots += int(bad.sum())
            total += len(pk)
            idx = np.nonzero(bad)[0]
            np.add.at(lanes, idx % 64, 1)
            dwords[:16] += d.sum(0)
            dwords[16] += int(dm.sum())
        out[hm] = {"slots": total, "bad_slots": bad_slots,
                   "bad_by_lane_mod4": [int(lanes[k::4].sum()) for k in range(4)],
                   "bad_dwords": [int(x) for x in dwords[:16]], "bad_meta": int(dwords[16])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
