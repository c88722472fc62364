"""How many ACL rule tiles / groups a wave of 64 packets runs, from the host's tile layout
(host.cpp build_acl_frags) and the prefilters - the ClassBench-style set (scenario.install_acl_wild)
over the headline's pod traffic.  CPU only.

r5 s10: 1726 ternary entries, 108 tiles, 14 groups; 9 groups pass every wave (72 tiles run with
group prefilters), 37 tiles can match.  Running only those (NFDP_ACL_PTILES) measured slower.
r6: with the rules placed source-first (host.cpp NFDP_ACL_ORDER=1) 29 tiles can match; the group
prefilters still pass 68.  Measured (profiles/r6_s20_*, r6_s21_*): prefilter tiles 7,386 Mpps,
+ source-first 8,060, + a batched cursor over them 7,217, against 8,002 for the group-prefilter
default - the 2-wave instance waits on its memory latency, not on its tile count.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.native import nfdp  # noqa: E402


def passes(rows: np.ndarray, keys: np.ndarray) -> np.ndarray:
    """[waves, rows]: some packet of the wave passes the (mask, value) row."""
    x = (keys[:, None, :] & rows[None, :, :4]) ^ rows[None, :, 4:]
    ok = (x == 0).all(axis=2)
    w = len(keys) // 64
    return ok[: w * 64].reshape(w, 64, -1).any(axis=1)


def main() -> None:
    nf = nfdp()
    dp = DataPlane(device="cpu", flow_buckets=1 << 16)
    sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 16, n_acl=256, seed=0)
    S.install_acl_wild(dp, 1024)
    val, msk, _, n = dp.acl.arrays()
    w, c, tiles = nf.build_acl_frags(np.ascontiguousarray(val[:n]), np.ascontiguousarray(msk[:n]))
    tiles = int(tiles)
    c = np.asarray(c).view(np.uint32).ravel()
    pf = c[tiles * 16: tiles * 24].reshape(tiles, 8)
    ng = (tiles + 7) // 8
    gpf = c[tiles * 24: tiles * 24 + ng * 8].reshape(ng, 8)
    _, _, f = S.traffic(sc, 1 << 16, seed=9001, return_flows=True)
    keys = sc.keys[f].astype(np.uint32)
    gp, tp = passes(gpf, keys), passes(pf, keys)
    print(f"entries {n} tiles {tiles} groups {ng}")
    print(f"groups passing per wave {gp.sum(1).mean():.2f} -> tiles run {gp.sum(1).mean() * 8:.1f}; "
          f"tiles that can match {tp.sum(1).mean():.1f}")


if __name__ == "__main__":
    main()
