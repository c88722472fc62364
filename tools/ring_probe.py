"""Ring-kernel latency / throughput sweep on one GPU (cost attribution for csrc/nfdp/ring.hip).

RTT = host publish -> host sees the completion flag (steady clock); svc = device time from
the chunk becoming visible to its flag store (s_memrealtime, 10 ns ticks).
"""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
from dpu_operator_amd.dataplane import scenario as S  # noqa: E402
from dpu_operator_amd.dataplane.engine import DataPlane  # noqa: E402
from dpu_operator_amd.dataplane.ring import RingPath  # noqa: E402


def main():
    dp = DataPlane(device="cuda", flow_buckets=1 << 19, hash_mode="lds", acl_mode="mfma")
    sc = S.build_sfc(dp, n_pods=8, n_flows=1 << 20, n_acl=256, seed=0)
    dp.commit(full=True)
    pk, im = S.traffic(sc, 1 << 16, seed=1)
    rows = []
    for wgs, knobs, coop in ((1, 0, True), (1, 32, True), (1, 0, False), (1, 64, False), (2, 0, False)):
        ring = RingPath(dp, capacity=1 << 16, wgs_per_cu=wgs, deadline_s=60.0, knobs=knobs, coop=coop)
        ring.stage(pk, im)
        ring.start()
        res = {"wgs": wgs, "knobs": knobs, "coop": coop}
        for batch, inflight, nb in ((64, 16, 3000), (1024, 16, 2000), (4096, 16, 1000), (8192, 7, 500), (64, 1, 3000)):
            lat, el = ring.probe(nb, batch, inflight)
            lat = lat[nb // 10:]
            res[f"b{batch}x{inflight}"] = {"p50_us": round(float(np.median(lat)), 2),
                                           "p99_us": round(float(np.percentile(lat, 99)), 2),
                                           "mpps": round(nb * batch / el / 1e6, 1)}
        ring.stop()
        svc = ring.service_ticks().astype(np.float64) * 0.01
        res["svc_p50_us"] = round(float(np.median(svc[svc > 0])), 2)
        if knobs & 32:
            ph = ring.service_ticks(phases=True).astype(np.float64) * 0.01
            ph = ph[ph[:, 7] > 0]
            res["phases_p50_us"] = {n: round(float(np.median(ph[:, k])), 2) for k, n in enumerate(
                ["frame", "ingress+classify", "probe", "chain+emit+store", "fence", "counters(after flag)", "_", "total"])}
        ring.close()
        rows.append(res)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
