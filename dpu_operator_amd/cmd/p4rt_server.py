"""`p4rt-server` — the pipeline server (the role of the reference's P4 "infrapod": infrap4d +
set-pipe, vendor/.../infrapod/infrapod.go).

Hosts bridge `br0` on a DataPlane (GPU by default) behind the p4rt-ctl service on --address
(127.0.0.1:9559), loads the MI355X linux-networking P4Info (or --p4info FILE), optional LAG
group -> port mapping (--lag 0:4093).
"""
from __future__ import annotations

import argparse
import logging
import signal
import sys
import threading


def main(argv=None, stop: threading.Event | None = None, dataplane=None) -> int:
    ap = argparse.ArgumentParser(prog="p4rt-server")
    ap.add_argument("--address", default="127.0.0.1:9559")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--flow-buckets", type=int, default=1 << 16)
    ap.add_argument("--p4info", default="")
    ap.add_argument("--lag", action="append", default=[])
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ..dataplane.p4info import MI355X_P4INFO, MI355X_P4INFO_TEXT, P4Info
    from ..dataplane.p4rt import P4Runtime
    from ..dataplane.p4server import P4rtServer

    if dataplane is None:
        from ..dataplane.engine import DataPlane

        dataplane = DataPlane(device=a.device, flow_buckets=a.flow_buckets)
        dataplane.commit(full=True)
    text = open(a.p4info).read() if a.p4info else MI355X_P4INFO_TEXT
    info = P4Info.from_text(text) if a.p4info else MI355X_P4INFO
    lag = {int(g): int(p) for g, p in (x.split(":") for x in a.lag)}
    srv = P4rtServer({"br0": P4Runtime(dataplane, info, lag_ports=lag)}, text).start(a.address)
    print(f"p4rt-server listening on port {srv.port}", flush=True)
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    srv.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
