"""`p4rt-server` — the pipeline server (the role of the reference's P4 "infrapod": infrap4d +
set-pipe, vendor/.../infrapod/infrapod.go).

Hosts bridge `br0` on a DataPlane (GPU by default) behind the p4rt-ctl service on --address
(127.0.0.1:9559), loads the MI355X linux-networking P4Info (or --p4info FILE), optional LAG
group -> port mapping (--lag 0:4093).

--gpus N|all: the pipeline spans the node's GPUs (dataplane/multi.py MultiDataPlane): P4 entries are
compiled ONCE into the shared table models and every commit replicates them to each GPU; flows
are sharded by RSS owner.  --memif PORT=PATH (repeatable): live shared-memory ports served by the
native I/O engine (--io-queues rx threads), frames steered to their owner GPU.
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
    ap.add_argument("--gpus", default="1", help="GPUs behind the pipeline (a number or 'all')")
    ap.add_argument("--memif", action="append", default=[], help="PORT=PATH: a live shared-memory port")
    ap.add_argument("--io-queues", type=int, default=2)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    from ..dataplane.p4info import MI355X_P4INFO, MI355X_P4INFO_TEXT, P4Info
    from ..dataplane.p4rt import P4Runtime
    from ..dataplane.p4server import P4rtServer

    if dataplane is None:
        dataplane = build_dataplane(a.device, a.gpus, a.flow_buckets)
    text = open(a.p4info).read() if a.p4info else MI355X_P4INFO_TEXT
    info = P4Info.from_text(text) if a.p4info else MI355X_P4INFO
    lag = {int(g): int(p) for g, p in (x.split(":") for x in a.lag)}
    srv = P4rtServer({"br0": P4Runtime(dataplane, info, lag_ports=lag)}, text).start(a.address)
    live = None
    if a.memif:
        from ..dataplane.native_io import MemifVport, NativeLivePath

        ports = {int(k): MemifVport(v) for k, v in (x.split("=", 1) for x in a.memif)}
        live = NativeLivePath(dataplane, ports, queues=a.io_queues).start()
    print(f"p4rt-server listening on port {srv.port}", flush=True)
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    if live is not None:
        live.stop()
    srv.stop()
    return 0


def build_dataplane(device: str, gpus="1", flow_buckets: int = 1 << 16):
    """One DataPlane, or a MultiDataPlane over `gpus` devices (CPU oracle planes without a GPU)."""
    from ..dataplane.engine import DataPlane
    from ..dataplane.multi import MultiDataPlane, visible_devices

    n = len(visible_devices()) if gpus == "all" and device != "cpu" else (1 if gpus == "all" else int(gpus))
    if n <= 1:
        dp = DataPlane(device=device, flow_buckets=flow_buckets)
    else:
        devs = [f"cuda:{i}" for i in range(n)] if device != "cpu" else ["cpu"] * n
        dp = MultiDataPlane(devs, flow_buckets=flow_buckets)
    dp.commit(full=True)
    return dp


if __name__ == "__main__":
    sys.exit(main())
