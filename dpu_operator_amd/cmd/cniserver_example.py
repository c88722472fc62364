"""Standalone NF CNI server for manual testing (reference dpu-cni/example/cniserver_main.go, C6).

Serves the dpu-cni protocol on the given socket and handles ADD/DEL with the NF-side handler
(networkfn: move a netdev into the pod namespace and back).
"""
from __future__ import annotations

import argparse
import logging
import signal
import sys
import threading

from ..cni import networkfn
from ..cni.server import Server
from ..utils.paths import PathManager


def main(argv=None, nl=None, stop: threading.Event | None = None) -> int:
    ap = argparse.ArgumentParser(prog="cniserver-example")
    ap.add_argument("--socket", default="")
    ap.add_argument("--root", default="/")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if nl is None:
        from ..cni.netlink import RtNetlink

        nl = RtNetlink()
    pm = PathManager(a.root)
    srv = Server(lambda r: networkfn.cmd_add(r, nl), lambda r: networkfn.cmd_del(r, nl), pm,
                 socket_path=a.socket or None).listen().start()
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    srv.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
