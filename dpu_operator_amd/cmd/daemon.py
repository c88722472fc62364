"""`dpu-daemon` — node daemon entry (reference cmd/daemon/daemon.go:18-40).

`--mode` is accepted (the reference stores it and never uses it; detection decides the side).
Real node: sysfs platform, rtnetlink, SR-IOV manager, VSP client over the vendor-plugin socket.
"""
from __future__ import annotations

import argparse
import logging
import signal
import sys
import threading

from ..daemon.daemon import Daemon
from ..platform.platform import SysfsPlatform
from ..utils.paths import PathManager


def main(argv=None, api=None, stop: threading.Event | None = None) -> int:
    ap = argparse.ArgumentParser(prog="dpu-daemon")
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--root", default="/", help="path-manager root (tests)")
    ap.add_argument("--cni-src", default="/dpu-cni")
    ap.add_argument("--node-config", default="", help="node policy YAML (config.py); also DPU_NODE_CONFIG")
    a = ap.parse_args(argv)
    if a.node_config:
        from ..config import NodeConfig, set_node_config

        set_node_config(NodeConfig.load(a.node_config))
    logging.basicConfig(level=logging.DEBUG)
    from ..cni.netlink import RtNetlink
    from ..cni.sriov import SriovManager

    pm = PathManager(a.root)
    nl = RtNetlink()
    d = Daemon(SysfsPlatform(a.root), a.mode, api, None, pm, cni_src=a.cni_src, nl=nl, sriov_manager=SriovManager(nl))
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: d.stop_event.set())
        signal.signal(signal.SIGINT, lambda *_: d.stop_event.set())
    if stop is not None:
        threading.Thread(target=lambda: (stop.wait(), d.stop_event.set()), daemon=True).start()
    err = d.prepare_and_serve()
    if err is not None:
        logging.error("daemon failed: %s", err)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
