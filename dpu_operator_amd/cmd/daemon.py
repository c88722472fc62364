"""`dpu-daemon` — node daemon entry (reference cmd/daemon/daemon.go:18-40).

`--mode` is accepted (the reference stores it and never uses it; detection decides the side).
Real node: sysfs platform, rtnetlink, SR-IOV manager, VSP client over the vendor-plugin socket,
and the cluster API (k8s/rest.py: --kubeconfig, $KUBECONFIG or the pod's service account) for the
SFC reconciler and the VSP DaemonSet; --standalone keeps an in-process API server.
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
    ap.add_argument("--kubeconfig", default="", help="cluster API config (default: $KUBECONFIG, then in-cluster)")
    ap.add_argument("--standalone", action="store_true", help="in-process API server (no cluster)")
    a = ap.parse_args(argv)
    if api is None:
        if a.standalone:
            from ..api.scheme import SCHEME
            from ..k8s.apiserver import ApiServer

            api = ApiServer(scheme=SCHEME)
        else:
            from ..k8s.rest import connect

            api = connect(a.kubeconfig or None)
            if api is None:
                logging.error("no cluster configuration (--kubeconfig, $KUBECONFIG or in-cluster service account); "
                              "use --standalone for an in-process API server")
                return 2
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
