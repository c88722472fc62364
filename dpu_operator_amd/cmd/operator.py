"""`operator` — the DPU operator manager (reference cmd/main.go:43-133).

Flags kept: --metrics-bind-address (:18090), --health-probe-bind-address (:18091), --bindata,
--leader-elect (Lease id `1e46962d.openshift.io`), webhook server on :9443 with certificates from
--cert-dir (tls.crt / tls.key), ENABLE_WEBHOOKS=false disables the webhook.  Controllers:
DpuOperatorConfig + ServiceFunctionChain.  The API is the cluster's (k8s/rest.py RestClient:
--kubeconfig, $KUBECONFIG or the in-cluster service account, as controller-runtime's
GetConfigOrDie); --standalone runs against an in-process API server instead (demos, tests).
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import socket
import sys
import threading

from .. import vars as V
from ..api.v1 import crd_manifests
from ..controller.operator import setup_operator
from ..api.scheme import SCHEME
from ..k8s.apiserver import AlreadyExists, ApiServer
from ..k8s.leader import LeaderElector
from ..utils.metrics import MetricsServer, ProbeServer

LEADER_ELECTION_ID = "1e46962d.openshift.io"
log = logging.getLogger("dpu.operator")


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="dpu-operator")
    ap.add_argument("--metrics-bind-address", default=":18090")
    ap.add_argument("--health-probe-bind-address", default=":18091")
    ap.add_argument("--bindata", default="")
    ap.add_argument("--leader-elect", action="store_true")
    ap.add_argument("--webhook-port", type=int, default=9443)
    ap.add_argument("--cert-dir", default="/tmp/k8s-webhook-server/serving-certs")
    ap.add_argument("--identity", default=f"{socket.gethostname()}_{os.getpid()}")
    ap.add_argument("--lease-duration", type=float, default=15.0)
    ap.add_argument("--renew-interval", type=float, default=2.0)
    ap.add_argument("--kubeconfig", default="", help="cluster API config (default: $KUBECONFIG, then in-cluster)")
    ap.add_argument("--standalone", action="store_true", help="in-process API server (no cluster)")
    return ap


def cluster_api(args):
    """The cluster API client, or an in-process ApiServer with --standalone; exits without one."""
    if getattr(args, "standalone", False):
        return ApiServer(scheme=SCHEME)
    from ..k8s.rest import connect

    api = connect(args.kubeconfig or None)
    if api is None:
        raise SystemExit("no cluster configuration (--kubeconfig, $KUBECONFIG or in-cluster service account); "
                         "use --standalone for an in-process API server")
    return api


class Operator:
    def __init__(self, args, api: ApiServer | None = None, image_manager=None):
        self.args = args
        self.api = api if api is not None else cluster_api(args)
        for crd in crd_manifests():
            try:
                self.api.create(crd)
            except AlreadyExists:
                pass
        self.enable_webhooks = os.environ.get("ENABLE_WEBHOOKS") != "false"
        if image_manager is None:
            from ..images import EnvImageManager

            image_manager = EnvImageManager()
        self.mgr = setup_operator(self.api, image_manager=image_manager, enable_webhooks=self.enable_webhooks)
        self.metrics = MetricsServer(args.metrics_bind_address)
        self.probes = ProbeServer(args.health_probe_bind_address)
        self.webhook = None
        self.elector = None
        self.started = threading.Event()

    def _start_manager(self):
        self.mgr.start()
        self.started.set()

    def start(self) -> "Operator":
        self.metrics.start()
        self.probes.ready["manager"] = self.started.is_set
        self.probes.start()
        if self.enable_webhooks:
            crt, key = os.path.join(self.args.cert_dir, "tls.crt"), os.path.join(self.args.cert_dir, "tls.key")
            if os.path.exists(crt) and os.path.exists(key):
                from ..controller.webhook_server import WebhookServer
                from ..nri.server import KeyPairReloader

                self.webhook = WebhookServer(KeyPairReloader(crt, key, insecure=True), port=self.args.webhook_port).start()
            else:
                log.warning("webhook certificates not found in %s; admission runs in-process only", self.args.cert_dir)
        if self.args.leader_elect:
            self.elector = LeaderElector(self.api, LEADER_ELECTION_ID, V.NAMESPACE, self.args.identity,
                                         lease_duration=self.args.lease_duration, renew=self.args.renew_interval,
                                         on_started=self._start_manager, on_stopped=self.mgr.stop).start()
        else:
            self._start_manager()
        return self

    def stop(self) -> None:
        if self.elector is not None:
            self.elector.stop()
        self.mgr.stop()
        for s in (self.webhook, self.metrics, self.probes):
            if s is not None:
                s.stop()


def main(argv=None, api=None, stop: threading.Event | None = None) -> int:
    logging.basicConfig(level=logging.INFO)
    op = Operator(build_parser().parse_args(argv), api).start()
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    op.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
