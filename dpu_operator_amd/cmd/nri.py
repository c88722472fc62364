"""`nri` — Network Resources Injector webhook server (reference cmd/nri/networkresourcesinjector.go).

Flags kept: --port 8443, --bind-address 0.0.0.0, --tls-cert-file cert.pem, --tls-private-key-file
key.pem, --insecure, --client-ca (repeatable), --health-check-port 8444, --enable-http2 (accepted;
HTTP/1.1 only here, like the reference's default), --injectHugepageDownApi,
--network-resource-name-keys, --honor-resources.  Exits with an error for invalid ports or when
resource-name injection is disabled (the injector would have nothing to do).
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import sys
import threading

from ..nri.server import InjectorServer, KeyPairReloader, valid_port
from ..nri.webhook import DEFAULT_RESOURCE_NAME_KEY, ControlSwitches, NadCache

DEFAULT_CLIENT_CA = "/var/run/secrets/kubernetes.io/serviceaccount/ca.crt"


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="nri")
    ap.add_argument("--port", type=int, default=8443)
    ap.add_argument("--bind-address", default="0.0.0.0")
    ap.add_argument("--tls-cert-file", default="cert.pem")
    ap.add_argument("--tls-private-key-file", default="key.pem")
    ap.add_argument("--insecure", action="store_true")
    ap.add_argument("--client-ca", action="append", default=[])
    ap.add_argument("--health-check-port", type=int, default=8444)
    ap.add_argument("--enable-http2", action="store_true")
    ap.add_argument("--injectHugepageDownApi", action="store_true")
    ap.add_argument("--network-resource-name-keys", default=DEFAULT_RESOURCE_NAME_KEY)
    ap.add_argument("--honor-resources", action="store_true")
    return ap


def main(argv=None, api=None, nad_getter=None, stop: threading.Event | None = None) -> int:
    logging.basicConfig(level=logging.INFO)
    a = build_parser().parse_args(argv)
    switches = ControlSwitches(a.injectHugepageDownApi, a.honor_resources, a.network_resource_name_keys)
    if not switches.resource_names_enabled():
        print("resource name injection is disabled: nothing to do", file=sys.stderr)
        return 1
    if not valid_port(a.port):
        print("invalid port number. Choose between 1024 and 65535", file=sys.stderr)
        return 1
    if not a.bind_address or not a.tls_cert_file or not a.tls_private_key_file:
        print("input argument(s) not defined correctly", file=sys.stderr)
        return 1
    if not valid_port(a.health_check_port) or a.health_check_port == a.port:
        print("invalid health check port (1024-65535, different from --port)", file=sys.stderr)
        return 1
    if not a.client_ca:
        a.client_ca = [DEFAULT_CLIENT_CA]
    namespace = os.environ.get("NAMESPACE") or "kube-system"
    getter = nad_getter or (lambda ns, name: api.try_get("NetworkAttachmentDefinition", name, ns) if api else None)
    srv = InjectorServer(NadCache(getter), switches,
                         KeyPairReloader(a.tls_cert_file, a.tls_private_key_file, a.client_ca, a.insecure),
                         a.bind_address, a.port, a.health_check_port, api=api, namespace=namespace).start()
    stop = stop or threading.Event()
    if threading.current_thread() is threading.main_thread():
        signal.signal(signal.SIGTERM, lambda *_: stop.set())
        signal.signal(signal.SIGINT, lambda *_: stop.set())
    stop.wait()
    srv.stop()
    return 0


if __name__ == "__main__":
    sys.exit(main())
