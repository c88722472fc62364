"""HTTPS admission endpoint for the DpuOperatorConfig validating webhook.

Reference: api/v1/dpuoperatorconfig_webhook.go:34-83 served by controller-runtime's webhook server
on :9443 at `/validate-config-openshift-io-v1-dpuoperatorconfig`.  Create and update
are validated (name must be `dpu-operator-config`, mode in host/dpu/auto); delete is allowed.
"""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler

from ..api.v1 import ValidationError, validate_dpu_operator_config
from ..nri.server import KeyPairReloader, _TLSServer

VALIDATE_PATH = "/validate-config-openshift-io-v1-dpuoperatorconfig"


def review_response(review: dict) -> dict:
    req = review.get("request") or {}
    resp = {"uid": req.get("uid", ""), "allowed": True}
    if req.get("operation") in ("CREATE", "UPDATE"):
        try:
            validate_dpu_operator_config(req.get("object") or {})
        except ValidationError as e:
            resp = {"uid": req.get("uid", ""), "allowed": False, "status": {"code": 403, "reason": "Forbidden",
                                                                          "message": str(e)}}
    return {"apiVersion": review.get("apiVersion", "admission.k8s.io/v1"), "kind": "AdmissionReview", "response": resp}


class WebhookServer:
    def __init__(self, reloader: KeyPairReloader, address: str = "0.0.0.0", port: int = 9443):
        self.reloader = reloader
        self.address, self.port = address, port
        self._srv = None

    def start(self) -> "WebhookServer":
        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):
                if self.path != VALIDATE_PATH:
                    self.send_response(404)
                    self.end_headers()
                    return
                n = int(self.headers.get("Content-Length", "0") or 0)
                try:
                    body = json.dumps(review_response(json.loads(self.rfile.read(n)))).encode()
                    code = 200
                except ValueError:
                    body, code = b"bad AdmissionReview", 400
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        self._srv = _TLSServer((self.address, self.port), H, self.reloader)
        self.port = self._srv.server_address[1]
        threading.Thread(target=self._srv.serve_forever, daemon=True).start()
        return self

    def stop(self) -> None:
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
