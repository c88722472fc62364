"""Operator-side reconcilers.

DpuOperatorConfigReconciler (reference: internal/controller/dpuoperatorconfig_controller.go:98-204):
  Get CR (NotFound -> ignore) -> ensure daemon DaemonSet (+RBAC) from bindata -> ensure the
  network-function NAD for the configured mode (dpu / host; anything else incl. "auto" is a
  BadRequest, exactly like the reference) -> ensure the Network Resources Injector (errors only
  logged).  Template vars: Namespace, ImagePullPolicy, Mode="auto", ResourceName, CniDir (from
  cluster flavour x filesystem mode), plus every image key.
ServiceFunctionChainReconciler: the operator-side SFC controller is a no-op in the reference too
  (servicefunctionchain_controller.go:49-55); NF pods are created by the node daemon's SFC
  reconciler (daemon/sfc.py).
"""
from __future__ import annotations

import logging

from .. import images as I
from .. import render
from .. import vars as V
from ..api.v1 import KIND_DPU_OPERATOR_CONFIG, validate_dpu_operator_config
from ..k8s.apiserver import ApiServer, BadRequest, NotFound
from ..k8s.manager import Manager, Request, Result
from ..utils.environment import ClusterEnvironment, FilesystemModeDetector
from ..utils.paths import PathManager

log = logging.getLogger("dpu.operator")


class DpuOperatorConfigReconciler:
    def __init__(self, api: ApiServer, image_manager=None, path_manager: PathManager | None = None,
                 image_pull_policy: str = "IfNotPresent", fs_detector: FilesystemModeDetector | None = None):
        self.api = api
        self.images = image_manager or I.EnvImageManager()
        self.paths = path_manager or PathManager("/")
        self.pull_policy = image_pull_policy
        self.fs = fs_detector or FilesystemModeDetector()

    def yaml_vars(self) -> dict:
        flavour = ClusterEnvironment(self.api).flavour()
        mode = self.fs.detect_mode()
        return {
            "Namespace": V.NAMESPACE,
            "ImagePullPolicy": self.pull_policy,
            "Mode": "auto",
            "ResourceName": V.RESOURCE_NAME,
            "CniDir": self.paths.cni_host_dir(flavour, mode),
        }

    def _apply(self, subdir: str, cfg: dict) -> list[dict]:
        data = I.merge_vars_with_images(self.images, self.yaml_vars())
        return render.apply_all_from_bindata(self.api, subdir, data, owner=cfg)

    def reconcile(self, req: Request) -> Result:
        try:
            cfg = self.api.get(KIND_DPU_OPERATOR_CONFIG, req.name)
        except NotFound:
            log.info("DpuOperatorConfig %s not found; ignoring", req.name)
            return Result()
        self.images.get_image(I.DPU_OPERATOR_DAEMON_IMAGE)  # the daemon image must be configured
        self._apply("daemon", cfg)
        mode = (cfg.get("spec") or {}).get("mode", "")
        if mode == "dpu":
            self._apply("networkfn-nad-dpu", cfg)
        elif mode == "host":
            self._apply("networkfn-nad-host", cfg)
        else:
            raise BadRequest(f"Invalid Mode: {mode}")
        try:
            self._apply("network-resources-injector", cfg)
        except Exception as e:  # noqa: BLE001 - logged only, as in the reference
            log.error("failed to ensure Network Resources Injector: %s", e)
        return Result()


class ServiceFunctionChainReconciler:
    def reconcile(self, req: Request) -> Result:
        return Result()


def install_webhook(api: ApiServer) -> None:
    """Register the validating admission webhook for DpuOperatorConfig (create + update)."""

    def validate(op: str, obj: dict, old: dict | None) -> None:
        if op in ("CREATE", "UPDATE"):
            validate_dpu_operator_config(obj)

    api.register_validating(KIND_DPU_OPERATOR_CONFIG, validate)


def setup_operator(api: ApiServer, image_manager=None, path_manager=None, fs_detector=None,
                   enable_webhooks: bool = True) -> Manager:
    mgr = Manager(api)
    rec = DpuOperatorConfigReconciler(api, image_manager, path_manager, fs_detector=fs_detector)
    mgr.add("dpuoperatorconfig", rec, KIND_DPU_OPERATOR_CONFIG,
            owns=("DaemonSet", "NetworkAttachmentDefinition", "Deployment"))
    mgr.add("servicefunctionchain", ServiceFunctionChainReconciler(), "ServiceFunctionChain")
    if enable_webhooks:
        install_webhook(api)
    return mgr
