"""Container image bookkeeping (reference: internal/images/images.go:6-58, env_manager.go, dummy_manager.go).

Image keys are the env-var names the operator Deployment sets; the GPU build adds the GPU VSP image.
"""
from __future__ import annotations

import os

DPU_OPERATOR_DAEMON_IMAGE = "DpuOperatorDaemonImage"
NRI_WEBHOOK_IMAGE = "NRIWebhookImage"
VSP_IMAGE_INTEL = "IntelVspImage"
VSP_IMAGE_MARVELL = "MarvellVspImage"
VSP_IMAGE_INTEL_NETSEC = "IntelNetSecVspImage"
VSP_IMAGE_P4_INTEL = "IntelVspP4Image"
VSP_IMAGE_AMD_GPU = "AmdGpuVspImage"


def all_image_keys() -> list[str]:
    return [DPU_OPERATOR_DAEMON_IMAGE, NRI_WEBHOOK_IMAGE, VSP_IMAGE_INTEL, VSP_IMAGE_MARVELL,
            VSP_IMAGE_INTEL_NETSEC, VSP_IMAGE_P4_INTEL, VSP_IMAGE_AMD_GPU]


class ImageNotFound(KeyError):
    pass


class EnvImageManager:
    def __init__(self, env: dict | None = None):
        self.env = os.environ if env is None else env

    def get_image(self, key: str) -> str:
        v = self.env.get(key)
        if not v:
            raise ImageNotFound(key)
        return v

    def get_all_keys(self) -> list[str]:
        return all_image_keys()


class DummyImageManager:
    def get_image(self, key: str) -> str:
        return f"{key}-mock-image"

    def get_all_keys(self) -> list[str]:
        return all_image_keys()


def merge_vars_with_images(manager, extra: dict | None) -> dict:
    out = {}
    for k in manager.get_all_keys():
        try:
            out[k] = manager.get_image(k)
        except ImageNotFound:
            out[k] = ""
    out.update(extra or {})
    return out
