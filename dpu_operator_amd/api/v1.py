"""config.openshift.io/v1 API: DpuOperatorConfig and ServiceFunctionChain.

Wire-compatible with the reference CRDs (field names / JSON shape), re-expressed as Python
dataclasses over the unstructured (dict) objects the in-process API server stores.

Reference:
* DpuOperatorConfig spec {mode, logLevel}, cluster-scoped singleton named
  ``dpu-operator-config`` — api/v1/dpuoperatorconfig_types.go:29-36,46,70-73
* ServiceFunctionChain spec {networkFunctions: [{name, image}]}, shortName sfc —
  api/v1/servicefunctionchain_types.go:27-38
* validating webhook (create + update): name must be the standard name, mode in
  {host, dpu, auto} — api/v1/dpuoperatorconfig_webhook.go:46-61
"""
from __future__ import annotations

import copy
from dataclasses import asdict, dataclass, field

from .. import vars as V

GROUP = "config.openshift.io"
VERSION = "v1"
API_VERSION = f"{GROUP}/{VERSION}"

KIND_DPU_OPERATOR_CONFIG = "DpuOperatorConfig"
KIND_SFC = "ServiceFunctionChain"

VALID_MODES = ("host", "dpu", "auto")
WEBHOOK_PATH = "/validate-config-openshift-io-v1-dpuoperatorconfig"


class ValidationError(ValueError):
    """Raised by the admission webhook; the API server turns it into a 403 Forbidden."""


@dataclass
class DpuOperatorConfigSpec:
    mode: str = ""
    logLevel: int = 0


@dataclass
class DpuOperatorConfig:
    name: str = V.DPU_OPERATOR_CONFIG_NAME
    spec: DpuOperatorConfigSpec = field(default_factory=DpuOperatorConfigSpec)
    status: dict = field(default_factory=dict)
    metadata: dict = field(default_factory=dict)

    def to_obj(self) -> dict:
        md = dict(self.metadata)
        md["name"] = self.name
        spec = {k: v for k, v in asdict(self.spec).items() if v not in ("", 0, None)}
        return {"apiVersion": API_VERSION, "kind": KIND_DPU_OPERATOR_CONFIG, "metadata": md, "spec": spec,
                "status": dict(self.status)}

    @classmethod
    def from_obj(cls, obj: dict) -> "DpuOperatorConfig":
        spec = obj.get("spec") or {}
        return cls(
            name=obj["metadata"]["name"],
            spec=DpuOperatorConfigSpec(mode=spec.get("mode", ""), logLevel=int(spec.get("logLevel", 0) or 0)),
            status=copy.deepcopy(obj.get("status") or {}),
            metadata=copy.deepcopy(obj["metadata"]),
        )


def validate_dpu_operator_config(obj: dict) -> list[str]:
    """Webhook validation (create and update).  Returns warnings; raises ValidationError.

    Mirrors dpuoperatorconfig_webhook.go:50-61 exactly, including accepting ``auto``, which the
    reconciler later rejects for the network-function NAD (dpuoperatorconfig_controller.go:189-202).
    """
    name = (obj.get("metadata") or {}).get("name")
    if name != V.DPU_OPERATOR_CONFIG_NAME:
        raise ValidationError(f'DpuOperatorConfig must have standard name "{V.DPU_OPERATOR_CONFIG_NAME}"')
    mode = (obj.get("spec") or {}).get("mode", "")
    if mode not in VALID_MODES:
        raise ValidationError("Invalid mode")
    return []


@dataclass
class NetworkFunction:
    name: str
    image: str


@dataclass
class ServiceFunctionChain:
    name: str
    namespace: str = V.NAMESPACE
    network_functions: list[NetworkFunction] = field(default_factory=list)
    metadata: dict = field(default_factory=dict)

    def to_obj(self) -> dict:
        md = dict(self.metadata)
        md.update(name=self.name, namespace=self.namespace)
        return {
            "apiVersion": API_VERSION,
            "kind": KIND_SFC,
            "metadata": md,
            "spec": {"networkFunctions": [{"name": n.name, "image": n.image} for n in self.network_functions]},
            "status": {},
        }

    @classmethod
    def from_obj(cls, obj: dict) -> "ServiceFunctionChain":
        spec = obj.get("spec") or {}
        nfs = [NetworkFunction(n["name"], n.get("image", "")) for n in spec.get("networkFunctions") or []]
        md = obj["metadata"]
        return cls(md["name"], md.get("namespace", V.NAMESPACE), nfs, copy.deepcopy(md))


def validate_sfc(obj: dict) -> list[str]:
    """Schema-level checks the CRD's OpenAPI schema enforces (name/image are strings)."""
    for nf in (obj.get("spec") or {}).get("networkFunctions") or []:
        if not isinstance(nf, dict) or not isinstance(nf.get("name"), str) or not isinstance(nf.get("image", ""), str):
            raise ValidationError("spec.networkFunctions[]: name and image must be strings")
    return []


def crd_manifests() -> list[dict]:
    """CustomResourceDefinitions (the kubebuilder artefacts, A4) generated from the types."""

    def crd(kind, plural, singular, scope, short, spec_schema):
        return {
            "apiVersion": "apiextensions.k8s.io/v1",
            "kind": "CustomResourceDefinition",
            "metadata": {"name": f"{plural}.{GROUP}"},
            "spec": {
                "group": GROUP,
                "names": {"kind": kind, "listKind": kind + "List", "plural": plural, "singular": singular,
                          **({"shortNames": short} if short else {})},
                "scope": scope,
                "versions": [{
                    "name": VERSION, "served": True, "storage": True,
                    "subresources": {"status": {}},
                    "schema": {"openAPIV3Schema": {
                        "type": "object",
                        "properties": {
                            "apiVersion": {"type": "string"}, "kind": {"type": "string"},
                            "metadata": {"type": "object"}, "spec": spec_schema,
                            "status": {"type": "object"},
                        },
                    }},
                }],
            },
        }

    return [
        crd(KIND_DPU_OPERATOR_CONFIG, "dpuoperatorconfigs", "dpuoperatorconfig", "Cluster", None, {
            "type": "object",
            "properties": {"mode": {"type": "string"}, "logLevel": {"type": "integer"}},
        }),
        crd(KIND_SFC, "servicefunctionchains", "servicefunctionchain", "Namespaced", ["sfc"], {
            "type": "object",
            "properties": {"networkFunctions": {"type": "array", "items": {
                "type": "object", "required": ["name", "image"],
                "properties": {"name": {"type": "string"}, "image": {"type": "string"}},
            }}},
        }),
    ]
