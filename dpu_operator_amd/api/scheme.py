"""Type scheme (A6): which (apiVersion, kind) pairs the control plane understands.

Reference: internal/scheme/scheme.go:13-22 registers config/v1, the core types, apiextensions and
the NetworkAttachmentDefinition types into one runtime.Scheme shared by the operator, daemon and
webhook clients.  Here the scheme is a registry of group/version/kind -> (scope, typed decoder,
schema validator) used by:

* `ApiServer(scheme=...)` to reject objects of unknown kinds or with a mismatched apiVersion
  (the 400 a real API server gives for an unregistered resource),
* `Scheme.decode(obj)` to obtain the typed view (DpuOperatorConfig / ServiceFunctionChain) from
  an unstructured object, as controller-runtime's typed client does.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

from . import v1


@dataclass(frozen=True)
class Gvk:
    group: str
    version: str
    kind: str

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version


@dataclass
class TypeInfo:
    gvk: Gvk
    namespaced: bool
    decode: Callable[[dict], object] | None = None
    validate: Callable[[dict], list[str]] | None = None


class Scheme:
    def __init__(self):
        self._by_kind: dict[str, TypeInfo] = {}

    def add(self, group: str, version: str, kind: str, namespaced: bool = True, decode=None, validate=None) -> None:
        self._by_kind[kind] = TypeInfo(Gvk(group, version, kind), namespaced, decode, validate)

    def recognizes(self, api_version: str, kind: str) -> bool:
        t = self._by_kind.get(kind)
        return t is not None and t.gvk.api_version == api_version

    def info(self, kind: str) -> TypeInfo:
        try:
            return self._by_kind[kind]
        except KeyError:
            raise KeyError(f"no kind {kind!r} is registered in the scheme") from None

    def kinds(self) -> list[str]:
        return sorted(self._by_kind)

    def cluster_scoped(self) -> set[str]:
        return {k for k, t in self._by_kind.items() if not t.namespaced}

    def check(self, obj: dict) -> None:
        """Raises ValueError for an unregistered kind, a wrong apiVersion or a schema violation."""
        kind, av = obj.get("kind", ""), obj.get("apiVersion", "")
        t = self._by_kind.get(kind)
        if t is None:
            raise ValueError(f"no matches for kind {kind!r}")
        if av and av != t.gvk.api_version:
            raise ValueError(f"no matches for kind {kind!r} in version {av!r}")
        if t.validate is not None:
            t.validate(obj)

    def decode(self, obj: dict):
        t = self.info(obj.get("kind", ""))
        return t.decode(obj) if t.decode else obj


def _schema_sfc(obj: dict) -> list[str]:
    return v1.validate_sfc(obj)


def new_scheme() -> Scheme:
    """config/v1 + core/v1 + apps/v1 + rbac + coordination + apiextensions + admission + NAD."""
    s = Scheme()
    s.add(v1.GROUP, v1.VERSION, v1.KIND_DPU_OPERATOR_CONFIG, namespaced=False,
          decode=v1.DpuOperatorConfig.from_obj)
    s.add(v1.GROUP, v1.VERSION, v1.KIND_SFC, decode=v1.ServiceFunctionChain.from_obj, validate=_schema_sfc)
    for kind in ("Pod", "ConfigMap", "Secret", "Service", "ServiceAccount", "Event", "Endpoints"):
        s.add("", "v1", kind)
    for kind in ("Namespace", "Node", "PersistentVolume"):
        s.add("", "v1", kind, namespaced=False)
    for kind in ("DaemonSet", "Deployment"):
        s.add("apps", "v1", kind)
    s.add("rbac.authorization.k8s.io", "v1", "Role")
    s.add("rbac.authorization.k8s.io", "v1", "RoleBinding")
    s.add("rbac.authorization.k8s.io", "v1", "ClusterRole", namespaced=False)
    s.add("rbac.authorization.k8s.io", "v1", "ClusterRoleBinding", namespaced=False)
    s.add("coordination.k8s.io", "v1", "Lease")
    s.add("apiextensions.k8s.io", "v1", "CustomResourceDefinition", namespaced=False)
    s.add("admissionregistration.k8s.io", "v1", "MutatingWebhookConfiguration", namespaced=False)
    s.add("admissionregistration.k8s.io", "v1", "ValidatingWebhookConfiguration", namespaced=False)
    s.add("k8s.cni.cncf.io", "v1", "NetworkAttachmentDefinition")
    s.add("config.openshift.io", "v1", "ClusterVersion", namespaced=False)
    return s


SCHEME = new_scheme()
