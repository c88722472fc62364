"""Cluster flavour and filesystem deployment-mode detection.

Reference: internal/utils/cluster_environment.go:34-108 (MicroShift = ConfigMap
kube-public/microshift-version; OpenShift = CRD clusterversions.config.openshift.io; Kind = a single
node running a docker.io/kindest image) and internal/utils/filesystem_mode_detector.go:42-86
(image mode iff /host-run/ostree-booted or /run/ostree-booted exists; EPERM counts as present).
"""
from __future__ import annotations

import errno
import os

from ..k8s.apiserver import ApiServer
from .paths import FilesystemMode, Flavour


class ClusterEnvironment:
    def __init__(self, api: ApiServer):
        self.api = api

    def flavour(self) -> Flavour:
        if self.api.try_get("ConfigMap", "microshift-version", "kube-public") is not None:
            return Flavour.MICROSHIFT
        if self.api.try_get("CustomResourceDefinition", "clusterversions.config.openshift.io") is not None:
            return Flavour.OPENSHIFT
        nodes = self.api.list("Node")
        if len(nodes) == 1:
            for img in (nodes[0].get("status") or {}).get("images") or []:
                names = img.get("names") or []
                if names and "docker.io/kindest" in names[0]:
                    return Flavour.KIND
        return Flavour.UNKNOWN


class FilesystemModeDetector:
    PATHS = ("/host-run/ostree-booted", "/run/ostree-booted")

    def __init__(self, root: str = "/", stat_fn=None):
        self.root = root
        self._stat = stat_fn or os.stat

    def _exists(self, p: str) -> bool:
        path = os.path.join(self.root, p.lstrip("/")) if self.root not in ("", "/") else p
        try:
            self._stat(path)
            return True
        except FileNotFoundError:
            return False
        except PermissionError:
            return True
        except OSError as e:
            if e.errno in (errno.EPERM, errno.EACCES):
                return True
            if e.errno == errno.ENOENT:
                return False
            raise

    def detect_mode(self) -> FilesystemMode:
        return FilesystemMode.IMAGE if any(self._exists(p) for p in self.PATHS) else FilesystemMode.PACKAGE
