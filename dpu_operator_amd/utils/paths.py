"""Socket / file path policy, relocatable under a root dir for tests.

Reference: internal/utils/path_manager.go:12-100 (every path is re-rooted by ``PathManager(root)``
so tests can run the CNI server, device plugin and VSP sockets under /tmp/<cluster>).
GPU additions: the data-plane journal and the host<->device control mailbox live under
/var/run/dpu-daemon as well.
"""
from __future__ import annotations

import os
import stat
from enum import Enum
from pathlib import Path


class Flavour(str, Enum):
    MICROSHIFT = "MicroShift"
    OPENSHIFT = "OpenShift"
    KIND = "Kind"
    UNKNOWN = "Unknown"


class FilesystemMode(str, Enum):
    IMAGE = "image"
    PACKAGE = "package"


class PathManager:
    def __init__(self, root_dir: str = "/"):
        self.root = root_dir

    def wrap(self, p: str) -> str:
        return os.path.join(self.root, p.lstrip("/")) if self.root not in ("", "/") else p

    def cni_server_path(self) -> str:
        return self.wrap("/var/run/dpu-daemon/dpu-cni/dpu-cni-server.sock")

    def kubelet_endpoint(self) -> str:
        return self.wrap("/var/lib/kubelet/device-plugins/kubelet.sock")

    def plugin_endpoint(self) -> str:
        return self.wrap("/var/lib/kubelet/device-plugins/dpuNet.sock")

    def plugin_endpoint_filename(self) -> str:
        return os.path.basename(self.plugin_endpoint())

    def cni_path(self) -> str:
        return self.wrap("/var/lib/cni/bin/dpu-cni")

    def vendor_plugin_socket(self) -> str:
        return self.wrap("/var/run/dpu-daemon/vendor-plugin/vendor-plugin.sock")

    def journal_dir(self) -> str:
        return self.wrap("/var/run/dpu-daemon/journal")

    def mailbox_path(self) -> str:
        return self.wrap("/var/run/dpu-daemon/ctrl-mbox")

    def memif_dir(self) -> str:
        """Shared-memory vport regions (<vport name>.memif): created by the GPU VSP, mounted into
        the pod that was allocated the vport by the device plugin."""
        return self.wrap("/var/run/dpu-daemon/memif")

    @staticmethod
    def memif_container_path(device_id: str) -> str:
        """Where a pod finds the region of its vport (the device plugin's mount target)."""
        return f"/var/run/dpu/memif/{device_id}.memif"

    def cni_host_dir(self, flavour: Flavour, fs_mode: FilesystemMode) -> str:
        if flavour == Flavour.MICROSHIFT and fs_mode == FilesystemMode.IMAGE:
            return self.wrap("/run/cni")
        if flavour == Flavour.OPENSHIFT:
            return self.wrap("/var/lib/cni")
        if (flavour == Flavour.MICROSHIFT and fs_mode == FilesystemMode.PACKAGE) or flavour == Flavour.KIND:
            return self.wrap("/opt/cni")
        raise ValueError(f"unknown combination of cluster flavour ({flavour}) and filesystem mode ({fs_mode})")

    @staticmethod
    def ensure_socket_dir_exists(socket_path: str) -> None:
        """Fresh 0700 directory for a unix socket; refuse a pre-existing insecure one
        (path_manager.go:66-96)."""
        run_dir = Path(socket_path).parent
        if run_dir.exists():
            st = run_dir.stat()
            if st.st_uid != os.getuid():
                raise PermissionError(f"insecure owner of socket directory {run_dir}: {st.st_uid}")
            if stat.S_IMODE(st.st_mode) & 0o077:
                os.chmod(run_dir, 0o700)
            if Path(socket_path).exists() or Path(socket_path).is_socket():
                os.unlink(socket_path)
        else:
            run_dir.mkdir(parents=True, mode=0o700, exist_ok=True)
            os.chmod(run_dir, 0o700)
