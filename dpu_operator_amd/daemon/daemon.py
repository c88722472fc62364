"""Node daemon: install the CNI shim, detect the offload engine, run one side manager.

Reference: internal/daemon/daemon.go:30-209.  Behaviour kept:
* prepare(): copy the `dpu-cni` shim to the host CNI bin path and make it executable;
* serve(): a detection tick (1 s) until a platform is found, then the side manager is brought up
  in a worker thread (StartVsp -> SetupDevices -> Listen -> Serve); any failure of that worker
  stops every manager and serve() returns the error; cancellation stops managers and returns.
Side manager selection (the reference's createDaemon): colocated VSP spec (MI355X GPU data plane)
-> ColocatedSideManager, dpu mode -> DpuSideManager, otherwise HostSideManager.
"""
from __future__ import annotations

import logging
import os
import queue
import threading

from ..cni.netlink import FakeNetlink
from ..cni.sriov import SriovManagerStub
from ..platform.detectors import DpuDetectorManager
from ..utils import fileutils
from ..utils.paths import PathManager
from .managers import ColocatedSideManager, DpuSideManager, HostSideManager
from .plugin import GrpcPlugin

log = logging.getLogger("dpu.daemon")


class Daemon:
    def __init__(self, platform, mode: str = "auto", api=None, image_manager=None,
                 path_manager: PathManager | None = None, cni_src: str = "/dpu-cni", nl=None, sriov_manager=None,
                 plugin_factory=None, tick: float = 1.0, manager_kw: dict | None = None):
        self.platform = platform
        self.mode = mode
        self.api = api
        self.images = image_manager
        self.pm = path_manager or PathManager("/")
        self.cni_src = cni_src
        self.nl = nl or FakeNetlink()
        self.sm = sriov_manager or SriovManagerStub()
        self.plugin_factory = plugin_factory
        self.tick = tick
        self.manager_kw = manager_kw or {}
        self.detector = DpuDetectorManager(platform)
        self.managers: list = []
        self._threads: list[threading.Thread] = []
        self._errors: queue.Queue = queue.Queue()
        self.stop_event = threading.Event()

    # ------------------------------------------------------------------ prepare
    def prepare(self) -> None:
        dst = self.pm.cni_path()
        src = self.cni_src if os.path.isabs(self.cni_src) and os.path.exists(self.cni_src) else self.pm.wrap(self.cni_src)
        try:
            fileutils.copy_file(src, dst)
        except OSError as e:
            raise RuntimeError(f"Failed to prepare CNI binary from {self.cni_src} to {dst}: {e}") from e
        fileutils.make_executable(dst)
        log.info("Prepared CNI binary at %s", dst)

    # ------------------------------------------------------------------ managers
    def _plugin(self, spec):
        if self.plugin_factory is not None:
            return self.plugin_factory(spec)
        return GrpcPlugin(spec.dpu_mode, spec.identifier, api=self.api, path_manager=self.pm, spec=spec,
                          image_manager=self.images)

    def create_side_manager(self):
        spec = self.detector.detect()
        if spec is None:
            return None
        plugin = self._plugin(spec)
        if spec.colocated:
            return ColocatedSideManager(plugin, self.sm, self.nl, self.api, self.pm, **self.manager_kw)
        if spec.dpu_mode:
            return DpuSideManager(plugin, self.nl, self.api, self.pm, **self.manager_kw)
        return HostSideManager(plugin, self.sm, self.api, self.pm, **self.manager_kw)

    def _run_manager(self, mgr) -> None:
        try:
            mgr.start_vsp()
            mgr.setup_devices()
            mgr.listen()
            mgr.serve()
        except Exception as e:  # noqa: BLE001
            log.error("side manager failed: %s", e)
            self._errors.put(e)
            return
        self.stop_event.wait()

    # ------------------------------------------------------------------ serve
    def serve(self) -> Exception | None:
        log.info("Starting detection loop")
        err: Exception | None = None
        while not self.stop_event.is_set():
            try:
                err = self._errors.get(timeout=self.tick)
                log.error("Side manager failed, stopping all managers: %s", err)
                break
            except queue.Empty:
                pass
            if self.managers:
                continue
            try:
                mgr = self.create_side_manager()
            except Exception as e:  # noqa: BLE001
                err = RuntimeError(f"Failed to detect DPUs: {e}")
                break
            if mgr is not None:
                self.managers.append(mgr)
                t = threading.Thread(target=self._run_manager, args=(mgr,), daemon=True, name="side-manager")
                self._threads.append(t)
                t.start()
        self.shutdown()
        return err

    def prepare_and_serve(self) -> Exception | None:
        self.prepare()
        return self.serve()

    def shutdown(self) -> None:
        self.stop_event.set()
        for m in self.managers:
            try:
                m.stop()
            except Exception as e:  # noqa: BLE001
                log.warning("stopping manager: %s", e)
        for t in self._threads:
            t.join(timeout=5)
