"""VendorPlugin: the node daemon's client of the VSP over the vendor-plugin unix socket.

Reference: internal/daemon/plugin/vendorplugin.go:29-265.  Start(): render the VSP DaemonSet
from bindata (owned by the DpuOperatorConfig; skipped when no VSP image is configured), then poll
every 100 ms for up to 10 s: connect + LifeCycle.Init{dpu_mode, dpu_identifier} -> (ip, port).
All other calls are thin forwards: OPI Create/DeleteBridgePort, Create/DeleteNetworkFunction,
GetDevices, SetNumVfs.
"""
from __future__ import annotations

import logging
import time

import grpc

from .. import render
from .. import vars as V
from ..k8s.apiserver import ApiServer
from ..platform.detectors import VspSpec
from ..proto import opi, vendor
from ..proto.grpcutil import Stub, unix_target
from ..utils.paths import PathManager

log = logging.getLogger("dpu.vendorplugin")


class VendorPlugin:
    def start(self) -> tuple[str, int]: ...
    def close(self) -> None: ...
    def create_bridge_port(self, req) -> object: ...
    def delete_bridge_port(self, req) -> None: ...
    def create_network_function(self, inp: str, out: str) -> None: ...
    def delete_network_function(self, inp: str, out: str) -> None: ...
    def get_devices(self) -> object: ...
    def set_num_vfs(self, n: int) -> object: ...


class GrpcPlugin(VendorPlugin):
    def __init__(self, dpu_mode: bool, dpu_identifier: str = "", api: ApiServer | None = None,
                 path_manager: PathManager | None = None, spec: VspSpec | None = None, image_manager=None,
                 image_pull_policy: str = "Always", start_timeout: float = 10.0, poll: float = 0.1):
        self.dpu_mode = dpu_mode
        self.dpu_identifier = dpu_identifier
        self.api = api
        self.pm = path_manager or PathManager("/")
        self.spec = spec
        self.image_manager = image_manager
        self.pull_policy = image_pull_policy
        self.start_timeout = start_timeout
        self.poll = poll
        self.channel: grpc.Channel | None = None
        self.lifecycle = self.nf = self.devices = self.opi = None

    def _template_vars(self) -> dict:
        d = {"VendorSpecificPluginImage": "", "Namespace": V.NAMESPACE, "ImagePullPolicy": self.pull_policy,
             "Command": "[ ]", "Args": "[ ]"}
        if self.spec is not None and self.image_manager is not None:
            d.update(self.spec.template_vars(self.image_manager))
        return d

    def deploy_vsp(self) -> list[dict]:
        tv = self._template_vars()
        if not tv["VendorSpecificPluginImage"] or self.api is None:
            return []
        cfg = self.api.get("DpuOperatorConfig", V.DPU_OPERATOR_CONFIG_NAME)
        return render.apply_all_from_bindata(self.api, "vsp-ds", tv, owner=cfg)

    def ensure_connected(self) -> None:
        if self.channel is not None:
            return
        ch = grpc.insecure_channel(unix_target(self.pm.vendor_plugin_socket()))
        grpc.channel_ready_future(ch).result(timeout=max(self.poll, 0.05))
        self.channel = ch
        self.lifecycle = Stub(ch, vendor, "LifeCycleService")
        self.nf = Stub(ch, vendor, "NetworkFunctionService")
        self.devices = Stub(ch, vendor, "DeviceService")
        self.opi = Stub(ch, opi, "BridgePortService")

    def start(self) -> tuple[str, int]:
        t0 = time.monotonic()
        self.deploy_vsp()
        last = None
        while True:
            try:
                self.ensure_connected()
                ipport = self.lifecycle.Init(vendor.InitRequest(dpu_mode=self.dpu_mode,
                                                                dpu_identifier=self.dpu_identifier), timeout=5)
                log.info("VSP started in %.2fs (dpu_mode=%s)", time.monotonic() - t0, self.dpu_mode)
                return ipport.ip, ipport.port
            except Exception as e:  # noqa: BLE001
                last = e
                if self.channel is not None and not isinstance(e, grpc.RpcError):
                    self.close()
            if time.monotonic() - t0 >= self.start_timeout:
                raise TimeoutError(f"failed to start VSP after {self.start_timeout}s: {last}")
            time.sleep(self.poll)

    def close(self) -> None:
        if self.channel is not None:
            self.channel.close()
        self.channel = None
        self.lifecycle = self.nf = self.devices = self.opi = None

    def _need(self):
        if self.channel is None:
            self.ensure_connected()

    def create_bridge_port(self, req):
        self._need()
        return self.opi.CreateBridgePort(req, timeout=30)

    def delete_bridge_port(self, req) -> None:
        self._need()
        self.opi.DeleteBridgePort(req, timeout=30)

    def create_network_function(self, inp: str, out: str) -> None:
        self._need()
        self.nf.CreateNetworkFunction(vendor.NFRequest(input=inp, output=out), timeout=30)

    def delete_network_function(self, inp: str, out: str) -> None:
        self._need()
        self.nf.DeleteNetworkFunction(vendor.NFRequest(input=inp, output=out), timeout=30)

    def get_devices(self):
        self._need()
        return self.devices.GetDevices(vendor.Empty(), timeout=30)

    def set_num_vfs(self, n: int):
        self._need()
        return self.devices.SetNumVfs(vendor.VfCount(vf_cnt=n), timeout=60)
