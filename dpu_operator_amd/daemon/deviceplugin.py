"""kubelet device plugin for the `openshift.io/dpu` extended resource + the device handler.

Reference: internal/daemon/device-plugin/deviceplugin.go:24-353 and
internal/daemon/device-handler/dpu-device-handler/dpudevicehandler.go:48-106.
* DeviceHandler.setup_devices: VSP SetNumVfs(8) (an error is tolerated on the device side);
  get_devices: wait until setup ran, map VSP devices to {ID, health}; on the host side device IDs
  must be PCI addresses.
* ListAndWatch polls the handler every `poll` s (5 s in the reference) and streams the list when it
  changes; Allocate rejects unknown or unhealthy devices and returns env NF-DEV="<id>,<id>,".
  GPU-VSP shared-memory vports: a device whose region exists (<PathManager.memif_dir>/<id>.memif)
  is also mounted into the container (PathManager.memif_container_path) and listed in NF-MEMIF,
  the way memif / vhost-user device plugins hand over their sockets; netdev vports (veth, TAP)
  reach the pod through the CNI instead (networkfn.cmd_add moves the netdev named <id>).
* Serve: gRPC on the plugin socket, self-dial until ready (the reference's WithBlock workaround),
  then Register{v1beta1, endpoint filename, resource name} with the kubelet.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from concurrent import futures

import grpc

from .. import vars as V
from ..cni.sriov.utils import is_valid_pci_address
from ..proto import DEVICE_PLUGIN_VERSION, HEALTHY, deviceplugin as dp
from ..proto.grpcutil import Stub, service_handler, unix_target
from ..utils.faults import FAULTS
from ..utils.metrics import CONTROL
from ..utils.paths import PathManager

log = logging.getLogger("dpu.deviceplugin")

DEFAULT_VF_COUNT = 8


class DeviceHandler:
    def __init__(self, vsp, dpu_mode: bool, vf_count: int | None = None, numa_of=None):
        """`numa_of(device_id) -> int` (optional): NUMA node advertised to kubelet's topology
        manager (-1 = unknown); e.g. devutils.get_numa_node for PCI ids, or the data-plane GPU's
        node for GPU vports."""
        self.vsp = vsp
        self.dpu_mode = dpu_mode
        if vf_count is None:
            from ..config import node_config

            vf_count = node_config().vf_count
        self.vf_count = vf_count
        self.numa_of = numa_of
        self._setup = threading.Event()

    def setup_devices(self) -> None:
        try:
            self.vsp.set_num_vfs(self.vf_count)
        except Exception as e:  # noqa: BLE001
            if not self.dpu_mode:
                raise
            log.warning("SetNumVfs failed on the device side (tolerated): %s", e)
        self._setup.set()

    def get_devices(self, timeout: float = 30.0) -> dict[str, tuple[str, str]]:
        if not self._setup.wait(timeout):
            raise TimeoutError("devices not set up")
        resp = self.vsp.get_devices()
        out = {}
        for key, dev in resp.devices.items():
            if not self.dpu_mode and not is_valid_pci_address(dev.ID):
                raise ValueError(f"host-side device id must be a PCI address, got {dev.ID}")
            out[dev.ID or key] = (dev.ID or key, dev.health)
        return out


class DevicePluginServer:
    def __init__(self, handler: DeviceHandler, path_manager: PathManager | None = None,
                 resource_name: str = V.RESOURCE_NAME, poll: float = 5.0):
        self.handler = handler
        self.pm = path_manager or PathManager("/")
        self.resource_name = resource_name
        self.poll = poll
        self.devices: dict[str, tuple[str, str]] = {}
        self._server: grpc.Server | None = None
        self._stop = threading.Event()
        self.registered = False

    def _device(self, dev_id: str, health: str):
        numa = self.handler.numa_of(dev_id) if self.handler.numa_of else -1
        if numa is not None and numa >= 0:
            return dp.Device(ID=dev_id, health=health, topology=dp.TopologyInfo(nodes=[dp.NUMANode(ID=numa)]))
        return dp.Device(ID=dev_id, health=health)

    # ------------------------------------------------------------------ gRPC service
    def GetDevicePluginOptions(self, request, context):
        return dp.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=False)

    def ListAndWatch(self, request, context):
        old: dict | None = None
        while not self._stop.is_set() and context.is_active():
            try:
                FAULTS.check("deviceplugin.GetDevices")
                new = self.handler.get_devices()
            except Exception as e:  # noqa: BLE001
                log.error("GetDevices failed: %s", e)
                context.abort(grpc.StatusCode.UNAVAILABLE, str(e))
                return
            if new != old:
                self.devices = dict(new)
                yield dp.ListAndWatchResponse(devices=[self._device(i, h) for i, h in sorted(new.values())])
                old = new
            self._stop.wait(self.poll)

    def Allocate(self, request, context):
        CONTROL.allocations.inc()
        resp = dp.AllocateResponse()
        for creq in request.container_requests:
            names, regions = "", []
            cr = resp.container_responses.add()
            for did in creq.devices_ids:
                dev = self.devices.get(did)
                if dev is None:
                    context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                                  f"invalid allocation request with non-existing device: {did}")
                if dev[1] != HEALTHY:
                    context.abort(grpc.StatusCode.INVALID_ARGUMENT,
                                  f"invalid allocation request with unhealthy device: {did}")
                names += did + ","
                host = os.path.join(self.pm.memif_dir(), f"{did}.memif")
                if "/" not in did and os.path.exists(host):
                    target = self.pm.memif_container_path(did)
                    cr.mounts.add(container_path=target, host_path=host, read_only=False)
                    regions.append(target)
            cr.envs["NF-DEV"] = names
            if regions:
                cr.envs["NF-MEMIF"] = ",".join(regions)
        return resp

    def GetPreferredAllocation(self, request, context):
        resp = dp.PreferredAllocationResponse()
        for creq in request.container_requests:
            ids = list(creq.must_include_deviceIDs)
            for d in creq.available_deviceIDs:
                if len(ids) >= creq.allocation_size:
                    break
                if d not in ids:
                    ids.append(d)
            resp.container_responses.add(deviceIDs=ids)
        return resp

    def PreStartContainer(self, request, context):
        return dp.PreStartContainerResponse()

    # ------------------------------------------------------------------ lifecycle
    def setup_devices(self) -> None:
        self.handler.setup_devices()

    def listen(self) -> "DevicePluginServer":
        ep = self.pm.plugin_endpoint()
        os.makedirs(os.path.dirname(ep), exist_ok=True)
        try:
            os.unlink(ep)
        except FileNotFoundError:
            pass
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        self._server.add_generic_rpc_handlers((service_handler(dp, "DevicePlugin", self),))
        self._server.add_insecure_port(unix_target(ep))
        return self

    def serve(self, register: bool = True) -> None:
        assert self._server is not None
        self._server.start()
        ch = grpc.insecure_channel(unix_target(self.pm.plugin_endpoint()))
        grpc.channel_ready_future(ch).result(timeout=5)  # ensureDevicePluginServerStarted
        ch.close()
        if register:
            self.register_with_kubelet()

    def register_with_kubelet(self, timeout: float = 10.0) -> None:
        ch = grpc.insecure_channel(unix_target(self.pm.kubelet_endpoint()))
        try:
            grpc.channel_ready_future(ch).result(timeout=timeout)
            Stub(ch, dp, "Registration").Register(dp.RegisterRequest(
                version=DEVICE_PLUGIN_VERSION, endpoint=self.pm.plugin_endpoint_filename(),
                resource_name=self.resource_name, options=dp.DevicePluginOptions()), timeout=timeout)
            self.registered = True
        finally:
            ch.close()

    def stop(self) -> None:
        self._stop.set()
        if self._server is not None:
            self._server.stop(grace=0.5)
            self._server = None
        try:
            os.unlink(self.pm.plugin_endpoint())
        except FileNotFoundError:
            pass


def wait_until(pred, timeout: float, interval: float = 0.05) -> bool:
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout:
        if pred():
            return True
        time.sleep(interval)
    return pred()
