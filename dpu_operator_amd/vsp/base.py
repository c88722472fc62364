"""VSP gRPC server scaffolding: serves Vendor.{LifeCycle,NetworkFunction,Device}Service and the OPI
BridgePortService on the vendor-plugin unix socket (internal/utils/path_manager.go:58-60).

A VSP implementation subclasses `VspBase` and implements the python-level hooks
(`init`, `create_bridge_port`, `delete_bridge_port`, `create_network_function`,
`delete_network_function`, `get_devices`, `set_num_vfs`); this module maps them onto the wire
messages.  Every hook runs under one lock: the reference's VSPs mutate shared maps from concurrent
RPCs without synchronisation, this one does not.
"""
from __future__ import annotations

import logging
import os
import threading
from concurrent import futures

import grpc

from ..proto import GoogleEmpty, opi, vendor
from ..proto.grpcutil import service_handler, unix_target
from ..utils.faults import FAULTS, FaultError
from ..utils.metrics import CONTROL
from ..utils.trace import TRACER
from ..utils.paths import PathManager

log = logging.getLogger("dpu.vsp")


def _fault_code(e: FaultError) -> grpc.StatusCode:
    return grpc.StatusCode.UNAVAILABLE if e.kind == "unavailable" else grpc.StatusCode.INTERNAL


class VspBase:
    name = "vsp"

    def __init__(self, path_manager: PathManager | None = None):
        self.pm = path_manager or PathManager("/")
        self._lock = threading.RLock()
        self._server: grpc.Server | None = None
        self.calls: list[tuple[str, tuple]] = []

    # -------------------------------------------------------------- hooks (override)
    def init(self, dpu_mode: bool, dpu_identifier: str) -> tuple[str, int]:
        raise NotImplementedError

    def create_bridge_port(self, name: str, mac: bytes, ptype: int, logical_bridges: list[str]) -> None:
        pass

    def delete_bridge_port(self, name: str) -> None:
        pass

    def create_network_function(self, inp: str, out: str) -> None:
        pass

    def delete_network_function(self, inp: str, out: str) -> None:
        pass

    def get_devices(self) -> dict[str, str]:
        return {}

    def set_num_vfs(self, n: int) -> int:
        return n

    # -------------------------------------------------------------- wire adapters
    def _call(self, name, fn, *args):
        FAULTS.check(f"vsp.{name}")
        with self._lock, TRACER.span(f"vsp.{name}"):
            self.calls.append((name, args))
            try:
                out = fn(*args)
            except Exception:
                CONTROL.vsp_calls.labels(name, "error").inc()
                raise
            CONTROL.vsp_calls.labels(name, "success").inc()
            self._journal(name, args)
            return out

    def _journal(self, name: str, args: tuple) -> None:
        """Hook for state journaling of mutating RPCs (see vsp/gpu.py)."""

    def Init(self, request, context):
        try:
            ip, port = self._call("Init", self.init, request.dpu_mode, request.dpu_identifier)
        except FaultError as e:
            context.abort(grpc.StatusCode.UNAVAILABLE if e.kind == "unavailable" else grpc.StatusCode.INTERNAL, str(e))
        except Exception as e:  # noqa: BLE001
            context.abort(grpc.StatusCode.INTERNAL, f"Init failed: {e}")
        return vendor.IpPort(ip=ip, port=port)

    def CreateNetworkFunction(self, request, context):
        try:
            self._call("CreateNetworkFunction", self.create_network_function, request.input, request.output)
        except FaultError as e:
            context.abort(_fault_code(e), str(e))
        except Exception as e:  # noqa: BLE001
            context.abort(grpc.StatusCode.INTERNAL, str(e))
        return vendor.Empty()

    def DeleteNetworkFunction(self, request, context):
        try:
            self._call("DeleteNetworkFunction", self.delete_network_function, request.input, request.output)
        except FaultError as e:
            context.abort(_fault_code(e), str(e))
        except Exception as e:  # noqa: BLE001
            context.abort(grpc.StatusCode.INTERNAL, str(e))
        return vendor.Empty()

    def GetDevices(self, request, context):
        try:
            devs = self._call("GetDevices", self.get_devices)
        except FaultError as e:
            context.abort(_fault_code(e), str(e))
        resp = vendor.DeviceListResponse()
        for did, health in devs.items():
            resp.devices[did].ID = did
            resp.devices[did].health = health
        return resp

    def SetNumVfs(self, request, context):
        try:
            n = self._call("SetNumVfs", self.set_num_vfs, request.vf_cnt)
        except FaultError as e:
            context.abort(_fault_code(e), str(e))
        except Exception as e:  # noqa: BLE001
            context.abort(grpc.StatusCode.INTERNAL, f"SetNumVfs failed: {e}")
        return vendor.VfCount(vf_cnt=n)

    def CreateBridgePort(self, request, context):
        bp = request.bridge_port
        try:
            self._call("CreateBridgePort", self.create_bridge_port, bp.name, bytes(bp.spec.mac_address),
                       bp.spec.ptype, list(bp.spec.logical_bridges))
        except FaultError as e:
            context.abort(_fault_code(e), str(e))
        except Exception as e:  # noqa: BLE001
            context.abort(grpc.StatusCode.INTERNAL, f"CreateBridgePort failed: {e}")
        out = opi.BridgePort()
        out.CopyFrom(bp)
        out.status.oper_status = opi.BP_OPER_STATUS_UP
        return out

    def DeleteBridgePort(self, request, context):
        try:
            self._call("DeleteBridgePort", self.delete_bridge_port, request.name)
        except FaultError as e:
            context.abort(_fault_code(e), str(e))
        except Exception as e:  # noqa: BLE001
            context.abort(grpc.StatusCode.INTERNAL, f"DeleteBridgePort failed: {e}")
        return GoogleEmpty()

    # -------------------------------------------------------------- serving
    def start(self) -> "VspBase":
        sock = self.pm.vendor_plugin_socket()
        PathManager.ensure_socket_dir_exists(sock)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        self._server.add_generic_rpc_handlers((
            service_handler(vendor, "LifeCycleService", self),
            service_handler(vendor, "NetworkFunctionService", self),
            service_handler(vendor, "DeviceService", self),
            service_handler(opi, "BridgePortService", self),
        ))
        self._server.add_insecure_port(unix_target(sock))
        self._server.start()
        log.info("%s serving on %s", self.name, sock)
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=0.5)
            self._server = None
        try:
            os.unlink(self.pm.vendor_plugin_socket())
        except FileNotFoundError:
            pass

    def wait(self) -> None:
        if self._server is not None:
            self._server.wait_for_termination()


class MockVsp(VspBase):
    """Reference: internal/daemon/vendor-specific-plugins/mock-vsp/mockvsp.go:31-152."""

    name = "mock-vsp"

    def __init__(self, path_manager=None, opi_port: int = 50051):
        super().__init__(path_manager)
        self.opi_port = opi_port
        self.bridge_ports: dict[str, dict] = {}
        self.network_functions: list[tuple[str, str]] = []
        self.num_vfs = 0

    def init(self, dpu_mode, dpu_identifier):
        return "127.0.0.1", self.opi_port

    def create_bridge_port(self, name, mac, ptype, logical_bridges):
        self.bridge_ports[name] = {"mac": mac, "ptype": ptype, "bridges": logical_bridges}

    def delete_bridge_port(self, name):
        self.bridge_ports.pop(name, None)

    def create_network_function(self, inp, out):
        self.network_functions.append((inp, out))

    def delete_network_function(self, inp, out):
        if (inp, out) in self.network_functions:
            self.network_functions.remove((inp, out))

    def get_devices(self):
        return {f"ens5f{i}": "Healthy" for i in range(4)}

    def set_num_vfs(self, n):
        self.num_vfs = n
        return n
