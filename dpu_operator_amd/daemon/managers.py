"""Side managers: what the node daemon runs on the host side, the device side, or both (GPU).

Reference: internal/daemon/hostsidemanager.go:29-346 and internal/daemon/dpusidemanager.go:33-292.

HostSideManager — CNI ADD for a workload pod: SR-IOV attach, then OPI CreateBridgePort
  {name "host<pf>-<vf>", ptype ACCESS, mac, logical_bridges ["<vf+2>"]} to the device side over gRPC
  with the reference's retry policy (40 attempts, 1 s -> 16 s, UNAVAILABLE); DEL is symmetric.
DpuSideManager — serves OPI BridgePortService on the address the VSP's Init returned and forwards to
  the VSP; CNI ADD for an NF pod moves its vport netdev in, and once the pod's netns has two MACs it
  calls CreateNetworkFunction(mac0, mac1); DEL tears down.  The reference's unsynchronised macStore is
  guarded by a lock here.
ColocatedSideManager — MI355X nodes are both: one CNI server dispatches NF pods (operator namespace)
  to the device-side handler and everything else to the host-side handler; the host side talks OPI
  to the device side over loopback.
Every manager also runs the SFC reconciler (namespace-scoped) and the device plugin.
"""
from __future__ import annotations

import logging
import threading
from concurrent import futures

import grpc

from .. import vars as V
from ..api.v1 import KIND_SFC
from ..cni import networkfn
from ..cni.ipam import HostLocalIpam
from ..cni.netlink import NetlinkManager
from ..cni.server import Server as CniServer
from ..cni.types import PodRequest
from ..k8s.apiserver import ApiServer
from ..k8s.manager import Manager
from ..proto import GoogleEmpty, opi
from ..config import node_config
from ..proto.grpcutil import Stub, retry_service_config, service_handler
from ..utils.paths import PathManager
from .deviceplugin import DeviceHandler, DevicePluginServer
from .sfc import SfcReconciler

log = logging.getLogger("dpu.sidemanager")


def parse_mac(mac: str) -> bytes:
    parts = mac.split(":")
    if len(parts) != 6:
        raise ValueError(f"Failed to parse Mac '{mac}'")
    return bytes(int(p, 16) for p in parts)


class _Base:
    kind = "base"

    def __init__(self, vsp, api: ApiServer | None, path_manager: PathManager | None, dpu_mode: bool,
                 dp_poll: float = 5.0, register_device_plugin: bool = True, numa_of=None):
        self.vsp = vsp
        self.api = api
        self.pm = path_manager or PathManager("/")
        self.addr, self.port = "", 0
        self.dp = DevicePluginServer(DeviceHandler(vsp, dpu_mode, numa_of=numa_of), self.pm, poll=dp_poll)
        self.register_dp = register_device_plugin
        self.cni: CniServer | None = None
        self.manager: Manager | None = None
        self._stop = threading.Event()
        self.errors: list[Exception] = []

    def start_vsp(self) -> None:
        self.addr, self.port = self.vsp.start()

    def setup_devices(self) -> None:
        self.dp.setup_devices()

    def _setup_reconcilers(self, on_gpu_chain=None) -> None:
        if self.api is None:
            return
        self.manager = Manager(self.api, namespace=V.NAMESPACE)
        self.manager.add("sfc", SfcReconciler(self.api, on_gpu_chain), KIND_SFC, owns=("Pod",))

    def serve_common(self) -> None:
        self.cni.start()
        self.dp.serve(register=self.register_dp)
        if self.manager is not None:
            self.manager.start()

    def wait(self, timeout: float | None = None) -> bool:
        return self._stop.wait(timeout)

    def stop(self) -> None:
        self._stop.set()
        if self.cni is not None:
            self.cni.shutdown()
        self.dp.stop()
        if self.manager is not None:
            self.manager.stop()
        try:
            self.vsp.close()
        except Exception:  # noqa: BLE001
            pass


class HostSideManager(_Base):
    kind = "host"

    def __init__(self, vsp, sriov_manager, api: ApiServer | None = None, path_manager: PathManager | None = None,
                 pf: int = 0, **kw):
        super().__init__(vsp, api, path_manager, dpu_mode=False, **kw)
        self.sm = sriov_manager
        self.pf = pf
        self._conn: grpc.Channel | None = None
        self._client = None
        self._lock = threading.Lock()

    def connect_with_retry(self):
        with self._lock:
            if self._client is None:
                self._conn = grpc.insecure_channel(
                    f"{self.addr}:{self.port}", options=[("grpc.service_config", retry_service_config()),
                                                         ("grpc.enable_retries", 1)])
                self._client = Stub(self._conn, opi, "BridgePortService")
            return self._client

    def create_bridge_port(self, pf: int, vf: int, vlan: int, mac: str):
        client = self.connect_with_retry()
        req = opi.CreateBridgePortRequest(bridge_port=opi.BridgePort(
            name=f"host{pf}-{vf}",
            spec=opi.BridgePortSpec(ptype=opi.BRIDGE_PORT_TYPE_ACCESS, mac_address=parse_mac(mac),
                                    logical_bridges=[str(node_config().logical_bridge(vf))])))
        return client.CreateBridgePort(req, timeout=60)

    def delete_bridge_port(self, pf: int, vf: int, vlan: int, mac: str) -> None:
        client = self.connect_with_retry()
        client.DeleteBridgePort(opi.DeleteBridgePortRequest(name=f"host{pf}-{vf}"), timeout=60)

    def cni_add(self, req: PodRequest) -> dict:
        try:
            res = self.sm.cmd_add(req)
        except Exception as e:
            raise RuntimeError(f"SRIOV manager failed in add handler: {e}") from e
        vf = req.cni_conf.VFID
        mac = req.cni_conf.OrigVfState.EffectiveMAC
        self.create_bridge_port(self.pf, vf, 2, mac)
        return res

    def cni_del(self, req: PodRequest) -> None:
        try:
            self.sm.cmd_del(req)
        except Exception as e:
            raise RuntimeError("SRIOV manager failed in del handler") from e
        try:
            self.delete_bridge_port(self.pf, req.cni_conf.VFID, 2, req.cni_conf.OrigVfState.EffectiveMAC)
        except grpc.RpcError as e:
            log.warning("DeleteBridgePort failed: %s", e)
        return None

    def listen(self) -> None:
        self._setup_reconcilers()
        self.cni = CniServer(self.cni_add, self.cni_del, self.pm).listen()
        self.dp.listen()

    def serve(self) -> None:
        self.serve_common()

    def stop(self) -> None:
        super().stop()
        if self._conn is not None:
            self._conn.close()


class _OpiServicer:
    """OPI BridgePortService on the device side; forwards to the VSP, keeps a port registry."""

    def __init__(self, vsp):
        self.vsp = vsp
        self.ports: dict[str, object] = {}
        self._lock = threading.Lock()

    def CreateBridgePort(self, request, context):
        try:
            bp = self.vsp.create_bridge_port(request)
        except grpc.RpcError as e:
            context.abort(e.code(), e.details())
        with self._lock:
            self.ports[request.bridge_port.name] = bp
        return bp

    def DeleteBridgePort(self, request, context):
        with self._lock:
            known = request.name in self.ports
        if not known and request.allow_missing:
            return GoogleEmpty()
        try:
            self.vsp.delete_bridge_port(request)
        except grpc.RpcError as e:
            context.abort(e.code(), e.details())
        with self._lock:
            self.ports.pop(request.name, None)
        return GoogleEmpty()

    def GetBridgePort(self, request, context):
        with self._lock:
            bp = self.ports.get(request.name)
        if bp is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"unable to find key {request.name}")
        return bp

    def ListBridgePorts(self, request, context):
        with self._lock:
            return opi.ListBridgePortsResponse(bridge_ports=list(self.ports.values()))


class DpuSideManager(_Base):
    kind = "dpu"

    def __init__(self, vsp, nl: NetlinkManager, api: ApiServer | None = None, path_manager: PathManager | None = None,
                 ipam: HostLocalIpam | None = None, on_gpu_chain=None, **kw):
        super().__init__(vsp, api, path_manager, dpu_mode=True, **kw)
        self.nl = nl
        self.ipam = ipam
        self.on_gpu_chain = on_gpu_chain
        self.mac_store: dict[str, list[str]] = {}
        self._mac_lock = threading.Lock()
        self.opi_servicer = _OpiServicer(vsp)
        self.grpc: grpc.Server | None = None

    def nf_add(self, req: PodRequest) -> dict:
        res = networkfn.cmd_add(req, self.nl, self.ipam)
        with self._mac_lock:
            macs = self.mac_store.setdefault(req.netns, [])
            macs.append(req.cni_conf.MAC)
            pair = list(macs) if len(macs) == 2 else None
        if pair:
            self.vsp.create_network_function(pair[0], pair[1])
        return res

    def nf_del(self, req: PodRequest) -> None:
        networkfn.cmd_del(req, self.nl, self.ipam)
        with self._mac_lock:
            macs = self.mac_store.get(req.netns, [])
            pair = list(macs) if len(macs) == 2 else None
            if macs:
                macs.pop()
            if not macs:
                self.mac_store.pop(req.netns, None)
        if pair:
            self.vsp.delete_network_function(pair[0], pair[1])
        return None

    def listen(self, with_cni: bool = True) -> None:
        self._setup_reconcilers(self.on_gpu_chain)
        self.grpc = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        self.grpc.add_generic_rpc_handlers((service_handler(opi, "BridgePortService", self.opi_servicer),))
        bound = self.grpc.add_insecure_port(f"{self.addr}:{self.port}")
        if bound == 0:
            raise OSError(f"Failed to start listening on {self.addr}:{self.port}")
        self.port = bound
        if with_cni:
            self.cni = CniServer(self.nf_add, self.nf_del, self.pm).listen()
        self.dp.listen()

    def serve(self) -> None:
        self.grpc.start()
        self.serve_common()

    def stop(self) -> None:
        if self.grpc is not None:
            self.grpc.stop(grace=0.5)
        super().stop()


class ColocatedSideManager:
    """Device side + host side in one daemon (MI355X: the GPUs are in the host)."""
    kind = "colocated"

    def __init__(self, vsp, sriov_manager, nl: NetlinkManager, api: ApiServer | None = None,
                 path_manager: PathManager | None = None, ipam: HostLocalIpam | None = None, on_gpu_chain=None, **kw):
        if "numa_of" not in kw:
            # GPU vports live on the data-plane GPU: advertise its NUMA node (KFD topology)
            try:
                from .devutils import data_plane_numa

                node = data_plane_numa((path_manager or PathManager("/")).root)
            except Exception:  # noqa: BLE001 - no KFD on this host / native module unavailable
                node = -1
            kw["numa_of"] = (lambda _dev, n=node: n) if node >= 0 else None
        self.dpu = DpuSideManager(vsp, nl, api, path_manager, ipam, on_gpu_chain, **kw)
        self.host = HostSideManager(vsp, sriov_manager, None, path_manager, **{k: v for k, v in kw.items() if k != "numa_of"})
        self.pm = self.dpu.pm

    def start_vsp(self) -> None:
        self.dpu.start_vsp()

    def setup_devices(self) -> None:
        self.dpu.setup_devices()

    @staticmethod
    def _gpu_vport(req: PodRequest) -> int | None:
        """Index of the GPU vport a workload pod was allocated (deviceID = the vport netdev name,
        e.g. dpuvp3 -> 3); None for an SR-IOV VF (PCI address) or no device."""
        import re

        from ..cni.sriov.utils import is_valid_pci_address

        dev = getattr(req.cni_conf, "deviceID", "") if req.cni_conf is not None else ""
        if not dev or is_valid_pci_address(dev):
            return None
        m = re.fullmatch(r"[A-Za-z][\w.-]*?(\d+)", dev)
        return int(m.group(1)) if m else None

    def cni_add(self, req: PodRequest) -> dict:
        if req.pod_namespace == V.NAMESPACE:
            return self.dpu.nf_add(req)
        idx = self._gpu_vport(req)
        if idx is None:
            return self.host.cni_add(req)
        # a GPU vport (veth / TAP netdev): the pod gets the netdev itself (networkfn moves it into
        # its namespace), then the host side's CreateBridgePort host<pf>-<idx> programs the VF port
        res = networkfn.cmd_add(req, self.dpu.nl, self.dpu.ipam)
        try:
            self.host.create_bridge_port(self.host.pf, idx, node_config().logical_bridge(idx), req.cni_conf.MAC)
        except Exception:
            networkfn.cmd_del(req, self.dpu.nl, self.dpu.ipam)
            raise
        return res

    def cni_del(self, req: PodRequest) -> None:
        if req.pod_namespace == V.NAMESPACE:
            return self.dpu.nf_del(req)
        idx = self._gpu_vport(req)
        if idx is None:
            return self.host.cni_del(req)
        networkfn.cmd_del(req, self.dpu.nl, self.dpu.ipam)
        try:
            self.host.delete_bridge_port(self.host.pf, idx, 0, "")
        except grpc.RpcError as e:
            log.warning("DeleteBridgePort failed: %s", e)
        return None

    def listen(self) -> None:
        self.dpu.listen(with_cni=False)
        self.dpu.cni = CniServer(self.cni_add, self.cni_del, self.pm).listen()
        self.host.addr, self.host.port = ("127.0.0.1" if self.dpu.addr in ("", "0.0.0.0", "::") else self.dpu.addr,
                                          self.dpu.port)

    def serve(self) -> None:
        self.dpu.serve()

    @property
    def dp(self):
        return self.dpu.dp

    @property
    def manager(self):
        return self.dpu.manager

    def wait(self, timeout=None) -> bool:
        return self.dpu.wait(timeout)

    def stop(self) -> None:
        self.dpu.stop()
        if self.host._conn is not None:
            self.host._conn.close()
