"""In-process kubelet + cluster stand-ins for control-plane tests.

The reference's daemon tests run against a Kind cluster (internal/testutils/kindcluster.go) and a
real kubelet picks up the device plugin; here:
* FakeKubelet serves the device-plugin Registration service on the kubelet socket; on Register it
  dials the plugin endpoint, consumes ListAndWatch and mirrors the healthy-device count into the
  Node's capacity/allocatable (what makes `openshift.io/dpu` schedulable), and can Allocate.
* cni_call() drives the CNI server exactly as the `dpu-cni` shim does (CNI_* env + stdin config).
"""
from __future__ import annotations

import json
import os
import threading
from concurrent import futures

import grpc

from .. import vars as V
from ..cni.shim import Plugin
from ..k8s.apiserver import ApiServer, make_node
from ..proto import HEALTHY, deviceplugin as dp
from ..proto.grpcutil import Stub, service_handler, unix_target
from ..utils.paths import PathManager


class FakeKubelet:
    def __init__(self, pm: PathManager, api: ApiServer | None = None, node: str = "worker-0"):
        self.pm = pm
        self.api = api
        self.node = node
        self.registrations: list[dp.RegisterRequest] = []
        self.devices: dict[str, dict[str, str]] = {}   # resource -> {id: health}
        self.updates = 0
        self._server: grpc.Server | None = None
        self._watchers: list[threading.Thread] = []
        self._stop = threading.Event()
        self._chans: list[grpc.Channel] = []
        if api is not None and api.try_get("Node", node) is None:
            api.create(make_node(node, labels={"dpu": "true"}))

    # Registration service
    def Register(self, request, context):
        self.registrations.append(request)
        t = threading.Thread(target=self._watch, args=(request,), daemon=True)
        self._watchers.append(t)
        t.start()
        return dp.Empty()

    def _endpoint(self, req) -> str:
        return os.path.join(os.path.dirname(self.pm.kubelet_endpoint()), req.endpoint)

    def _watch(self, req) -> None:
        ch = grpc.insecure_channel(unix_target(self._endpoint(req)))
        self._chans.append(ch)
        stub = Stub(ch, dp, "DevicePlugin")
        try:
            for resp in stub.ListAndWatch(dp.Empty()):
                self.devices[req.resource_name] = {d.ID: d.health for d in resp.devices}
                self.updates += 1
                self._update_node(req.resource_name)
                if self._stop.is_set():
                    break
        except grpc.RpcError:
            pass

    def _update_node(self, resource: str) -> None:
        if self.api is None:
            return
        n = sum(1 for h in self.devices[resource].values() if h == HEALTHY)
        node = self.api.get("Node", self.node)
        st = node.setdefault("status", {})
        st.setdefault("capacity", {})[resource] = str(len(self.devices[resource]))
        st.setdefault("allocatable", {})[resource] = str(n)
        self.api.update_status(node)

    def allocatable(self, resource: str = V.RESOURCE_NAME) -> int:
        return sum(1 for h in self.devices.get(resource, {}).values() if h == HEALTHY)

    def allocate(self, ids: list[str], resource: str = V.RESOURCE_NAME):
        req = next(r for r in self.registrations if r.resource_name == resource)
        ch = grpc.insecure_channel(unix_target(self._endpoint(req)))
        try:
            return Stub(ch, dp, "DevicePlugin").Allocate(
                dp.AllocateRequest(container_requests=[dp.ContainerAllocateRequest(devices_ids=ids)]), timeout=5)
        finally:
            ch.close()

    def start(self) -> "FakeKubelet":
        ep = self.pm.kubelet_endpoint()
        os.makedirs(os.path.dirname(ep), exist_ok=True)
        if os.path.exists(ep):
            os.unlink(ep)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        self._server.add_generic_rpc_handlers((service_handler(dp, "Registration", self),))
        self._server.add_insecure_port(unix_target(ep))
        self._server.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        for ch in self._chans:
            ch.close()
        if self._server is not None:
            self._server.stop(grace=0.2)
            self._server = None


def cni_call(socket_path: str, command: str, conf: dict, *, netns: str = "fakenetns", ifname: str = "eth0",
             container_id: str = "fakecontainerid", pod_ns: str = "x", pod_name: str = "y", pod_uid: str = "z"):
    """POST one CNI request like the dpu-cni shim (cni/shim.py) -> response dict."""
    env = {"CNI_COMMAND": command, "CNI_CONTAINERID": container_id, "CNI_NETNS": netns, "CNI_IFNAME": ifname,
           "CNI_PATH": "/opt/cni/bin",
           "CNI_ARGS": f"K8S_POD_NAMESPACE={pod_ns};K8S_POD_NAME={pod_name};K8S_POD_UID={pod_uid}"}
    return Plugin(socket_path).post_request(env, json.dumps(conf).encode())
