"""Device-side SFC reconciler: one NF pod per network function of a ServiceFunctionChain.

Reference: internal/daemon/sfc-reconciler/sfc.go:32-144.  Each NF becomes a Pod in the operator
namespace with two `dpunfcni-conf` attachments (NF ingress + egress vports), `openshift.io/dpu: 2`
requests/limits, privileged with NET_RAW/NET_ADMIN, owned by the SFC.  Create-or-update.
Differences from the reference (documented quirks fixed): a deleted SFC is NOT requeued forever
(its pods go away through owner-reference GC), and per-NF errors are reported instead of ignored.

GPU extension: an NF whose image is `gpu-nf://<kind>[,<kind>...]` (acl, nat, l2fwd, ttl, vlan,
hairpin) needs no pod — it runs inside the GPU pipeline; the reconciler records it in the SFC
status and the GPU VSP programs it as a chain hop (see vsp/gpu.py).  `<kind>@<gpu>` places the hop
on one of the node's GPUs: the chain hands its frames over to that GPU mid-chain (the SFC hop
pipeline across GPUs, parallel/hops.py).
"""
from __future__ import annotations

import copy
import logging

from .. import vars as V
from ..api.v1 import KIND_SFC, ServiceFunctionChain
from ..config import node_config
from ..k8s.apiserver import ApiServer, NotFound, set_controller_reference
from ..k8s.manager import Request, Result

log = logging.getLogger("dpu.sfc")
GPU_NF_PREFIX = "gpu-nf://"


def network_function_pod(name: str, image: str) -> dict:
    cfg = node_config()
    nets = ", ".join([cfg.nf_nad_name] * cfg.nf_devices_per_pod)
    return {
        "apiVersion": "v1", "kind": "Pod",
        "metadata": {"name": name, "namespace": V.NAMESPACE,
                     "annotations": {"k8s.v1.cni.cncf.io/networks": nets}},
        "spec": {"containers": [{
            "name": name, "image": image,
            "ports": [{"name": "web", "containerPort": 8080}],
            "resources": {"requests": {cfg.resource_name: str(cfg.nf_devices_per_pod)},
                          "limits": {cfg.resource_name: str(cfg.nf_devices_per_pod)}},
            "securityContext": {"privileged": True,
                                "capabilities": {"drop": ["ALL"], "add": ["NET_RAW", "NET_ADMIN"]}},
        }]},
    }


class SfcReconciler:
    def __init__(self, api: ApiServer, on_gpu_chain=None):
        self.api = api
        self.on_gpu_chain = on_gpu_chain  # callback(sfc_name, [kinds]) for gpu-nf:// functions

    def _create_or_update(self, pod: dict) -> None:
        cur = self.api.try_get("Pod", pod["metadata"]["name"], pod["metadata"]["namespace"])
        if cur is None:
            self.api.create(pod)
        else:
            upd = copy.deepcopy(cur)
            upd["metadata"]["annotations"] = pod["metadata"]["annotations"]
            upd["metadata"]["ownerReferences"] = pod["metadata"]["ownerReferences"]
            upd["spec"]["containers"] = pod["spec"]["containers"]
            self.api.update(upd)

    def reconcile(self, req: Request) -> Result:
        try:
            obj = self.api.get(KIND_SFC, req.name, req.namespace or V.NAMESPACE)
        except NotFound:
            return Result()
        sfc = ServiceFunctionChain.from_obj(obj)
        gpu_kinds, errors = [], []
        for nf in sfc.network_functions:
            if nf.image.startswith(GPU_NF_PREFIX):
                gpu_kinds.extend(k.strip() for k in nf.image[len(GPU_NF_PREFIX):].split(",") if k.strip())
                continue
            pod = network_function_pod(nf.name, nf.image)
            set_controller_reference(obj, pod)
            try:
                self._create_or_update(pod)
            except Exception as e:  # noqa: BLE001
                errors.append(f"{nf.name}: {e}")
        if gpu_kinds and self.on_gpu_chain is not None:
            self.on_gpu_chain(sfc.name, gpu_kinds)
        status = {"networkFunctions": [n.name for n in sfc.network_functions], "gpuHops": gpu_kinds}
        if errors:
            status["errors"] = errors
        obj = self.api.get(KIND_SFC, req.name, req.namespace or V.NAMESPACE)
        if obj.get("status") != status:
            obj["status"] = status
            self.api.update_status(obj)
        return Result(requeue=bool(errors))
