"""Drain helper (reference pkgs/drain/drain_test.go): drain cordons the node and evicts its
workload, a new pod cannot land on the cordoned node, completing the drain makes it schedulable
and the pending pod runs again."""
from dpu_operator_amd.drain import Drainer
from dpu_operator_amd.k8s.apiserver import ApiServer, make_node


def _pod(name, node=None, owner_kind=None):
    p = {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "namespace": "default"},
         "spec": {"containers": [{"name": "c", "image": "ubi"}]}}
    if node:
        p["spec"]["nodeName"] = node
    if owner_kind:
        p["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": owner_kind, "name": "o", "uid": "u-" + name,
                                             "controller": True}]
    return p


def test_drain_and_complete():
    api = ApiServer()
    api.create(make_node("worker-0"))
    api.create(_pod("ds", "worker-0", "DaemonSet"))
    api.create(_pod("managed", "worker-0", "ReplicaSet"))
    api.create(_pod("bare", "worker-0"))
    hooks = []
    d = Drainer(api, on_drain=lambda n: hooks.append(("drain", n)), on_complete=lambda n: hooks.append(("done", n)))
    assert d.drain_node("worker-0") is False          # the unmanaged pod blocks a non-forced drain
    names = {p["metadata"]["name"] for p in api.list("Pod")}
    assert names == {"ds", "bare"}
    assert api.get("Node", "worker-0")["spec"]["unschedulable"] is True
    assert d.drain_node(api.get("Node", "worker-0"), force=True) is True
    assert {p["metadata"]["name"] for p in api.list("Pod")} == {"ds"}
    api.create(_pod("test-pod"))
    assert api.get("Pod", "test-pod")["status"]["phase"] == "Pending"
    d.complete_drain_node("worker-0")
    assert not api.get("Node", "worker-0")["spec"]["unschedulable"]
    api.update(api.get("Node", "worker-0"))  # node update triggers the scheduler
    p = api.get("Pod", "test-pod")
    assert p["spec"]["nodeName"] == "worker-0" and p["status"]["phase"] == "Running"
    assert hooks == [("drain", "worker-0"), ("drain", "worker-0"), ("done", "worker-0")]
