"""API scheme (A6), CRD generation (A4) and typed decoding."""
from __future__ import annotations

import pytest

from dpu_operator_amd import render
from dpu_operator_amd import vars as V
from dpu_operator_amd.api import v1
from dpu_operator_amd.api.scheme import SCHEME
from dpu_operator_amd.controller.operator import DpuOperatorConfigReconciler, setup_operator
from dpu_operator_amd.images import DummyImageManager
from dpu_operator_amd.k8s.apiserver import ApiServer, BadRequest
from dpu_operator_amd.k8s.manager import Request


def test_scheme_rejects_unknown_and_wrong_version():
    api = ApiServer(scheme=SCHEME)
    with pytest.raises(BadRequest):
        api.create({"apiVersion": "v1", "kind": "Frobnicator", "metadata": {"name": "x"}})
    with pytest.raises(BadRequest):
        api.create({"apiVersion": "config.openshift.io/v2", "kind": v1.KIND_SFC, "metadata": {"name": "x"}})
    with pytest.raises(BadRequest):  # schema: image must be a string
        api.create({"apiVersion": v1.API_VERSION, "kind": v1.KIND_SFC, "metadata": {"name": "x"},
                    "spec": {"networkFunctions": [{"name": "a", "image": 3}]}})
    o = api.create({"apiVersion": v1.API_VERSION, "kind": v1.KIND_SFC, "metadata": {"name": "x"},
                    "spec": {"networkFunctions": [{"name": "a", "image": "img"}]}})
    sfc = SCHEME.decode(o)
    assert isinstance(sfc, v1.ServiceFunctionChain) and sfc.network_functions[0].image == "img"


def test_scheme_scope_matches_apiserver():
    from dpu_operator_amd.k8s.apiserver import CLUSTER_SCOPED

    assert SCHEME.cluster_scoped() <= CLUSTER_SCOPED


def test_crds_are_registered_kinds():
    for crd in v1.crd_manifests():
        SCHEME.check(crd)
        names = crd["spec"]["names"]
        assert SCHEME.recognizes(f'{crd["spec"]["group"]}/{crd["spec"]["versions"][0]["name"]}', names["kind"])


@pytest.mark.parametrize("mode", ["host", "dpu"])
def test_operator_objects_pass_scheme(mode):
    """Everything the operator renders from bindata (daemon, NADs, NRI, VSP DaemonSets) is a
    registered kind at the right apiVersion."""
    api = ApiServer(scheme=SCHEME)
    api.create({"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                "metadata": {"name": "clusterversions.config.openshift.io"}})
    setup_operator(api, image_manager=DummyImageManager())
    rec = DpuOperatorConfigReconciler(api, DummyImageManager())
    api.create({"apiVersion": v1.API_VERSION, "kind": v1.KIND_DPU_OPERATOR_CONFIG,
                "metadata": {"name": V.DPU_OPERATOR_CONFIG_NAME}, "spec": {"mode": mode}})
    rec.reconcile(Request("", V.DPU_OPERATOR_CONFIG_NAME))
    assert api.list("DaemonSet", V.NAMESPACE)
    assert api.list("NetworkAttachmentDefinition")
    for sub in ("vsp-ds",):
        for f in render.bindata_files(sub):
            obj = render.render_file(f, {"Namespace": V.NAMESPACE, "VendorSpecificPluginImage": "img",
                                         "ImagePullPolicy": "IfNotPresent", "Command": "[]", "Args": "[]"})
            SCHEME.check(obj)
