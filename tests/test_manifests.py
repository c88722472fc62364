"""Deployment packaging (config/, examples/, bundle/) is generated from the code and stays in sync
with what the operator actually does (reference: config/**, examples/*.yaml, bundle/)."""
import os

import yaml

from dpu_operator_amd import manifests as M
from dpu_operator_amd import vars as V
from dpu_operator_amd.api import v1
from dpu_operator_amd.k8s.apiserver import ApiServer
from dpu_operator_amd.k8s.manager import Request

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# kind -> (api group, resource) for everything the operator renders
RESOURCES = {
    "DaemonSet": ("apps", "daemonsets"), "Deployment": ("apps", "deployments"), "Service": ("", "services"),
    "ServiceAccount": ("", "serviceaccounts"), "ConfigMap": ("", "configmaps"), "Secret": ("", "secrets"),
    "ClusterRole": ("rbac.authorization.k8s.io", "clusterroles"),
    "ClusterRoleBinding": ("rbac.authorization.k8s.io", "clusterrolebindings"),
    "Role": ("rbac.authorization.k8s.io", "roles"), "RoleBinding": ("rbac.authorization.k8s.io", "rolebindings"),
    "NetworkAttachmentDefinition": ("k8s.cni.cncf.io", "network-attachment-definitions"),
    "MutatingWebhookConfiguration": ("admissionregistration.k8s.io", "mutatingwebhookconfigurations"),
    "ValidatingWebhookConfiguration": ("admissionregistration.k8s.io", "validatingwebhookconfigurations"),
}


def _load(rel):
    with open(os.path.join(REPO, rel)) as f:
        return [d for d in yaml.safe_load_all(f) if d is not None]


def test_checked_in_manifests_are_up_to_date():
    stale = []
    for rel, docs in M.tree().items():
        path = os.path.join(REPO, rel)
        if not os.path.exists(path) or open(path).read() != M.render(docs):
            stale.append(rel)
    assert not stale, f"regenerate with `python -m dpu_operator_amd.manifests --out .`: {stale}"


def test_all_yaml_parses_and_kustomizations_resolve():
    for rel in M.tree():
        docs = _load(rel)
        assert docs, rel
        for d in docs:
            if d.get("kind") == "Kustomization":
                base = os.path.dirname(os.path.join(REPO, rel))
                for r in d["resources"]:
                    assert os.path.exists(os.path.join(base, r)), (rel, r)


def test_samples_and_examples_are_admitted():
    from dpu_operator_amd.controller.operator import install_webhook

    api = ApiServer(scheduler=False)
    for c in _load("config/crd/bases/config.openshift.io_dpuoperatorconfigs.yaml") + \
            _load("config/crd/bases/config.openshift.io_servicefunctionchains.yaml"):
        api.create(c)
    install_webhook(api)
    for rel in ("examples/dpu.yaml", "config/samples/config_v1_servicefunctionchain.yaml", "examples/sfc.yaml"):
        for d in _load(rel):
            if d["kind"] == v1.KIND_SFC:
                v1.validate_sfc(d)
            else:
                v1.validate_dpu_operator_config(d)
            if api.try_get(d["kind"], d["metadata"]["name"], d["metadata"].get("namespace")) is None:
                api.create(d)
    assert api.get(v1.KIND_DPU_OPERATOR_CONFIG, V.DPU_OPERATOR_CONFIG_NAME)["spec"]["mode"] == "dpu"


def test_manager_args_are_operator_flags():
    from dpu_operator_amd.cmd.operator import build_parser

    dep = [d for d in _load("config/manager/manager.yaml") if d["kind"] == "Deployment"][0]
    c = dep["spec"]["template"]["spec"]["containers"][0]
    a = build_parser().parse_args(c["args"])
    assert a.leader_elect and a.metrics_bind_address == f":{M.METRICS_PORT}"
    probe = c["livenessProbe"]["httpGet"]
    assert probe["port"] == M.PROBE_PORT and f":{probe['port']}" == a.health_probe_bind_address
    envs = {e["name"] for e in c["env"]}
    from dpu_operator_amd.images import all_image_keys

    assert set(all_image_keys()) <= envs


def _allowed(rules, group, resource, verb):
    for r in rules:
        if group in r["apiGroups"] and (resource in r["resources"] or "*" in r["resources"]) and \
                (verb in r["verbs"] or "*" in r["verbs"]):
            return True
    return False


def test_manager_role_covers_everything_the_operator_renders():
    from dpu_operator_amd.controller.operator import DpuOperatorConfigReconciler, install_webhook
    from dpu_operator_amd.images import DummyImageManager

    rules = _load("config/rbac/role.yaml")[0]["rules"]
    for mode in ("host", "dpu"):
        api = ApiServer(scheduler=False)
        api.create({"apiVersion": "apiextensions.k8s.io/v1", "kind": "CustomResourceDefinition",
                    "metadata": {"name": "clusterversions.config.openshift.io"}})  # OpenShift flavour marker
        install_webhook(api)
        rec = DpuOperatorConfigReconciler(api, DummyImageManager())
        api.create({"apiVersion": v1.API_VERSION, "kind": v1.KIND_DPU_OPERATOR_CONFIG,
                    "metadata": {"name": V.DPU_OPERATOR_CONFIG_NAME}, "spec": {"mode": mode}})
        rec.reconcile(Request("", V.DPU_OPERATOR_CONFIG_NAME))
        kinds = {k[0] for k in api._objs}
        rendered = kinds & set(RESOURCES)
        assert "DaemonSet" in rendered and "NetworkAttachmentDefinition" in rendered
        for kind in rendered:
            g, res = RESOURCES[kind]
            for verb in ("create", "get", "update"):
                assert _allowed(rules, g, res, verb), (kind, verb)
    # the operator's own CRs and leader election
    for res in ("dpuoperatorconfigs", "servicefunctionchains"):
        assert _allowed(rules, v1.GROUP, res, "watch")
    lease = _load("config/rbac/leader_election_role.yaml")[0]["rules"]
    assert _allowed(lease, "coordination.k8s.io", "leases", "update")


def test_bundle_csv_owns_the_crds_and_ships_the_manager():
    csv = _load(f"bundle/manifests/{M.PROJECT}.clusterserviceversion.yaml")[0]
    owned = {o["name"] for o in csv["spec"]["customresourcedefinitions"]["owned"]}
    assert owned == {c["metadata"]["name"] for c in v1.crd_manifests()}
    dep = csv["spec"]["install"]["spec"]["deployments"][0]
    assert dep["spec"]["template"]["spec"]["containers"][0]["command"][-1] == "dpu_operator_amd.cmd.operator"
    examples = yaml.safe_load(csv["metadata"]["annotations"]["alm-examples"])
    assert {e["kind"] for e in examples} == {v1.KIND_DPU_OPERATOR_CONFIG, v1.KIND_SFC}


def test_dockerfile_targets_run_real_entry_points():
    """Every image target of the Dockerfile starts an existing entry point with accepted flags, and
    the Makefile builds exactly those targets."""
    import importlib
    import re

    text = open(os.path.join(REPO, "Dockerfile")).read()
    targets = re.findall(r"^FROM \S+ AS (\S+)$", text, flags=re.M)
    images = [t for t in targets if t not in ("build", "runtime")]
    mk = open(os.path.join(REPO, "Makefile")).read()
    assert re.search(r"^IMAGES := (.*)$", mk, flags=re.M).group(1).split() == images
    for ep in re.findall(r"^ENTRYPOINT (\[.*\])$", text, flags=re.M):
        argv = __import__("json").loads(ep)
        if argv[0] != "python3":
            assert argv[0].endswith("dpu-cp-agent")
            continue
        mod = importlib.import_module(argv[2])
        if argv[3:] and hasattr(mod, "build_parser"):
            mod.build_parser().parse_args(argv[3:])
        elif argv[3:]:
            src = open(mod.__file__).read()
            for a in argv[3:]:
                if not a.startswith("--"):
                    assert f'"{a}"' in src, (argv, a)
