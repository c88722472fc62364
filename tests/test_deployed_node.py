"""The deployed MI355X node with real traffic (dpu_operator_amd/testutils/deployed.py): the VSP the
detector deploys (its exact argument list: live, native engine, veth vports, a wire port) behind
the node daemon, device plugin and CNI; netns pods and an external host; pod <-> pod,
pod <-> external, an SFC network-function pod (pod -> NF -> external, NF -> external, pod <-> NF)
— the reference's e2e traffic suite (e2e_test/e2e_test.go:399-512) on one node.

On CPU the data plane is the bit-exact oracle; the `gpu` tests run with the resident ring kernel
on cuda:0.  Namespaces need CAP_NET_ADMIN: where the tests run as an ordinary user the netns
scenario runs in a child process in a user + network + mount namespace of its own
(`unshare -Urnm`).  The MI355X box of this pool has neither (uid nobody, no capabilities,
user.max_user_namespaces = 0: profiles/r5_s1_box_probe.txt), so there the same VSP arguments run
with shared-memory vports and a shared-memory wire (`run_memif`: the same pod / NF / external
checks, frames asserted per endpoint) in front of the GPU ring."""
import json
import os
import shutil
import subprocess
import sys
import tempfile

import pytest

from dpu_operator_amd.testutils import netns as NS

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECKS = ["pod_pod", "pod_pod_udp", "pod_ext", "ext_pod", "ext_udp", "nf_pod_pod", "pod_nf", "nf_pod", "nf_ext",
          "pod_ext_nf", "after_nf_del"]


def _unshare_ok() -> bool:
    if not shutil.which("unshare"):
        return False
    try:
        return subprocess.run(["unshare", "-Urnm", "true"], capture_output=True, timeout=20).returncode == 0
    except (OSError, subprocess.TimeoutExpired):
        return False


def _run_isolated(device: str) -> dict:
    """The scenario in `unshare -Urnm` (a child process: this one keeps its namespaces)."""
    d = tempfile.mkdtemp(prefix="dpns", dir="/tmp")
    env = dict(os.environ, DPU_NETNS_DIR=d, PYTHONPATH=REPO + os.pathsep + os.environ.get("PYTHONPATH", ""))
    try:
        r = subprocess.run(["unshare", "-Urnm", sys.executable, "-u", "-m", "dpu_operator_amd.testutils.deployed",
                            "--device", device, "--json"], cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    finally:
        shutil.rmtree(d, ignore_errors=True)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, f"rc={r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-4000:]}"
    return json.loads(line[-1])


def _check(res: dict) -> None:
    assert "--uplink" in res["vsp_args"] and {"--live", "native", "all"} <= set(res["vsp_args"])
    failed = [k for k in CHECKS if not res.get(k)]
    assert not failed, (failed, res)
    assert res["error"] is None and res["ok"]
    assert res["nf_forwarded"] > 0


@pytest.mark.skipif(not NS.privileged(), reason="needs CAP_NET_ADMIN + CAP_SYS_ADMIN (netns, veth)")
def test_deployed_node_traffic_cpu_oracle():
    from dpu_operator_amd.testutils import deployed

    res = deployed.run("cpu")
    _check(res)
    assert not res["ring_on_gpu"]


@pytest.mark.gpu
def test_deployed_node_traffic_on_the_gpu_ring():
    """The deployed default in front of the resident ring kernel on cuda:0."""
    if NS.privileged():
        from dpu_operator_amd.testutils import deployed

        res = deployed.run("cuda:0")
    elif _unshare_ok():
        res = _run_isolated("cuda:0")
    else:
        pytest.skip("no CAP_NET_ADMIN and no user namespaces")
    _check(res)
    assert res["ring_on_gpu"]


def _check_memif(res: dict) -> None:
    assert {"--live", "native", "all", "--uplink"} <= set(res["vsp_args"])
    failed = [k for k in res["checks"] if not res.get(k)]
    assert not failed, (failed, res)
    assert res["error"] is None and res["ok"] and res["engine"]["learn_events"] >= 1


def test_deployed_node_memif_cpu_oracle():
    from dpu_operator_amd.testutils import deployed

    res = deployed.run_memif("cpu")
    _check_memif(res)
    assert not res["ring_on_gpu"]


@pytest.mark.gpu
def test_deployed_node_memif_on_the_gpu_ring():
    """The detector's VSP (memif vports, memif wire) in front of the resident ring on cuda:0:
    pod <-> pod, flooding then learning on the wire, pod -> NF -> external, external -> NF -> pod,
    the NF hairpin, and the plain bridge again after the NF is gone."""
    from dpu_operator_amd.testutils import deployed

    res = deployed.run_memif("cuda:0")
    _check_memif(res)
    assert res["ring_on_gpu"]
