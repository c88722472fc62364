"""Real multi-GPU (>= 2 visible MI355X) checks: a 2-rank RCCL device all-to-all and the N = 2
bench path (rss flow sharding over RCCL/xGMI).  Skipped on boxes with fewer than 2 GPUs (the
1-GPU path is rehearsed in test_dataplane_gpu.py::test_bench_multirank_rehearsal_on_one_gpu)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpus() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


needs2 = pytest.mark.skipif(_gpus() < 2, reason="needs >= 2 GPUs")


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


_A2A = r"""
import os, torch, torch.distributed as dist
r = int(os.environ["RANK"]); w = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(r)
dist.init_process_group("nccl", device_id=torch.device("cuda", r))
x = torch.arange(w * 1024, dtype=torch.int32, device="cuda") + r * 100000
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
exp = torch.cat([torch.arange(r * 1024, (r + 1) * 1024, dtype=torch.int32, device="cuda") + s * 100000 for s in range(w)])
assert torch.equal(y, exp)
dist.barrier(); dist.destroy_process_group()
print("A2A_OK", r)
"""


@needs2
def test_rccl_all_to_all_2ranks(tmp_path):
    f = tmp_path / "a2a.py"
    f.write_text(_A2A)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(f)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0 and r.stdout.count("A2A_OK") == 2, r.stderr[-2000:]


@needs2
def test_bench_rss_two_gpus():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2", "--steps", "5",
           "--warmup", "2", "--batch", str(1 << 18), "--flows", str(1 << 17), "--no-variants"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    import bench

    assert line["n_gpus"] == 2 and line["forwarded_fraction"] == 1.0
    assert line["exchange"]["a2a_per_step"] == bench.RSS_A2A_PER_STEP
    assert set(line["exchange"]) == set(bench.RSS_EXCHANGE_KEYS)
    # the exchange-bound variant: unsteered traffic, half of every batch over xGMI at N = 2
    assert set(line["unsteered"]) == set(bench.RSS_UNSTEERED_KEYS)
    assert line["unsteered"]["remote_frac"] == 0.5 and line["unsteered"]["sent_per_gpu_per_step"] > 0
