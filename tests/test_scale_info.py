"""The N > 1 bench line describes the run it measured (bench.py scale_info):
world size, backend, RCCL version, local GPUs, every rank's own ms per step and the peer-access
matrix.  Checked here with gloo process groups of 2 and 4 CPU ranks (the collective it runs is the
same one the GPU ranks run over RCCL)."""
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        info = bench.scale_info(dist, torch, elapsed_s=0.01 * (rank + 1), steps=10, cdev=torch.device("cpu"))
        q.put((rank, info))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_scale_info_keys_at_world(world):
    sys.path.insert(0, REPO)
    import bench

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r, info in got.items():
        assert set(bench.SCALE_KEYS) <= set(info), info
        assert info["world_size"] == world and info["backend"] == "gloo"
        # every rank sees every rank's own step time (rank r ran (r + 1) ms per step)
        assert info["per_rank_ms_per_step"] == [round(float(k + 1), 4) for k in range(world)]
        assert info["step_skew"] == pytest.approx(world, rel=1e-3)
        assert isinstance(info["peer_access"], list) and len(info["peer_access"]) == info["device_count"]
