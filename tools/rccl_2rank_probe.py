"""Can two ranks share one GPU over RCCL on this box?  (Rehearsal of the N>1 bench path on a
1-GPU box: correctness only, not performance.)  torchrun --nproc-per-node 2 tools/rccl_2rank_probe.py"""
import os

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((world * 4,), rank, dtype=torch.int32, device=dev)
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
torch.cuda.synchronize()
print(rank, y.tolist(), flush=True)
dist.barrier()
dist.destroy_process_group()
