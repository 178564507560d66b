"""Probe: can two ranks share one GPU over RCCL (backend nccl)?  Used only to rehearse the
multi-GPU exchange path on a one-GPU box; run with torch.distributed.run --nproc-per-node 2."""
import os
import sys

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
x = torch.arange(8, dtype=torch.int64, device="cuda:0") + 100 * rank
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
s = torch.tensor([rank + 1], dtype=torch.int64, device="cuda:0")
dist.all_reduce(s)
torch.cuda.synchronize()
print(f"rank {rank}: a2a {y.tolist()} allreduce {s.item()}", flush=True)
dist.barrier()
dist.destroy_process_group()
