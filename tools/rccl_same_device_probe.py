"""Probe: can two ranks share one GPU under the nccl (RCCL) backend on this box? (Rehearsal of the
multi-rank bench path on a one-GPU box; run with torch.distributed.run --nproc-per-node 2.)"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=int(os.environ["WORLD_SIZE"]))
x = torch.arange(8, dtype=torch.int64, device="cuda") + 100 * rank
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
t = torch.tensor([float(rank)], device="cuda")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {rank}: all_to_all {y.tolist()} all_reduce {t.item()}", flush=True)
dist.destroy_process_group()
