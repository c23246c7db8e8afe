"""Can RCCL put two ranks on ONE GPU?  (The split's RCCL branch has only run over gloo / device copies on the
1-GPU boxes.)  Two processes, backend nccl, device 0 for both; all_to_all_single + all_reduce of small tensors."""
import os
import sys

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
x = torch.arange(8, dtype=torch.int32, device="cuda") + 100 * rank
y = torch.empty_like(x)
dist.all_to_all_single(y, x)
z = torch.ones(4, device="cuda") * (rank + 1)
dist.all_reduce(z)
torch.cuda.synchronize()
print(f"rank {rank}: all_to_all {y.tolist()} all_reduce {z.tolist()}", flush=True)
dist.destroy_process_group()
