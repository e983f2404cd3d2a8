"""Probe: can two RCCL ranks share one GPU on this box?  (tools only)"""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((4,), float(rank + 1), device=dev)
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {x.tolist()}", flush=True)
dist.destroy_process_group()
