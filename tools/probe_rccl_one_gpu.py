"""Probe: can two RCCL ("nccl" backend) ranks share one GPU on this box?  If
so the N>1 RCCL halo path of bench.py can be exercised on a 1-GPU box.
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/probe_rccl_one_gpu.py"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
x = torch.full((4,), float(rank), device=dev)
out = torch.empty(8, device=dev)
dist.all_gather_into_tensor(out, x)
torch.cuda.synchronize()
print(f"rank {rank}: all_gather -> {out.tolist()}", flush=True)
dist.destroy_process_group()
