"""Probe: can two ranks share one GPU over RCCL (nccl backend)?  If so, the graph-captured bucketed
all-reduce (GradAllReduce inside GraphedTrainStep) can be tested at world size 2 on a 1-GPU box.
    python tools/probes/rccl_one_gpu.py   (spawns 2 ranks itself)"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE="2")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {rank} eager all_reduce -> {x[0].item()}", flush=True)
    g = torch.cuda.CUDAGraph()
    y = torch.full((1 << 20,), float(rank + 1), device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
        dist.all_reduce(y)
    y.fill_(float(rank + 1))
    g.replay()
    torch.cuda.synchronize()
    print(f"rank {rank} captured all_reduce -> {y[0].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(29533,), nprocs=2, join=True)
    print("RCCL_ONE_GPU_OK")
