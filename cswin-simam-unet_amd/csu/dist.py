"""Data-parallel plumbing: one process per GPU over RCCL (torch.distributed 'nccl' on ROCm).

The reference is single-device (cswin:865); SURVEY §8e: CSWin-UNet has no BatchNorm, so averaging
per-rank gradients of equal per-rank batches equals the global-batch gradient.  Buckets are sized
for xGMI point-to-point rings: 94 MB of fp32 gradients go in 64 MB buckets (2 all-reduces per step,
the first overlapped with the rest of backward)."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_distributed(backend: str = None):
    """Initialise from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).
    Returns (rank, world, device).  Single-process when WORLD_SIZE is unset or 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", local) if use_cuda else torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if use_cuda:
            torch.cuda.set_device(local)
            dist.init_process_group(backend or "nccl", device_id=device)
        else:
            dist.init_process_group(backend or "gloo")
    return rank, world, device


def wrap_ddp(model: torch.nn.Module, device: torch.device, bucket_cap_mb: int = 64):
    """DistributedDataParallel with gradient buckets as views (no copy into the bucket) and a
    static graph (every parameter receives a gradient every step, SURVEY §4 KAT iii)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    ids = [device.index] if device.type == "cuda" else None
    return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids, gradient_as_bucket_view=True,
                                                     static_graph=True, bucket_cap_mb=bucket_cap_mb)


def make_loader(dataset, batch_size: int, shuffle: bool, seed: int = 42, num_workers: int = 0, drop_last=False):
    """DataLoader whose sampler shards the dataset across ranks (each rank sees len/world samples)."""
    sampler = None
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(dataset, shuffle=shuffle, seed=seed,
                                                                  drop_last=drop_last)
        shuffle = False
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, sampler=sampler,
                                       num_workers=num_workers, pin_memory=torch.cuda.is_available(),
                                       drop_last=drop_last)
