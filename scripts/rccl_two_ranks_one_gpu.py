#!/usr/bin/env python3
"""Probe: can two RCCL ranks share one GPU on this box (a real multi-rank collective on a 1-GPU machine)?

usage: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
           scripts/rccl_two_ranks_one_gpu.py
Each rank all-reduces rank + 1 on cuda:0 through the nccl (RCCL) backend and prints what it got.
"""
import os

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(t)
    torch.cuda.synchronize()
    want = world * (world + 1) / 2
    print(f"rank {rank}/{world}: got {t[0].item()} want {want} ok={bool((t == want).all())}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
