"""Process-group bring-up for torchrun-style launches (one process per GPU).

``torchrun --nproc-per-node N --master-addr 127.0.0.1 ...`` exports RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT; ``init_distributed`` binds the process to ``cuda:LOCAL_RANK`` and joins
the group over RCCL (backend "nccl" on ROCm, which runs over xGMI inside a node) or gloo on CPU.
Errors are re-raised tagged with the rank so a failing replica is identifiable in merged logs.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def init_distributed(backend: Optional[str] = None) -> Tuple[int, int, torch.device]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        be = backend or os.environ.get("RDP_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
        dist.init_process_group(backend=be, device_id=dev if be == "nccl" else None)
    return rank, world, dev


def shutdown_distributed() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


@contextlib.contextmanager
def rank_tagged_errors():
    rank = os.environ.get("RANK", "0")
    try:
        yield
    except Exception as e:
        raise RuntimeError(f"[rank {rank}] {type(e).__name__}: {e}") from e
