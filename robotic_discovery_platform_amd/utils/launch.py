"""Process-group bring-up for torchrun-style launches (one process per GPU).

``torchrun --nproc-per-node N --master-addr 127.0.0.1 ...`` exports RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT; ``init_distributed`` binds the process to ``cuda:LOCAL_RANK`` and joins
the group over RCCL (backend "nccl" on ROCm, which runs over xGMI inside a node) or gloo on CPU.
Errors are re-raised tagged with the rank so a failing replica is identifiable in merged logs.
"""
from __future__ import annotations

import contextlib
import datetime
import os
from typing import Optional, Tuple

import torch
import torch.distributed as dist


def dist_timeout(seconds: Optional[float] = None) -> datetime.timedelta:
    """Process-group timeout (``RDP_DIST_TIMEOUT_S``, default 600 s): a rank that dies or hangs makes
    the others' collectives fail with an error after this long instead of blocking forever (the
    torchrun agent then tears the job down and ``--resume auto`` relaunches from the checkpoint)."""
    if seconds is None:
        seconds = float(os.environ.get("RDP_DIST_TIMEOUT_S", "600"))
    return datetime.timedelta(seconds=float(seconds))


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None,
                     force: bool = False) -> Tuple[int, int, torch.device]:
    """Join the job's process group. ``force=True`` also initialises a 1-rank group (world == 1), so
    the RCCL code paths (bucketed all-reduce, stream semantics) run on a single GPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        be = backend or os.environ.get("RDP_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
        with rank_tagged_errors():
            dist.init_process_group(backend=be, rank=rank, world_size=world, timeout=dist_timeout(timeout_s),
                                    device_id=dev if be == "nccl" else None)
    return rank, world, dev


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def shutdown_distributed() -> None:
    from ..parallel.watchdog import close_all
    close_all()  # they poll communicators of the groups destroyed here
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


@contextlib.contextmanager
def rank_tagged_errors():
    rank = os.environ.get("RANK", "0")
    try:
        yield
    except Exception as e:
        raise RuntimeError(f"[rank {rank}] {type(e).__name__}: {e}") from e


def maybe_crash(epoch: int, rank: Optional[int] = None) -> None:
    """Fault injection for relaunch tests: ``RDP_FAULT_CRASH="<rank>:<epoch>"`` makes that rank die
    (``os._exit(17)``, no cleanup, like a killed process) when it reaches the start of that epoch.
    The surviving ranks then fail their next collective (peer gone / process-group timeout), the
    launcher tears the job down, and a relaunch with ``--resume auto`` continues from the last
    epoch checkpoint."""
    spec = os.environ.get("RDP_FAULT_CRASH", "")
    if not spec:
        return
    r, _, e = spec.partition(":")
    me = int(os.environ.get("RANK", "0")) if rank is None else rank
    if int(r) == me and int(e) == epoch:
        import sys
        print(f"[rank {me}] RDP_FAULT_CRASH: exiting at epoch {epoch}", file=sys.stderr, flush=True)
        os._exit(17)
