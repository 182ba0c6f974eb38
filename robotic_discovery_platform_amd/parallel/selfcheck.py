"""Self-check of the DDP collective path before a multi-rank run is timed (bench.py, world > 1).

The reference trains on one device (``/root/reference/scripts/train_segmenter.py:156-165``); the DDP
step here all-reduces gradient buckets with ``ncclAllReduce`` issued natively on the wgrad side stream
(``parallel/ddp.py`` native_comm_group, ``csrc/bindings.cpp`` comm_all_reduce). A one-GPU box can only
run that path at world 1, where RCCL moves nothing, so the first real multi-rank run of it must check
itself and report what it saw:

  * ``rccl_ranks``: the rank count of the gradient communicator as RCCL sees it (ncclCommCount); a count
    different from WORLD_SIZE is fatal (:class:`CommMismatch`) -- the numbers would be meaningless;
  * a correctness probe through the SAME call and issue path as the buckets (fp32 and bf16 buffers
    filled with rank + 1, all-reduced on a side stream, checked against N (N + 1) / 2 everywhere),
    bounded by a host timeout; every rank's verdict is combined over the default process group, so all
    ranks take the same decision;
  * on a failed probe the run falls back to torch.distributed issue (``RDP_DDP_COMM=torch``, c10d's
    own work objects and timeouts) and reports ``ddp_comm: "torch (native probe failed: ...)"``
    instead of dying or printing numbers from a broken reduction;
  * the bus bandwidth of 16 MB and 64 MB all-reduces on the path that will run
    (``allreduce_busbw_gbps``: 2 (n - 1) / n x bytes / time, the figure the one-GPU emulation of
    ``RDP_DDP_EMULATE`` assumed).

The all-reduce callables are injectable so the decision logic is tested on CPU with gloo
(``tests/test_bench_cli_cpu.py``); ``RDP_COMM_PROBE_FAIL=1`` corrupts the probe's result (test hook).
"""
from __future__ import annotations

import os
import time
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.distributed as dist

from .ddp import dist_info, native_comm_group


class CommMismatch(RuntimeError):
    """The gradient communicator does not span the job's ranks."""


def _sync_wait(dev: torch.device, stream, timeout_s: float, poll_err: Optional[Callable[[], Tuple[int, str]]]):
    """Wait for ``stream``'s work with a host-side bound; raises TimeoutError / RuntimeError."""
    if dev.type != "cuda":
        return
    ev = torch.cuda.Event()
    ev.record(stream)
    t0 = time.monotonic()
    while not ev.query():
        if poll_err is not None:
            code, text = poll_err()
            if code:
                raise RuntimeError(f"RCCL async error {code}: {text}")
        if time.monotonic() - t0 > timeout_s:
            raise TimeoutError(f"probe all-reduce incomplete after {timeout_s:.0f} s")
        time.sleep(0.001)


def probe_all_reduce(all_reduce: Callable[[torch.Tensor], None], dev: torch.device, rank: int, world: int,
                     numel: int = 1 << 20, timeout_s: float = 120.0,
                     poll_err: Optional[Callable[[], Tuple[int, str]]] = None,
                     inject: bool = False) -> Tuple[bool, str]:
    """Every rank fills rank + 1 (fp32 and bf16) and all-reduces through ``all_reduce`` on a side
    stream; the result must be N (N + 1) / 2 in every element (exact in bf16 up to N = 21).
    ``inject``: report the sums off by one (test hook for the fallback path)."""
    want = world * (world + 1) / 2
    try:
        side = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        bufs = []
        for dt in (torch.float32, torch.bfloat16):
            if dt == torch.bfloat16 and (world > 21 or dev.type != "cuda"):
                continue  # bf16 sums stop being exact / gloo has no bf16 SUM on every build
            t = torch.full((numel,), float(rank + 1), dtype=dt, device=dev)
            if side is not None:
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    all_reduce(t)
            else:
                all_reduce(t)
            bufs.append(t)
        _sync_wait(dev, side, timeout_s, poll_err)
        for t in bufs:
            got = t.float()
            if inject:
                got = got + 1.0
            bad = int((got != want).sum().item())
            if bad:
                first = float(got[(got != want).nonzero()[0, 0]].item())
                return False, f"{bad} of {numel} {str(t.dtype).replace('torch.', '')} elements wrong " \
                              f"(expected {want:g}, e.g. {first:g})"
        return True, "ok"
    except Exception as e:  # the verdict is combined over ranks below; never raise from one rank
        return False, f"{type(e).__name__}: {e}"


def busbw(all_reduce: Callable[[torch.Tensor], None], dev: torch.device, world: int, mb: float,
          iters: int = 10, warmup: int = 3) -> Dict[str, float]:
    """Time ``iters`` back-to-back all-reduces of ``mb`` MB fp32 on the issue path; bus bandwidth as
    nccl-tests define it: algbw x 2 (n - 1) / n."""
    n = int(mb * (1 << 20) // 4)
    t = torch.ones(n, dtype=torch.float32, device=dev)
    for _ in range(warmup):
        all_reduce(t)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        all_reduce(t)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / iters
    alg = n * 4 / dt / 1e9
    return {"us": round(dt * 1e6, 1), "algbw_gbps": round(alg, 2),
            "busbw_gbps": round(alg * 2 * (world - 1) / world, 2)}


class NativePath:
    """The gradient buckets' native collective: RCCL's view of the communicator and its exact call."""

    def __init__(self, dev: torch.device):
        from ..ops import native
        self.C = C = native(build_if_missing=False)
        _, self.ptr = native_comm_group(dev)
        self.all_reduce = lambda t: C.comm_all_reduce(t, self.ptr)  # what FlatBucketer._launch issues

    def info(self) -> Tuple[int, int, int]:
        return tuple(self.C.comm_info(self.ptr))  # (ranks, this rank, device)

    def poll(self) -> Tuple[int, str]:
        return tuple(self.C.comm_async_error(self.ptr))

    def abort(self) -> None:
        self.C.comm_abort(self.ptr)


def comm_selfcheck(dev: torch.device, want_native: bool, measure_bw: bool = True,
                   timeout_s: Optional[float] = None, native_path: Optional[Callable[[], object]] = None
                   ) -> Dict[str, object]:
    """Run before the trainer is built (its DDP path reads ``RDP_DDP_COMM``). Returns the JSON fields;
    raises :class:`CommMismatch` if RCCL's communicator does not span WORLD_SIZE ranks, RuntimeError if
    no collective path passes the probe. ``native_path``: factory of the native path (tests inject
    fakes with the :class:`NativePath` interface)."""
    rank, world = dist_info()
    timeout_s = float(os.environ.get("RDP_COMM_PROBE_TIMEOUT_S", "120")) if timeout_s is None else timeout_s
    out: Dict[str, object] = {"dist_backend": dist.get_backend(), "world_size": world}
    native_ar, poll, nat = None, None, None
    why = "not requested"
    if want_native:
        try:
            nat = NativePath(dev) if native_path is None else native_path()
            n, crank, cdev = nat.info()
            out["rccl_ranks"] = int(n)
            out["rccl_device"] = int(cdev)
            if int(n) != world or int(crank) != rank:
                raise CommMismatch(f"[rank {rank}] RCCL gradient communicator has {n} ranks (this one is rank "
                                   f"{crank}) but WORLD_SIZE is {world}")
            native_ar, poll = nat.all_reduce, nat.poll
        except CommMismatch:
            raise
        except Exception as e:
            why = f"{type(e).__name__}: {e}"
    torch_ar = lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM)  # noqa: E731

    def agree(ok: bool) -> bool:  # every rank takes the same decision (default group, c10d)
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                            device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())

    ok = False
    if native_ar is not None:
        ok, why = probe_all_reduce(native_ar, dev, rank, world, timeout_s=timeout_s, poll_err=poll,
                                   inject=os.environ.get("RDP_COMM_PROBE_FAIL", "0") == "1")
    ok = agree(ok)
    if native_ar is not None and not ok and why.startswith(("TimeoutError", "RuntimeError: RCCL async error")):
        # a probe collective may still wait on a peer: release it (the buckets go through c10d now; the
        # aborted communicator's group then fails its own teardown, which bench.py tolerates). A probe
        # that completed with wrong sums leaves the communicator intact.
        try:
            nat.abort()
        except Exception:
            pass
    if want_native and ok:
        out["ddp_comm"] = "native"
        out["comm_probe"] = "ok"
        chosen = native_ar
    else:
        # torch.distributed issue: c10d work objects, its own timeouts (RDP_DDP_COMM is read by NativeTrainer)
        if want_native:
            os.environ["RDP_DDP_COMM"] = "torch"
        tok, twhy = probe_all_reduce(torch_ar, dev, rank, world, timeout_s=timeout_s)
        tok = agree(tok)
        if not tok:
            raise RuntimeError(f"[rank {rank}] no collective path passed the all-reduce probe "
                               f"(native: {why}; torch.distributed: {twhy})")
        out["ddp_comm"] = f"torch (native probe failed: {why})" if want_native else "torch"
        out["comm_probe"] = "ok (torch.distributed)"
        chosen = torch_ar
    if measure_bw and world > 1:
        for mb in (16, 64):
            r = busbw(chosen, dev, world, mb)
            out[f"allreduce_{mb}mb_us"] = r["us"]
            out[f"allreduce_{mb}mb_busbw_gbps"] = r["busbw_gbps"]
        out["allreduce_busbw_gbps"] = out["allreduce_64mb_busbw_gbps"]
    return out
