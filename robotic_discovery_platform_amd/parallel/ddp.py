"""Data parallelism over RCCL (xGMI) / gloo with flat-buffer gradient buckets.

The reference trains on one device only (``scripts/train_segmenter.py:50,143``).
This module adds the north-star DDP: one process per GPU, parameters broadcast from rank 0,
gradients all-reduced in buckets that are launched *while backward is still running*.

Design (MI355X-first):
  * All gradients live in ONE flat fp32 buffer whose layout is the parameter registration order.
    Backward produces gradients in exactly the reverse order, so buckets are contiguous reverse
    ranges of that buffer -- no gradient copies, no per-parameter launches.
  * A bucket is launched (``all_reduce(SUM, async_op=True)``) as soon as the last parameter in it is
    final; RCCL's internal stream waits on the ISSUING stream at issue time and runs concurrently
    with the remaining backward kernels. ``finish()`` makes the compute stream wait for all buckets.
  * Stream ordering: RCCL (and gloo's CUDA path) orders a collective after the current stream only.
    The native executor produces gradients on two streams (BN / head gradients on the main stream,
    conv weight gradients on the wgrad side stream), so a bucket may only be issued from a stream
    that is ordered after EVERY producer of its gradients. ``launch_ctx`` supplies that stream
    (the executor's wgrad side stream, forked from the main stream where needed:
    ``UNetExecutor.comm_stream``); the bf16 narrowing copy runs there too. :class:`StreamOrderChecker` verifies it with vector clocks.
  * A parameter of at least half a bucket that would overflow the open bucket starts a new one, so
    the small decoder layers whose gradients are final first (outc, up4 .. up1.conv.3, 12.5 MB) go
    out before the 18.9 MB up1.conv.0 gradient exists.
  * Bucket size: 17.3 M params = 69 MB fp32. On xGMI each GPU has 7 links (~153 GB/s each), and a
    ring all-reduce moves 2(n-1)/n of the bucket per GPU, so ~16 MB buckets (≈4-5 per step) keep
    every bucket well above the latency-bound regime while still giving backward-overlap.
  * The 1/world averaging is folded into the fused Adam kernel (gscale), not a separate pass.
  * Native RCCL issue (``native_comm``, the default for the nccl backend on GPUs): each bucket is
    all-reduced by ``ncclAllReduce`` on a dedicated process group's communicator, enqueued by the
    native runtime straight onto the issuing HIP stream (``csrc/bindings.cpp`` comm_all_reduce) --
    stream order is the dependency, no per-bucket ProcessGroupNCCL work objects, events or waits,
    and the launch is recorded into the step's launch plan like a kernel. ``RDP_DDP_COMM=torch``
    issues through torch.distributed instead (gloo always does).
  * Issue stream at world > 1 (``RDP_DDP_STREAM``): ``side`` enqueues each collective on the wgrad side
    stream itself (every later weight gradient then waits for it), ``dedicated`` on a collective stream
    of its own that waits for the side stream (and the main stream where the bucket needs it), so the
    remaining weight gradients run beside the collective. The default per world size comes from the
    emulated A/B in ``profiles/ddp_emulated.md``: ``RDP_DDP_EMULATE=<n>:<GB/s>[:<blocks>[:<alpha_us>]]``
    replaces each native all-reduce by a resident spin of the modelled ring time
    2 (n - 1) / n x bytes / bw + alpha on ``blocks`` CUs (``csrc/comm.hip``), so a one-GPU box measures
    what an n-rank collective does to the step.
  * ``comm_dtype=torch.bfloat16`` (SURVEY.md §7.4 option): each ready bucket is cast into a bf16
    mirror of the gradient buffer on the producing stream and all-reduced there (half the xGMI bytes:
    34.5 MB instead of 69 MB per step for the bilinear U-Net); ``finish()`` widens the reduced sums
    back into the fp32 buffer, so Adam still accumulates its moments and the master in fp32.
"""
from __future__ import annotations

import contextlib
from typing import Callable, ContextManager, Dict, Iterable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def emulate_spec(spec: Optional[str] = None) -> Optional[Tuple[int, float, int, float, float]]:
    """Parse ``RDP_DDP_EMULATE`` = ``<n>:<GB/s>[:<blocks>[:<alpha_us>[:<traffic_x>]]]`` -> (n, GB/s, blocks,
    alpha_us, traffic_x), or None. ``blocks`` resident workgroups (default 16, RCCL's channel count order on
    xGMI), ``alpha_us`` the fixed latency of one ring all-reduce (default 15 us: 2 (n - 1) hops of ~1 us),
    ``traffic_x`` the HBM traffic the emulated collective streams, in multiples of the bucket read AND
    written over its duration (default 0: residency only; a ring all-reduce moves ~3x the bucket)."""
    import os
    spec = os.environ.get("RDP_DDP_EMULATE", "") if spec is None else spec
    if not spec:
        return None
    parts = spec.split(":")
    if len(parts) < 2:
        raise ValueError(f"RDP_DDP_EMULATE must be <n>:<GB/s>[:<blocks>[:<alpha_us>[:<traffic_x>]]], got {spec!r}")
    n, bw = int(parts[0]), float(parts[1])
    blocks = int(parts[2]) if len(parts) > 2 and parts[2] else 16
    alpha = float(parts[3]) if len(parts) > 3 and parts[3] else 15.0
    traffic = float(parts[4]) if len(parts) > 4 and parts[4] else 0.0
    if n < 2 or bw <= 0 or not 1 <= blocks <= 4096 or alpha < 0 or not 0 <= traffic <= 16:
        raise ValueError(f"RDP_DDP_EMULATE out of range: {spec!r}")
    return n, bw, blocks, alpha, traffic


def ring_allreduce_us(nbytes: int, n: int, gbps: float, alpha_us: float) -> float:
    """Modelled time of one ring all-reduce of ``nbytes`` over ``n`` ranks at ``gbps`` per-rank bus rate."""
    return alpha_us + 2.0 * (n - 1) / n * nbytes / (gbps * 1e3)


def dist_info() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class FlatBucketer:
    """Reverse-order contiguous gradient buckets over a flat buffer."""

    def __init__(self, grad_flat: torch.Tensor, param_ranges: Sequence[Tuple[str, int, int]],
                 bucket_mb: float = 16.0, group=None, comm_dtype: Optional[torch.dtype] = None,
                 launch_ctx: Optional[Callable[[], ContextManager]] = None, native_comm: Optional[int] = None,
                 join: Optional[Callable[[], None]] = None,
                 emulate: Optional[Tuple[int, float, int, float, float]] = None):
        self.grad = grad_flat
        # (n, GB/s, blocks, alpha_us): a modelled collective instead of ncclAllReduce (native issue only)
        self.emulate = emulate
        self._emu_scratch: Optional[torch.Tensor] = None  # the emulated collectives' HBM traffic buffer
        # RCCL communicator (ncclComm_t as int) for native issue, and the callable that orders the
        # caller's stream after the issuing stream once every bucket is out (native mode has no handles)
        self.native_comm = native_comm
        self.join = join
        # context that makes the current stream one ordered after every gradient producer (None: the
        # caller's current stream already is, e.g. single-stream autograd)
        self.launch_ctx = launch_ctx
        self.checker: Optional["StreamOrderChecker"] = None
        # host_call(fn) runs a bucket launch; a launch-plan recorder (NativeTrainer) replaces it to keep
        # the launch as a host call point of the plan (csrc/bindings.cpp plan_mark)
        self.host_call: Optional[Callable[[Callable[[], None]], None]] = None
        self.group = group
        self.comm_dtype = comm_dtype if comm_dtype not in (None, grad_flat.dtype) else None
        # bf16 mirror of the whole gradient buffer (buckets are slices of it, like of ``grad``)
        self.comm = torch.empty_like(grad_flat, dtype=self.comm_dtype) if self.comm_dtype is not None else None
        elt = (self.comm if self.comm is not None else grad_flat).element_size()
        cap = max(1, int(bucket_mb * 1024 * 1024 / elt))
        # walk parameters in reverse registration order, cutting at parameter boundaries
        self.buckets: List[Tuple[int, int]] = []
        self.bucket_params: List[List[str]] = []
        self.param_bucket: Dict[str, int] = {}
        cur_hi: Optional[int] = None
        cur_lo = None
        names: List[str] = []
        end_of = {}
        ordered = sorted(param_ranges, key=lambda r: r[1])
        for i, (n, lo, hi) in enumerate(ordered):  # extend each param to the next param's start (padding)
            end_of[n] = ordered[i + 1][1] if i + 1 < len(ordered) else grad_flat.numel()
        for name, lo, hi in reversed(ordered):
            hi = end_of[name]
            if cur_hi is not None and (cur_hi - lo) > cap and hi - lo >= cap // 2:
                # a parameter of at least half a bucket that would overflow the open bucket closes it
                # first: the gradients already final go out now instead of waiting for the big one
                self._close(cur_lo, cur_hi, names)
                cur_hi, names = None, []
            if cur_hi is None:
                cur_hi, cur_lo, names = hi, lo, [name]
            else:
                cur_lo = lo
                names.append(name)
            if cur_hi - cur_lo >= cap:
                self._close(cur_lo, cur_hi, names)
                cur_hi, names = None, []
        if cur_hi is not None and names:
            self._close(ordered[0][1] if cur_lo is None else cur_lo, cur_hi, names)
        # the first bucket must start at 0 so every element is covered
        lo0, hi0 = self.buckets[-1]
        self.buckets[-1] = (0, hi0)
        self.pending: List[int] = [len(p) for p in self.bucket_params]
        self.handles: List = []

    def _close(self, lo, hi, names):
        b = len(self.buckets)
        self.buckets.append((lo, hi))
        self.bucket_params.append(list(names))
        for n in names:
            self.param_bucket[n] = b

    def reset(self):
        self.pending = [len(p) for p in self.bucket_params]
        self.handles = []

    def _launch(self, b: int, producer=None):
        """Issue bucket ``b``; ``producer``: the stream of the gradient that completed it (launch_ctx may
        use it to skip a wait)."""
        # issued exactly once per step: a launch-plan replay re-runs this recorded call after reset()
        # without going through mark_ready, and finish() must not issue the bucket a second time
        self.pending[b] = 0
        with (self.launch_ctx(producer) if self.launch_ctx is not None else contextlib.nullcontext()):
            if self.checker is not None:
                self.checker.check_launch(self.bucket_params[b], torch.cuda.current_stream())
            lo, hi = self.buckets[b]
            buf = self.grad[lo:hi]
            if self.native_comm is not None:
                from ..ops import native
                C = native(build_if_missing=False)
                if self.comm is not None:
                    buf = self.comm[lo:hi]
                    C.cast_bf16(self.grad[lo:hi], buf)  # narrowing cast, ordered after every producer
                if self.emulate is not None:
                    n, bw, blocks, alpha, traffic = self.emulate
                    nbytes = buf.numel() * buf.element_size()
                    tb = int(traffic * nbytes) // 16 * 16
                    if tb > 0 and (self._emu_scratch is None or self._emu_scratch.numel() < 2 * tb):
                        self._emu_scratch = torch.zeros(2 * tb, dtype=torch.uint8, device=buf.device)
                    C.comm_emulate(ring_allreduce_us(nbytes, n, bw, alpha), blocks,
                                   self._emu_scratch if tb > 0 else None, tb)
                else:
                    C.comm_all_reduce(buf, self.native_comm)
                self.handles.append((b, None))
                return
            if self.comm is not None:
                buf = self.comm[lo:hi]
                buf.copy_(self.grad[lo:hi])  # narrowing cast, ordered after every producer (launch_ctx)
            self.handles.append((b, dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)))

    def mark_ready(self, names: Iterable[str], stream=None):
        """``names`` are final once the work issued so far on ``stream`` (their producer; None: the
        current stream) has run."""
        names = list(names)
        if self.checker is not None:
            self.checker.produced(names, stream)
        for n in names:
            b = self.param_bucket[n]
            self.pending[b] -= 1
            if self.pending[b] == 0:
                if self.host_call is not None:
                    self.host_call(lambda b=b, s=stream: self._launch(b, s))
                else:
                    self._launch(b, stream)

    def finish(self):
        """Every bucket issued; the caller's stream is ordered after the reductions. With native issue
        and bf16 comm the reduced sums stay in ``comm`` (bf16) for the optimizer to read directly."""
        for b, p in enumerate(self.pending):  # anything never marked (unused params) goes now
            if p > 0:
                self.pending[b] = 0
                self._launch(b)
        if self.native_comm is not None:
            if self.join is not None:
                self.join()
            self.handles = []
            return
        for b, h in self.handles:
            h.wait()  # the caller's stream now waits for the collective (RCCL: no host block)
            if self.comm is not None:
                lo, hi = self.buckets[b]
                self.grad[lo:hi].copy_(self.comm[lo:hi])  # widen the reduced sums back to fp32
        self.handles = []


class StreamOrderChecker:
    """Vector-clock model of HIP stream ordering, to prove every bucket is issued after its producers.

    Each stream keeps a clock {stream: count}. Producing gradients on stream ``p`` ticks ``p``'s own
    entry and stamps the gradients with (p, count); ``waiter`` waiting on ``waitee`` (an event recorded
    on waitee, waited on waiter: ``stream_wait``) merges waitee's clock into waiter's. A collective
    issued on stream ``s`` reads its bucket correctly iff ``clock[s][p] >= count`` for every stamped
    gradient. Install with :meth:`install` (hooks ``UNetExecutor``'s stream waits)."""

    def __init__(self):
        self.clock: Dict[int, Dict[int, int]] = {}
        self.stamp: Dict[str, Tuple[int, int]] = {}
        self.launches = 0
        self.violations: List[str] = []

    @staticmethod
    def _key(stream) -> int:
        if stream is None:
            stream = torch.cuda.current_stream()
        return int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream)

    def _vc(self, k: int) -> Dict[int, int]:
        return self.clock.setdefault(k, {k: 0})

    def produced(self, names: Iterable[str], stream=None):
        k = self._key(stream)
        vc = self._vc(k)
        vc[k] = vc.get(k, 0) + 1
        for n in names:
            self.stamp[n] = (k, vc[k])

    def wait(self, waiter, waitee):
        w, e = self._vc(self._key(waiter)), self._vc(self._key(waitee))
        for s, c in e.items():
            if w.get(s, 0) < c:
                w[s] = c

    def check_launch(self, names: Iterable[str], stream=None):
        self.launches += 1
        vc = self._vc(self._key(stream))
        for n in names:
            st = self.stamp.get(n)
            if st is not None and vc.get(st[0], 0) < st[1]:
                self.violations.append(f"{n}: produced on stream {st[0]:#x} at {st[1]}, bucket issued on a stream "
                                       f"ordered only up to {vc.get(st[0], 0)}")

    def install(self):
        """Observe every cross-stream wait the native executor issues (``models.unet._stream_wait``)."""
        from ..models import unet
        unet._STREAM_OBSERVERS.append(self)
        return self

    def uninstall(self):
        from ..models import unet
        if self in unet._STREAM_OBSERVERS:
            unet._STREAM_OBSERVERS.remove(self)


_GRAD_GROUPS: Dict[Tuple[int, str], object] = {}


def native_comm_group(device: torch.device, tag: str = "grad"):
    """(process group, ncclComm_t as int) for natively issued all-reduces on ``device``: a dedicated
    nccl group per (device, ``tag``) -- "grad" for the gradient buckets (wgrad side stream), "syncbn" for
    the SyncBatchNorm statistics (main stream: a communicator of its own, so the two streams never
    interleave operations of one communicator in a rank-dependent order). The two communicators' kernels
    run at once without a wait cycle: every rank issues both in the same host order (one executor / launch
    plan); an RCCL kernel holds only its channel blocks, so one of each fits on the GPU beside the convs;
    and the wait edges between the streams point one way per step (the side stream waits on backward
    events of the same step, the main stream on the side stream's Adam event only at the next forward, by
    when every bucket of this step is issued) -- so a SyncBN collective never waits, through its own
    stream, on a bucket collective that waits on it. The watchdog polls and aborts both
    (``native_comm_ptrs``). Created once (collective:
    every rank calls this in the same order) with BLOCKING communicators (eager-init groups default to
    non-blocking ones, whose calls may return ncclInProgress), initialised by one all-reduce before its
    communicator is taken."""
    from torch._C._distributed_c10d import ProcessGroupNCCL
    key = (device.index or 0, tag)
    if key not in _GRAD_GROUPS:
        opts = ProcessGroupNCCL.Options()
        opts.config.blocking = 1
        grp = dist.new_group(backend="nccl", pg_options=opts)
        dist.all_reduce(torch.zeros(1, device=device), group=grp)
        torch.cuda.synchronize(device)
        with torch.cuda.device(device):
            ptr = int(grp._get_backend(device)._comm_ptr())
        if ptr == 0:
            raise RuntimeError("native_comm_group: the RCCL communicator is not initialised")
        from ..ops import native
        native(build_if_missing=False).comm_bind()
        _GRAD_GROUPS[key] = (grp, ptr)
    return _GRAD_GROUPS[key]


def native_comm_ptrs() -> List[int]:
    """Every natively used RCCL communicator of this process (the comm watchdog polls and aborts all)."""
    return [ptr for _, ptr in _GRAD_GROUPS.values()]


def broadcast_module_state(tensors: Iterable[torch.Tensor], src: int = 0, group=None):
    """Broadcast parameters/buffers from ``src`` so every replica starts identical."""
    for t in tensors:
        dist.broadcast(t, src=src, group=group)


def all_reduce_mean_(t: torch.Tensor, group=None) -> torch.Tensor:
    _, world = dist_info()
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t /= world
    return t


class DistributedShardSampler(torch.utils.data.Sampler):
    """Deterministic per-epoch shuffled shard of ``range(n)`` for this rank (DistributedSampler semantics).

    Pads by wrapping so every rank gets the same number of samples (keeps collectives in lockstep).
    """

    def __init__(self, n: int, rank: int, world: int, shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        self.n, self.rank, self.world, self.shuffle, self.seed = n, rank, world, shuffle, seed
        self.drop_last = drop_last
        self.epoch = 0
        if drop_last:
            self.per_rank = n // world
        else:
            self.per_rank = (n + world - 1) // world

    def set_epoch(self, e: int):
        self.epoch = e

    def __iter__(self):
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g).tolist()
        else:
            idx = list(range(self.n))
        total = self.per_rank * self.world
        if len(idx) < total:
            idx = (idx * ((total + len(idx) - 1) // max(1, len(idx))))[:total]
        else:
            idx = idx[:total]
        return iter(idx[self.rank:total:self.world])

    def __len__(self):
        return self.per_rank
