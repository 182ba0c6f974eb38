"""Training engines: the native (HIP kernel) step and the eager (plain torch) step.

Both implement the reference step (``/root/reference/scripts/train_segmenter.py:156-165``):
zero_grad -> forward -> BCEWithLogits (optionally + Dice) -> backward -> Adam(lr 1e-4), and
optionally DDP over RCCL with flat-buffer gradient buckets (``parallel/ddp.py``).

``NativeTrainer`` runs everything on the hand-written gfx950 kernels, as eager launches of ~220
kernels per step on two streams (main: forward, dgrad, BN backward; side: weight gradients). The
whole step (forward + backward + Adam + weight re-layout) can instead be captured once into a
hipGraph (``torch.cuda.CUDAGraph`` is hipGraph on ROCm; ``graph=True``) and replayed, but measured
on MI355X the replay is slower at every batch size (img/s eager vs graph: bs4 1369 vs 1189, bs16
2308 vs 2225, bs32 2607 vs 2525, bs64 2710 vs 2664): the replayed graph spreads the wgrad side
branch over two extra hardware queues, and the extra contention slows the critical-path main
stream, while ~10 us of host time per launch stays ahead of the GPU even at bs 4. ``graph="auto"``
therefore means eager launches for training; serving (N=1, latency-bound) keeps its graphs.
With world > 1 the bucketed all-reduces overlap backward on RCCL's stream.

Plan mode (``plan=True``; "auto" = on unless a graph or SyncBN is used): the third step
is recorded by the native runtime (``csrc/bindings.cpp``: every kernel launch and cross-stream wait of
the step, with its validated raw arguments and stream) and every later step is ONE ``plan_replay``
call that re-issues the same launches on the same two streams from C++. The executor's Python
(~8 us of host time per launch) then runs once instead of every step; at small batch the host no
longer falls behind the GPU. Requirements, all true of the training step: static buffers, no
host-side decisions that change between steps, a constant learning rate and the same current stream
at every call. ``RDP_PLAN=0`` disables it. Under DDP the bucket all-reduces (and ``finish``'s waits / bf16 widening)
are torch.distributed calls the runtime cannot replay: each is recorded as a host call point of the
plan (``plan_mark``), run with recording paused, and replay calls back into Python at that point, so
every collective keeps its place between the recorded kernels. Measured (one MI355X, interleaved): host enqueue per bs-4
step 1.55 -> 1.37 ms, step time unchanged (bs 4 2.53 ms, bs 64 20.1 ms either way) -- the remaining
host cost is HIP's own ~7 us per kernel launch, which the GPU still outruns only in runs of
sub-10-us kernels. (Compiling each single-stream run of the plan into a hipGraph and a high-priority
main stream measured slower / neutral: profiles/dead_ends.md.)

``EagerTrainer`` is the reference execution model (torch autograd + MIOpen) used for the CPU path,
CPU/gloo DDP tests and as the measured comparison baseline.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.nn as nn

from ..models.unet import NativeAdam, UNetNative
from ..models.unet_ref import UNetRef
from ..parallel.ddp import FlatBucketer, broadcast_module_state, dist_info, emulate_spec, native_comm_group
from ..utils import trace


class NativeTrainer:
    # per-GPU pixels per step at or below which the step is graph-captured in "auto" mode
    # (0: never -- eager launches measured faster at every batch, see the module docstring)
    GRAPH_AUTO_MAX_PIXELS = 0

    def __init__(self, model: UNetNative, batch: int, h: int, w: int, lr: float = 1e-4, loss: str = "bce",
                 dice_weight: float = 1.0, graph="auto", bucket_mb: float = 16.0, sync_bn: bool = False,
                 grad_comm: Optional[str] = None, ddp_force: Optional[bool] = None, plan="auto"):
        self.model = model
        self.ex = model.executor(batch, h, w, training=True, loss=loss, dice_weight=dice_weight)
        self.opt = NativeAdam(model, lr=lr)
        self.rank, self.world = dist_info()
        self.bucketer = None
        self.watchdog = None
        # DDP machinery (broadcast, bucketer, side-stream hooks, gscale) also at world == 1 when forced
        # (RDP_DDP_FORCE=1): exercises the RCCL path on a single GPU (all_reduce over one rank)
        if ddp_force is None:
            ddp_force = os.environ.get("RDP_DDP_FORCE", "0") != "0"
        # gradient all-reduce dtype: "fp32" (default) or "bf16" (half the bytes; fp32 accumulate in Adam)
        grad_comm = grad_comm or os.environ.get("RDP_GRAD_COMM", "fp32")
        if grad_comm not in ("fp32", "bf16"):
            raise ValueError(f"grad_comm must be 'fp32' or 'bf16', got {grad_comm!r}")
        self.grad_comm = grad_comm
        import torch.distributed as dist
        self.ddp = self.world > 1 or (bool(ddp_force) and dist.is_available() and dist.is_initialized())
        if self.ddp:
            st = model.store
            broadcast_module_state([st.flat] + [b for _, b in model.named_buffers()])
            model.refresh_weights()
            ranges = [(n, st.offsets[n], st.offsets[n] + _numel(st.shapes[n])) for n in st.names]
            # buckets are issued from a stream ordered after both gradient streams (main: BN / head,
            # side: conv weights), never from whichever stream a hook happens to run on
            group, comm_ptr, join = None, None, None
            launch_ctx = self.ex.comm_stream
            emu = emulate_spec()
            self.ddp_stream = None
            if self._native_comm_wanted(model):
                group, comm_ptr = native_comm_group(model.store.device)
                self.ddp_stream = self.ddp_stream_mode(emu[0] if emu else self.world)
                if self.ddp_stream == "dedicated":
                    launch_ctx, join = self.ex.comm_stream_dedicated, self.ex.join_comm_dedicated
                else:
                    join = self.ex.join_comm
                if self.world > 1 or os.environ.get("RDP_COMM_WATCHDOG") == "1":
                    self.watchdog = self._make_watchdog(comm_ptr)
            elif emu is not None:
                raise ValueError("RDP_DDP_EMULATE needs native RCCL issue (nccl backend, RDP_DDP_COMM=native)")
            self.bucketer = FlatBucketer(st.grad, ranges, bucket_mb, group=group,
                                         comm_dtype=torch.bfloat16 if grad_comm == "bf16" else None,
                                         launch_ctx=launch_ctx, native_comm=comm_ptr, join=join, emulate=emu)
            self.ex.set_sync_bn(enabled=sync_bn)
        if graph == "auto":
            graph = batch * h * w <= self.GRAPH_AUTO_MAX_PIXELS
        self.use_graph = bool(graph) and not self.ddp and torch.cuda.is_available()
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        if plan == "auto":
            plan = os.environ.get("RDP_PLAN", "1") != "0"
        # SyncBN's statistics all-reduces sit inside the executor's kernel sequence: a plan holds them only
        # when they are native launches (nccl: fold kernel + ncclAllReduce, UNetExecutor._sync_rows)
        sync_py = self.ddp and sync_bn and self.ex.sync_comm is None
        self.use_plan = (bool(plan) and not sync_py and not self.use_graph
                         and torch.cuda.is_available() and model.store.device.type == "cuda")
        self.plan_id: Optional[int] = None
        self._plan_calls: list = []  # host call points of the recorded plan (DDP collectives), by tag
        if self.bucketer is not None and self.use_plan and self.bucketer.native_comm is None:
            self.bucketer.host_call = self._host_call  # torch.distributed issue: plan host call points
        self._plan_version = None
        self.steps = 0

    def __del__(self):
        if getattr(self, "watchdog", None) is not None:
            self.watchdog.close()
        if getattr(self, "plan_id", None) is not None:
            try:
                from ..ops import native
                native(build_if_missing=False).plan_free(self.plan_id)
            except Exception:  # interpreter teardown
                pass

    # Issue stream of the natively issued bucket all-reduces by (emulated) world size, from the A/B in
    # profiles/ddp_emulated.md (RDP_DDP_EMULATE on one MI355X); RDP_DDP_STREAM=side|dedicated overrides.
    # World 1 (forced DDP): RCCL launches nothing, an extra stream wait would only cost (ddp_world1.md).
    # World > 1: a dedicated collective stream on a hardware queue of its own (models.unet.concurrent_stream)
    # -- round 6, n = 8 emulated: bs 64 19.16-19.22 vs 19.94-19.98 ms on the side stream, bs 4 2.68 vs 3.19-3.20
    # (150 GB/s, 16 CUs); 19.39-19.59 vs 19.56-19.62 and 2.45 vs 2.80 at 300 GB/s, 32 CUs. Round 5 measured the
    # opposite (22.3 vs 20.3 ms) with a dedicated stream that shared a queue with the main or side stream:
    # the same stream placed by creation order alone gave 21.8-22.2 ms this round.
    DDP_STREAM_BY_WORLD = {1: "side"}
    DDP_STREAM_DEFAULT = "dedicated"

    @classmethod
    def ddp_stream_mode(cls, world: int) -> str:
        mode = os.environ.get("RDP_DDP_STREAM", "auto")
        if mode not in ("auto", "side", "dedicated"):
            raise ValueError(f"RDP_DDP_STREAM must be auto, side or dedicated, got {mode!r}")
        if mode != "auto":
            return mode
        return cls.DDP_STREAM_BY_WORLD.get(int(world), cls.DDP_STREAM_DEFAULT)

    def _make_watchdog(self, comm_ptr: int):
        """Host watchdog over the natively issued collectives (parallel/watchdog.py): they bypass
        ProcessGroupNCCL's work objects, so its timeout would not see a dead peer. It polls EVERY native
        communicator of the process (the gradient buckets' and, with SyncBN, the statistics'), read at
        each poll so a communicator created later is covered, and aborts all of them on a failure."""
        from ..ops import native
        from ..parallel.ddp import native_comm_ptrs
        from ..parallel.watchdog import CommWatchdog
        C = native(build_if_missing=False)

        def comms():
            return native_comm_ptrs() or [comm_ptr]

        def poll():
            for p in comms():
                code, text = C.comm_async_error(p)
                if code:
                    return code, text
            return 0, ""

        def abort():
            for p in comms():
                C.comm_abort(p)

        return CommWatchdog(poll=poll, abort=abort, rank=self.rank)

    def _arm_watchdog(self):
        if self.watchdog is not None:
            ev = torch.cuda.Event()
            ev.record()
            self.watchdog.arm(ev)

    @staticmethod
    def native_comm_wanted_env() -> bool:
        """RCCL issued natively (parallel.ddp native_comm_group) unless RDP_DDP_COMM=torch: nccl backend
        and the executor's wgrad side stream to issue from (the device is checked by the caller)."""
        import torch.distributed as dist
        mode = os.environ.get("RDP_DDP_COMM", "native")
        if mode not in ("native", "torch"):
            raise ValueError(f"RDP_DDP_COMM must be 'native' or 'torch', got {mode!r}")
        return (mode == "native" and dist.is_initialized() and dist.get_backend() == "nccl"
                and os.environ.get("RDP_WGRAD_OVERLAP", "1") != "0")

    @classmethod
    def _native_comm_wanted(cls, model) -> bool:
        return model.store.device.type == "cuda" and cls.native_comm_wanted_env()

    def _host_call(self, fn):
        """Run ``fn`` (torch.distributed work); while a plan is being recorded, also make it a host call
        point of the plan, run with recording paused."""
        from ..ops import native
        C = native(build_if_missing=False)
        if not C.plan_recording():
            fn()
            return
        C.plan_mark(len(self._plan_calls))
        self._plan_calls.append(fn)
        C.plan_pause()
        try:
            fn()
        finally:
            C.plan_resume()

    def _plan_host(self, tag: int):
        self._plan_calls[tag]()

    def _hook(self, spec, stream=None):
        """Gradient hook of one layer (head, BN, conv or ConvTranspose2d: ``spec.param_names()``), final
        once the work issued so far on ``stream`` has run."""
        self.bucketer.mark_ready(spec.param_names(), stream)

    def _step_body(self):
        ex = self.ex
        with trace.range("train.forward"):
            ex.forward()
        if self.bucketer is not None:
            self.bucketer.reset()
            with trace.range("train.backward+allreduce"):
                ex.backward(grad_hook=self._hook)  # every layer's hook fires inside, the head's first
                if self.use_plan and self.bucketer.native_comm is None:
                    self._host_call(self.bucketer.finish)
                else:  # native issue: finish is only the stream join (recorded in the plan)
                    self.bucketer.finish()
            with trace.range("train.adam"):
                # native bf16 comm: Adam reads the reduced bf16 sums straight from the comm buffer
                g = self.bucketer.comm if self.bucketer.native_comm is not None else None
                self.opt.step(gscale=1.0 / self.world, side=self._wprep_side(), grad=g)
        else:
            with trace.range("train.backward"):
                ex.backward()
            with trace.range("train.adam"):
                self.opt.step(side=self._wprep_side())

    def _wprep_side(self):
        """The stream for the dgrad weight re-layout after Adam (NativeAdam.step): the executor's wgrad
        stream, idle during the next forward; inline under graph capture (no work left unjoined)."""
        # (measured: bs 64 3,198 / 3,195 vs 3,187 / 3,188 img/s inline, bs 4 within noise; interleaved)
        return None if self.use_graph else getattr(self.ex, "side", None)

    def set_batch(self, x: torch.Tensor, target: torch.Tensor):
        self.ex.set_input(x, target)

    def step(self) -> torch.Tensor:
        """One training step on the current input buffers; returns the (device) loss tensor."""
        if self.use_plan:
            from ..ops import native
            C = native(build_if_missing=False)
            version = (self.model.__dict__.get("_layout_version"), self.opt.hyper_key())
            if self.plan_id is not None and self._plan_version != version:
                # buffers re-laid out or optimizer hyper-parameters changed (lr schedule, Adam
                # load_state_dict): the recorded launches bake those in, so record again
                C.plan_free(self.plan_id)
                self.plan_id = None
            if self.plan_id is not None:
                if self._plan_calls:
                    self.bucketer.reset()
                    C.plan_replay(self.plan_id, self._plan_host)
                else:
                    C.plan_replay(self.plan_id)
            elif self.steps < 2:  # first steps eagerly (first-launch costs, flags that settle)
                self._step_body()
            else:
                self._plan_calls = []
                C.plan_begin()
                try:
                    self._step_body()
                except BaseException:
                    C.plan_abort()
                    raise
                self.plan_id = C.plan_end()
                self._plan_version = version
            self.steps += 1
            self._arm_watchdog()
            return self.ex.loss
        if self.use_graph:
            if self.graph is None:
                if self.steps < 2:  # warm up eagerly (allocator, first-launch costs) before capture
                    self._step_body()
                    self.steps += 1
                    return self.ex.loss
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s):
                        self._step_body()
                torch.cuda.current_stream().wait_stream(s)
                self.graph = g
            self.graph.replay()
        else:
            self._step_body()
        self.steps += 1
        self._arm_watchdog()
        return self.ex.loss

    def eval_loss(self) -> torch.Tensor:
        """Validation forward (batch statistics are NOT updated: eval-mode BN)."""
        ev = self.model.executor(self.ex.N, self.ex.H, self.ex.W, training=False)
        ev.target.copy_(self.ex.target)
        ev.x_in.copy_(self.ex.x_in)
        ev.dice_w = self.ex.dice_w
        ev.forward()
        return ev.loss


def _numel(shape):
    n = 1
    for s in shape:
        n *= s
    return n


class EagerTrainer:
    """Plain-torch trainer (reference execution model) with the same flat-bucket DDP."""

    def __init__(self, model: nn.Module, lr: float = 1e-4, loss: str = "bce", dice_weight: float = 1.0,
                 bucket_mb: float = 16.0, amp: Optional[torch.dtype] = None):
        self.model = model
        self.opt = torch.optim.Adam(model.parameters(), lr=lr)
        self.loss_kind, self.dice_w = loss, dice_weight
        self.amp = amp
        self.rank, self.world = dist_info()
        self.bucketer = None
        if self.world > 1:
            params = list(model.named_parameters())
            broadcast_module_state([p.data for _, p in params] + [b for _, b in model.named_buffers()])
            # flat grad buffer; each param.grad is a view into it (autograd accumulates in place)
            total = sum(p.numel() for _, p in params)
            dev = params[0][1].device
            self.flat_grad = torch.zeros(total, dtype=params[0][1].dtype, device=dev)
            ranges, off = [], 0
            for n, p in params:
                p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
                ranges.append((n, off, off + p.numel()))
                off += p.numel()
            self.bucketer = FlatBucketer(self.flat_grad, ranges, bucket_mb)
            for n, p in params:
                p.register_post_accumulate_grad_hook(lambda _p, n=n: self.bucketer.mark_ready([n]))

    def compute_loss(self, logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        logits = logits.float()
        loss = nn.functional.binary_cross_entropy_with_logits(logits, target)
        if self.loss_kind == "bce_dice":
            p = torch.sigmoid(logits)
            dice = 1 - (2 * (p * target).sum() + 1.0) / (p.sum() + target.sum() + 1.0)
            loss = loss + self.dice_w * dice
        return loss

    def step(self, x: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        if self.bucketer is not None:
            self.flat_grad.zero_()
            self.bucketer.reset()
        else:
            self.opt.zero_grad(set_to_none=True)
        ctx = torch.autocast(device_type=x.device.type, dtype=self.amp) if self.amp else contextlib.nullcontext()
        with ctx:
            out = self.model(x)
        loss = self.compute_loss(out, target)
        loss.backward()
        if self.bucketer is not None:
            self.bucketer.finish()
            self.flat_grad /= self.world
        self.opt.step()
        return loss.detach()


def build_bench_step(batch: int, size: int, decoder: str, device: torch.device, world: int, graph: bool,
                     bucket_mb: float, loss: str = "bce", sync_bn: bool = False, grad_comm: str = "fp32",
                     ddp_force: bool = False):
    """bench.py hook: returns a zero-arg callable running one full native training step."""
    bilinear = decoder == "bilinear"
    torch.manual_seed(0)
    ref = UNetRef(3, 1, bilinear=bilinear)
    model = UNetNative(3, 1, bilinear=bilinear, device=device, init_from=ref)
    tr = NativeTrainer(model, batch, size, size, loss=loss, graph=graph, bucket_mb=bucket_mb, sync_bn=sync_bn,
                       grad_comm=grad_comm, ddp_force=ddp_force)
    g = torch.Generator(device="cpu").manual_seed(1234 + tr.rank)
    x = torch.rand(batch, 3, size, size, generator=g).to(device)
    y = (torch.rand(batch, 1, size, size, generator=g) > 0.5).float().to(device)
    tr.set_batch(x, y)

    def step():
        return tr.step()

    step.trainer = tr
    return step
