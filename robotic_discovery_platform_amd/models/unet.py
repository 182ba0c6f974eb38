"""MI355X-native U-Net: flat parameter store + static-shape executor over the HIP kernels.

Architecture and state_dict are those of the reference ``UNet(3, 1)``
(``/root/reference/pkg/segmentation_model.py:86-120``, mirrored by :class:`UNetRef`), but the
execution model is MI355X-first:

* **Parameters** live in ONE flat fp32 master buffer (grads, Adam moments and a bf16 shadow share
  its layout). Each reference-named parameter is a view into it; conv weights are stored
  channels_last (physical OHWI = the [Cout][tap][Cin] K-contiguous layout the implicit-GEMM kernels
  read), so ``state_dict()`` has the reference's 110 keys / shapes while the kernels read weights
  with zero re-layout. Derived bf16 layouts (dgrad's flipped/transposed weights, the packed first
  layer) are rebuilt by one ``wprep`` launch after each optimizer step.
* **Activations** are NHWC bf16, preallocated once per (batch, H, W): every launch is static, so
  the whole train step (forward, backward, Adam) is capturable in one hipGraph.
* **Kernels**: implicit-GEMM MFMA convs with BN statistics fused in the epilogue; the Up block's
  concat is never materialised (dual-source conv operand; dual-destination dgrad);
  maxpool backward fuses the skip-gradient add; head + BCE(+Dice) are fused.
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from .unet_ref import UNetRef, unet_widths

ALIGN = 64  # elements; keeps every parameter 256-B aligned in fp32, 128-B in bf16


@dataclass
class UpTSpec:
    """ConvTranspose2d(cin, cout, 2, stride=2) of a transposed-decoder Up block, run as a 1x1 GEMM
    [pixels, cin] x [cin, 4*cout] (conv kernel, taps=1) + sub-pixel shuffle with bias."""
    name: str  # reference module path, e.g. "up1.up"
    cin: int
    cout: int

    def param_names(self) -> List[str]:
        return [self.name + ".weight", self.name + ".bias"]


@dataclass
class HeadSpec:
    """The 1x1 head ``outc`` (conv + bias): its gradients are final as soon as backward starts, so its
    DDP hook fires first (before any conv layer's)."""
    name: str = "outc"

    def param_names(self) -> List[str]:
        return [self.name + ".conv.weight", self.name + ".conv.bias"]


HEAD_SPEC = HeadSpec()


@dataclass
class ConvSpec:
    name: str  # reference module path of the conv, e.g. "down1.maxpool_conv.1.double_conv.0"
    bn: str  # reference module path of its BatchNorm
    cin: int
    cout: int
    taps: int = 9
    packed: bool = False  # first layer: Cin padded to 8, 8 taps per K step
    cin_real: int = 0

    def param_names(self) -> List[str]:
        """The conv weight (its BN's gamma / beta are final earlier: :class:`BNHook`)."""
        return [self.name + ".weight"]


@dataclass
class BNHook:
    """Gradient hook of a conv layer's BatchNorm: gamma / beta gradients are final right after the BN
    backward (main stream), before that layer's weight gradient (side stream) is."""
    conv: ConvSpec

    @property
    def name(self) -> str:
        return self.conv.bn

    def param_names(self) -> List[str]:
        return [self.conv.bn + ".weight", self.conv.bn + ".bias"]


class ParamStore:
    """Flat fp32 master/grad/Adam buffers + bf16 shadow, with reference-named parameter views."""

    def __init__(self, ref: nn.Module, device: torch.device):
        self.device = device
        self.names: List[str] = []
        self.offsets: Dict[str, int] = {}
        self.shapes: Dict[str, torch.Size] = {}
        off = 0
        for name, p in ref.named_parameters():
            self.names.append(name)
            self.offsets[name] = off
            self.shapes[name] = p.shape
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.grad = torch.zeros(off, dtype=torch.float32, device=device)
        self.exp_avg = torch.zeros(off, dtype=torch.float32, device=device)
        self.exp_avg_sq = torch.zeros(off, dtype=torch.float32, device=device)
        self.shadow = torch.zeros(off, dtype=torch.bfloat16, device=device)
        self.step = torch.zeros(1, dtype=torch.int32, device=device)
        with torch.no_grad():
            for name, p in ref.named_parameters():
                self.view(name).copy_(p.detach().to(device))

    def _phys(self, buf: torch.Tensor, name: str) -> torch.Tensor:
        o, shp = self.offsets[name], self.shapes[name]
        n = 1
        for s in shp:
            n *= s
        return buf[o:o + n]

    def view(self, name: str, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Logical (reference-shaped) view; 4-D conv weights are channels_last (physical OHWI)."""
        buf = self.flat if buf is None else buf
        t = self._phys(buf, name)
        shp = self.shapes[name]
        if len(shp) == 4:
            co, ci, kh, kw = shp
            return t.view(co, kh, kw, ci).permute(0, 3, 1, 2)
        return t.view(shp)

    def flat_slice(self, name: str, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        return self._phys(self.flat if buf is None else buf, name)


def unet_conv_specs(depth: int, base: int, in_ch: int, bilinear: bool) -> List[ConvSpec]:
    """Conv layers in forward order with reference module paths."""
    f = 2 if bilinear else 1
    enc = unet_widths(base, depth, bilinear)
    specs: List[ConvSpec] = []

    def dc(prefix: str, cin: int, cout: int, cmid: Optional[int] = None, first: bool = False):
        cmid = cmid or cout
        specs.append(ConvSpec(f"{prefix}.double_conv.0", f"{prefix}.double_conv.1", cin, cmid,
                              packed=first, cin_real=cin if first else 0))
        specs.append(ConvSpec(f"{prefix}.double_conv.3", f"{prefix}.double_conv.4", cmid, cout))

    dc("inc", in_ch, enc[0], first=True)
    for i in range(1, depth + 1):
        dc(f"down{i}.maxpool_conv.1", enc[i - 1], enc[i])
    for i in range(1, depth + 1):
        lvl = depth - i
        cin = base * (2 ** (lvl + 1))
        cout = base * (2 ** lvl) // (f if i < depth else 1)
        dc(f"up{i}.conv", cin, cout, cin // 2 if bilinear else None)
    return specs


class UNetNative(nn.Module):
    """Reference-keyed U-Net whose compute runs on the native HIP kernels (training + inference)."""

    def __init__(self, n_channels: int = 3, n_classes: int = 1, bilinear: bool = True, base_width: int = 64,
                 depth: int = 4, device: Optional[torch.device] = None, init_from: Optional[nn.Module] = None):
        super().__init__()
        if n_classes != 1:
            raise NotImplementedError("native head supports n_classes == 1 (reference: UNet(3, 1))")
        if n_channels > 8:
            raise NotImplementedError("native first layer packs <= 8 input channels")
        if base_width != 64:
            raise NotImplementedError("native head assumes 64 channels")
        self.n_channels, self.n_classes, self.bilinear = n_channels, n_classes, bilinear
        self.depth, self.base_width = depth, base_width
        device = device or torch.device("cuda")
        ref = init_from if init_from is not None else UNetRef(n_channels, n_classes, bilinear, base_width, depth)
        self.store = ParamStore(ref, device)
        # reference-named parameters (views into the flat master) and BN buffers
        self._pnames = list(self.store.names)
        self._bn_names: List[str] = []
        for name in self.store.names:
            self._register_view(name, nn.Parameter(self.store.view(name), requires_grad=False))
        for name, buf in ref.named_buffers():
            self._register_buffer_path(name, buf.detach().clone().to(device))
        self.specs = unet_conv_specs(depth, base_width, n_channels, bilinear)
        # transposed decoder: the Up blocks' ConvTranspose2d(cin, cin // 2, 2, 2), up1 .. up_depth
        self.up_specs: List[UpTSpec] = []
        if not bilinear:
            for i in range(1, depth + 1):
                cin = base_width * (2 ** (depth - i + 1))
                self.up_specs.append(UpTSpec(f"up{i}.up", cin, cin // 2))
        self._derived_built = False
        self._build_derived()

    # ---- module plumbing: keep reference key names ("inc.double_conv.0.weight", ...) ----
    def _holder(self, path: str) -> Tuple[nn.Module, str]:
        parts = path.split(".")
        mod: nn.Module = self
        for p in parts[:-1]:
            if p not in mod._modules:
                mod._modules[p] = nn.Module()
            mod = mod._modules[p]
        return mod, parts[-1]

    def _register_view(self, path: str, param: nn.Parameter):
        mod, leaf = self._holder(path)
        mod._parameters[leaf] = param

    def _register_buffer_path(self, path: str, t: torch.Tensor):
        mod, leaf = self._holder(path)
        mod._buffers[leaf] = t

    def buf(self, path: str) -> torch.Tensor:
        mod, leaf = self._holder(path)
        return mod._buffers[leaf]

    def _join_wprep(self):
        """Order the current stream after the work NativeAdam.step left on a training executor's side
        stream (the dgrad re-layout; with the overlapped update also Adam's group B, i.e. most masters,
        the bf16 shadow and the step counter) before the masters / derived buffers are touched here."""
        pend = self.__dict__.pop("_wprep_pending", None)
        self.__dict__.pop("_adam_ev_pending", None)
        if pend is not None:
            _stream_wait(torch.cuda.current_stream(), pend)

    def _join_adam(self):
        """Order the current stream after the side stream's Adam group B only (not the re-layouts queued
        behind it): the next forward's join before its first group-B layer. While a launch plan is
        recorded the wait is unconditional once the overlap has ever run: an eval or state_dict between
        steps clears the pending flag, but every replay of the plan follows a replayed overlapped Adam
        (a wait on a completed event costs almost nothing)."""
        C = _native()
        pending = self.__dict__.pop("_adam_ev_pending", False)
        ev = self.__dict__.get("_adam_ev")
        if ev is not None and (pending or C.plan_recording()):
            C.stream_wait_event(torch.cuda.current_stream().cuda_stream, ev)

    def state_dict(self, *args, **kwargs):
        # the masters of the Adam update's group B may still be written on the side stream
        self._join_wprep()
        return super().state_dict(*args, **kwargs)

    def load_state_dict(self, sd, strict: bool = True):  # keep flat-buffer views intact
        self._join_wprep()
        own = dict(self.named_parameters())
        ownb = dict(self.named_buffers())
        missing = [k for k in list(own) + list(ownb) if k not in sd]
        unexpected = [k for k in sd if k not in own and k not in ownb]
        if strict and (missing or unexpected):
            raise RuntimeError(f"state_dict mismatch: missing={missing} unexpected={unexpected}")
        with torch.no_grad():
            for k, v in sd.items():
                if k in own:
                    own[k].copy_(v.to(own[k].device))
                elif k in ownb:
                    ownb[k].copy_(v.to(ownb[k].device))
        # the derived layouts are rebuilt IN PLACE: launch plans and serving graphs captured against
        # these buffers stay valid and see the new weights
        self.refresh_weights()
        return missing, unexpected

    # ---- derived bf16 weight layouts ----
    def _build_derived(self):
        C = _native()
        st = self.store
        segs = []
        off = 0
        self._dw: Dict[str, Tuple[int, int]] = {}  # name -> (offset, numel) in derived
        for sp in self.specs:
            wname = sp.name + ".weight"
            if sp.packed:
                n = sp.cout * 128
                segs.append((st.offsets[wname], off, 1, sp.cout, sp.cin_real, sp.taps))
            else:
                n = sp.cout * sp.taps * sp.cin
                segs.append((st.offsets[wname], off, 0, sp.cout, sp.cin, sp.taps))
            self._dw[sp.name] = (off, n)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        for us in self.up_specs:
            # master (channels_last view of [cin, cout, 2, 2]) is physically [cin][(dh, dw, cout)];
            # the forward GEMM needs its transpose [(dh, dw, cout)][cin] (a taps=1 "dgrad" re-layout)
            n = us.cin * 4 * us.cout
            segs.append((st.offsets[us.name + ".weight"], off, 0, us.cin, 4 * us.cout, 1))
            self._dw[us.name] = (off, n)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.derived = torch.zeros(max(off, 1), dtype=torch.bfloat16, device=st.device)
        # launch plans recorded against the previous derived buffers are stale from here (NativeTrainer
        # re-records when this changes)
        self.__dict__["_layout_version"] = self.__dict__.get("_layout_version", 0) + 1
        seg_size = C.wseg_size()
        import struct

        def tiles(s):  # wprep work tiles of a segment (csrc/optim.hip wseg_tiles)
            _, _, kind, co, ci, taps = s
            return (co * 128 + 2047) // 2048 if kind == 1 else taps * ((co + 63) // 64) * ((ci + 63) // 64)

        def table(ss):  # records carry their first tile: the launch walks one flat range of real tiles
            raw = bytearray()
            t0 = 0
            for s in ss:
                rec = struct.pack("<qqiiiiii", *s, t0, 0)
                raw += rec + b"\0" * (seg_size - len(rec))
                t0 += tiles(s)
            return torch.tensor(list(raw) or [0], dtype=torch.uint8).to(st.device), len(ss)

        def blocks(ss):  # the table's total tile count (wprep's `blocks` argument)
            return sum(tiles(s) for s in ss)

        self._segs, self._nseg = table(segs)
        self._wblk = blocks(segs)
        # the conv dgrad layouts (kind 0 with 9 or 1 taps of a ConvSpec) are read only by backward; the
        # packed first layer and the transposed decoder's forward weights by the next forward
        n_conv = len(self.specs)
        bwd = [s for i, s in enumerate(segs) if i < n_conv and not self.specs[i].packed]
        fwd = [s for i, s in enumerate(segs) if not (i < n_conv and not self.specs[i].packed)]
        self._segs_fwd, self._nseg_fwd = table(fwd)
        self._segs_bwd, self._nseg_bwd = table(bwd)
        self._wblk_fwd, self._wblk_bwd = blocks(fwd), blocks(bwd)
        # Adam split for the overlap with the next forward (NativeAdam.step with a side stream): group A =
        # the parameters of the first two DoubleConvs (inc, down1; ~1.5 % of the U-Net), updated on the
        # main stream; group B = the rest, on the side stream, which the next forward joins just before the
        # first layer that reads them (UNetExecutor._wait_layer). The derived forward layouts split the
        # same way: the packed first layer (A) and the transposed decoder's ConvTranspose2d weights (B).
        self._adam_split = 0
        if len(self.specs) > 4:
            split = st.offsets[self.specs[4].name + ".weight"]
            names_a = [n for n in st.names if st.offsets[n] < split]
            own_a = {sp.name for sp in self.specs[:4]}
            def in_a(n):
                return n.rsplit(".", 1)[0] in own_a or any(n.startswith(sp.bn + ".") for sp in self.specs[:4])

            def end(n):
                return st.offsets[n] + math.prod(st.shapes[n])

            # both directions: group A holds only specs[:4]'s parameters, and ALL of them (else the side
            # stream's group B would update one the next forward's first layers read before the join)
            if all(in_a(n) for n in names_a) and all(end(n) <= split for n in st.names if in_a(n)):
                self._adam_split = split
        fwd_a = [s for i, s in enumerate(segs) if i < n_conv and self.specs[i].packed and i < 4]
        fwd_b = [s for s in fwd if s not in fwd_a]
        self._segs_fwd_a, self._nseg_fwd_a = table(fwd_a)
        self._segs_fwd_b, self._nseg_fwd_b = table(fwd_b)
        self._wblk_fwd_a, self._wblk_fwd_b = blocks(fwd_a), blocks(fwd_b)
        self.refresh_weights()

    def refresh_weights(self):
        """Rebuild the bf16 shadow + derived layouts from the fp32 master (after load / manual edits)."""
        self._join_wprep()
        C = _native()
        C.cast_bf16(self.store.flat, self.store.shadow)
        C.wprep(self.store.flat, self.derived, self._segs, self._nseg, None, self._wblk)

    def fwd_weight(self, sp: ConvSpec) -> torch.Tensor:
        if sp.packed:
            o, n = self._dw[sp.name]
            return self.derived[o:o + n].view(sp.cout, 128)
        return self.store.flat_slice(sp.name + ".weight", self.store.shadow).view(sp.cout, sp.taps * sp.cin)

    def eval_frag_weight(self, sp: ConvSpec) -> Optional[torch.Tensor]:
        """The fragment-major copy of ``sp``'s forward weights for the row-band eval conv, or None
        (built by the eval executor's prepare_eval for its small-map layers)."""
        return self.__dict__.get("_wfrag", {}).get(sp.name)

    def refresh_eval_frag(self, specs) -> None:
        """(Re)build the fragment-major eval weights of ``specs`` in place (stable pointers for captured
        graphs): after a weight change, like the BN eval coefficients."""
        d = self.__dict__.setdefault("_wfrag", {})
        for sp in specs:
            src = rowband_frag_weights(self.fwd_weight(sp))
            buf = d.get(sp.name)
            if buf is None or buf.shape != src.shape:
                d[sp.name] = src
            else:
                buf.copy_(src)

    def dgrad_weight(self, sp: ConvSpec) -> torch.Tensor:
        o, n = self._dw[sp.name]
        return self.derived[o:o + n].view(sp.cin, sp.taps * sp.cout)

    def upT_fwd_weight(self, us: UpTSpec) -> torch.Tensor:
        o, n = self._dw[us.name]
        return self.derived[o:o + n].view(4 * us.cout, us.cin)

    def upT_dgrad_weight(self, us: UpTSpec) -> torch.Tensor:
        return self.store.flat_slice(us.name + ".weight", self.store.shadow).view(us.cin, 4 * us.cout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """NCHW float input -> NCHW fp32 logits (inference helper; training uses UNetExecutor)."""
        ex = self.executor(x.shape[0], x.shape[2], x.shape[3], training=False)
        ex.set_input(x)
        ex.forward()
        return ex.logits_nchw()

    def executor(self, batch: int, h: int, w: int, training: bool = True, loss: str = "bce",
                 dice_weight: float = 1.0) -> "UNetExecutor":
        key = (batch, h, w, training, loss, dice_weight)
        cache = self.__dict__.setdefault("_executors", {})
        if key not in cache:
            cache[key] = UNetExecutor(self, batch, h, w, training, loss, dice_weight)
        return cache[key]


class _Ablated:
    """``RDP_ABLATE=<binding>[,<binding>...]`` -- PROFILING ONLY, results are wrong: the listed kernel
    bindings become no-ops in the executor (e.g. ``bn_relu_bwd_reduce``, ``bn_relu_bwd_apply``,
    ``bn_relu_apply``, ``conv_wgrad``), and ``wgsum`` / ``wgred`` drop the weight-gradient slab
    reductions inside ``conv_wgrad`` (csrc/conv_wgrad.hip). The step time without a kernel class bounds
    what fusing or speeding it up can gain (profiles/step_ablation.md)."""
    RET = {"bn_relu_bwd_reduce": 1, "conv_wgrad": 1, "wgrad_first_bn": 0, "conv_dgrad_bnred": 0}

    def __init__(self, C, names):
        self._C, self._names = C, frozenset(names)

    def __getattr__(self, n):
        # only inside a launch plan being recorded (NativeTrainer: step 3 on, replayed after): the eager
        # steps before it fill every skipped output with real values, so the knocked-out step still runs
        # on realistic data (zero-filled operands let the chip hold a ~19 % higher clock:
        # MI355X_MICROARCH.md 'DVFS give-back')
        if n in self._names and self._C.plan_recording():
            return lambda *a, **k: self.RET.get(n)
        return getattr(self._C, n)


_ABLATED = None



def rowband_frag_weights(w: torch.Tensor) -> torch.Tensor:
    """OHWI [Cout][9 Cin] bf16 -> the row-band eval conv's fragment-major layout
    [Cout/16][9 Cin/32][64 lanes][8] (lane = 16 * 8-channel group + output row): every MFMA A fragment
    is one contiguous KiB, 8 full cache lines per load instead of 16 half lines (csrc/conv_rowband.hip)."""
    co, k = w.shape
    return w.view(co // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().view(co, k)

def _native():
    from ..ops import native
    global _ABLATED
    spec = os.environ.get("RDP_ABLATE", "")
    if not spec:
        return native()
    if _ABLATED is None:
        _ABLATED = _Ablated(native(), [n for n in spec.split(",") if n and n not in ("wgsum", "wgred")])
    return _ABLATED


@dataclass
class _Layer:
    spec: ConvSpec
    x1: torch.Tensor
    x2: Optional[torch.Tensor]
    y: torch.Tensor
    a: torch.Tensor
    coef: torch.Tensor
    coef2: torch.Tensor
    da: Optional[torch.Tensor] = None  # gradient w.r.t. a (filled by the consumer)
    dy: Optional[torch.Tensor] = None
    dx1: Optional[torch.Tensor] = None  # dgrad destinations (None => no dgrad)
    dx1_owner: Optional["_Layer"] = None  # layer whose BN input gradient dx1 is (None: a pool / concat grad)
    dx2: Optional[torch.Tensor] = None
    splits: int = 1
    bwd_rows: int = 0  # BN-backward partial rows already produced by a fused producer of da
    # training: this conv reads its producer's PRE-BN output and applies that BN + ReLU itself (the
    # row-ring kernels, 64 -> 64 channels at W % 64 == 0): bnin = the producer layer, whose `a` that
    # kernel also writes; consumer_bnin marks the producer (no bn_relu_apply pass)
    bnin: Optional["_Layer"] = None
    consumer_bnin: bool = False


# observers of every cross-stream wait (parallel.ddp.StreamOrderChecker, tests)
_STREAM_OBSERVERS: List = []


_CONCURRENT_CACHE: Dict[tuple, bool] = {}


def _runs_concurrently(a: "torch.cuda.Stream", b: "torch.cuda.Stream") -> bool:
    """Whether kernels of streams ``a`` and ``b`` overlap on the GPU: a 300 us single-block resident kernel
    (csrc/comm.hip, the collective emulator's spin) on each; on one hardware queue they serialize (~600 us).
    The GPU must be idle (called while an executor is set up, never inside a step or a plan)."""
    key = (a.cuda_stream, b.cuda_stream)
    if key in _CONCURRENT_CACHE:
        return _CONCURRENT_CACHE[key]
    import time
    C = _native()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(2):
        t0 = time.perf_counter()
        with torch.cuda.stream(a):
            C.comm_emulate(300.0, 1)
        with torch.cuda.stream(b):
            C.comm_emulate(300.0, 1)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    ok = best < 450e-6
    _CONCURRENT_CACHE[key] = _CONCURRENT_CACHE[(key[1], key[0])] = ok
    return ok


def concurrent_stream(dev, others, tries: int = 8) -> "torch.cuda.Stream":
    """A new stream whose kernels run concurrently with every stream of ``others``. HIP gives streams hardware
    queues round-robin in creation order (GPU_MAX_HW_QUEUES, 4 by default; torch.cuda.Stream draws from a
    pre-created pool), so a plain new stream may share a queue with the main or the weight-gradient stream --
    and then everything issued on it waits behind their work. Measured under emulated n = 8 collectives
    (profiles/ddp_emulated.md, round 6): the same dedicated collective stream gave 19.2 or 21.9 ms per bs-64
    step depending only on how many streams the process had drawn before it (a high-priority stream did not
    help: 22.1 ms). Draws up to ``tries`` streams and returns the first that overlaps every stream of
    ``others`` in a timed probe (``RDP_STREAM_PROBE=0``: no probe, the next pool stream)."""
    others = [o for o in others if o is not None]
    if os.environ.get("RDP_STREAM_PROBE", "1") == "0" or torch.device(dev).type != "cuda":
        return torch.cuda.Stream(dev)
    s = None
    with torch.cuda.device(dev):
        for _ in range(tries):
            s = torch.cuda.Stream(dev)
            if all(_runs_concurrently(s, o) for o in others):
                return s
    return s


def _stream_wait(waiter: "torch.cuda.Stream", waitee: "torch.cuda.Stream"):
    """``waiter.wait_stream(waitee)`` through the native runtime, so that a launch plan being recorded
    (NativeTrainer plan mode, csrc/bindings.cpp) also holds the cross-stream dependency."""
    _native().stream_wait(waiter.cuda_stream, waitee.cuda_stream)
    for o in _STREAM_OBSERVERS:
        o.wait(waiter, waitee)


class UNetExecutor:
    """Static-shape forward/backward/step program for one (batch, H, W)."""

    def __init__(self, model: UNetNative, N: int, H: int, W: int, training: bool, loss: str, dice_weight: float):
        self.m, self.N, self.H, self.W = model, N, H, W
        self.training = training
        self.dice_w = float(dice_weight) if loss == "bce_dice" else 0.0
        self.dice_eps = 1.0
        dev = model.store.device
        self.dev = dev
        # Fusions (each measured against its separate-kernel form, profiles/dead_ends.md): BN apply +
        # maxpool (forward) and maxpool backward + BN reduce (backward) in one pass each at the Down
        # boundaries, upsample backward + BN reduce at the Up boundaries; in training the 1x1 head
        # applies the last conv's BN+ReLU itself (forward) and produces that BN's backward partials and
        # dy from the logits (backward), so the 64-ch activation and its gradient are never stored.
        self.fuse_head = training
        C = _native()
        D = model.depth
        bf = torch.bfloat16
        specs = model.specs
        enc = unet_widths(model.base_width, D, model.bilinear)
        sizes = [(H, W)]
        for _ in range(D):
            h, w = sizes[-1]
            sizes.append((h // 2, w // 2))
        self.sizes = sizes

        def t(h, w, c):
            return torch.zeros(N, h, w, c, dtype=bf, device=dev)

        self.x_in = t(H, W, 8)
        self.target = torch.zeros(N * H * W, dtype=torch.float32, device=dev)
        self.layers: List[_Layer] = []
        it = iter(specs)

        def mk(spec, x1, x2, h, w):
            a = t(h, w, spec.cout)
            y = t(h, w, spec.cout) if training else a  # eval writes BN+ReLU output directly
            L = _Layer(spec, x1, x2, y, a,
                       torch.zeros(4 * spec.cout, device=dev), torch.zeros(3 * spec.cout, device=dev))
            self.layers.append(L)
            return L

        # encoder
        h, w = sizes[0]
        l0 = mk(next(it), self.x_in, None, h, w)
        l1 = mk(next(it), l0.a, None, h, w)
        self.skips = [l1.a]
        self.pools: List[torch.Tensor] = []
        self.down_layers: List[Tuple[_Layer, _Layer]] = [(l0, l1)]
        for i in range(1, D + 1):
            h, w = sizes[i]
            p = t(h, w, enc[i - 1])
            self.pools.append(p)
            la = mk(next(it), p, None, h, w)
            lb = mk(next(it), la.a, None, h, w)
            self.down_layers.append((la, lb))
            self.skips.append(lb.a)
        # decoder
        self.ups: List[torch.Tensor] = []
        self.up_layers: List[Tuple[_Layer, _Layer]] = []
        low = self.skips[D]
        self.yTs: List[torch.Tensor] = []  # transposed decoder: [N, h_low, w_low, 4 * cout] GEMM outputs
        for i in range(1, D + 1):
            lv = D - i
            h, w = sizes[lv]
            uc = low.shape[3] if model.bilinear else model.up_specs[i - 1].cout
            u = t(h, w, uc)
            self.ups.append(u)
            if not model.bilinear:
                self.yTs.append(t(low.shape[1], low.shape[2], 4 * uc))
            la = mk(next(it), self.skips[lv], u, h, w)
            lb = mk(next(it), la.a, None, h, w)
            self.up_layers.append((la, lb))
            low = lb.a
        self.final = low
        # overlapped Adam (NativeAdam.step): join the side stream before the first layer of group B
        self._wait_layer = self.layers[4] if model._adam_split and len(self.layers) > 4 else None
        # BN + ReLU of the first layer of the full-resolution DoubleConvs (inc, up4) applied by the
        # consumer conv instead of a separate pass (training; the forward and the weight-gradient
        # row-ring kernels stage the pre-BN rows and form the activation in LDS)
        # (measured: bs 64 3,178 / 3,195 vs 3,169 / 3,179 img/s without, bs 4 neutral; same box, 2 rounds)
        if training and dev.type == "cuda":
            pairs = [self.down_layers[0]] + ([self.up_layers[-1]] if self.up_layers else [])
            for la, lb in pairs:
                n, h, w, c = la.y.shape
                if (lb.x1 is la.a and lb.x2 is None and c == 64 and lb.spec.cout == 64 and lb.spec.taps == 9
                        and not lb.spec.packed and w % 64 == 0 and h % 2 == 0 and n * h * w * c * 2 < (1 << 31)):
                    lb.bnin = la
                    la.consumer_bnin = True
        # ... and the forward also stores that activation (one extra write) so the weight gradient runs the
        # plain row-ring kernel on it (re-forming it in the wgrad measured 1 % slower: dead_ends.md)
        # training, bilinear decoder: the BN + ReLU of the layer under each Up block is applied by the
        # upsample itself on its 4 source taps (that layer's activation is never written; its backward
        # reads only y). Pays at small batch, where each of the 4 apply launches is mostly launch /
        # dependent-load latency; at bs 64 the 4x re-application cost 0.3-0.5 % (profiles/dead_ends.md).
        fu = os.environ.get("RDP_FUSE_UP_BN")
        self.fuse_up_bn = (training and model.bilinear and dev.type == "cuda" and
                           (fu == "1" if fu is not None else N * H * W <= (1 << 20)))
        M = N * H * W
        self.M = M
        self.logits = torch.zeros(M, dtype=torch.float32, device=dev)
        self.head_partial = torch.zeros(C.head_partial_blocks(M) * 65, dtype=torch.float32, device=dev)
        # BCE-only training with the BN-fused head: the forward pass also emits the head's backward
        # partials (d loss / d logit is local), so backward only finalizes them (no second read of y)
        self.head_grads_in_fwd = self.fuse_head and self.dice_w == 0.0
        self.head_gscale = 1.0  # loss scale assumed by those partials (backward falls back if it differs)
        self._head_fwd_grads = False
        self.head_gpart = (torch.zeros(C.head_partial_blocks(M) * 65, dtype=torch.float32, device=dev)
                           if self.head_grads_in_fwd else None)
        self.loss_sums = torch.zeros(4, dtype=torch.float32, device=dev)
        self.loss = torch.zeros(2, dtype=torch.float32, device=dev)
        # stats slab (reused by every conv; finalize runs right after each conv)
        max_rows = max(C.conv_stats_rows(L.x1.shape[0] * L.x1.shape[1] * L.x1.shape[2], L.spec.cout, 0) * 2 * L.spec.cout
                       for L in self.layers)
        self.stats = torch.zeros(max_rows, dtype=torch.float32, device=dev)
        # SyncBatchNorm (optional): process group whose ranks share batch statistics.
        # The per-block partial rows are folded to one [2][C] row, all-reduced (one 2C-float call per
        # layer, forward and backward) and finalized with the global pixel count.
        self.sync_group = None
        self.sync_world = 1
        self.sync_comm = None  # native RCCL communicator of the statistics all-reduces (set_sync_bn)
        self.sync_emulate = None
        self._sync_on = False
        self.red_ws = torch.zeros(64 * 2 * max(L.spec.cout for L in self.layers), dtype=torch.float32, device=dev)
        # split-K workspace (fp32 partial tiles) for the convs whose tile grid alone underfills the
        # chip (deep layers at small batch, e.g. serving at N=1); shared: convs run in sequence
        ws = 0
        for L in self.layers:
            n, h, w, c1 = L.x1.shape
            c2 = L.x2.shape[3] if L.x2 is not None else 0
            ws = max(ws, C.conv_ws_elems(n, h, w, c1, c2, L.spec.cout, L.spec.taps, int(L.spec.packed), 0))
            if training and not L.spec.packed:  # dgrad: dy (cout ch) -> d(input) (c1 + c2 ch)
                ws = max(ws, C.conv_ws_elems(n, h, w, L.spec.cout, 0, c1 + c2, L.spec.taps, 0, 0))
        for i, us in enumerate(model.up_specs):
            n, h, w, _ = self.yTs[i].shape
            ws = max(ws, C.conv_ws_elems(n, h, w, us.cin, 0, 4 * us.cout, 1, 0, 0))
            if training:
                ws = max(ws, C.conv_ws_elems(n, h, w, 4 * us.cout, 0, us.cin, 1, 0, 0))
        self.kws = torch.zeros(ws, dtype=torch.float32, device=dev) if ws else None
        self._frag_names = frozenset()  # layers whose fragment-major eval weights prepare_eval refreshed
        if training:
            self._alloc_backward(C)
        else:
            self._eval_coef_ready = False

    # ------------------------------------------------------------------ backward buffers
    def _alloc_backward(self, C):
        dev, bf = self.dev, torch.bfloat16
        # RDP_WGRAD_OVERLAP=0 serialises the wgrads on the main stream (clean per-kernel profiles)
        self.overlap_wgrad = dev.type == "cuda" and os.environ.get("RDP_WGRAD_OVERLAP", "1") != "0"
        # BN-backward partial rows from the split-K dgrad reduce (RDP_SPLITK_BNRED=0: the separate pass, A/B)
        self.splitk_bnred = os.environ.get("RDP_SPLITK_BNRED", "1") != "0"
        # a stream whose kernels overlap the main stream's (concurrent_stream: not on its hardware queue)
        self.side = concurrent_stream(dev, [torch.cuda.current_stream(dev)]) if self.overlap_wgrad else None
        # split-K grid target of the generic / packed weight-gradient kernels. Fewer splits = less fp32
        # slab traffic, more = more parallelism; 512 measured best at bs 4 .. 64 (the side stream's wgrads
        # overlap the main stream, so a lighter slab wins over the serialised optimum).
        self.wgrad_blocks = 512
        N = self.N
        D = self.m.depth

        def like(x):
            return torch.zeros_like(x)

        for L in self.layers:
            L.da = like(L.a)
            L.dy = like(L.y)
        # dgrad destinations
        enc_layers = self.down_layers
        # inc: conv1 has no dgrad; conv2 -> inc conv1 da
        (l0, l1) = enc_layers[0]
        l1.dx1 = l0.da
        l1.dx1_owner = l0
        self.dpools: List[torch.Tensor] = []
        self.dskips: List[torch.Tensor] = [like(s) for s in self.skips[:D]]  # grads from the decoder concat
        for i in range(1, D + 1):
            la, lb = enc_layers[i]
            lb.dx1 = la.da
            lb.dx1_owner = la
            dp = like(self.pools[i - 1])
            self.dpools.append(dp)
            la.dx1 = dp
        self.dups: List[torch.Tensor] = []
        for i in range(1, D + 1):
            lv = D - i
            la, lb = self.up_layers[i - 1]
            lb.dx1 = la.da
            lb.dx1_owner = la
            du = like(self.ups[i - 1])
            self.dups.append(du)
            la.dx1 = self.dskips[lv]
            la.dx2 = du
        # wgrad split-K choice + shared slab (one grid target for every layer: giving the first encoder
        # level -- the last side-stream work of the step -- the wide 2048-block grid to shorten the
        # tail measured 1.3% slower, 2900 / 2909 vs 2938 / 2950 img/s at bs64)
        slab = 0
        for L in self.layers:
            n, h, w, _ = L.x1.shape
            M = n * h * w
            cin = L.spec.cin if not L.spec.packed else 8
            ncols = 72 if L.spec.packed else L.spec.taps * cin
            tiles = ((ncols + 255) // 256) * (L.spec.cout // 64)
            L.splits = int(max(1, min((self.wgrad_blocks + tiles - 1) // tiles, M // 2048)))
            slab = max(slab, C.wgrad_slab_elems(n, h, w, cin, L.spec.cout, L.spec.taps, int(L.spec.packed), L.splits))
        self.dyTs: List[torch.Tensor] = [like(y) for y in self.yTs]
        self.upT_splits: List[int] = []
        for i, us in enumerate(self.m.up_specs):
            n, h, w, _ = self.yTs[i].shape
            M = n * h * w
            tiles = ((4 * us.cout + 255) // 256) * (us.cin // 64)
            sp_ = int(max(1, min((self.wgrad_blocks + tiles - 1) // tiles, max(1, M // 2048))))
            self.upT_splits.append(sp_)
            # roles swapped in conv_wgrad: "x" = dyT (4*cout ch), "dy" = the ConvT input (cin ch)
            slab = max(slab, C.wgrad_slab_elems(n, h, w, 4 * us.cout, us.cin, 1, 0, sp_))
        self.slab = torch.zeros(slab, dtype=torch.float32, device=dev)
        # The first layer's wgrad is the step's last gradient; the side stream is still working off
        # its backlog then while the main stream idles, so it runs on the main stream with its own slab
        # (moving the second-to-last layer's wgrad there too measured 1.3 % slower)
        self.slab_main = None
        if self.side is not None:
            L0 = self.down_layers[0][0]
            n, h, w, _ = L0.x1.shape
            cin = L0.spec.cin if not L0.spec.packed else 8
            self.slab_main = torch.zeros(C.wgrad_slab_elems(n, h, w, cin, L0.spec.cout, L0.spec.taps,
                                                            int(L0.spec.packed), L0.splits),
                                         dtype=torch.float32, device=dev)
        if self.m.up_specs:
            self.colsum_ws = torch.zeros((1024 * 4 + 64) * max(us.cout for us in self.m.up_specs), dtype=torch.float32,
                                         device=dev)
        maxc = max(L.spec.cout for L in self.layers)
        # (also the fused head's BN-backward partials: 128 floats per head block -- the larger need for
        # shallow / narrow models at large batch)
        self.bn_partial = torch.zeros(max(1024 * 2 * maxc, C.head_partial_blocks(self.M) * 128), dtype=torch.float32,
                                      device=dev)

    # ------------------------------------------------------------------ data
    def set_input(self, x: torch.Tensor, target: Optional[torch.Tensor] = None):
        """x: [N,C,H,W] (float, values in [0,1]) or NHWC8 bf16; target: [N,1,H,W] float masks."""
        with torch.no_grad():
            if x.dim() == 4 and x.shape[-1] == 8 and x.dtype == torch.bfloat16:
                self.x_in.copy_(x)
            else:
                self.x_in.zero_()
                self.x_in[..., : x.shape[1]].copy_(x.permute(0, 2, 3, 1))
            if target is not None:
                self.target.copy_(target.reshape(-1))

    # ------------------------------------------------------------------ forward
    def _conv_bn_relu(self, C, L: _Layer, pool: Optional[torch.Tensor] = None, apply: bool = True,
                      up: Optional[torch.Tensor] = None):
        """conv -> BN(train: batch stats) -> ReLU into ``L.a``; with ``pool`` also MaxPool2d(2) of
        ``L.a`` into ``pool`` (fused with the BN apply in training). Returns True if it pooled.
        ``apply=False`` (training) stops after the BN statistics: the consumer applies BN+ReLU.
        ``up`` (eval): also the decoder's bilinear x2 upsample of ``L.a`` into ``up`` (centred, as the
        F.pad of Up.forward); returns True when it was produced."""
        sp = L.spec
        m = self.m
        if L is self._wait_layer:  # the first layer whose parameters the side stream's Adam group B updates
            m._join_adam()
        w = m.fwd_weight(sp)
        if not self.training:  # eval: BN folded into the conv epilogue, ReLU fused, writes a directly
            # with ``pool`` / ``up``: MaxPool2d(2) / the upsample too (fused into the split-K reduce or
            # the row-ring epilogue where those run, else separate launches)
            # only a copy this executor's own prepare_eval refreshed (another executor's may be stale)
            wf = m.eval_frag_weight(sp) if sp.name in self._frag_names else None
            if up is not None:
                oy = (up.shape[1] - 2 * L.a.shape[1]) // 2
                ox = (up.shape[2] - 2 * L.a.shape[2]) // 2
                C.conv_fwd(L.x1, L.x2, w, sp.taps, int(sp.packed), L.a, None, None, 0, L.coef, 1, self.kws, None, up,
                           oy, ox, wf)
                return True
            C.conv_fwd(L.x1, L.x2, w, sp.taps, int(sp.packed), L.a, None, None, 0, L.coef, 1, self.kws, pool, None, 0, 0,
                       wf)
            return pool is not None
        if L.bnin is not None:  # the producer's BN + ReLU applied by this conv (row-ring BNIN)
            rows = C.conv_fwd_bnin(L.bnin.y, w, L.y, self.stats, L.bnin.coef, L.bnin.a)
            assert rows > 0, "conv_fwd_bnin: ring kernel not applicable"
        else:
            rows = C.conv_fwd(L.x1, L.x2, w, sp.taps, int(sp.packed), L.y, None, self.stats, 0, None, 0, self.kws)
        g = m.store.view(sp.bn + ".weight")
        b = m.store.view(sp.bn + ".bias")
        if self.training:
            M = L.y.shape[0] * L.y.shape[1] * L.y.shape[2]
            if self._sync_on:
                rows, M = self._sync_rows(self.stats, rows, sp.cout, (L.y.shape[1], L.y.shape[2]))
            C.bn_finalize(self.stats, rows, M, g, b, m.buf(sp.bn + ".running_mean"), m.buf(sp.bn + ".running_var"),
                          m.buf(sp.bn + ".num_batches_tracked"), 0.1, 1e-5, L.coef, self.red_ws)
        if pool is not None:
            C.bn_relu_apply_pool(L.y, L.a, pool, L.coef)
            return True
        if apply and not L.consumer_bnin:
            C.bn_relu_apply(L.y, L.a, L.coef, 1)
        return False

    def prepare_eval(self):
        C = _native()
        m = self.m
        m._join_wprep()  # reads every layer's BN parameters and running statistics
        for L in self.layers:
            sp = L.spec
            C.bn_eval_coef(m.store.view(sp.bn + ".weight"), m.store.view(sp.bn + ".bias"),
                           m.buf(sp.bn + ".running_mean"), m.buf(sp.bn + ".running_var"), 1e-5, L.coef)
        # the row-band eval conv's fragment-major weights for the small-map 3x3 layers (csrc/conv_rowband.hip;
        # conv_fwd picks the kernel per layer from its traffic model)
        if self.dev.type == "cuda":
            specs = [L.spec for L in self.layers if self._rowband_candidate(C, L)]
            m.refresh_eval_frag(specs)
            self._frag_names = frozenset(sp.name for sp in specs)

    def _rowband_candidate(self, C, L: "_Layer") -> bool:
        """Whether conv_fwd will run ``L`` on the row-band kernel: asked of the native selector itself
        (rdp_conv_rowband_frag_auto, csrc/conv_rowband.hip), so the two can never disagree."""
        sp = L.spec
        if sp.packed or sp.taps != 9:
            return False
        n, h, w, c1 = L.x1.shape
        c2 = L.x2.shape[3] if L.x2 is not None else 0
        return C.rowband_frag_mode(n, h, w, c1, c2, sp.cout) > 0

    def forward(self, head: bool = True, refresh_eval: bool = True, mask_head: Optional[tuple] = None):
        """Run the network; ``head=False`` stops after up4 (serving applies ``head_mask`` instead).

        Eval mode folds BN into the conv epilogues with coefficients from the running statistics;
        ``refresh_eval=False`` reuses the coefficients from the last ``prepare_eval()`` (the serving
        pipeline recomputes them only when the weights change, not per frame).
        ``mask_head=(head_w, head_b, logit_thr, mask_u8)`` (eval, with ``head=False``): the serving mask
        ``head(a_final) > logit_thr``; where the row-ring kernel runs the last conv, the head is fused
        into its epilogue and ``final`` is not materialised (elsewhere the separate ``head_mask`` launch)."""
        C = _native()
        D = self.m.depth
        if not self.training and refresh_eval:
            self.prepare_eval()
        l0, l1 = self.down_layers[0]
        self._conv_bn_relu(C, l0)
        pooled = self._conv_bn_relu(C, l1, self.pools[0] if D > 0 else None)
        # eval, bilinear decoder: each decoder input upsample is produced by the conv that makes `low`
        eval_up = not self.training and self.m.bilinear
        upsampled = False
        fuse_up = self.fuse_up_bn and head
        for i in range(1, D + 1):
            if not pooled:
                C.maxpool2_fwd(self.skips[i - 1], self.pools[i - 1])
            la, lb = self.down_layers[i]
            self._conv_bn_relu(C, la)
            if i == D and eval_up:
                upsampled = self._conv_bn_relu(C, lb, up=self.ups[0])
                continue
            pooled = self._conv_bn_relu(C, lb, self.pools[i] if i < D else None, apply=not (i == D and fuse_up))
        low = self.skips[D]
        low_layer = self.down_layers[D][1] if D else None
        for i in range(1, D + 1):
            lv = D - i
            u = self.ups[i - 1]
            oy = (u.shape[1] - 2 * low.shape[1]) // 2
            ox = (u.shape[2] - 2 * low.shape[2]) // 2
            if upsampled:
                upsampled = False
            elif fuse_up:  # relu(bn(y)) of the layer below formed on the upsample's source taps
                C.upsample2_fwd(low_layer.y, u, oy, ox, low_layer.coef)
            elif self.m.bilinear:
                C.upsample2_fwd(low, u, oy, ox)
            else:
                us = self.m.up_specs[i - 1]
                bias = self.m.store.view(us.name + ".bias")
                # the sub-pixel scatter + bias in the ping-pong GEMM's epilogue where that kernel takes the
                # shape (u's zero border is never written); else the GEMM into yT + the shuffle pass
                if C.conv_upT_fwd(low, self.m.upT_fwd_weight(us), bias, u, oy, ox) != 0:
                    C.conv_fwd(low, None, self.m.upT_fwd_weight(us), 1, 0, self.yTs[i - 1], None, None, 0, None, 0,
                               self.kws)
                    C.upT_shuffle(self.yTs[i - 1], bias, u, oy, ox)
            la, lb = self.up_layers[i - 1]
            self._conv_bn_relu(C, la)
            last = i == D
            if last and mask_head is not None and not head and self._conv_head_mask(C, lb, mask_head):
                return
            if not last and eval_up:
                upsampled = self._conv_bn_relu(C, lb, up=self.ups[i])
            else:
                self._conv_bn_relu(C, lb, apply=not ((last and self.fuse_head and head) or (not last and fuse_up)))
            low = lb.a
            low_layer = lb
        if not head:
            if mask_head is not None:
                C.head_mask(self.final, *mask_head)
            return
        head_w = self.m.store.view("outc.conv.weight").reshape(-1)
        head_b = self.m.store.view("outc.conv.bias")
        if self.fuse_head:
            lb = self.up_layers[-1][1] if D else self.down_layers[0][1]
            if self.head_grads_in_fwd:
                C.head_fwd(lb.y, head_w, head_b, self.target, self.logits, self.head_partial, self.loss_sums,
                           self.loss, self.dice_w, self.dice_eps, lb.coef, self.head_gpart, self.bn_partial,
                           self.head_gscale)
                self._head_fwd_grads = True
            else:
                C.head_fwd(lb.y, head_w, head_b, self.target, self.logits, self.head_partial, self.loss_sums,
                           self.loss, self.dice_w, self.dice_eps, lb.coef)
        else:
            C.head_fwd(self.final, head_w, head_b, self.target, self.logits, self.head_partial, self.loss_sums,
                       self.loss, self.dice_w, self.dice_eps)

    def _conv_head_mask(self, C, L: _Layer, mask_head: tuple) -> bool:
        """Eval: the last conv + BN fold + ReLU + 1x1 head + threshold in one row-ring launch."""
        sp = L.spec
        if self.training or L.x2 is not None or sp.taps != 9 or sp.packed:
            return False
        hw, hb, thr, mask = mask_head
        return bool(C.conv_head_mask(L.x1, self.m.fwd_weight(sp), L.coef, hw, hb, float(thr), mask))

    def logits_nchw(self) -> torch.Tensor:
        return self.logits.view(self.N, 1, self.H, self.W)

    # ------------------------------------------------------------------ backward
    def _bn_bwd(self, C, L: _Layer, head_gscale: Optional[float] = None, apply: bool = True):
        sp = L.spec
        st = self.m.store
        M = L.y.shape[0] * L.y.shape[1] * L.y.shape[2]
        # the reduction already ran inside the pool/head backward that produced L.da (fused), or runs now
        T = L.bwd_rows if L.bwd_rows else C.bn_relu_bwd_reduce(L.da, L.y, L.coef, 1, self.bn_partial)
        L.bwd_rows = 0
        if self._sync_on:
            # gamma/beta gradients stay local (DDP averages them like any weight); the input-gradient
            # coefficients use the globally reduced sums, as torch.nn.SyncBatchNorm does
            C.bn_bwd_finalize(self.bn_partial, T, M, st.view(sp.bn + ".weight"), L.coef,
                              st.view(sp.bn + ".weight", st.grad), st.view(sp.bn + ".bias", st.grad), L.coef2,
                              self.red_ws)
            T, M = self._sync_rows(self.bn_partial, T, sp.cout, (L.y.shape[1], L.y.shape[2]))
            C.bn_bwd_finalize(self.bn_partial, T, M, st.view(sp.bn + ".weight"), L.coef, None, None, L.coef2,
                              self.red_ws)
        else:
            C.bn_bwd_finalize(self.bn_partial, T, M, st.view(sp.bn + ".weight"), L.coef,
                              st.view(sp.bn + ".weight", st.grad), st.view(sp.bn + ".bias", st.grad), L.coef2,
                              self.red_ws)
        if not apply:  # the consumer (the first layer's fused wgrad) applies it on the fly
            return
        if head_gscale is not None:  # fused head: g recomputed from the logits, no da
            C.head_bn_bwd_apply(L.y, st.view("outc.conv.weight").reshape(-1), self.logits, self.target,
                                self.loss_sums, L.coef, L.coef2, L.dy, self.dice_w, self.dice_eps, head_gscale)
        else:
            C.bn_relu_bwd_apply(L.da, L.y, L.coef, L.coef2, L.dy, 1)

    def set_sync_bn(self, group=None, enabled: bool = True):
        """Share BN batch statistics across the ranks of ``group`` in training.

        Default group: a dedicated copy of WORLD created once per model (collective: every rank calls
        this in the same order), so the small per-layer statistics all-reduces get their own RCCL
        communicator and never queue behind the gradient buckets issued from the wgrad side stream.
        The ranks' (N, H, W) are all-gathered once here: the global pixel count of every BN layer is
        static, so ranks with different batch shapes get exact global moments (as torch's
        SyncBatchNorm, which gathers per-rank counts) without a per-layer host round trip."""
        import torch.distributed as dist
        if enabled and dist.is_available() and dist.is_initialized():
            if group is None:
                group = self.m.__dict__.get("_sync_bn_group")
                if group is None:
                    group = dist.new_group()
                    self.m.__dict__["_sync_bn_group"] = group
            self.sync_group, self.sync_world = group, dist.get_world_size(group)
            # nccl on GPUs: the per-layer statistics all-reduces issued natively on the main stream over a
            # communicator of their own (parallel.ddp.native_comm_group "syncbn"), folded by a kernel --
            # every step of it a recorded launch, so SyncBN keeps the launch plan
            self.sync_comm = None
            if (group is self.m.__dict__.get("_sync_bn_group") and dist.get_backend(group) == "nccl"
                    and self.dev.type == "cuda" and os.environ.get("RDP_DDP_COMM", "native") == "native"):
                from ..parallel.ddp import emulate_spec, native_comm_group
                self.sync_comm = native_comm_group(self.dev, "syncbn")[1]
                self.sync_emulate = emulate_spec()
            self.sync_ws64 = torch.zeros(2 * max(L.spec.cout for L in self.layers), dtype=torch.float64,
                                         device=self.dev)
            shp = torch.tensor([self.N, self.H, self.W], dtype=torch.int64)
            if dist.get_backend(group) != "gloo":
                shp = shp.to(self.dev)
            shapes = [torch.zeros_like(shp) for _ in range(self.sync_world)]
            dist.all_gather(shapes, shp, group=group)
            self._sync_m = {}
            for lvl, (h, w) in enumerate(self.sizes):
                tot = 0
                for t in shapes:
                    n, hh, ww = (int(v) for v in t.tolist())
                    for _ in range(lvl):
                        hh, ww = hh // 2, ww // 2
                    tot += n * hh * ww
                self._sync_m[(h, w)] = tot
        else:
            self.sync_group, self.sync_world = None, 1
            self.sync_comm = None
        # statistics shared across ranks (also at world 1 under RDP_DDP_EMULATE: the modelled collectives)
        self._sync_on = self.sync_world > 1 or (self.sync_comm is not None and self.sync_emulate is not None)

    def _sync_rows(self, buf: torch.Tensor, rows: int, c: int, hw: Tuple[int, int]) -> Tuple[int, int]:
        """Fold ``rows`` partial [2][C] rows of ``buf`` into row 0 (fp64 sum), all-reduce it over the
        sync group and return (1, global pixel count at spatial size ``hw``): the row count the
        finalize kernels then read and the pixels the reduced sums cover."""
        import torch.distributed as dist
        # the global sums travel in fp64 and come back as two fp32 rows (hi, lo) that the finalize kernels
        # add in fp64 (one fp32 rounding of the sums is enough to move small layers' bf16 gradients by tens
        # of percent through E[x^2] - mean^2)
        ws = self.sync_ws64
        if getattr(self, "sync_comm", None) is not None:  # native: fold kernel + ncclAllReduce on this stream
            C = _native()
            C.rows_fold(buf, rows, 2 * c, ws)
            emu = getattr(self, "sync_emulate", None)
            if emu is not None:  # RDP_DDP_EMULATE: the modelled collective instead (one-GPU A/B)
                from ..parallel.ddp import ring_allreduce_us
                n, bw, blocks, alpha, _traffic = emu  # (16 c bytes: traffic is negligible)
                C.comm_emulate(ring_allreduce_us(16 * c, n, bw, alpha), 1)
            else:
                C.comm_all_reduce(ws[: 2 * c], self.sync_comm)
            C.rows_hilo(ws, buf, 2 * c)
            return 2, self._sync_m[hw]
        tot = buf[: rows * 2 * c].view(rows, 2 * c).sum(0, dtype=torch.float64)
        if dist.get_backend(self.sync_group) == "gloo":  # host round trip (gloo tests: ranks share a GPU)
            tot = tot.cpu()
        dist.all_reduce(tot, group=self.sync_group)
        tot = tot.to(buf.device)
        hi = tot.float()
        buf[: 2 * c].copy_(hi)
        buf[2 * c: 4 * c].copy_((tot - hi.double()).float())
        return 2, self._sync_m[hw]

    def _on_wgrad_stream(self, fn):
        """Run ``fn(slab)`` (a weight gradient) on the side stream with its slab. (Several side streams,
        one per consecutive wgrad, measured slower: every extra stream lands on another hardware queue.)"""
        return self._on_side(lambda: fn(self.slab))

    @contextlib.contextmanager
    def comm_stream(self, producer=None):
        """Make the current stream one ordered after EVERY gradient issued so far, for the DDP bucket
        all-reduces (parallel.ddp.FlatBucketer ``launch_ctx``): the wgrad side stream (conv weight
        gradients), after a fork from the main stream (BN, head, bias gradients) -- skipped when the
        bucket was completed on the side stream (``producer``): every main-stream gradient of it was
        issued before the completing weight gradient's own fork. Without a side stream the current
        stream already is ordered.
        (Measured, forced DDP at world 1: a dedicated collective stream waiting on side + main instead
        cost 6.5 % at bs 64 and 7 % at bs 4 -- 20.96 vs 19.69 ms, 2.66 vs 2.49 ms -- and more with 8
        hardware queues, 23.3 / 5.5 ms; profiles/ddp_world1.md.)"""
        if self.side is None:
            yield
            return
        cur = torch.cuda.current_stream()
        if cur != self.side and (producer is None or producer != self.side):
            _stream_wait(self.side, cur)
        with torch.cuda.stream(self.side):
            yield

    def join_comm(self):
        """Order the current stream after the collectives issued on :meth:`comm_stream` (native RCCL issue
        has no work handles to wait on: stream order is the dependency)."""
        if self.side is not None:
            _stream_wait(torch.cuda.current_stream(), self.side)

    @contextlib.contextmanager
    def comm_stream_dedicated(self, producer=None):
        """A collective stream of its own (``RDP_DDP_STREAM=dedicated``): it waits for the wgrad side
        stream (every conv weight gradient issued so far) and, unless the bucket was completed there, for
        the current stream too (BN / head / bias gradients); the weight gradients issued after it keep
        running beside the collective instead of queueing behind it on the side stream."""
        if self.side is None:
            yield
            return
        if getattr(self, "comm_side", None) is None:
            # the main stream here is the caller's current one; the collective stream must not share a
            # hardware queue with it or with the weight-gradient stream
            self.comm_side = concurrent_stream(self.dev, [torch.cuda.current_stream(self.dev), self.side])
        cur = torch.cuda.current_stream()
        _stream_wait(self.comm_side, self.side)
        if cur != self.side and (producer is None or producer != self.side):
            _stream_wait(self.comm_side, cur)
        with torch.cuda.stream(self.comm_side):
            yield

    def join_comm_dedicated(self):
        """Order the current stream after the collectives of :meth:`comm_stream_dedicated`."""
        if getattr(self, "comm_side", None) is not None:
            _stream_wait(torch.cuda.current_stream(), self.comm_side)

    def _on_side(self, fn):
        """Run ``fn`` on the wgrad side stream after everything issued so far on the main stream
        (fork); without a side stream it runs inline. (One fork per two weight gradients, which saves
        the fork's event record in the main queue, measured 2 % slower at bs 4: profiles/dead_ends.md.)"""
        if self.side is None:
            return fn()
        _stream_wait(self.side, torch.cuda.current_stream())
        with torch.cuda.stream(self.side):
            return fn()

    def _conv_bwd(self, C, L: _Layer, hooks=None, head_gscale: Optional[float] = None):
        sp = L.spec
        st = self.m.store
        gw = st.flat_slice(sp.name + ".weight", st.grad)
        main = torch.cuda.current_stream() if self.dev.type == "cuda" else None
        if (self.dev.type == "cuda" and L is self.down_layers[0][0] and sp.packed and L.dx1 is None
                and head_gscale is None and sp.cout == 64):
            # first layer: its pre-BN gradient feeds only the weight gradient, so the BN-backward apply
            # runs inside that wgrad (wgrad_first_bn) and dz is never stored
            self._bn_bwd(C, L, None, apply=False)
            if hooks is not None:
                hooks(BNHook(sp), main)

            def fused(slab):
                r = C.wgrad_first_bn(L.x1, L.da, L.y, L.coef, L.coef2, slab, gw, sp.cin_real, 0, L.splits)
                if r < 0:  # shape outside the kernel (e.g. tensors past 2 GiB): separate passes
                    C.bn_relu_bwd_apply(L.da, L.y, L.coef, L.coef2, L.dy, 1)
                    C.conv_wgrad(L.x1, L.x2, L.dy, sp.taps, int(sp.packed), sp.cin_real, slab, gw, 0, L.splits, 0)

            if self.slab_main is not None:
                fused(self.slab_main)
            else:
                self._on_wgrad_stream(fused)
            if hooks is not None:  # the weight gradient is final once its stream's work so far has run
                hooks(sp, main if self.slab_main is not None or self.side is None else self.side)
            return
        self._bn_bwd(C, L, head_gscale)
        if hooks is not None:  # gamma / beta gradients are final (main stream)
            hooks(BNHook(sp), main)
        # wgrad (latency-bound on x / dY streams) overlaps the main stream's dgrad + next BN backward;
        # all wgrads share the slab, so they stay serialized on the one side stream
        wstream = self.side if self.side is not None else main
        if self.slab_main is not None and L is self.down_layers[0][0]:
            C.conv_wgrad(L.x1, L.x2, L.dy, sp.taps, int(sp.packed), sp.cin_real, self.slab_main, gw, 0, L.splits, 0)
            wstream = main
        else:
            self._on_wgrad_stream(lambda slab: C.conv_wgrad(L.x1, L.x2, L.dy, sp.taps, int(sp.packed), sp.cin_real,
                                                            slab, gw, 0, L.splits, 0))
        # dgrad into the da of a BN layer: where the row-ring kernel runs it (64 -> 64 channels), its
        # epilogue also produces that layer's BN-backward partial sums (no bn_relu_bwd_reduce pass)
        owner = L.dx1_owner
        fusable = owner is not None and L.dx2 is None and sp.taps == 9 and not owner.bwd_rows
        done = False
        if fusable:
            rows = C.conv_dgrad_bnred(L.dy, self.m.dgrad_weight(sp), L.dx1, owner.y, owner.coef, self.bn_partial)
            if rows > 0:
                owner.bwd_rows = rows
                done = True
        if fusable and not done and self.splitk_bnred:
            # where the dgrad runs split-K (the reference batch's deep layers), the split-K reduce writes the
            # owner's BN-backward partial rows too: no bn_relu_bwd_reduce pass (0 rows: another path ran)
            rows = C.conv_dgrad_splitk_bnred(L.dy, self.m.dgrad_weight(sp), L.dx1, owner.y, owner.coef,
                                             self.bn_partial, self.kws)
            if rows >= 0:
                owner.bwd_rows = rows
                done = True
        if L.dx1 is not None and not done:
            C.conv_fwd(L.dy, None, self.m.dgrad_weight(sp), sp.taps, 0, L.dx1, L.dx2, None, 0, None, 0, self.kws)
        if hooks is not None:  # the weight gradient is final once its stream's work so far has run
            hooks(sp, wstream)

    def backward(self, grad_hook=None, gscale: float = 1.0):
        """Full backward; ``grad_hook(spec, stream)`` fires as each layer's gradients are issued: they
        are final once the work issued so far on ``stream`` has run (a collective reading them must be
        issued from a stream ordered after it: :meth:`comm_stream`).

        Weight gradients run on a side stream (``overlap_wgrad``) and join the caller's stream at
        the end, so the optimizer (or a graph capture) sees every gradient complete."""
        C = _native()
        D = self.m.depth
        st = self.m.store
        main = torch.cuda.current_stream() if self.overlap_wgrad else None
        pend = self.m.__dict__.pop("_wprep_pending", None)
        if pend is None and self.overlap_wgrad and C.plan_recording():
            # recorded plans always join the side stream here: a replay follows a replayed Adam whose
            # dgrad re-layout runs there, even if an eval / checkpoint cleared the flag before recording
            pend = self.side
        if pend is not None:  # the dgrad weights rebuilt on a side stream after the last Adam step
            _stream_wait(torch.cuda.current_stream(), pend)
        try:
            self._backward(C, D, st, grad_hook, gscale)
        finally:
            if main is not None:
                _stream_wait(main, self.side)  # join

    def _backward(self, C, D, st, grad_hook, gscale):
        head_w = st.view("outc.conv.weight").reshape(-1)
        last = self.up_layers[-1][1] if D else self.down_layers[0][1]
        hgw, hgb = st.flat_slice("outc.conv.weight", st.grad), st.flat_slice("outc.conv.bias", st.grad)
        head_gscale = None
        if self.fuse_head and self._head_fwd_grads and gscale == self.head_gscale:
            C.head_grad_finalize(self.head_gpart, self.M, hgw, hgb)  # partials came with the forward
            last.bwd_rows = C.head_partial_blocks(self.M)
            head_gscale = gscale
        elif self.fuse_head:
            last.bwd_rows = C.head_bwd(last.y, head_w, self.logits, self.target, self.loss_sums, None,
                                       self.head_partial, hgw, hgb, self.dice_w, self.dice_eps, gscale, last.coef,
                                       self.bn_partial)
            head_gscale = gscale
        else:
            C.head_bwd(self.final, head_w, self.logits, self.target, self.loss_sums, last.da, self.head_partial, hgw,
                       hgb, self.dice_w, self.dice_eps, gscale)
        self._head_fwd_grads = False
        if grad_hook is not None:  # the head's gradients are final now: its bucket may go first
            grad_hook(HEAD_SPEC, torch.cuda.current_stream() if self.dev.type == "cuda" else None)
        for i in range(D, 0, -1):
            la, lb = self.up_layers[i - 1]
            self._conv_bwd(C, lb, grad_hook, head_gscale if i == D else None)
            self._conv_bwd(C, la, grad_hook)
            # d(low) = upsample / transposed-conv backward of du
            low_layer = self.down_layers[D][1] if i == 1 else self.up_layers[i - 2][1]
            du = self.dups[i - 1]
            oy = (du.shape[1] - 2 * low_layer.a.shape[1]) // 2
            ox = (du.shape[2] - 2 * low_layer.a.shape[2]) // 2
            if self.m.bilinear:  # + the BN-backward reduction of low_layer (like the pool boundary)
                low_layer.bwd_rows = C.upsample2_bwd(du, low_layer.da, oy, ox, low_layer.y, low_layer.coef,
                                                     self.bn_partial)
            else:
                us = self.m.up_specs[i - 1]
                dyT = self.dyTs[i - 1]
                bgrad = st.flat_slice(us.name + ".bias", st.grad)
                wgrad = st.flat_slice(us.name + ".weight", st.grad)
                ns = self.upT_splits[i - 1]
                exact = du.shape[1] == 2 * dyT.shape[1] and du.shape[2] == 2 * dyT.shape[2]  # no F.pad border
                if exact:
                    # bias / weight / input gradients read du's 2x2 sub-pixels in place (no unshuffled copy):
                    # bias = column sums of du, weight = the role-swapped GEMM over the sub-pixels (wgrad
                    # stream), input = the ping-pong GEMM with the sub-pixels as 4 taps where it takes the
                    # shape (else the unshuffle + 1x1 GEMM)
                    C.colsum_bf16(du, 1, self.colsum_ws, bgrad, 0)
                    self._on_wgrad_stream(lambda slab, du=du, xa=low_layer.a, ns=ns, g=wgrad:
                                          C.conv_wgrad_upT(du, xa, 0, 0, slab, g, 0, ns))
                    if C.conv_upT_dgrad(du, self.m.upT_dgrad_weight(us), low_layer.da, 0, 0) != 0:
                        C.upT_unshuffle(du, dyT, oy, ox)
                        C.conv_fwd(dyT, None, self.m.upT_dgrad_weight(us), 1, 0, low_layer.da, None, None, 0, None,
                                   0, self.kws)
                else:
                    C.upT_unshuffle(du, dyT, oy, ox)
                    C.colsum_bf16(dyT, 4, self.colsum_ws, bgrad, 0)
                    self._on_wgrad_stream(lambda slab, dyT=dyT, xa=low_layer.a, us=us, ns=ns, g=wgrad:
                                          C.conv_wgrad(dyT, None, xa, 1, 0, 4 * us.cout, slab, g, 0, ns, 0))
                    C.conv_fwd(dyT, None, self.m.upT_dgrad_weight(us), 1, 0, low_layer.da, None, None, 0, None, 0,
                               self.kws)
                if grad_hook is not None:  # bias (main) + weight (side, forked after the bias)
                    grad_hook(us, self.side if self.side is not None else torch.cuda.current_stream())
        for i in range(D, 0, -1):
            la, lb = self.down_layers[i]
            self._conv_bwd(C, lb, grad_hook)
            self._conv_bwd(C, la, grad_hook)
            prev = self.down_layers[i - 1][1]
            prev.bwd_rows = C.maxpool2_bwd_bn_reduce(self.dpools[i - 1], self.skips[i - 1], self.dskips[i - 1],
                                                     prev.da, prev.y, prev.coef, self.bn_partial)
        l0, l1 = self.down_layers[0]
        self._conv_bwd(C, l1, grad_hook)
        self._conv_bwd(C, l0, grad_hook)

    def backward_order(self) -> List:
        """Gradient hooks in the order backward() fires them (see :func:`backward_hook_order`)."""
        return backward_hook_order(self.m.specs, self.m.up_specs, self.m.depth)


def backward_hook_order(specs: List[ConvSpec], up_specs: List[UpTSpec], depth: int) -> List:
    """The gradient hooks of ``UNetExecutor.backward`` in firing order: the head first (its gradients
    come with the loss), then per conv layer from the output back to the input its BN's gamma / beta
    (:class:`BNHook`) and its weight; a transposed decoder's ConvTranspose2d after its Up block's
    first conv. ``specs`` is the forward order of :func:`unet_conv_specs`."""
    D = depth
    enc = specs[: 2 * (D + 1)]
    dec = specs[2 * (D + 1):]
    out: List = [HEAD_SPEC]

    def conv(sp):
        out.extend([BNHook(sp), sp])

    for i in range(D, 0, -1):
        conv(dec[2 * (i - 1) + 1])
        conv(dec[2 * (i - 1)])
        if up_specs:
            out.append(up_specs[i - 1])
    for i in range(D, -1, -1):
        conv(enc[2 * i + 1])
        conv(enc[2 * i])
    return out


class NativeAdam:
    """torch.optim.Adam semantics over the flat store, one fused launch (+ derived-weight rebuild).

    (Measured dead end: per-layer Adam segments on the weight-gradient side stream as each layer's
    gradient became final -- neutral at bs64, 3% slower at bs4 from the 18 extra launches.)"""

    def __init__(self, model: UNetNative, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0):
        self.m = model
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay

    # Overlap the update with the next forward (RDP_ADAM_OVERLAP, default on; needs ``side`` and a model
    # whose parameter layout splits, UNetNative._adam_split)
    OVERLAP = os.environ.get("RDP_ADAM_OVERLAP", "1") != "0"
    # grid cap of the side-stream group (0: full grid)
    # (measured: 256 blocks 19.00 / 19.10 ms bs 64 and 2.392 / 2.387 ms bs 4 vs 19.10 / 19.12 and 2.405 / 2.394
    # with the full grid, vs 19.10 / 19.28 and 2.400 / 2.391 without the overlap; one box, interleaved)
    SIDE_BLOCKS = int(os.environ.get("RDP_ADAM_SIDE_BLOCKS", "256"))

    def step(self, gscale: float = 1.0, side: Optional["torch.cuda.Stream"] = None,
             grad: Optional[torch.Tensor] = None):
        """``grad``: the gradients to apply (default the store's fp32 grad; the DDP bf16 all-reduce buffer
        is read as is). ``side``: the training executor's weight-gradient stream. The dgrad weight layouts are then
        rebuilt there, off the critical path, overlapping the next forward (which reads only the packed
        first layer and the transposed decoder's weights, rebuilt here); the next backward waits for
        them (:meth:`UNetExecutor.backward`)."""
        C = _native()
        st = self.m.store
        m = self.m
        g = st.grad if grad is None else grad
        split = m._adam_split
        if side is not None and self.OVERLAP and 0 < split < st.numel and m._nseg_bwd > 0:
            # group A (inc, down1) on the main stream, then the rest of the update and every derived layout
            # but the packed first layer on the side stream: the next forward runs its first two
            # DoubleConvs meanwhile and joins the side stream before down2 (UNetExecutor._wait_layer); the
            # step counter advances once, after both groups read it. Per element the same arithmetic as
            # the single launch, so the result is bitwise the same.
            a, b = slice(0, split), slice(split, st.numel)
            C.adam(st.flat[a], g[a], st.exp_avg[a], st.exp_avg_sq[a], st.shadow[a], self.lr, self.betas[0],
                   self.betas[1], self.eps, self.wd, gscale, st.step, False)
            if m._nseg_fwd_a:
                C.wprep(st.flat, m.derived, m._segs_fwd_a, m._nseg_fwd_a, None, m._wblk_fwd_a)
            if m.__dict__.get("_adam_ev") is None:
                m.__dict__["_adam_ev"] = C.event_create()
            _stream_wait(side, torch.cuda.current_stream())
            with torch.cuda.stream(side):
                C.adam(st.flat[b], g[b], st.exp_avg[b], st.exp_avg_sq[b], st.shadow[b], self.lr, self.betas[0],
                       self.betas[1], self.eps, self.wd, gscale, st.step, False, self.SIDE_BLOCKS)
                if m._nseg_fwd_b:  # the transposed decoder's ConvTranspose2d forward layouts
                    C.wprep(st.flat, m.derived, m._segs_fwd_b, m._nseg_fwd_b, None, m._wblk_fwd_b)
                C.event_record(m._adam_ev, side.cuda_stream)  # the next forward's join point
                # dgrad layouts, read only by the next backward (+ the step counter advance, after both
                # groups read it)
                C.wprep(st.flat, m.derived, m._segs_bwd, m._nseg_bwd, st.step, m._wblk_bwd)
            m.__dict__["_wprep_pending"] = side
            m.__dict__["_adam_ev_pending"] = True
            return
        C.adam(st.flat, g, st.exp_avg, st.exp_avg_sq, st.shadow, self.lr,
               self.betas[0], self.betas[1], self.eps,
               self.wd, gscale, st.step, False)
        if side is None or m._nseg_bwd == 0:
            C.wprep(st.flat, m.derived, m._segs, m._nseg, st.step, m._wblk)  # + the step counter advance
            return
        C.wprep(st.flat, m.derived, m._segs_fwd, m._nseg_fwd, st.step, m._wblk_fwd)
        _stream_wait(side, torch.cuda.current_stream())
        with torch.cuda.stream(side):
            C.wprep(st.flat, m.derived, m._segs_bwd, m._nseg_bwd, None, m._wblk_bwd)
        m.__dict__["_wprep_pending"] = side

    def hyper_key(self) -> tuple:
        """The hyper-parameters a recorded launch plan bakes in (NativeTrainer re-records on change)."""
        return (float(self.lr), tuple(float(b) for b in self.betas), float(self.eps), float(self.wd))

    def state_dict(self):
        st = self.m.store
        self.m._join_wprep()
        return {"step": st.step.clone(), "exp_avg": st.exp_avg.clone(), "exp_avg_sq": st.exp_avg_sq.clone(),
                "lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.wd}

    def load_state_dict(self, sd):
        st = self.m.store
        self.m._join_wprep()
        with torch.no_grad():
            st.step.copy_(sd["step"])
            st.exp_avg.copy_(sd["exp_avg"])
            st.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.lr, self.betas, self.eps, self.wd = sd["lr"], tuple(sd["betas"]), sd["eps"], sd["weight_decay"]
