#!/usr/bin/env python3
"""Headline benchmark: U-Net train imgs/sec at 256x256 (BASELINE.json metric, config 2/3).

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``. Both launch forms run N ranks,
one per GPU:
  * under a launcher (``torch.distributed.run --nproc-per-node N ... bench.py --gpus N``): every rank
    reads RANK / LOCAL_RANK / WORLD_SIZE from the env; a WORLD_SIZE different from ``--gpus`` is an
    error (exit 2), never a silent 1-GPU run;
  * directly (``python bench.py --gpus N``, no WORLD_SIZE in the env, N > 1): this process touches no
    GPU -- it starts ``torch.distributed.run`` with N ranks as a child process (never exec),
    its rank 0 prints the JSON line to the inherited stdout, and the parent exits with the child's
    return code (torchrun's: non-zero if any rank failed).
W untimed warm-up steps, then exactly K timed steps bracketed by barrier + device sync on both
sides; the time is the MAX over ranks; rank 0 prints one JSON line. ``value`` is the whole-job
aggregate (images/s over all ranks).

The step is the full reference training step (``scripts/train_segmenter.py:156-165``): forward,
BCEWithLogits loss, backward, Adam(lr=1e-4) -- on random-init weights of the reference
architecture (``UNet(3, 1)``, bilinear decoder) and synthetic 256x256 RGB images / binary masks.

Implementations:
  * ``--impl native`` (default): the framework's HIP/CDNA4 kernels (NHWC bf16 implicit-GEMM convs,
    fused BN/ReLU/pool/upsample/loss kernels, flat fused Adam), optional hipGraph capture, RCCL
    bucketed gradient all-reduce.
  * ``--impl eager``: the reference execution model on the same GPU (torch eager + MIOpen,
    bf16 autocast, channels_last) -- the comparison baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# reference training throughput (bs4 256^2 fp32, measured on the sandbox CPU).
BASELINE_TRAIN_IMGS_PER_S = 2.14
METRIC = "U-Net train imgs/sec at 256×256 (1/2/4/8 GPU); e2e frames/sec + p50 latency"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=64, help="per-GPU batch (weak scaling: fixed per GPU)")
    p.add_argument("--size", type=int, default=256)
    p.add_argument("--impl", choices=["native", "eager"], default="native")
    p.add_argument("--decoder", choices=["bilinear", "transposed"], default="bilinear")
    p.add_argument("--graph", type=int, default=-1,
                   help="capture the native step in a hipGraph (1), eager launches (0), -1: auto by batch size")
    p.add_argument("--bucket-mb", type=float, default=16.0)
    p.add_argument("--loss", choices=["bce", "bce_dice"], default="bce")
    p.add_argument("--sync-bn", type=int, default=0, help="1: SyncBatchNorm across ranks (not the reference's BN)")
    p.add_argument("--grad-comm", choices=["fp32", "bf16"], default="fp32",
                   help="gradient all-reduce dtype (bf16: half the xGMI bytes, fp32 accumulate in Adam)")
    p.add_argument("--ddp-force", type=int, default=0,
                   help="1: run the DDP path (RCCL process group, bucketed all-reduce hooks) even at world 1")
    p.add_argument("--extras", type=int, default=-1,
                   help="also report ref_batch_imgs_per_s (bs 4 step) and train_model_imgs_per_s (train_model on an "
                        "on-disk synthetic PNG dataset, incl. data gather/H2D) and transposed_imgs_per_s (the "
                        "transposed-conv decoder at the same batch); default: on for 1-GPU native runs")
    p.add_argument("--serve", type=int, default=-1,
                   help="also measure e2e serving FPS / p50 latency (default: on for single-GPU runs)")
    return p.parse_args()


def self_launch(args) -> "int | None":
    """``--gpus N`` without a launcher: start N ranks as a child ``torch.distributed.run`` job and
    return its exit code. Returns None when this process is (or should act as) the rank itself.
    Nothing here initialises the GPU (``device_count`` does not on this ROCm image)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks; "
                  f"pass --gpus {env_world} (or launch {args.gpus} ranks)", file=sys.stderr, flush=True)
            sys.exit(2)
        return None
    if args.gpus <= 1:
        return None
    shared = os.environ.get("RDP_DIST_BACKEND") == "gloo"  # test mode: ranks may share one GPU
    if args.impl == "native" and not shared:
        have = torch.cuda.device_count()
        if have < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {have} GPU(s) are visible", file=sys.stderr, flush=True)
            sys.exit(2)
    import subprocess
    from robotic_discovery_platform_amd.utils.launch import _free_port
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        # test mode: several gloo ranks may share one GPU (RCCL refuses that; the real runs use nccl)
        if os.environ.get("RDP_DIST_BACKEND") == "gloo" and local >= torch.cuda.device_count():
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if world > 1 or args.ddp_force:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            from robotic_discovery_platform_amd.utils.launch import _free_port
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # nccl == RCCL on ROCm (xGMI); RDP_DIST_BACKEND=gloo lets several ranks share one GPU in tests
        backend = os.environ.get("RDP_DIST_BACKEND") or ("nccl" if dev.type == "cuda" else "gloo")
        from robotic_discovery_platform_amd.utils.launch import dist_timeout
        dist.init_process_group(backend=backend, timeout=dist_timeout(),
                                device_id=dev if dev.type == "cuda" and backend == "nccl" else None)
    return rank, world, dev


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def barrier(world, dev):
    if world > 1:
        dist.barrier()
    sync(dev)


def make_eager_step(args, dev, world):
    from robotic_discovery_platform_amd.models.unet_ref import UNet
    model = UNet(3, 1, bilinear=(args.decoder == "bilinear")).to(dev).to(memory_format=torch.channels_last)
    if world > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if dev.type == "cuda" else None,
                                                          bucket_cap_mb=args.bucket_mb)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    crit = torch.nn.BCEWithLogitsLoss()
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.rand(args.batch, 3, args.size, args.size, generator=g).to(dev).to(memory_format=torch.channels_last)
    y = (torch.rand(args.batch, 1, args.size, args.size, generator=g) > 0.5).float().to(dev)
    amp = dev.type == "cuda"

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast(device_type=dev.type, dtype=torch.bfloat16, enabled=amp):
            out = model(x)
        loss = crit(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    return step


def make_native_step(args, dev, world):
    from robotic_discovery_platform_amd.train.engine import build_bench_step
    return build_bench_step(batch=args.batch, size=args.size, decoder=args.decoder, device=dev,
                            world=world, graph="auto" if args.graph < 0 else bool(args.graph), bucket_mb=args.bucket_mb, loss=args.loss,
                            sync_bn=bool(args.sync_bn), grad_comm=args.grad_comm, ddp_force=bool(args.ddp_force))


def quiesce_gc() -> None:
    """Collect once and move every object alive now out of the cyclic collector's reach (``gc.freeze``,
    as the server does after start-up): a full collection of the framework's start-up heap landing inside
    a short timed region shows up as a slow step."""
    import gc
    if os.environ.get("RDP_BENCH_GC_FREEZE", "1") == "0":  # A/B
        return
    gc.collect()
    gc.freeze()


def measure_ref_batch(args, dev, steps: int = 200, warmup: int = 20) -> dict:
    """The reference's batch (bs 4, train_segmenter.py:46) through the same native step. (200 timed steps,
    ~0.5 s: 50 steps left the number at the mercy of a single host hiccup -- 1,342-1,384 vs 1,689-1,703 img/s
    in otherwise equal runs, profiles/bench_recheck_r6.jsonl.)"""
    from robotic_discovery_platform_amd.train.engine import build_bench_step
    step = build_bench_step(batch=4, size=args.size, decoder=args.decoder, device=dev, world=1, graph="auto",
                            bucket_mb=args.bucket_mb, loss=args.loss)
    for _ in range(warmup):
        step()
    sync(dev)
    quiesce_gc()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync(dev)
    dt = time.perf_counter() - t0
    return {"ref_batch_imgs_per_s": round(4 * steps / dt, 2), "ref_batch_ms_per_step": round(dt / steps * 1e3, 3)}


def measure_transposed(args, dev, steps: int = 20, warmup: int = 5) -> dict:
    """BASELINE.json's north-star decoder ("transposed-conv decoder", the reference's
    ``bilinear=False`` path, fixed: ``segmentation_model.py:63-65,75-76``) through the same timed step
    at the headline's per-GPU batch: forward, BCE, backward, Adam, device syncs around the K steps."""
    if args.decoder == "transposed":
        return {}
    from robotic_discovery_platform_amd.train.engine import build_bench_step
    step = build_bench_step(batch=args.batch, size=args.size, decoder="transposed", device=dev, world=1,
                            graph="auto", bucket_mb=args.bucket_mb, loss=args.loss)
    for _ in range(warmup):
        step()
    sync(dev)
    quiesce_gc()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync(dev)
    dt = time.perf_counter() - t0
    return {"transposed_imgs_per_s": round(args.batch * steps / dt, 2),
            "transposed_ms_per_step": round(dt / steps * 1e3, 3),
            "transposed_config": f"UNet(3,1) transposed decoder (fixed), 31.04M params, bs {args.batch}, "
                                 f"{steps} timed steps"}


def measure_train_model(args, dev, samples: int = 160, epochs: int = 3) -> dict:
    """``train_model`` (the train_segmenter.py entry point) on an on-disk synthetic PNG dataset at the
    reference's batch 4: device-resident data build, per-epoch shuffled batches gathered on the GPU,
    native steps, eval-mode validation, checkpoints and registry writes. Reports the last epoch's
    training throughput (validation excluded) and the epoch wall time."""
    import logging
    import tempfile
    from robotic_discovery_platform_amd.config import TrainConfig
    from robotic_discovery_platform_amd.data.synthetic import write_dataset
    from robotic_discovery_platform_amd.train.trainer import train_model
    root = tempfile.mkdtemp(prefix="rdp_bench_tm_")
    write_dataset(os.path.join(root, "data"), samples, seed=0)
    logging.getLogger("rdp.train").setLevel(logging.WARNING)
    cfg = TrainConfig(epochs=epochs, batch_size=4, image_size=args.size, bilinear=args.decoder == "bilinear",
                      dataset_dir=os.path.join(root, "data"), mlruns_dir=os.path.join(root, "mlruns"),
                      model_output_dir=os.path.join(root, "models"), backend="native")
    res = train_model(cfg)
    last = res["history"][-1]
    return {"train_model_imgs_per_s": round(last["train_imgs_per_s"], 2),
            "train_model_epoch_s": round(last["epoch_s"], 4),
            "train_model_config": f"bs4, {samples} on-disk PNG scenes (80/20 split), epoch {epochs} of {epochs}"}


class _Progress:
    """Prints the current phase to stderr every 30 s until the timed region is done (rank 0)."""

    def __init__(self, rank: int, period: float = 30.0):
        import threading
        self.phase, self.t0 = "setup", time.perf_counter()
        if rank == 0:
            self._stop = threading.Event()
            th = threading.Thread(target=self._run, args=(period,), daemon=True)
            th.start()

    def _run(self, period):
        while not self._stop.wait(period):
            print(f"[bench] {self.phase} ({time.perf_counter() - self.t0:.0f} s)", file=sys.stderr, flush=True)


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    rank, world, dev = setup_dist(args)
    comm = {}
    if dist.is_initialized() and os.environ.get("RDP_COMM_SELFCHECK", "1") != "0":
        # the first real multi-rank run of the native collective path checks itself before anything is
        # timed: RCCL's rank count, a rank-sum probe through the buckets' exact call, fallback to
        # torch.distributed issue if it fails, measured all-reduce bus bandwidth (parallel/selfcheck.py)
        from robotic_discovery_platform_amd.parallel.selfcheck import CommMismatch, comm_selfcheck
        from robotic_discovery_platform_amd.train.engine import NativeTrainer
        want_native = args.impl == "native" and dev.type == "cuda" and NativeTrainer.native_comm_wanted_env()
        try:
            comm = comm_selfcheck(dev, want_native)
        except CommMismatch as e:
            print(f"bench.py: {e}", file=sys.stderr, flush=True)
            sys.exit(3)
    step = make_eager_step(args, dev, world) if args.impl == "eager" else make_native_step(args, dev, world)
    tr = getattr(step, "trainer", None)
    used_graph = bool(tr.use_graph) if tr is not None else False
    progress = _Progress(rank)  # stderr heartbeat: first eager steps can spend minutes in MIOpen kernel builds
    for i in range(args.warmup):
        progress.phase = f"warmup step {i + 1}/{args.warmup}"
        step()
    progress.phase = "timed steps"
    quiesce_gc()
    barrier(world, dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier(world, dev)
    dt = time.perf_counter() - t0
    dt_own = dt
    t = torch.tensor([dt], dtype=torch.float64, device=dev if world > 1 and dev.type == "cuda" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1e3
    rank_ms = [ms]
    if world > 1:  # every rank's own timed-region length (the headline uses the max)
        own = torch.tensor([dt_own / args.steps * 1e3], dtype=torch.float64,
                           device=dev if dev.type == "cuda" and dist.get_backend() == "nccl" else "cpu")
        allt = [torch.zeros_like(own) for _ in range(world)]
        dist.all_gather(allt, own)
        rank_ms = [float(x.item()) for x in allt]
    imgs = args.batch * world * args.steps / dt
    extra = {}
    extras = args.extras if args.extras >= 0 else int(world == 1 and args.impl == "native" and dev.type == "cuda")
    if extras and rank == 0:
        progress.phase = "extras (reference batch, transposed decoder, train_model)"
        for fn in (measure_ref_batch, measure_transposed, measure_train_model):
            try:  # never let it break the training result line
                extra.update(fn(args, dev))
            except Exception as e:  # pragma: no cover - reported in the JSON
                extra[fn.__name__ + "_error"] = f"{type(e).__name__}: {e}"
    serve = args.serve if args.serve >= 0 else int(world == 1 and args.impl == "native" and dev.type == "cuda")
    if serve and rank == 0:
        progress.phase = "serving"
        try:  # second half of the metric; never let it break the training result line
            from robotic_discovery_platform_amd.serve.bench_serve import measure_serving
            extra.update(measure_serving(dev))
        except Exception as e:  # pragma: no cover - reported in the JSON
            extra["serve_error"] = f"{type(e).__name__}: {e}"
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(imgs, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(imgs / BASELINE_TRAIN_IMGS_PER_S, 2),
            "dtype": "bf16",
            "data": "synthetic (random 256x256 RGB + binary masks), random-init weights",
            "config": {
                "model": f"UNet(3,1) {args.decoder} decoder, 17.26M params" if args.decoder == "bilinear"
                else "UNet(3,1) transposed decoder (fixed), 31.04M params",
                "global_batch": args.batch * world,
                "per_gpu_batch": args.batch,
                "seq_len": None,
                "image_size": args.size,
                "parallelism": f"dp{world}",
                "impl": args.impl,
                "optimizer": "Adam(lr=1e-4)",
                "loss": args.loss,
                # statistics actually shared (world > 1, or the emulated collective of RDP_DDP_EMULATE)
                "sync_bn": bool(getattr(getattr(tr, "ex", None), "_sync_on", False)),
                "hipgraph": used_graph,
                "grad_comm": args.grad_comm if (world > 1 or args.ddp_force) else None,
                "ddp_stream": getattr(tr, "ddp_stream", None),
                "ddp_emulate": os.environ.get("RDP_DDP_EMULATE") or None,
            },
            "baseline_note": "vs_baseline = value / 2.14 img/s (BASELINE.md: reference bs4 fp32 on CPU; "
                             "no published GPU number exists)",
        }
        if world > 1:
            out["rank_ms_per_step_min"] = round(min(rank_ms), 3)
            out["rank_ms_per_step_max"] = round(max(rank_ms), 3)
        out.update(comm)
        out.update(extra)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        from robotic_discovery_platform_amd.parallel.watchdog import close_all
        close_all()  # the comm watchdog polls communicators of the groups destroyed next
        try:
            dist.destroy_process_group()
        except Exception as e:  # the result line is out; e.g. a communicator the self-check aborted
            print(f"bench.py: process-group teardown: {type(e).__name__}: {e}", file=sys.stderr, flush=True)
    return bool(serve) and rank == 0


if __name__ == "__main__":
    if main():
        # The result line is out and the serving measurement ran: skip interpreter teardown so the
        # gRPC core's threads cannot turn a finished run into an abort at exit. (Not taken with
        # --serve 0 -- profilers such as rocprofv3 write their output in exit handlers.)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
