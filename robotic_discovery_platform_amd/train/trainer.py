"""``train_model()``: the reference training + registration pipeline on the native engine.

Mirrors ``/root/reference/scripts/train_segmenter.py:103-210`` step by step:
  * MLflow setup: tracking URI = file store ``ml/mlruns``, experiment "Actuator Segmentation" (:112-113)
  * params logged: learning_rate, batch_size, epochs, validation_split, image_size, device, architecture (:119-128)
  * dataset ``ml/datasets/processed/{images,masks}`` paired by filename, 80/20 split (:132-136) -- seeded here;
    synthetic scenes are generated when the directory is missing (no camera/data in this environment)
  * UNet(3,1), Adam(lr 1e-4), BCEWithLogitsLoss (:143-145); optional BCE+Dice (north star)
  * per epoch: train loss (mean over batches), eval-mode val loss, both logged with step=epoch (:151-184)
  * best-val checkpoint ``best_segmentation_model.pth`` (state_dict, :186-189), ``best_val_loss`` metric (:191)
  * best weights logged as artifact "model" and registered as "Actuator-Segmenter" (:195-207)

MI355X-native differences: the step runs on the HIP kernels (hipGraph-captured on one GPU), the
loss is accumulated on device and read once per epoch (the reference syncs with ``.item()`` every
step), DDP over RCCL with rank-0-only store writes, and a full resume checkpoint
(model + Adam state + epoch + best val + RNG) beside the best-only one.
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import asdict
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import mlstore
from ..config import TrainConfig
from ..data.dataset import SegmentationDataset, SyntheticSegmentationDataset, preload, split_dataset
from ..data.synthetic import write_dataset
from ..models.unet_ref import UNetRef
from ..parallel.ddp import DistributedShardSampler, dist_info

log = logging.getLogger("rdp.train")


def _device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    return torch.device("cpu")


def _pick_backend(cfg: TrainConfig, dev: torch.device) -> str:
    if cfg.backend != "auto":
        return cfg.backend
    return "native" if dev.type == "cuda" else "eager"


class _NativeRunner:
    """Per-batch-shape native executors (+ hipGraphs) over one model / one Adam state."""

    def __init__(self, model, cfg: TrainConfig):
        from ..models.unet import NativeAdam
        from .engine import NativeTrainer
        self.model, self.cfg = model, cfg
        self._trainers = {}
        self._cls = NativeTrainer
        self._shared_opt = NativeAdam(model, lr=cfg.learning_rate)

    def _get(self, n, h, w):
        key = (n, h, w)
        if key not in self._trainers:
            tr = self._cls(self.model, n, h, w, lr=self.cfg.learning_rate, loss=self.cfg.loss,
                           dice_weight=self.cfg.dice_weight, graph=self.cfg.graph, bucket_mb=self.cfg.grad_bucket_mb,
                           sync_bn=self.cfg.sync_bn, grad_comm=self.cfg.grad_comm)
            tr.opt = self._shared_opt
            self._trainers[key] = tr
        return self._trainers[key]

    def train_step(self, x, y) -> torch.Tensor:
        tr = self._get(x.shape[0], x.shape[2], x.shape[3])
        tr.set_batch(x, y)
        return tr.step()[0]

    def eval_loss(self, x, y) -> torch.Tensor:
        ex = self.model.executor(x.shape[0], x.shape[2], x.shape[3], training=False, loss=self.cfg.loss,
                                 dice_weight=self.cfg.dice_weight)
        ex.set_input(x, y)
        ex.forward()
        return ex.loss[0]

    def optimizer_state(self):
        return self._shared_opt.state_dict()

    def load_optimizer_state(self, sd):
        self._shared_opt.load_state_dict(sd)


class _EagerRunner:
    def __init__(self, model, cfg: TrainConfig, dev):
        from .engine import EagerTrainer
        amp = torch.bfloat16 if (dev.type == "cuda" and cfg.dtype == "bf16") else None
        self.tr = EagerTrainer(model, lr=cfg.learning_rate, loss=cfg.loss, dice_weight=cfg.dice_weight,
                               bucket_mb=cfg.grad_bucket_mb, amp=amp)
        self.model = model

    def train_step(self, x, y):
        self.model.train()
        return self.tr.step(x, y)

    @torch.no_grad()
    def eval_loss(self, x, y):
        self.model.eval()
        return self.tr.compute_loss(self.model(x), y)

    def optimizer_state(self):
        return self.tr.opt.state_dict()

    def load_optimizer_state(self, sd):
        self.tr.opt.load_state_dict(sd)


def _batches(x: torch.Tensor, y: torch.Tensor, order, bs: int, dev):
    """Batches (float NCHW image, float N1HW mask) in ``order``; u8 device-resident data is gathered
    and converted on the device."""
    if x.dtype == torch.uint8:
        from ..data.device_data import batch_to_float
        order = order.to(x.device)
        for i in range(0, len(order), bs):
            idx = order[i:i + bs]
            yield batch_to_float(x.index_select(0, idx), y.index_select(0, idx))
        return
    for i in range(0, len(order), bs):
        idx = order[i:i + bs]
        yield x[idx].to(dev, non_blocking=True), y[idx].to(dev, non_blocking=True)


def build_dataset(cfg: TrainConfig):
    img_dir = os.path.join(cfg.dataset_dir, "images")
    mask_dir = os.path.join(cfg.dataset_dir, "masks")
    size = (cfg.image_size, cfg.image_size)
    if os.path.isdir(img_dir) and os.path.isdir(mask_dir) and os.listdir(img_dir):
        return SegmentationDataset(img_dir, mask_dir, size)
    if not cfg.synthetic_if_missing:
        raise FileNotFoundError(f"dataset not found at {cfg.dataset_dir}")
    log.info("dataset %s missing: using %d synthetic scenes", cfg.dataset_dir, cfg.synthetic_samples)
    return SyntheticSegmentationDataset(cfg.synthetic_samples, size, seed=cfg.seed)


def train_model(cfg: Optional[TrainConfig] = None, resume: Optional[str] = None) -> dict:
    cfg = cfg or TrainConfig()
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    rank, world = dist_info()
    dev = _device()
    backend = _pick_backend(cfg, dev)
    is_main = rank == 0
    torch.manual_seed(cfg.seed)
    np.random.seed(cfg.seed)
    os.makedirs(cfg.model_output_dir, exist_ok=True)

    if is_main:
        mlstore.set_tracking_uri(cfg.mlruns_dir if "://" in cfg.mlruns_dir else os.path.abspath(cfg.mlruns_dir))
        mlstore.set_experiment(cfg.experiment_name)
        run = mlstore.start_run()
        log.info("Starting run %s", run.info.run_name)
        mlstore.log_params({"learning_rate": cfg.learning_rate, "batch_size": cfg.batch_size, "epochs": cfg.epochs,
                            "validation_split": cfg.validation_split, "image_size": cfg.image_size,
                            "device": str(dev), "architecture": "UNet", "backend": backend, "world_size": world,
                            "loss": cfg.loss, "dtype": cfg.dtype})

    # ---- data ----
    # GPU: the processed dataset is built once on the device (u8 NHWC; INTER_AREA / nearest resizes
    # as kernels) and batches are gathered there -- no per-step host work or H2D copy. CPU: host
    # float tensors (the reference's item format).
    ds = build_dataset(cfg)
    train_set, val_set = split_dataset(ds, cfg.validation_split, cfg.seed)
    size = (cfg.image_size, cfg.image_size)
    device_data = cfg.device_data and dev.type == "cuda" and hasattr(ds, "raw_arrays")
    if device_data:
        from ..data.device_data import build_device_dataset
        xtr, ytr = build_device_dataset(ds, train_set.indices, dev, size)
        xva, yva = build_device_dataset(ds, val_set.indices, dev, size) if len(val_set) else (None, None)
    else:
        xtr, ytr = preload(ds, train_set.indices)
        xva, yva = preload(ds, val_set.indices) if len(val_set) else (None, None)
    log.info("Dataset: %d training, %d validation samples (%s)", len(train_set), len(val_set),
             "device-resident u8" if device_data else "host")
    sampler = DistributedShardSampler(len(train_set), rank, world, shuffle=True, seed=cfg.seed)

    # ---- model / engine ----
    ref = UNetRef(3, 1, bilinear=cfg.bilinear, depth=cfg.model_depth)
    if backend == "native":
        from ..models.unet import UNetNative
        model = UNetNative(3, 1, bilinear=cfg.bilinear, depth=cfg.model_depth, device=dev, init_from=ref)
        runner = _NativeRunner(model, cfg)
    else:
        model = ref.to(dev)
        if cfg.sync_bn and dev.type == "cuda" and dist_info()[1] > 1:  # torch's SyncBatchNorm is GPU-only
            model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
        runner = _EagerRunner(model, cfg, dev)

    start_epoch, best_val = 0, float("inf")
    ckpt_last = os.path.join(cfg.model_output_dir, "last_checkpoint.pt")
    best_path = os.path.join(cfg.model_output_dir, "best_segmentation_model.pth")
    if resume:
        state = torch.load(resume if resume != "auto" else ckpt_last, map_location="cpu", weights_only=True)
        model.load_state_dict(state["model"])
        runner.load_optimizer_state(state["optimizer"])
        start_epoch, best_val = int(state["epoch"]) + 1, float(state["best_val"])
        torch.set_rng_state(state["rng_cpu"])
        log.info("Resumed from epoch %d (best val %.4f)", start_epoch, best_val)

    history = []
    from ..utils.launch import maybe_crash
    for epoch in range(start_epoch, cfg.epochs):
        maybe_crash(epoch, rank)
        t0 = time.time()
        sampler.set_epoch(epoch)
        order = torch.tensor(list(iter(sampler)), dtype=torch.long)
        tl = torch.zeros((), device=dev)
        nb = 0
        for xb, yb in _batches(xtr, ytr, order, cfg.batch_size, dev):
            tl += runner.train_step(xb, yb).float()
            nb += 1
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        t_train = time.time() - t0
        if world > 1:
            stats = torch.stack([tl, torch.tensor(float(nb), device=dev)])
            dist.all_reduce(stats)
            tl, nb = stats[0], int(stats[1].item())
        avg_train = float(tl.item()) / max(nb, 1)
        vl, nv = torch.zeros((), device=dev), 0
        if xva is not None and len(xva):
            for xb, yb in _batches(xva, yva, torch.arange(len(xva)), cfg.batch_size, dev):
                vl += runner.eval_loss(xb, yb).float()
                nv += 1
        avg_val = float(vl.item()) / max(nv, 1) if nv else avg_train
        dt = time.time() - t0
        history.append({"epoch": epoch, "train_loss": avg_train, "val_loss": avg_val, "epoch_s": dt,
                        "train_s": t_train, "train_imgs_per_s": len(order) * world / max(t_train, 1e-9)})
        if is_main:
            mlstore.log_metric("train_loss", avg_train, step=epoch)
            mlstore.log_metric("val_loss", avg_val, step=epoch)
            mlstore.log_metric("epoch_time_s", dt, step=epoch)
            mlstore.log_metric("train_imgs_per_s", len(order) * world / max(t_train, 1e-9), step=epoch)
            log.info("Epoch %d/%d: train %.4f val %.4f (%.1fs)", epoch + 1, cfg.epochs, avg_train, avg_val, dt)
            if avg_val < best_val:
                best_val = avg_val
                torch.save({k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()}, best_path)
                log.info("New best model at epoch %d: val %.4f", epoch + 1, best_val)
            torch.save({"model": {k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()},
                        "optimizer": _to_cpu(runner.optimizer_state()), "epoch": epoch, "best_val": best_val,
                        "rng_cpu": torch.get_rng_state()}, ckpt_last)
        if world > 1:
            dist.barrier()

    result = {"history": history, "best_val_loss": best_val, "backend": backend}
    if is_main:
        mlstore.log_metric("best_val_loss", best_val)
        if os.path.exists(best_path):
            model.load_state_dict(torch.load(best_path, map_location="cpu", weights_only=True))
        info = mlstore.pytorch.log_model(model, name="model", registered_model_name=cfg.registered_model_name)
        log.info("Model '%s' registered with version %s", cfg.registered_model_name, info.registered_model_version)
        result.update(run_id=info.run_id, registered_version=info.registered_model_version)
        if os.path.exists(best_path):
            os.remove(best_path)  # reference removes the temporary checkpoint (:210)
        mlstore.end_run()
    if world > 1:
        dist.barrier()
    return result


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj
