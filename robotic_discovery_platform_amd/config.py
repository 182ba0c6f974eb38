"""Typed configuration for every subsystem, with defaults equal to the reference constants.

The reference hard-codes its constants in each script (SURVEY.md §5 "Config / flag system",
App. C). Here they live in one place as dataclasses, overridable from the CLI
(``--key value`` via :func:`add_dataclass_args`) or the environment (``RDP_<SECTION>_<KEY>``).

Reference citations (``/root/reference``):
  * training: ``scripts/train_segmenter.py:45-63``
  * serving:  ``services/vision_analysis/server.py:52-65,172,176``
  * client:   ``services/vision_analysis/client.py:43-45,92``
  * camera:   ``pkg/camera.py:35,62-63``
  * geometry: ``pkg/geometry_utils.py:64,69,78,83,119,144,155``
  * calibration: ``scripts/01_calibrate_camera.py:37-38,42,93``
  * collection: ``scripts/02_collect_segmentation_data.py:40-42``
  * drift: ``scripts/monitoring/drift_detector.py:16-22,37,71,84``
"""
from __future__ import annotations

import argparse
import dataclasses
import os
from dataclasses import dataclass, field, fields
from pathlib import Path
from typing import Any, Optional

# Project root = the directory containing the package (the reference resolves
# MLRUNS_DIR relative to its project root: train_segmenter.py:57).
PROJECT_ROOT = Path(os.environ.get("RDP_PROJECT_ROOT", Path(__file__).resolve().parent.parent))

MLFLOW_EXPERIMENT_NAME = "Actuator Segmentation"  # train_segmenter.py:62
MLFLOW_MODEL_NAME = "Actuator-Segmenter"  # train_segmenter.py:63
MLFLOW_ARTIFACT_NAME = "model"  # train_segmenter.py:202
PROMOTION_ALIAS = "staging"  # retraining_pipeline.py:72


@dataclass
class ModelConfig:
    n_channels: int = 3
    n_classes: int = 1
    base_width: int = 64
    depth: int = 4  # number of Down blocks (reference: 4)
    bilinear: bool = True  # reference default decoder (segmentation_model.py:91)


@dataclass
class TrainConfig:
    learning_rate: float = 1e-4
    batch_size: int = 4
    epochs: int = 50
    validation_split: float = 0.2
    image_size: int = 256
    loss: str = "bce"  # "bce" (reference) or "bce_dice" (north star)
    dice_weight: float = 1.0
    seed: int = 0  # the reference split is unseeded; we seed it
    dataset_dir: str = os.path.join("ml", "datasets", "processed")  # CWD-relative like the reference
    mlruns_dir: str = str(PROJECT_ROOT / "ml" / "mlruns")
    model_output_dir: str = str(PROJECT_ROOT / "ml" / "models" / "segmentation")
    experiment_name: str = MLFLOW_EXPERIMENT_NAME
    registered_model_name: str = MLFLOW_MODEL_NAME
    backend: str = "auto"  # "native" (HIP kernels), "eager" (plain torch), "auto"
    dtype: str = "bf16"
    num_workers: int = 0
    synthetic_if_missing: bool = True
    synthetic_samples: int = 64
    grad_bucket_mb: float = 16.0
    device_data: bool = True  # GPU: build the processed dataset once on the device (u8), batches gathered there
    grad_comm: str = "fp32"  # gradient all-reduce dtype: "fp32" or "bf16" (fp32 accumulate in Adam)
    dist_timeout_s: float = 600.0  # process-group timeout: a hung collective fails the job instead of hanging
    sync_bn: bool = False  # share BN batch statistics across DDP ranks (SyncBatchNorm semantics)
    graph: bool = False  # hipGraph-capture the train step (measured slower than eager launches, engine.py)
    model_depth: int = 4  # U-Net levels (reference: 4; the plumbing config uses 2)
    bilinear: bool = True  # decoder: bilinear upsample (reference default) or transposed conv (fixed)


@dataclass
class ServeConfig:
    host: str = "[::]"
    port: int = 50051
    max_workers: int = 10
    model_img_size: int = 256
    default_depth_scale: float = 0.001
    model_uri: str = f"models:/{MLFLOW_MODEL_NAME}/latest"
    mlruns_dir: str = str(PROJECT_ROOT / "ml" / "mlruns")
    calib_file: str = str(PROJECT_ROOT / "ml" / "configs" / "calibration_data.npz")
    metrics_log: str = str(PROJECT_ROOT / "logs" / "vision_service_metrics.csv")
    mask_threshold: float = 0.5
    backend: str = "auto"
    graph: bool = True
    devices: str = ""  # comma-separated GPU indices for per-GPU replicas ("" = current device only; "all")
    replicas_per_device: int = 2  # independent stream pipelines (hipGraph + buffers) per GPU
    frame_errors: str = "degrade"  # "degrade": bad frame -> error status, stream goes on; "abort": reference
    gpu_jpeg: bool = True  # baseline JPEGs: native entropy decode on the host, pixel stage in the frame graph
    workers: int = 1  # server processes sharing the port (SO_REUSEPORT): one interpreter lock each
    hot_reload_alias: Optional[str] = None  # e.g. "staging": reload when alias moves


@dataclass
class ClientConfig:
    server_address: str = "localhost:50051"
    smoothing_window: int = 10
    pairing_queue: int = 20
    calib_file: str = str(PROJECT_ROOT / "ml" / "configs" / "calibration_data.npz")


@dataclass
class CameraConfig:
    width: int = 640
    height: int = 480
    fps: int = 30
    backend: str = "synthetic"  # "synthetic" or "realsense"


@dataclass
class GeometryConfig:
    min_points: int = 100
    min_edge_points: int = 20
    num_bins: int = 50
    top_k_percent: float = 0.05
    smoothing: float = 0.1
    spline_degree: int = 3
    num_samples: int = 100
    deriv_eps: float = 1e-6


@dataclass
class CalibrationConfig:
    checkerboard: tuple = (9, 7)
    square_size_m: float = 0.027
    min_captures: int = 5
    subpix_window: tuple = (11, 11)
    subpix_max_iter: int = 30
    subpix_eps: float = 0.001
    out_file: str = str(PROJECT_ROOT / "ml" / "configs" / "calibration_data.npz")


@dataclass
class CollectConfig:
    save_interval_s: float = 0.5
    raw_dir: str = str(PROJECT_ROOT / "ml" / "raw_data")


@dataclass
class DriftConfig:
    log_file: str = os.path.join("logs", "vision_service_metrics.csv")  # CWD-relative like the reference
    reports_dir: str = "reports"
    min_rows: int = 50
    baseline_frac: float = 0.5
    threshold: float = 0.25
    rolling_window: int = 20
    dpi: int = 150
    metric: str = "mask_coverage_percent"


def _coerce(tp: Any, value: str) -> Any:
    if isinstance(tp, str):
        tp = {"int": int, "float": float, "bool": bool, "str": str, "tuple": tuple}.get(
            tp.replace("Optional[", "").rstrip("]"), str)
    if tp is bool:
        return value.lower() in ("1", "true", "yes", "on")
    if tp is tuple:
        return tuple(int(v) for v in value.split(","))
    if tp in (int, float, str):
        return tp(value)
    return value


def apply_env(cfg: Any, section: str) -> Any:
    """Override dataclass fields from ``RDP_<SECTION>_<FIELD>`` environment variables."""
    for f in fields(cfg):
        key = f"RDP_{section.upper()}_{f.name.upper()}"
        if key in os.environ:
            setattr(cfg, f.name, _coerce(f.type, os.environ[key]))
    return cfg


def add_dataclass_args(parser: argparse.ArgumentParser, cfg: Any, prefix: str = "") -> None:
    for f in fields(cfg):
        name = f"--{prefix}{f.name.replace('_', '-')}"
        default = getattr(cfg, f.name)
        if isinstance(default, bool):
            parser.add_argument(name, type=lambda v: v.lower() in ("1", "true", "yes"), default=default)
        elif isinstance(default, tuple):
            parser.add_argument(name, type=lambda v: tuple(int(x) for x in v.split(",")), default=default)
        elif default is None:
            parser.add_argument(name, type=str, default=None)
        else:
            parser.add_argument(name, type=type(default), default=default)


def from_args(cfg_cls: Any, args: argparse.Namespace, prefix: str = "") -> Any:
    cfg = cfg_cls()
    for f in fields(cfg):
        key = f"{prefix}{f.name}"
        if hasattr(args, key):
            setattr(cfg, f.name, getattr(args, key))
    return cfg


def to_dict(cfg: Any) -> dict:
    return dataclasses.asdict(cfg)
