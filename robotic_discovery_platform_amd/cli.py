"""Command-line entry points (``python -m robotic_discovery_platform_amd <command> [--flags]``).

One command per reference entry point, with the reference constants as defaults
(config.py) and every field overridable by ``--flag`` or ``RDP_<SECTION>_<FIELD>``:

  train        scripts/train_segmenter.py            (torchrun-compatible: one rank per GPU)
  serve        services/vision_analysis/server.py
  client       services/vision_analysis/client.py    (headless; --save-dir writes overlays)
  calibrate    scripts/01_calibrate_camera.py
  collect      scripts/02_collect_segmentation_data.py (+ --label to build the processed dataset)
  drift        scripts/monitoring/drift_detector.py
  retrain      workflows/retraining_pipeline.py
  bench-serve  serving FPS / latency benchmark
"""
from __future__ import annotations

import argparse
import json
import logging
import sys

from . import config as C

LOG_FORMAT = "%(asctime)s - %(levelname)s - %(message)s"  # the reference's format everywhere


def _section(p: argparse.ArgumentParser, cls, section: str):
    cfg = C.apply_env(cls(), section)
    C.add_dataclass_args(p, cfg)
    return cfg


def _cfg_from(cls, args, section):
    cfg = C.apply_env(cls(), section)
    for f in C.fields(cfg):
        if hasattr(args, f.name):
            setattr(cfg, f.name, getattr(args, f.name))
    return cfg


def cmd_train(args) -> int:
    from .train.trainer import train_model
    from .utils.launch import init_distributed, rank_tagged_errors, shutdown_distributed
    init_distributed()
    try:
        with rank_tagged_errors():
            res = train_model(_cfg_from(C.TrainConfig, args, "train"), resume=args.resume)
        if "run_id" in res:  # rank 0 (the only writer)
            print(json.dumps({k: v for k, v in res.items() if k in ("run_id", "registered_version", "best_val_loss")}))
    finally:
        shutdown_distributed()
    return 0


def cmd_serve(args) -> int:
    from .serve.server import serve
    out = serve(_cfg_from(C.ServeConfig, args, "serve"), block=True)
    return 0 if out is not None else 1


def cmd_client(args) -> int:
    from .camera import Camera
    from .serve.client import run_client
    cfg = _cfg_from(C.ClientConfig, args, "client")
    cam = Camera(backend=args.camera)
    if not cam.start():
        return 1
    try:
        recs = run_client(cfg, cam=cam, max_frames=args.max_frames, save_dir=args.save_dir)
    finally:
        cam.stop()
    for r in recs[-5:]:
        logging.info("mean %.4f max %.4f (smoothed %.4f / %.4f) coverage %.2f%% proc %.2f ms rtt %.2f ms",
                     r["mean_curvature"], r["max_curvature"], r["smoothed_mean"], r["smoothed_max"],
                     r["mask_coverage"], r["proc_time_ms"], r["rtt_ms"])
    return 0 if recs else 1


def cmd_calibrate(args) -> int:
    from .calibration.tool import run_calibration
    cfg = _cfg_from(C.CalibrationConfig, args, "calibration")
    res = run_calibration(cfg, image_glob=args.images, n_captures=args.captures)
    print(f"mean reprojection error: {res['mean_error']:.4f} px (rms {res['rms']:.4f}, {res['n_views']} views)")
    print(f"camera matrix:\n{res['mtx']}\ndistortion: {res['dist'].ravel()}\nsaved: {res['path']}")
    return 0


def cmd_collect(args) -> int:
    from .camera import Camera
    from .data.collect import collect_raw_data, label_capture
    cfg = _cfg_from(C.CollectConfig, args, "collect")
    cam = Camera(backend=args.camera)
    if not cam.start():
        return 1
    try:
        out, n = collect_raw_data(cam, cfg, n_frames=args.frames, duration_s=args.duration)
    finally:
        cam.stop()
    print(f"saved {n} frame pairs to {out}")
    if args.label:
        m = label_capture(out, args.label, cam.depth_scale or 0.001)
        print(f"labelled {m} pairs into {args.label}")
    return 0


def cmd_drift(args) -> int:
    from .monitoring.drift import analyze_drift
    cfg = _cfg_from(C.DriftConfig, args, "drift")
    res = analyze_drift(cfg.log_file, cfg)
    print(json.dumps({k: v for k, v in res.items() if not hasattr(v, "shape")}, default=str))
    return 0


def cmd_retrain(args) -> int:
    from .utils.launch import init_distributed, shutdown_distributed
    from .workflows.retrain import run_retraining_pipeline
    init_distributed()
    try:
        res = run_retraining_pipeline(_cfg_from(C.TrainConfig, args, "train"), alias=args.alias,
                                      only_if_drift=args.only_if_drift)
        print(json.dumps(res, default=str))
    finally:
        shutdown_distributed()
    return 0


def cmd_bench_serve(args) -> int:
    import torch
    from .serve.bench_serve import measure_serving
    print(json.dumps(measure_serving(torch.device("cuda"), args.frames, args.warmup, args.train_steps)))
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="rdp", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("train")
    _section(p, C.TrainConfig, "train")
    p.add_argument("--resume", default=None, help="checkpoint path or 'auto'")
    p.set_defaults(fn=cmd_train)
    p = sub.add_parser("serve")
    _section(p, C.ServeConfig, "serve")
    p.set_defaults(fn=cmd_serve)
    p = sub.add_parser("client")
    _section(p, C.ClientConfig, "client")
    p.add_argument("--camera", default="auto")
    p.add_argument("--max-frames", type=int, default=None)
    p.add_argument("--save-dir", default=None)
    p.set_defaults(fn=cmd_client)
    p = sub.add_parser("calibrate")
    _section(p, C.CalibrationConfig, "calibration")
    p.add_argument("--images", default=None, help="glob of checkerboard images (else capture from the camera)")
    p.add_argument("--captures", type=int, default=10)
    p.set_defaults(fn=cmd_calibrate)
    p = sub.add_parser("collect")
    _section(p, C.CollectConfig, "collect")
    p.add_argument("--camera", default="auto")
    p.add_argument("--frames", type=int, default=None)
    p.add_argument("--duration", type=float, default=None)
    p.add_argument("--label", default=None, help="write images/ + masks/ (auto-labelled) into this directory")
    p.set_defaults(fn=cmd_collect)
    p = sub.add_parser("drift")
    _section(p, C.DriftConfig, "drift")
    p.set_defaults(fn=cmd_drift)
    p = sub.add_parser("retrain")
    _section(p, C.TrainConfig, "train")
    p.add_argument("--alias", default=C.PROMOTION_ALIAS)
    p.add_argument("--only-if-drift", action="store_true")
    p.set_defaults(fn=cmd_retrain)
    p = sub.add_parser("bench-serve")
    p.add_argument("--frames", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--train-steps", type=int, default=200)
    p.set_defaults(fn=cmd_bench_serve)
    return ap


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format=LOG_FORMAT)
    args = build_parser().parse_args(argv)
    return int(args.fn(args) or 0)


if __name__ == "__main__":
    sys.exit(main())
