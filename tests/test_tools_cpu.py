"""Calibration, data collection, legacy loader and the CLI entry points (CPU)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from robotic_discovery_platform_amd.calibration import (calibrate_camera, corner_subpix, find_chessboard_corners,
                                                        object_points, project_points, random_board_pose,
                                                        render_board_view, rodrigues)
from robotic_discovery_platform_amd.config import CalibrationConfig, CollectConfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K_TRUE = np.array([[615.0, 0, 322.5], [0, 612.0, 238.0], [0, 0, 1]])
D_TRUE = np.array([0.06, -0.12, 0.0008, -0.0004, 0.0])


def test_rodrigues_roundtrip():
    rng = np.random.default_rng(0)
    for _ in range(20):
        v = rng.normal(size=3)
        v *= rng.uniform(0.01, 3.0) / np.linalg.norm(v)
        R = rodrigues(v)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-12) and np.isclose(np.linalg.det(R), 1)
        assert np.allclose(rodrigues(R), v, atol=1e-9)


def test_corner_detection_subpixel():
    rng = np.random.default_rng(1)
    r, t = random_board_pose(rng, K_TRUE, dist=D_TRUE)
    img = render_board_view(K_TRUE, D_TRUE, r, t, ss=2, seed=1)
    ok, c = find_chessboard_corners(img, (9, 7))
    assert ok and c.shape == (63, 1, 2) and c.dtype == np.float32
    c2 = corner_subpix(img, c, (11, 11), 30, 0.001).reshape(-1, 2)
    true = project_points(object_points(), r, t, K_TRUE, D_TRUE)
    err = np.linalg.norm(c2 - true, axis=1)
    if err.mean() > 5:  # the (9,7) board is 180-degree symmetric: accept the flipped labelling
        err = np.linalg.norm(c2[::-1] - true, axis=1)
    assert err.mean() < 0.15 and err.max() < 0.5


def test_no_board_found():
    img = np.full((480, 640), 120, np.uint8)
    ok, c = find_chessboard_corners(img, (9, 7))
    assert not ok and c is None


def test_zhang_recovers_intrinsics_from_exact_points():
    rng = np.random.default_rng(2)
    objs, imgs = [], []
    for _ in range(8):
        r, t = random_board_pose(rng, K_TRUE, dist=D_TRUE)
        objs.append(object_points())
        imgs.append(project_points(object_points(), r, t, K_TRUE, D_TRUE) + rng.normal(0, 0.05, (63, 2)))
    rms, K, d, rv, tv = calibrate_camera(objs, imgs, (640, 480))
    assert rms < 0.1
    assert np.allclose(K, K_TRUE, rtol=5e-3, atol=1.0)
    assert abs(d[0, 0] - D_TRUE[0]) < 0.02 and len(rv) == 8 and rv[0].shape == (3, 1)


def test_calibration_tool_end_to_end(tmp_path):
    from robotic_discovery_platform_amd.calibration.tool import SyntheticBoardCamera, calibrate_views
    from robotic_discovery_platform_amd.camera import load_calibration
    cam = SyntheticBoardCamera(K=K_TRUE, dist=D_TRUE, seed=3)
    cam._open()
    views = [cam._grab()[1] for _ in range(6)]
    res = calibrate_views(views, CalibrationConfig(min_captures=5))
    assert res["n_views"] == 6 and res["mean_error"] < 0.3
    assert abs(res["mtx"][0, 0] - 615) < 6 and abs(res["mtx"][0, 2] - 322.5) < 6


def test_collect_and_label(tmp_path):
    from robotic_discovery_platform_amd.camera import SyntheticCamera
    from robotic_discovery_platform_amd.data.collect import collect_raw_data, label_capture
    from robotic_discovery_platform_amd.data.dataset import SegmentationDataset
    cam = SyntheticCamera(n_scenes=3, realtime=False)
    assert cam.start()
    out, n = collect_raw_data(cam, CollectConfig(save_interval_s=0.0, raw_dir=str(tmp_path / "raw")), n_frames=3)
    cam.stop()
    assert n == 3 and os.path.basename(out).startswith("capture_")
    colors = sorted(os.listdir(os.path.join(out, "color")))
    depths = sorted(os.listdir(os.path.join(out, "depth")))
    assert len(colors) == 3 and colors[0].startswith("color_") and depths[0].endswith(".npy")
    d = np.load(os.path.join(out, "depth", depths[0]))
    assert d.dtype == np.uint16 and d.shape == (480, 640)
    m = label_capture(out, str(tmp_path / "processed"))
    assert m == 3
    ds = SegmentationDataset(str(tmp_path / "processed" / "images"), str(tmp_path / "processed" / "masks"), (64, 64))
    x, y = ds[0]
    assert x.shape == (3, 64, 64) and 0 < y.mean() < 0.5


def test_legacy_loader(tmp_path):
    from robotic_discovery_platform_amd.camera import write_calibration
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.serve.vision_utils import load_vision_service_dependencies
    torch.save(UNetRef(3, 1).state_dict(), tmp_path / "m.pth")
    write_calibration(str(tmp_path / "c.npz"), K_TRUE)
    model, mtx, dist = load_vision_service_dependencies(str(tmp_path / "m.pth"), str(tmp_path / "c.npz"),
                                                        torch.device("cpu"))
    assert model is not None and not model.training and np.array_equal(mtx, K_TRUE) and dist.shape == (1, 5)
    assert load_vision_service_dependencies(str(tmp_path / "nope.pth"), str(tmp_path / "c.npz")) == (None, None, None)


def _run(args, cwd, env_extra=None):
    env = dict(os.environ, PYTHONPATH=ROOT, **(env_extra or {}))
    return subprocess.run([sys.executable, *args], cwd=cwd, env=env, capture_output=True, text=True, timeout=600)


def test_cli_train_and_drift_via_reference_paths(tmp_path):
    r = _run([os.path.join(ROOT, "scripts", "train_segmenter.py"), "--epochs", "1", "--image-size", "32",
              "--synthetic-samples", "6", "--model-depth", "2", "--backend", "eager",
              "--mlruns-dir", str(tmp_path / "mlruns"), "--model-output-dir", str(tmp_path / "models"),
              "--dataset-dir", str(tmp_path / "none")], tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["registered_version"] == "1"
    # drift: < 50 rows -> insufficient data
    (tmp_path / "logs").mkdir()
    (tmp_path / "logs" / "vision_service_metrics.csv").write_text(
        "timestamp,mean_curvature,max_curvature,mask_coverage_percent\n" + "1.0,0.1,0.2,5.0\n" * 10)
    r = _run([os.path.join(ROOT, "scripts", "monitoring", "drift_detector.py")], tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["status"] == "insufficient_data"


def test_cli_help_all_commands():
    from robotic_discovery_platform_amd.cli import build_parser
    p = build_parser()
    for cmd in ("train", "serve", "client", "calibrate", "collect", "drift", "retrain", "bench-serve"):
        with pytest.raises(SystemExit) as e:
            p.parse_args([cmd, "--help"])
        assert e.value.code == 0
