"""End-to-end MLOps slice on the GPU: device-resident data build (INTER_AREA / nearest kernels) ->
``train_model`` on the native backend (both decoders) -> registry -> ``mlstore.pytorch.load_model``
-> ``FramePipeline.process``.

Reference flow: /root/reference/scripts/train_segmenter.py:103-210 (train + register) and
/root/reference/services/vision_analysis/server.py:74-99,113-152 (load latest + analyse a frame).
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(3))
def test_resize_area_kernel_matches_oracle(seed):
    from robotic_discovery_platform_amd.data.device_data import resize_area_gpu, resize_nearest_gpu
    from robotic_discovery_platform_amd.data.image_io import bgr2rgb, resize_area, resize_nearest
    from robotic_discovery_platform_amd.data.synthetic import make_scene
    sc = make_scene(seed)
    got = resize_area_gpu(torch.from_numpy(sc.color).cuda(), (256, 256), swap_rb=True).cpu().numpy()
    exp = resize_area(bgr2rgb(sc.color), (256, 256))
    assert np.array_equal(got, exp), np.abs(got.astype(int) - exp).max()
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (333, 517, 3), dtype=np.uint8)  # non-integer scale factors both ways
    got = resize_area_gpu(torch.from_numpy(img).cuda(), (200, 100)).cpu().numpy()
    exp = resize_area(img, (200, 100))
    assert np.abs(got.astype(int) - exp).max() <= 1 and (got == exp).mean() > 0.999
    m = resize_nearest_gpu(torch.from_numpy(sc.mask).cuda(), (256, 256)).cpu().numpy()
    assert np.array_equal(m, resize_nearest(sc.mask, (256, 256)))


def test_device_dataset_matches_host_items(tmp_path):
    from robotic_discovery_platform_amd.data.dataset import SegmentationDataset, preload
    from robotic_discovery_platform_amd.data.device_data import batch_to_float, build_device_dataset
    from robotic_discovery_platform_amd.data.synthetic import write_dataset
    write_dataset(str(tmp_path), 6, seed=3)
    ds = SegmentationDataset(str(tmp_path / "images"), str(tmp_path / "masks"))
    idx = [4, 0, 2]
    x, y = build_device_dataset(ds, idx, torch.device("cuda"))
    xf, yf = batch_to_float(x, y)
    hx, hy = preload(ds, idx)
    assert torch.equal(xf.cpu(), hx) and torch.equal(yf.cpu(), hy)


@pytest.mark.parametrize("bilinear", [True, False])
def test_train_register_load_serve_native(tmp_path, bilinear):
    from robotic_discovery_platform_amd import mlstore
    from robotic_discovery_platform_amd.config import TrainConfig
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene, write_dataset
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.serve.engine import FramePipeline
    from robotic_discovery_platform_amd.train.trainer import train_model
    root = str(tmp_path)
    write_dataset(os.path.join(root, "data"), 10, seed=0)  # on-disk PNG dataset, reference layout
    cfg = TrainConfig(epochs=2, batch_size=4, image_size=128, model_depth=4, bilinear=bilinear,
                      dataset_dir=os.path.join(root, "data"), mlruns_dir=os.path.join(root, "mlruns"),
                      model_output_dir=os.path.join(root, "models"), backend="native", learning_rate=1e-3)
    res = train_model(cfg)
    assert res["backend"] == "native" and res["registered_version"] == "1"
    h = res["history"]
    assert len(h) == 2 and all(np.isfinite(e["train_loss"]) and np.isfinite(e["val_loss"]) for e in h)
    assert h[-1]["train_imgs_per_s"] > 0
    # registered weights have the reference architecture's keys and shapes (the advisor's check)
    from robotic_discovery_platform_amd.mlstore import pytorch as mlpt
    arch, sd = mlpt.load_state("models:/Actuator-Segmenter/latest", os.path.join(root, "mlruns"))
    assert arch["bilinear"] == bilinear
    ref_sd = UNetRef(3, 1, bilinear=bilinear).state_dict()
    assert list(sd.keys()) == list(ref_sd.keys())
    assert all(sd[k].shape == ref_sd[k].shape for k in ref_sd)
    # server-side load (native backend) and one analysed frame
    model = mlpt.load_model("models:/Actuator-Segmenter/latest", map_location=torch.device("cuda"),
                            backend="native", tracking_uri=os.path.join(root, "mlruns"))
    assert isinstance(model, UNetNative) and model.bilinear == bilinear
    for k, v in model.state_dict().items():
        assert torch.equal(v.cpu(), sd[k].cpu()), k
    sc = make_scene(7)
    p = FramePipeline(model, DEFAULT_K, 0.001, graph=True)
    r = p.process(sc.color, sc.depth)
    assert r.mask.shape == (480, 640) and 0.0 <= r.coverage <= 100.0
    assert r.curvature.status in ("ok", "too_few_points", "too_few_edge_points", "fit_failed")
    mlstore.set_tracking_uri(os.path.join(root, "mlruns"))
