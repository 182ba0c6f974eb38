"""PyTorch model flavor: ``log_model`` / ``load_model`` / ``load_state`` (weights-only, no pickling).

Reference: ``mlflow.pytorch.log_model(pytorch_model=model, name="model",
registered_model_name="Actuator-Segmenter")`` (``/root/reference/scripts/train_segmenter.py:200-204``)
and ``mlflow.pytorch.load_model("models:/Actuator-Segmenter/latest", map_location=device)``
(``services/vision_analysis/server.py:81``). The reference pickles the whole nn.Module; we store the
reference-keyed ``state_dict`` (110 keys for UNet(3,1)) + the architecture config, so loading
executes nothing from the file (``torch.load(weights_only=True)``).
"""
from __future__ import annotations

import json
import os
import tempfile
from pathlib import Path
from typing import Any, Dict, Optional, Tuple

import torch
import yaml

from . import fluent
from .store import FileStore, ModelInfo


def _arch_config(model) -> Dict[str, Any]:
    cfg = {"class": "UNet"}
    for k in ("n_channels", "n_classes", "bilinear", "base_width", "depth"):
        if hasattr(model, k):
            v = getattr(model, k)
            cfg[k] = bool(v) if isinstance(v, bool) else v
    return cfg


def save_model(model, path: str | os.PathLike, extra: Optional[dict] = None) -> Path:
    """Write an MLmodel directory: MLmodel, data/model.pth (state_dict), data/config.json."""
    path = Path(path)
    (path / "data").mkdir(parents=True, exist_ok=True)
    sd = {k: v.detach().to("cpu").contiguous() for k, v in model.state_dict().items()}
    torch.save(sd, path / "data" / "model.pth")
    cfg = _arch_config(model)
    if extra:
        cfg.update(extra)
    (path / "data" / "config.json").write_text(json.dumps(cfg, indent=1))
    (path / "MLmodel").write_text(yaml.safe_dump({
        "artifact_path": path.name,
        "flavors": {"pytorch": {"model_data": "data", "pytorch_version": str(torch.__version__), "format": "state_dict"},
                    "python_function": {"loader_module": "robotic_discovery_platform_amd.mlstore.pytorch",
                                        "data": "data"}},
        "model_size_bytes": int(sum(v.numel() * v.element_size() for v in sd.values())),
    }))
    (path / "requirements.txt").write_text(f"torch=={torch.__version__}\n")
    return path


def log_model(pytorch_model=None, name: str = "model", registered_model_name: Optional[str] = None,
              artifact_path: Optional[str] = None, **kw) -> ModelInfo:
    name = artifact_path or name
    st = FileStore(fluent.get_tracking_uri())
    rid = fluent._rid()
    dst = st.artifact_dir(rid) / name
    save_model(pytorch_model, dst)
    source = f"runs:/{rid}/{name}"
    version = None
    if registered_model_name:
        mv = st.create_model_version(registered_model_name, source, rid)
        version = mv.version
    return ModelInfo(artifact_path=name, model_uri=source, run_id=rid, registered_model_version=version)


def load_state(model_uri: str, tracking_uri: Optional[str] = None) -> Tuple[dict, Dict[str, torch.Tensor]]:
    """Resolve a model URI and return (architecture config, state_dict) without building a module."""
    st = FileStore(tracking_uri or fluent.get_tracking_uri())
    d = st.resolve(model_uri)
    cfg = json.loads((d / "data" / "config.json").read_text())
    sd = torch.load(d / "data" / "model.pth", map_location="cpu", weights_only=True)
    return cfg, sd


def build_model(cfg: dict, backend: str = "auto", device: Optional[torch.device] = None):
    """Instantiate the architecture: native HIP model on GPU, plain-torch model otherwise."""
    from ..models.unet_ref import UNetRef
    kw = dict(n_channels=cfg.get("n_channels", 3), n_classes=cfg.get("n_classes", 1),
              bilinear=cfg.get("bilinear", True), base_width=cfg.get("base_width", 64), depth=cfg.get("depth", 4))
    device = torch.device(device) if device is not None else (torch.device("cuda") if torch.cuda.is_available()
                                                              else torch.device("cpu"))
    use_native = backend == "native" or (backend == "auto" and device.type == "cuda")
    if use_native:
        from ..models.unet import UNetNative
        return UNetNative(device=device, **kw)
    return UNetRef(kw["n_channels"], kw["n_classes"], kw["bilinear"], kw["base_width"], kw["depth"]).to(device)


def load_model(model_uri: str, map_location=None, backend: str = "auto", tracking_uri: Optional[str] = None):
    """``mlflow.pytorch.load_model`` equivalent: returns an eval-mode model with the logged weights."""
    cfg, sd = load_state(model_uri, tracking_uri)
    model = build_model(cfg, backend, map_location)
    model.load_state_dict(sd)
    model.eval()
    return model
