"""Local (non-registry) loading of the service dependencies.

Equivalent of ``/root/reference/services/vision_analysis/vision_utils.py:29-83``:
``load_vision_service_dependencies(model_path, calib_path) -> (model, mtx, dist)`` from a
``state_dict`` ``.pth`` file (loaded with ``weights_only=True``) and the calibration npz; any missing
piece logs an error and returns ``(None, None, None)``.
"""
from __future__ import annotations

import logging
import os
from typing import Optional

import numpy as np
import torch

log = logging.getLogger(__name__)


def _load_segmentation_model(model_path: str, device: Optional[torch.device] = None, backend: str = "auto"):
    from ..mlstore.pytorch import build_model
    if not os.path.exists(model_path):
        log.error("trained model file not found at '%s' (run the training script first)", model_path)
        return None
    try:
        sd = torch.load(model_path, map_location="cpu", weights_only=True)
        model = build_model({"n_channels": 3, "n_classes": 1}, backend, device)
        model.load_state_dict(sd)
        model.eval()
        return model
    except Exception as e:
        log.error("failed to load model: %s", e)
        return None


def _load_calibration_data(calib_path: str):
    if not os.path.exists(calib_path):
        log.error("camera calibration file not found at '%s' (run the calibration script first)", calib_path)
        return None, None
    with np.load(calib_path, allow_pickle=False) as data:
        return data["mtx"], data["dist"]


def load_vision_service_dependencies(model_path: str, calib_path: str, device: Optional[torch.device] = None,
                                     backend: str = "auto"):
    model = _load_segmentation_model(model_path, device, backend)
    mtx, dist = _load_calibration_data(calib_path)
    if model is None or mtx is None:
        log.error("could not load model or calibration data")
        return None, None, None
    return model, mtx, dist
