"""Retraining workflow: train -> register -> set the ``staging`` alias (-> optional hot reload).

Mirrors ``/root/reference/workflows/retraining_pipeline.py:42-79``: run ``train_model()`` in
process, find the newest version in stage "None" with ``get_latest_versions``, then
``set_registered_model_alias(name, "staging", version)``. Exceptions are logged (and returned),
not raised, like the reference. Additions: an optional drift gate (only retrain when the drift
detector fires) and a ``promote`` callback used to notify a running server (hot reload).

Under torchrun every rank calls this (``train_model`` is collective), but only rank 0 evaluates the
drift gate (its decision is broadcast so all ranks agree on whether to train) and touches the
registry alias; the other ranks return after training.
"""
from __future__ import annotations

import logging
from typing import Callable, Optional

from .. import mlstore
from ..config import PROMOTION_ALIAS, TrainConfig
from ..train.trainer import train_model

log = logging.getLogger("rdp.workflow")


def run_retraining_pipeline(cfg: Optional[TrainConfig] = None, alias: str = PROMOTION_ALIAS,
                            only_if_drift: Optional[str] = None,
                            on_promote: Optional[Callable[[str, str], None]] = None) -> dict:
    cfg = cfg or TrainConfig()
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    log.info("Starting automated retraining pipeline...")
    out = {"promoted": False}
    from ..parallel.ddp import dist_info
    rank, world = dist_info()
    try:
        if only_if_drift:
            rep = None
            if rank == 0:
                from ..monitoring.drift import analyze_drift
                rep = analyze_drift(only_if_drift, make_plot=False)
            if world > 1:
                import torch.distributed as dist
                box = [rep]
                dist.broadcast_object_list(box, src=0)
                rep = box[0]
            out["drift"] = rep
            if not rep.get("drift_detected"):
                log.info("No drift detected: skipping retraining.")
                return out
        res = train_model(cfg)
        out["train"] = res
        if rank != 0:  # registry writes are rank 0's (train_model already registered there)
            return out
        uri = cfg.mlruns_dir
        client = mlstore.MlflowClient(uri if "://" in uri else __import__("os").path.abspath(uri))
        latest = client.get_latest_versions(cfg.registered_model_name, stages=["None"])
        if not latest:
            log.error("No new model version found after training. Aborting.")
            return out
        v = latest[0].version
        log.info("Promoting version %s by setting '%s' alias...", v, alias)
        client.set_registered_model_alias(cfg.registered_model_name, alias, v)
        out.update(promoted=True, version=v, alias=alias)
        if on_promote:
            on_promote(cfg.registered_model_name, v)
        log.info("Retraining pipeline finished successfully.")
    except Exception as e:  # reference: log, don't raise (retraining_pipeline.py:78-79)
        log.error("An error occurred during the retraining pipeline: %s", e, exc_info=True)
        out["error"] = repr(e)
    return out
