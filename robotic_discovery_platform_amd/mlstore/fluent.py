"""Fluent tracking API mirroring the ``mlflow.*`` calls of the reference trainer.

``set_tracking_uri`` / ``set_experiment`` / ``start_run`` / ``log_params`` / ``log_metric`` /
``end_run`` (``/root/reference/scripts/train_segmenter.py:112-128,183-191``).
"""
from __future__ import annotations

import contextlib
import os
import threading
from typing import Any, Dict, Optional

from .store import FileStore, Run

_state = threading.local()
_global = {"uri": os.environ.get("MLFLOW_TRACKING_URI", "file://" + os.path.abspath("mlruns")),
           "experiment_id": None, "active": []}


def set_tracking_uri(uri: str) -> None:
    _global["uri"] = str(uri)
    _global["experiment_id"] = None


def get_tracking_uri() -> str:
    return _global["uri"]


def _store() -> FileStore:
    return FileStore(_global["uri"])


def set_experiment(name: str) -> str:
    exp_id = _store().create_experiment(name)
    _global["experiment_id"] = exp_id
    return exp_id


class ActiveRun(contextlib.AbstractContextManager):
    def __init__(self, run: Run):
        self._run = run
        self.info = run.info
        self.data = run.data

    def __exit__(self, exc_type, exc, tb):
        end_run("FAILED" if exc_type else "FINISHED")
        return False


def start_run(run_name: Optional[str] = None, tags: Optional[Dict[str, Any]] = None) -> ActiveRun:
    st = _store()
    exp_id = _global["experiment_id"] or "0"
    info = st.create_run(exp_id, run_name, tags)
    _global["active"].append(info.run_id)
    return ActiveRun(st.get_run(info.run_id))


def active_run_id() -> Optional[str]:
    return _global["active"][-1] if _global["active"] else None


def end_run(status: str = "FINISHED") -> None:
    if _global["active"]:
        rid = _global["active"].pop()
        _store().end_run(rid, status)


def _rid() -> str:
    rid = active_run_id()
    if rid is None:
        raise RuntimeError("no active run; call start_run() first")
    return rid


def log_param(key: str, value: Any) -> None:
    _store().log_param(_rid(), key, value)


def log_params(params: Dict[str, Any]) -> None:
    st, rid = _store(), _rid()
    for k, v in params.items():
        st.log_param(rid, k, v)


def log_metric(key: str, value: float, step: Optional[int] = None) -> None:
    _store().log_metric(_rid(), key, value, step or 0)


def log_metrics(metrics: Dict[str, float], step: Optional[int] = None) -> None:
    for k, v in metrics.items():
        log_metric(k, v, step)


def set_tag(key: str, value: Any) -> None:
    _store().set_tag(_rid(), key, value)


def log_artifact(local_path: str, artifact_path: Optional[str] = None) -> None:
    _store().log_artifact(_rid(), local_path, artifact_path)
