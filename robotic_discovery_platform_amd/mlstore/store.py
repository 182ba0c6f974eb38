"""MLflow-compatible local file store: experiments, runs, params, metrics, tags, artifacts, registry.

The reference logs through the MLflow fluent API against a ``file://<root>/ml/mlruns`` store
(``/root/reference/scripts/train_segmenter.py:112-128,183-206``), the server loads
``models:/Actuator-Segmenter/latest`` (``services/vision_analysis/server.py:80-82``) and the
retraining workflow promotes via ``MlflowClient.get_latest_versions`` +
``set_registered_model_alias("staging")`` (``workflows/retraining_pipeline.py:50-74``). mlflow is not
installed here, so this module implements that subset natively with the same on-disk layout
(SURVEY.md App. B):

    mlruns/<exp_id>/meta.yaml
    mlruns/<exp_id>/<run_id>/{meta.yaml, params/<k>, metrics/<k>, tags/<k>, artifacts/...}
    mlruns/models/<name>/meta.yaml
    mlruns/models/<name>/version-<n>/meta.yaml
    mlruns/models/<name>/aliases/<alias>          (contains the version number)

Metric files hold lines ``<timestamp_ms> <value> <step>``. Models are stored as a weights-only
state_dict (``data/model.pth``, loadable with ``torch.load(weights_only=True)``) plus the
architecture config (``data/config.json``) and an ``MLmodel`` descriptor -- never a pickled module.

All writes are atomic (write to temp + rename) and guarded by a process-wide lock; in DDP only
rank 0 should write (see ``train/trainer.py``).
"""
from __future__ import annotations

import contextlib
import json
import os
import random
import shutil
import threading
import time
import uuid
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional
from urllib.parse import urlparse
from urllib.request import url2pathname

import yaml

_LOCK = threading.RLock()
_ADJ = ["bold", "calm", "eager", "fierce", "gentle", "happy", "jolly", "keen", "lively", "merry", "nimble",
        "proud", "quick", "sharp", "shy", "swift", "tidy", "vast", "wise", "zesty"]
_NOUN = ["ant", "bat", "crab", "deer", "eel", "fox", "gnu", "hawk", "ibis", "jay", "koi", "lark", "mole",
         "newt", "owl", "puma", "quail", "ram", "seal", "toad"]


def _now_ms() -> int:
    return int(time.time() * 1000)


def _atomic_write(path: Path, text: str) -> None:
    path.parent.mkdir(parents=True, exist_ok=True)
    tmp = path.with_name(f".{path.name}.{uuid.uuid4().hex}.tmp")
    tmp.write_text(text)
    os.replace(tmp, path)


def _read_yaml(path: Path) -> dict:
    with open(path) as f:
        return yaml.safe_load(f) or {}


def uri_to_path(uri: str) -> Path:
    if uri.startswith("file:"):
        p = urlparse(uri)
        return Path(url2pathname(p.path))
    return Path(uri)


@dataclass
class RunInfo:
    run_id: str
    run_name: str
    experiment_id: str
    artifact_uri: str
    status: str = "RUNNING"
    start_time: int = 0
    end_time: Optional[int] = None

    @property
    def run_uuid(self) -> str:
        return self.run_id


@dataclass
class Run:
    info: RunInfo
    data: Dict[str, Any] = field(default_factory=dict)


@dataclass
class ModelVersion:
    name: str
    version: str
    source: str
    run_id: str
    current_stage: str = "None"
    status: str = "READY"
    creation_timestamp: int = 0
    aliases: List[str] = field(default_factory=list)


@dataclass
class ModelInfo:
    artifact_path: str
    model_uri: str
    run_id: str
    registered_model_version: Optional[str] = None


class FileStore:
    """Tracking + model-registry store rooted at ``root`` (an ``mlruns`` directory)."""

    def __init__(self, root: str | os.PathLike):
        self.root = uri_to_path(str(root))
        self.root.mkdir(parents=True, exist_ok=True)
        default = self.root / "0" / "meta.yaml"
        if not default.exists():
            self._write_experiment("0", "Default")

    # ------------------------------------------------------------------ experiments
    def _write_experiment(self, exp_id: str, name: str) -> None:
        now = _now_ms()
        _atomic_write(self.root / exp_id / "meta.yaml", yaml.safe_dump({
            "artifact_location": (self.root / exp_id).resolve().as_uri(), "creation_time": now,
            "experiment_id": exp_id, "last_update_time": now, "lifecycle_stage": "active", "name": name}))

    def list_experiments(self) -> List[dict]:
        out = []
        for d in sorted(self.root.iterdir()):
            if d.is_dir() and d.name.isdigit() and (d / "meta.yaml").exists():
                out.append(_read_yaml(d / "meta.yaml"))
        return out

    def get_experiment_by_name(self, name: str) -> Optional[dict]:
        for e in self.list_experiments():
            if e.get("name") == name and e.get("lifecycle_stage", "active") == "active":
                return e
        return None

    def create_experiment(self, name: str) -> str:
        with _LOCK:
            e = self.get_experiment_by_name(name)
            if e:
                return str(e["experiment_id"])
            ids = [int(x["experiment_id"]) for x in self.list_experiments()]
            exp_id = str(max(ids + [0]) + 1)
            self._write_experiment(exp_id, name)
            return exp_id

    # ------------------------------------------------------------------ runs
    def _run_dir(self, run_id: str) -> Path:
        for e in self.root.iterdir():
            if e.is_dir() and (e / run_id / "meta.yaml").exists():
                return e / run_id
        raise KeyError(f"run {run_id} not found")

    def create_run(self, exp_id: str, run_name: Optional[str] = None, tags: Optional[dict] = None) -> RunInfo:
        run_id = uuid.uuid4().hex
        run_name = run_name or f"{random.choice(_ADJ)}-{random.choice(_NOUN)}-{random.randint(100, 999)}"
        d = self.root / exp_id / run_id
        info = RunInfo(run_id, run_name, exp_id, (d / "artifacts").resolve().as_uri(), "RUNNING", _now_ms())
        (d / "artifacts").mkdir(parents=True, exist_ok=True)
        for sub in ("params", "metrics", "tags"):
            (d / sub).mkdir(exist_ok=True)
        self._write_run_meta(d, info)
        base_tags = {"mlflow.runName": run_name, "mlflow.user": os.environ.get("USER", "rdp"),
                     "mlflow.source.type": "LOCAL", "mlflow.source.name": os.path.basename(os.sys.argv[0] or "rdp")}
        base_tags.update(tags or {})
        for k, v in base_tags.items():
            self.set_tag(run_id, k, v)
        return info

    def _write_run_meta(self, d: Path, info: RunInfo) -> None:
        _atomic_write(d / "meta.yaml", yaml.safe_dump({
            "artifact_uri": info.artifact_uri, "end_time": info.end_time, "entry_point_name": "",
            "experiment_id": info.experiment_id, "lifecycle_stage": "active", "run_id": info.run_id,
            "run_name": info.run_name, "run_uuid": info.run_id, "source_name": "", "source_type": 4,
            "source_version": "", "start_time": info.start_time, "status": {"RUNNING": 1, "FINISHED": 3, "FAILED": 4}
            .get(info.status, 1), "tags": [], "user_id": os.environ.get("USER", "rdp")}))

    def get_run(self, run_id: str) -> Run:
        d = self._run_dir(run_id)
        m = _read_yaml(d / "meta.yaml")
        status = {1: "RUNNING", 3: "FINISHED", 4: "FAILED"}.get(m.get("status"), "RUNNING")
        info = RunInfo(m["run_id"], m.get("run_name", ""), str(m["experiment_id"]), m["artifact_uri"], status,
                       m.get("start_time", 0), m.get("end_time"))
        data = {"params": self.get_params(run_id), "metrics": {k: v[-1][1] for k, v in self.get_metrics(run_id).items()},
                "tags": {p.name: p.read_text() for p in (d / "tags").iterdir()} if (d / "tags").exists() else {}}
        return Run(info, data)

    def end_run(self, run_id: str, status: str = "FINISHED") -> None:
        d = self._run_dir(run_id)
        run = self.get_run(run_id)
        run.info.status, run.info.end_time = status, _now_ms()
        self._write_run_meta(d, run.info)

    def search_runs(self, exp_id: str) -> List[Run]:
        d = self.root / exp_id
        return [self.get_run(r.name) for r in sorted(d.iterdir()) if (r / "meta.yaml").exists()]

    def log_param(self, run_id: str, key: str, value: Any) -> None:
        p = self._run_dir(run_id) / "params" / key
        if p.exists() and p.read_text() != str(value):
            raise ValueError(f"param {key} already logged with a different value")
        _atomic_write(p, str(value))

    def get_params(self, run_id: str) -> Dict[str, str]:
        d = self._run_dir(run_id) / "params"
        return {p.name: p.read_text() for p in sorted(d.iterdir())} if d.exists() else {}

    def log_metric(self, run_id: str, key: str, value: float, step: int = 0, timestamp: Optional[int] = None) -> None:
        p = self._run_dir(run_id) / "metrics" / key
        p.parent.mkdir(parents=True, exist_ok=True)
        with _LOCK, open(p, "a") as f:
            f.write(f"{timestamp or _now_ms()} {float(value)} {int(step)}\n")

    def get_metrics(self, run_id: str) -> Dict[str, List[tuple]]:
        d = self._run_dir(run_id) / "metrics"
        out = {}
        if d.exists():
            for p in sorted(d.iterdir()):
                rows = []
                for line in p.read_text().splitlines():
                    ts, v, s = line.split()
                    rows.append((int(ts), float(v), int(s)))
                out[p.name] = rows
        return out

    def set_tag(self, run_id: str, key: str, value: Any) -> None:
        _atomic_write(self._run_dir(run_id) / "tags" / key, str(value))

    def artifact_dir(self, run_id: str) -> Path:
        return self._run_dir(run_id) / "artifacts"

    def log_artifact(self, run_id: str, local_path: str, artifact_path: Optional[str] = None) -> None:
        dst = self.artifact_dir(run_id) / (artifact_path or "")
        dst.mkdir(parents=True, exist_ok=True)
        src = Path(local_path)
        if src.is_dir():
            shutil.copytree(src, dst / src.name, dirs_exist_ok=True)
        else:
            shutil.copy2(src, dst / src.name)

    # ------------------------------------------------------------------ registry
    def _model_dir(self, name: str) -> Path:
        return self.root / "models" / name

    def create_registered_model(self, name: str) -> None:
        with _LOCK:
            d = self._model_dir(name)
            if (d / "meta.yaml").exists():
                return
            now = _now_ms()
            _atomic_write(d / "meta.yaml", yaml.safe_dump({"name": name, "creation_timestamp": now,
                                                           "last_updated_timestamp": now, "description": ""}))

    def create_model_version(self, name: str, source: str, run_id: str) -> ModelVersion:
        with _LOCK:
            self.create_registered_model(name)
            d = self._model_dir(name)
            versions = [int(p.name.split("-")[1]) for p in d.glob("version-*")]
            v = max(versions + [0]) + 1
            now = _now_ms()
            mv = ModelVersion(name, str(v), source, run_id, "None", "READY", now)
            _atomic_write(d / f"version-{v}" / "meta.yaml", yaml.safe_dump({
                "name": name, "version": v, "source": source, "run_id": run_id, "current_stage": "None",
                "status": "READY", "creation_timestamp": now, "last_updated_timestamp": now, "description": "",
                "user_id": os.environ.get("USER", "rdp")}))
            meta = _read_yaml(d / "meta.yaml")
            meta["last_updated_timestamp"] = now
            _atomic_write(d / "meta.yaml", yaml.safe_dump(meta))
            return mv

    def _aliases_of(self, name: str) -> Dict[str, str]:
        d = self._model_dir(name) / "aliases"
        return {p.name: p.read_text().strip() for p in d.iterdir()} if d.exists() else {}

    def get_model_version(self, name: str, version: str | int) -> ModelVersion:
        p = self._model_dir(name) / f"version-{int(version)}" / "meta.yaml"
        if not p.exists():
            raise KeyError(f"model version {name}/{version} not found")
        m = _read_yaml(p)
        aliases = [a for a, v in self._aliases_of(name).items() if v == str(m["version"])]
        return ModelVersion(m["name"], str(m["version"]), m["source"], m["run_id"], m.get("current_stage", "None"),
                            m.get("status", "READY"), m.get("creation_timestamp", 0), aliases)

    def search_model_versions(self, name: str) -> List[ModelVersion]:
        d = self._model_dir(name)
        vs = sorted(int(p.name.split("-")[1]) for p in d.glob("version-*"))
        return [self.get_model_version(name, v) for v in vs]

    def get_latest_versions(self, name: str, stages: Optional[Iterable[str]] = None) -> List[ModelVersion]:
        """Latest version per stage (MLflow semantics); ``stages=None`` => every stage."""
        vs = self.search_model_versions(name)
        latest: Dict[str, ModelVersion] = {}
        for v in vs:
            if stages is None or v.current_stage in stages:
                cur = latest.get(v.current_stage)
                if cur is None or int(v.version) > int(cur.version):
                    latest[v.current_stage] = v
        return list(latest.values())

    def set_registered_model_alias(self, name: str, alias: str, version: str | int) -> None:
        self.get_model_version(name, version)  # must exist
        _atomic_write(self._model_dir(name) / "aliases" / alias, str(int(version)))

    def delete_registered_model_alias(self, name: str, alias: str) -> None:
        p = self._model_dir(name) / "aliases" / alias
        if p.exists():
            p.unlink()

    def get_model_version_by_alias(self, name: str, alias: str) -> ModelVersion:
        al = self._aliases_of(name)
        if alias not in al:
            raise KeyError(f"alias {name}@{alias} not set")
        return self.get_model_version(name, al[alias])

    def transition_model_version_stage(self, name: str, version: str | int, stage: str) -> ModelVersion:
        p = self._model_dir(name) / f"version-{int(version)}" / "meta.yaml"
        m = _read_yaml(p)
        m["current_stage"] = stage
        m["last_updated_timestamp"] = _now_ms()
        _atomic_write(p, yaml.safe_dump(m))
        return self.get_model_version(name, version)

    # ------------------------------------------------------------------ URIs
    def resolve(self, uri: str) -> Path:
        """``models:/n/latest`` | ``models:/n/<v>`` | ``models:/n@alias`` | ``runs:/<id>/<path>`` | path."""
        if uri.startswith("models:/"):
            spec = uri[len("models:/"):]
            if "@" in spec:
                name, alias = spec.split("@", 1)
                mv = self.get_model_version_by_alias(name, alias)
            else:
                name, _, ver = spec.partition("/")
                if ver in ("", "latest"):
                    vs = self.search_model_versions(name)
                    if not vs:
                        raise KeyError(f"no versions of {name}")
                    mv = vs[-1]
                elif ver[0].isdigit():
                    mv = self.get_model_version(name, ver)
                else:  # stage name (Staging / Production / None)
                    vs = self.get_latest_versions(name, [ver])
                    if not vs:
                        raise KeyError(f"no {ver} version of {name}")
                    mv = vs[0]
            return self.resolve(mv.source)
        if uri.startswith("runs:/"):
            rid, _, path = uri[len("runs:/"):].partition("/")
            return self.artifact_dir(rid) / path
        return uri_to_path(uri)


class MlflowClient:
    """The subset of ``mlflow.MlflowClient`` the reference uses (retraining_pipeline.py:51,60,70)."""

    def __init__(self, tracking_uri: Optional[str] = None):
        from . import fluent
        self.store = FileStore(tracking_uri or fluent.get_tracking_uri())

    def __getattr__(self, item):
        return getattr(self.store, item)
