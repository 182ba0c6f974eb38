"""MLflow-compatible file store: layout, params/metrics, registry versions, aliases, URI resolution."""
import json

import pytest
import torch
import yaml

from robotic_discovery_platform_amd import mlstore
from robotic_discovery_platform_amd.mlstore.store import FileStore
from robotic_discovery_platform_amd.models.unet_ref import UNetRef


@pytest.fixture()
def store_uri(tmp_path):
    uri = (tmp_path / "mlruns").as_uri()
    mlstore.set_tracking_uri(uri)
    return uri


def test_run_layout_params_metrics(store_uri, tmp_path):
    exp = mlstore.set_experiment("Actuator Segmentation")
    with mlstore.start_run() as run:
        mlstore.log_params({"learning_rate": 1e-4, "batch_size": 4, "architecture": "UNet"})
        for e in range(3):
            mlstore.log_metric("train_loss", 1.0 / (e + 1), step=e)
        mlstore.log_metric("best_val_loss", 0.25)
        rid = run.info.run_id
    root = tmp_path / "mlruns"
    meta = yaml.safe_load((root / exp / "meta.yaml").read_text())
    assert meta["name"] == "Actuator Segmentation" and meta["lifecycle_stage"] == "active"
    rdir = root / exp / rid
    assert (rdir / "params" / "learning_rate").read_text() == "0.0001"
    assert (rdir / "params" / "batch_size").read_text() == "4"
    lines = (rdir / "metrics" / "train_loss").read_text().splitlines()
    assert len(lines) == 3
    ts, v, step = lines[2].split()
    assert int(ts) > 0 and float(v) == pytest.approx(1 / 3) and step == "2"
    rmeta = yaml.safe_load((rdir / "meta.yaml").read_text())
    assert rmeta["run_id"] == rid and len(rid) == 32 and rmeta["status"] == 3  # FINISHED
    assert (rdir / "tags" / "mlflow.runName").read_text() == rmeta["run_name"]
    # same experiment name -> same id
    assert mlstore.set_experiment("Actuator Segmentation") == exp


def test_registry_versions_latest_alias(store_uri):
    mlstore.set_experiment("Actuator Segmentation")
    models = []
    for i in range(3):
        torch.manual_seed(i)
        m = UNetRef(3, 1, base_width=64, depth=2)
        with mlstore.start_run():
            info = mlstore.pytorch.log_model(m, name="model", registered_model_name="Actuator-Segmenter")
        assert info.registered_model_version == str(i + 1)
        models.append(m)
    client = mlstore.MlflowClient()
    latest = client.get_latest_versions("Actuator-Segmenter", stages=["None"])
    assert [v.version for v in latest] == ["3"]
    client.set_registered_model_alias("Actuator-Segmenter", "staging", "2")
    assert client.get_model_version_by_alias("Actuator-Segmenter", "staging").version == "2"
    # URI resolution: latest, explicit version, alias
    for uri, idx in [("models:/Actuator-Segmenter/latest", 2), ("models:/Actuator-Segmenter/1", 0),
                     ("models:/Actuator-Segmenter@staging", 1)]:
        cfg, sd = mlstore.pytorch.load_state(uri)
        assert cfg["depth"] == 2 and cfg["bilinear"] is True
        ref = models[idx].state_dict()
        assert list(sd) == list(ref)
        assert all(torch.equal(sd[k], ref[k]) for k in ref)
    loaded = mlstore.pytorch.load_model("models:/Actuator-Segmenter@staging", map_location="cpu")
    assert not loaded.training
    x = torch.rand(1, 3, 32, 32)
    models[1].eval()
    assert torch.allclose(loaded(x), models[1](x))
    with pytest.raises(KeyError):
        mlstore.pytorch.load_state("models:/Actuator-Segmenter@production")


def test_model_file_is_weights_only(store_uri, tmp_path):
    mlstore.set_experiment("x")
    with mlstore.start_run() as run:
        mlstore.pytorch.log_model(UNetRef(3, 1, depth=1), name="model")
        rid = run.info.run_id
    st = FileStore(store_uri)
    d = st.resolve(f"runs:/{rid}/model")
    sd = torch.load(d / "data" / "model.pth", weights_only=True)  # must not need pickle
    assert "inc.double_conv.0.weight" in sd
    mlm = yaml.safe_load((d / "MLmodel").read_text())
    assert mlm["flavors"]["pytorch"]["format"] == "state_dict"
    assert json.loads((d / "data" / "config.json").read_text())["depth"] == 1


def test_param_conflict_and_stage_transition(store_uri):
    mlstore.set_experiment("y")
    with mlstore.start_run():
        mlstore.log_param("a", 1)
        mlstore.log_param("a", 1)  # idempotent
        with pytest.raises(ValueError):
            mlstore.log_param("a", 2)
        mlstore.pytorch.log_model(UNetRef(3, 1, depth=1), registered_model_name="M")
    c = mlstore.MlflowClient()
    c.transition_model_version_stage("M", 1, "Production")
    assert c.get_latest_versions("M", ["Production"])[0].version == "1"
    assert c.get_latest_versions("M", ["None"]) == []
