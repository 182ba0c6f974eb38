"""MLflow-compatible tracking + registry file store (mlflow is not a dependency).

Usage mirrors the reference's ``mlflow`` calls::

    from robotic_discovery_platform_amd import mlstore as mlflow
    mlflow.set_tracking_uri(uri); mlflow.set_experiment("Actuator Segmentation")
    with mlflow.start_run() as run:
        mlflow.log_params({...}); mlflow.log_metric("train_loss", v, step=epoch)
        info = mlflow.pytorch.log_model(model, name="model", registered_model_name="Actuator-Segmenter")
    client = mlflow.MlflowClient(); client.set_registered_model_alias(name, "staging", v)
"""
from . import pytorch  # noqa: F401
from .fluent import (end_run, get_tracking_uri, log_artifact, log_metric, log_metrics, log_param, log_params,  # noqa: F401
                     set_experiment, set_tag, set_tracking_uri, start_run, active_run_id)
from .store import FileStore, MlflowClient, ModelInfo, ModelVersion, Run, RunInfo  # noqa: F401
