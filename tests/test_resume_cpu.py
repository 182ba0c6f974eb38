"""Kill-a-rank and relaunch: DDP training (2 gloo ranks) where rank 1 dies at the start of epoch 1
(``RDP_FAULT_CRASH``), then the job is relaunched with ``resume="auto"`` and must finish with exactly
the weights and losses of an uninterrupted run. The reference has no resume at all (best-only
checkpoint, /root/reference/scripts/train_segmenter.py:186-210); SURVEY.md §5 asks for a
torchrun-style relaunch from the last checkpoint.
"""
import json
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, root, tag, resume, crash):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if crash:
        os.environ["RDP_FAULT_CRASH"] = crash
    torch.set_num_threads(2)
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    try:
        from robotic_discovery_platform_amd.config import TrainConfig
        from robotic_discovery_platform_amd.train.trainer import train_model
        c = TrainConfig(epochs=3, batch_size=2, image_size=32, synthetic_samples=10, model_depth=2,
                        dataset_dir=os.path.join(root, "nodata"), mlruns_dir=os.path.join(root, f"mlruns_{tag}"),
                        model_output_dir=os.path.join(root, f"models_{tag.split('_')[0]}"), backend="eager",
                        learning_rate=1e-3)
        res = train_model(c, resume=resume)
        if rank == 0:
            json.dump({"history": res["history"]}, open(os.path.join(root, f"{tag}.json"), "w"))
    finally:
        dist.destroy_process_group()


def _run(root, tag, resume=None, crash=None):
    mp.spawn(_entry, args=(2, _free_port(), root, tag, resume, crash), nprocs=2, join=True)


def _registered_state(root, tag):
    from robotic_discovery_platform_amd.mlstore import pytorch as mlpt
    _, sd = mlpt.load_state("models:/Actuator-Segmenter/latest", os.path.join(root, f"mlruns_{tag}"))
    return sd


@pytest.mark.slow
def test_killed_rank_relaunch_resumes_to_identical_weights(tmp_path):
    root = str(tmp_path)
    _run(root, "clean")
    with pytest.raises(Exception):  # rank 1 dies at epoch 1 -> the job fails
        _run(root, "job_a", crash="1:1")
    assert os.path.exists(os.path.join(root, "models_job", "last_checkpoint.pt"))
    assert not os.path.exists(os.path.join(root, "job_a.json"))
    _run(root, "job_b", resume="auto")  # relaunch, same checkpoint dir
    clean = json.load(open(os.path.join(root, "clean.json")))["history"]
    resumed = json.load(open(os.path.join(root, "job_b.json")))["history"]
    assert [h["epoch"] for h in resumed] == [1, 2]  # epoch 0 came from the checkpoint
    for a, b in zip(clean[1:], resumed):
        assert a["train_loss"] == b["train_loss"] and a["val_loss"] == b["val_loss"]
    sa, sb = _registered_state(root, "clean"), _registered_state(root, "job_b")
    assert sa.keys() == sb.keys()
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
