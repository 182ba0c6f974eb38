"""bench.py's multi-rank contract, end to end: torch.distributed.run launches 2 ranks (sharing the one
GPU of the test box over gloo; the driver's real N-GPU runs use RCCL), rank 0 prints ONE JSON line
whose value aggregates both ranks. Also exercises --sync-bn through the launcher."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("sync_bn", [0, 1])
def test_bench_two_ranks_json_contract(sync_bn):
    env = dict(os.environ, RDP_DIST_BACKEND="gloo", RDP_NO_BUILD="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--batch", "2", "--size", "64", "--sync-bn", str(sync_bn)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "weak"
    assert d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    assert d["config"]["sync_bn"] is bool(sync_bn)
    assert d["value"] > 0 and abs(d["value"] - 4 * 1000.0 / d["ms_per_step"]) / d["value"] < 0.02
    # the collective self-check and per-rank spread (parallel/selfcheck.py)
    assert d["dist_backend"] == "gloo" and d["world_size"] == 2 and d["comm_probe"].startswith("ok")
    assert d["allreduce_busbw_gbps"] > 0 and d["rank_ms_per_step_min"] <= d["rank_ms_per_step_max"]


def test_plain_bench_gpus2_self_launches():
    """The driver's form ``python bench.py --gpus N`` (no launcher): bench.py starts the N ranks
    itself, from a parent that never touches the GPU (native implementation, gloo sharing one GPU)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RDP_DIST_BACKEND="gloo", RDP_NO_BUILD="1")
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "2",
           "--size", "64"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    assert d["config"]["impl"] == "native"


@pytest.mark.parametrize("fail", [0, 1])
def test_bench_ddp_force_world1_native_selfcheck(fail):
    """World 1 under nccl with the DDP path forced: the self-check runs the native ncclAllReduce probe
    (RCCL reports 1 rank) -- and with RDP_COMM_PROBE_FAIL=1 the run falls back to torch.distributed
    issue, says why in the JSON, still prints its line and exits 0."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RDP_NO_BUILD="1", RDP_COMM_PROBE_FAIL=str(fail))
    cmd = [sys.executable, "bench.py", "--ddp-force", "1", "--steps", "2", "--warmup", "1", "--batch", "2",
           "--size", "64", "--extras", "0", "--serve", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["dist_backend"] == "nccl" and d["rccl_ranks"] == 1 and d["world_size"] == 1
    if fail:
        assert d["ddp_comm"].startswith("torch (native probe failed: ") and d["config"]["ddp_stream"] is None
    else:
        assert d["ddp_comm"] == "native" and d["comm_probe"] == "ok" and d["config"]["ddp_stream"] == "side"
