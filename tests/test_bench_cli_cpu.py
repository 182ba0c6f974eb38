"""bench.py's ``--gpus N`` contract without a launcher (CPU, gloo): a plain ``python bench.py --gpus 2``
must start two ranks itself and report ``n_gpus == 2`` / ``dp2``; a launcher whose WORLD_SIZE
disagrees with ``--gpus`` must fail loudly instead of measuring a different job. The eager
implementation is used so the test needs no GPU; the GPU variant of the same check is in
``tests/test_bench_dist_gpu.py``. Reference step per rank: ``scripts/train_segmenter.py:156-165``."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["RDP_NO_BUILD"] = "1"
    return env


def test_plain_bench_gpus2_launches_two_ranks():
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--impl", "eager", "--steps", "2", "--warmup", "1",
           "--batch", "1", "--size", "32"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 2
    assert d["steps"] == 2 and d["warmup"] == 1
    assert abs(d["value"] - 2 * 1000.0 / d["ms_per_step"]) / d["value"] < 0.02


def test_world_size_mismatch_fails():
    env = _env()
    env.update(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--impl", "eager"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=3" in r.stderr and not r.stdout.strip()
