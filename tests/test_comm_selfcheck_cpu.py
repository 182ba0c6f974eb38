"""bench.py's collective self-check (parallel/selfcheck.py) on a 2-rank gloo job (CPU).

The native RCCL path cannot run here, so fakes with the NativePath interface stand in for it: a
healthy one (the probe passes, ``ddp_comm == "native"``), one whose reduction is wrong (every rank falls
back to torch.distributed issue together, ``RDP_DDP_COMM`` becomes ``torch`` and the JSON field says
why), one that raises, and one whose communicator spans the wrong number of ranks (fatal). The last test
runs ``bench.py --gpus 2`` end to end and checks the self-check and per-rank fields of its JSON line.
Reference step per rank: ``/root/reference/scripts/train_segmenter.py:156-165``."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, kind, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    os.environ.pop("RDP_DDP_COMM", None)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from robotic_discovery_platform_amd.parallel.selfcheck import CommMismatch, comm_selfcheck

        class Fake:
            aborted = 0

            def info(self):
                return (world + 1 if kind == "mismatch" else world), rank, rank

            def all_reduce(self, t):
                if kind == "raises":
                    raise TimeoutError("probe all-reduce incomplete after 120 s")
                dist.all_reduce(t)
                if kind == "wrong" and rank == 1:  # one rank sees a broken sum: both must fall back
                    t += 1

            def poll(self):
                return 0, ""

            def abort(self):
                Fake.aborted += 1

        fake = Fake()
        try:
            res = comm_selfcheck(torch.device("cpu"), True, native_path=lambda: fake)
            res["env_comm"] = os.environ.get("RDP_DDP_COMM")
            res["aborted"] = Fake.aborted
        except CommMismatch as e:
            res = {"mismatch": str(e)}
        with open(f"{out}.{rank}", "w") as f:
            json.dump(res, f)
    finally:
        dist.destroy_process_group()


def _run(kind, tmp_path):
    out = str(tmp_path / "res")
    mp.spawn(_entry, args=(2, _free_port(), kind, out), nprocs=2, join=True)
    return [json.load(open(f"{out}.{r}")) for r in range(2)]


def test_native_probe_passes(tmp_path):
    res = _run("ok", tmp_path)
    for r in res:
        assert r["ddp_comm"] == "native" and r["comm_probe"] == "ok" and r["rccl_ranks"] == 2
        assert r["env_comm"] is None and r["aborted"] == 0
        assert r["allreduce_busbw_gbps"] > 0 and r["allreduce_16mb_us"] > 0


@pytest.mark.parametrize("kind", ["wrong", "raises"])
def test_failed_native_probe_falls_back_on_every_rank(kind, tmp_path):
    res = _run(kind, tmp_path)
    for r in res:
        assert r["ddp_comm"].startswith("torch (native probe failed: "), r
        # a hung probe aborts the communicator; one that returned wrong sums leaves it alone
        assert r["env_comm"] == "torch" and r["aborted"] == (1 if kind == "raises" else 0)
        assert r["comm_probe"] == "ok (torch.distributed)"
    if kind == "raises":
        assert "incomplete after" in res[0]["ddp_comm"]
    else:  # rank 0's own probe passed; it still falls back because rank 1's failed
        assert "elements wrong" in res[1]["ddp_comm"]


def test_rank_count_mismatch_is_fatal(tmp_path):
    res = _run("mismatch", tmp_path)
    for r in res:
        assert "RCCL gradient communicator has 3 ranks" in r["mismatch"]


def test_bench_json_reports_selfcheck_and_rank_spread():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["RDP_NO_BUILD"] = "1"
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--impl", "eager", "--steps", "2", "--warmup", "1",
           "--batch", "1", "--size", "32"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert d["dist_backend"] == "gloo" and d["world_size"] == 2 and d["ddp_comm"] == "torch"
    assert d["comm_probe"].startswith("ok") and d["allreduce_busbw_gbps"] > 0
    assert d["rank_ms_per_step_min"] <= d["rank_ms_per_step_max"] <= d["ms_per_step"] * 1.001
