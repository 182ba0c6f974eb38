"""Data-parallel path on a fake 2-rank cluster (gloo, CPU processes).

Checks the pieces the RCCL path uses unchanged: FlatBucketer's bucket layout and all-reduce,
parameter broadcast, DDP gradient equivalence (2 ranks x bs b == 1 process averaging the two
shard gradients, per-replica BatchNorm like the native path), and rank-0-only store writes in
train_model.
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


def _run(fn, world, *args):
    port = _free_port()
    mp.spawn(_entry, args=(world, port, fn, args), nprocs=world, join=True)


def _entry(rank, world, port, fn, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- bucketer
def _bucketer_worker(rank, world, out):
    from robotic_discovery_platform_amd.parallel.ddp import FlatBucketer
    sizes = [5, 300, 17, 1024, 64, 3, 700]
    ranges, off = [], 0
    for i, n in enumerate(sizes):
        ranges.append((f"p{i}", off, off + n))
        off += n + (3 if i % 2 else 0)  # alignment gaps like the native ParamStore
    g = torch.arange(off, dtype=torch.float32) * (rank + 1)
    b = FlatBucketer(g, ranges, bucket_mb=1200 * 4 / 2 ** 20)
    # buckets: contiguous, reverse order, cover [0, numel)
    spans = sorted(b.buckets)
    assert spans[0][0] == 0 and spans[-1][1] == off
    assert all(spans[i][1] == spans[i + 1][0] for i in range(len(spans) - 1))
    assert b.buckets[0][1] == off  # first bucket launched holds the last parameters
    for _ in range(2):  # reuse across steps
        g.copy_(torch.arange(off, dtype=torch.float32) * (rank + 1))
        b.reset()
        for n, _, _ in reversed(ranges[2:]):
            b.mark_ready([n])
        b.finish()  # p0, p1 never marked -> flushed here
        exp = torch.arange(off, dtype=torch.float32) * sum(r + 1 for r in range(world))
        assert torch.equal(g, exp)
    if rank == 0:
        json.dump({"nbuckets": len(b.buckets)}, open(out, "w"))


def test_flat_bucketer_allreduce(tmp_path):
    out = str(tmp_path / "r.json")
    _run(_bucketer_worker, 2, out)
    assert json.load(open(out))["nbuckets"] > 1


def _replay_worker(rank, world, comm, out):
    """The launch-plan protocol of NativeTrainer (train/engine.py): the recorded step keeps every bucket
    launch (and finish) as host call points; a replay resets the bucketer and re-runs those calls
    WITHOUT mark_ready. Each bucket must still be reduced exactly once per step."""
    from robotic_discovery_platform_amd.parallel.ddp import FlatBucketer
    sizes = [5, 300, 17, 1024, 64, 3, 700]
    ranges, off = [], 0
    for i, n in enumerate(sizes):
        ranges.append((f"p{i}", off, off + n))
        off += n
    g = torch.zeros(off)
    b = FlatBucketer(g, ranges, bucket_mb=1200 * 4 / 2 ** 20,
                     comm_dtype=torch.bfloat16 if comm == "bf16" else None)
    recorded = []
    b.host_call = lambda fn: (recorded.append(fn), fn())
    calls = []
    for step in range(4):
        g.copy_(torch.arange(off, dtype=torch.float32) % 7 * (rank + 1))
        b.reset()
        if step == 0:  # recording
            for n, _, _ in reversed(ranges):
                b.mark_ready([n])
            b.host_call(b.finish)
        else:  # replay: the recorded host calls, in order
            for fn in list(recorded):
                fn()
        exp = torch.arange(off, dtype=torch.float32) % 7 * sum(r + 1 for r in range(world))
        calls.append(bool(torch.equal(g, exp)))
    if rank == 0:
        json.dump({"ok": calls}, open(out, "w"))


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_flat_bucketer_plan_replay_reduces_once(tmp_path, comm):
    out = str(tmp_path / "r.json")
    _run(_replay_worker, 2, comm, out)
    assert json.load(open(out))["ok"] == [True] * 4


def _bucketer_bf16_worker(rank, world, out):
    """bf16 comm mirror: buckets are narrowed to bf16, summed over the ranks, widened back."""
    from robotic_discovery_platform_amd.parallel.ddp import FlatBucketer
    sizes = [5, 300, 17, 1024, 64, 3, 700]
    ranges, off = [], 0
    for i, n in enumerate(sizes):
        ranges.append((f"p{i}", off, off + n))
        off += n
    gen = torch.Generator().manual_seed(rank)
    src = torch.randn(off, generator=gen)
    g = src.clone()
    b = FlatBucketer(g, ranges, bucket_mb=1200 * 2 / 2 ** 20, comm_dtype=torch.bfloat16)
    assert b.comm is not None and b.comm.dtype == torch.bfloat16
    b.reset()
    for n, _, _ in reversed(ranges):
        b.mark_ready([n])
    b.finish()
    assert g.dtype == torch.float32
    allsrc = [torch.zeros_like(src) for _ in range(world)]
    dist.all_gather(allsrc, src)
    exact = sum(allsrc)
    # each rank's share is rounded to bf16 once, the sum once more (2 ranks)
    mag = sum(a.abs() for a in allsrc)
    assert ((g - exact).abs() <= 2 ** -7 * mag + 1e-6).all(), (g - exact).abs().max()
    assert torch.equal(g, sum(a.bfloat16().float() for a in allsrc).bfloat16().float())
    if rank == 0:
        json.dump({"nbuckets": len(b.buckets)}, open(out, "w"))


def test_flat_bucketer_bf16_comm(tmp_path):
    out = str(tmp_path / "r.json")
    _run(_bucketer_bf16_worker, 2, out)
    assert json.load(open(out))["nbuckets"] > 1


# ----------------------------------------------------------------------------- SyncBN row fold
def _syncbn_rows_worker(rank, world):
    """UNetExecutor._sync_rows: T partial [2][C] rows per rank -> row 0 = sum over rows and ranks;
    set_sync_bn gathers the ranks' (N, H, W) once, so unequal per-rank batches get exact counts."""
    from types import SimpleNamespace
    from robotic_discovery_platform_amd.models.unet import UNetExecutor
    C, T = 8, 5
    # set_sync_bn: rank r runs batch r + 1 (unequal), 8x8 input, two levels
    ex = SimpleNamespace(m=SimpleNamespace(), N=rank + 1, H=8, W=8, sizes=[(8, 8), (4, 4)], dev="cpu",
                         layers=[SimpleNamespace(spec=SimpleNamespace(cout=C))])
    UNetExecutor.set_sync_bn(ex)
    assert ex.sync_world == world and ex.sync_group is not None
    nsum = sum(r + 1 for r in range(world))
    assert ex._sync_m == {(8, 8): 64 * nsum, (4, 4): 16 * nsum}
    grp = ex.sync_group
    UNetExecutor.set_sync_bn(ex)  # the dedicated group is created once per model
    assert ex.sync_group is grp
    buf = torch.zeros(64 * 2 * C)
    rows = torch.arange(T * 2 * C, dtype=torch.float32).view(T, 2 * C) * (rank + 1)
    buf[: T * 2 * C] = rows.reshape(-1)
    # the global fp64 sums come back as two rows, hi + lo (the finalize kernels add them in fp64)
    assert UNetExecutor._sync_rows(ex, buf, T, C, (4, 4)) == (2, 16 * nsum)
    exp = rows.double().sum(0) / (rank + 1) * nsum
    got = buf[: 2 * C].double() + buf[2 * C: 4 * C].double()
    assert torch.equal(got, exp)
    UNetExecutor.set_sync_bn(ex, enabled=False)
    assert ex.sync_world == 1 and ex.sync_group is None


def test_syncbn_row_fold_allreduce():
    _run(_syncbn_rows_worker, 3)


# ----------------------------------------------------------------------------- gradient equivalence
def _make(seed):
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(seed)
    return UNetRef(3, 1, True, base_width=8, depth=2)


def _data():
    g = torch.Generator().manual_seed(7)
    x = torch.rand(4, 3, 32, 32, generator=g)
    y = (torch.rand(4, 1, 32, 32, generator=g) > 0.5).float()
    return x, y


def _ddp_worker(rank, world, out):
    from robotic_discovery_platform_amd.train.engine import EagerTrainer
    model = _make(seed=100 + rank)  # different init per rank: broadcast must fix it
    tr = EagerTrainer(model, lr=1e-3, bucket_mb=0.01)
    x, y = _data()
    sl = slice(rank * 2, rank * 2 + 2)
    tr.step(x[sl], y[sl])
    grad = tr.flat_grad.clone()  # all-reduced mean gradient of the step
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    gathered = [torch.zeros_like(flat) for _ in range(world)]
    dist.all_gather(gathered, flat)
    assert torch.equal(gathered[0], gathered[1])
    if rank == 0:
        torch.save({"p": flat, "g": grad}, out)


def test_ddp_matches_single_process_shard_average(tmp_path):
    out = str(tmp_path / "p.pt")
    _run(_ddp_worker, 2, out)
    got = torch.load(out, weights_only=True)
    # single process: same init as rank 0, gradient = mean of the two shard gradients
    model = _make(seed=100)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    x, y = _data()
    opt.zero_grad()
    for r in range(2):
        sl = slice(r * 2, r * 2 + 2)
        loss = torch.nn.functional.binary_cross_entropy_with_logits(model(x[sl]), y[sl]) / 2
        loss.backward()
    g = torch.cat([p.grad.reshape(-1) for p in model.parameters()])
    opt.step()
    exp = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    assert torch.allclose(got["g"], g, rtol=1e-4, atol=1e-7), (got["g"] - g).abs().max()
    # Adam's first step is ~lr*sign(g): only elements with |g| ~ 0 may differ
    assert (got["p"] - exp).abs().max() < 2.1e-3 and ((got["p"] - exp).abs() > 1e-6).float().mean() < 1e-3


# ----------------------------------------------------------------------------- rank-0 writes
def _train_worker(rank, world, root):
    from robotic_discovery_platform_amd.config import TrainConfig
    from robotic_discovery_platform_amd.train.trainer import train_model
    c = TrainConfig(epochs=1, batch_size=2, image_size=32, synthetic_samples=8, model_depth=2,
                    dataset_dir=os.path.join(root, "nodata"), mlruns_dir=os.path.join(root, "mlruns"),
                    model_output_dir=os.path.join(root, "models"), backend="eager", learning_rate=1e-3)
    res = train_model(c)
    json.dump({"rank": rank, "version": res.get("registered_version")}, open(os.path.join(root, f"r{rank}.json"), "w"))


@pytest.mark.slow
def test_train_model_two_ranks_rank0_writes(tmp_path):
    _run(_train_worker, 2, str(tmp_path))
    r0 = json.load(open(tmp_path / "r0.json"))
    assert r0["version"] == "1"
    from robotic_discovery_platform_amd import mlstore
    st = mlstore.FileStore(str(tmp_path / "mlruns"))
    assert len(st.search_model_versions("Actuator-Segmenter")) == 1  # only rank 0 registered
    exp = st.get_experiment_by_name("Actuator Segmentation")
    runs = st.search_runs(exp["experiment_id"])
    assert len(runs) == 1 and runs[0].data["params"]["world_size"] == "2"


# ----------------------------------------------------------------------------- bucket launch order
def _hook_sequence_launches(bilinear: bool, bucket_mb: float):
    """Drive a FlatBucketer over the native ParamStore layout of UNet(3, 1) with the executor's hook
    order (no process group: launches are recorded, not reduced). Returns (hooks, launches) where
    launches[k] = (bucket, number of hooks fired when it was issued)."""
    from robotic_discovery_platform_amd.models.unet import (ALIGN, UpTSpec, backward_hook_order,
                                                             unet_conv_specs)
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.parallel.ddp import FlatBucketer
    ref = UNetRef(3, 1, bilinear=bilinear)
    ranges, off = [], 0
    for n, p in ref.named_parameters():
        ranges.append((n, off, off + p.numel()))
        off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
    b = FlatBucketer(torch.zeros(off), ranges, bucket_mb)
    launches, hooks = [], []
    b._launch = lambda k, s=None: launches.append((k, len(hooks)))
    specs = unet_conv_specs(4, 64, 3, bilinear)
    ups = [] if bilinear else [UpTSpec(f"up{i}.up", 64 * 2 ** (5 - i), 64 * 2 ** (4 - i)) for i in range(1, 5)]
    b.reset()
    for sp in backward_hook_order(specs, ups, 4):
        hooks.append(sp.name)
        b.mark_ready(sp.param_names())
    assert sorted(n for ns in b.bucket_params for n in ns) == sorted(n for n, _, _ in ranges)
    return b, hooks, launches


@pytest.mark.parametrize("bilinear", [True, False])
def test_bucket_launch_order_follows_backward_hooks(bilinear):
    """Every bucket is issued at the hook that completes it, in backward order; the decoder bucket
    (head + up4 .. up1.conv.3) goes out before the first encoder hook -- not after backward, as when
    the head's gradients were marked ready only once backward had returned."""
    b, hooks, launches = _hook_sequence_launches(bilinear, 16.0)
    assert [k for k, _ in launches] == list(range(len(b.buckets)))  # all launched inside backward, in order
    assert hooks[0] == "outc"
    first_enc = next(i for i, h in enumerate(hooks) if h.startswith(("down", "inc")))
    assert launches[0][1] <= first_enc
    # each bucket launches at the FIRST hook after which all its params are final
    for k, n_fired in launches:
        names = set(b.bucket_params[k])
        done_at = max(i for i, h in enumerate(hooks) if any(p.startswith(h + ".") for p in names)) + 1
        assert n_fired == done_at, (k, n_fired, done_at)
    if bilinear:  # bucket 0 leaves before the 18 MB up1.conv.0 weight gradient exists
        assert launches[0][1] <= hooks.index("up1.conv.double_conv.0")


def test_bucket_big_param_starts_new_bucket():
    from robotic_discovery_platform_amd.parallel.ddp import FlatBucketer
    ranges = [("a", 0, 1000), ("b", 1000, 1100), ("c", 1100, 1200)]  # reverse order: c, b, a
    b = FlatBucketer(torch.zeros(1200), ranges, bucket_mb=400 * 4 / 2 ** 20)
    assert b.bucket_params == [["c", "b"], ["a"]]


# ----------------------------------------------------------------------------- stream ordering model
def _simulate_issue(bilinear: bool, ordered: bool):
    """The native executor's two-stream protocol on fake stream ids, checked by StreamOrderChecker:
    BN / head gradients on the main stream, each conv / ConvTranspose weight gradient on the side
    stream after a fork from main; buckets issued either on the side stream (forked from main unless side
    completed the bucket: ``UNetExecutor.comm_stream``) or, unordered, on the stream the hook runs on
    (main)."""
    from robotic_discovery_platform_amd.models.unet import (ALIGN, BNHook, ConvSpec, UpTSpec, backward_hook_order,
                                                             unet_conv_specs)
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.parallel.ddp import FlatBucketer, StreamOrderChecker
    MAIN, SIDE = 1, 2
    ref = UNetRef(3, 1, bilinear=bilinear)
    ranges, off = [], 0
    for n, p in ref.named_parameters():
        ranges.append((n, off, off + p.numel()))
        off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
    ck = StreamOrderChecker()
    b = FlatBucketer(torch.zeros(off), ranges, 16.0)
    b.checker = ck

    def launch(k, producer=None):
        if ordered:  # UNetExecutor.comm_stream: on side, forked from main unless side completed the bucket
            if producer != SIDE:
                ck.wait(SIDE, MAIN)
            ck.check_launch(b.bucket_params[k], SIDE)
        else:
            ck.check_launch(b.bucket_params[k], MAIN)
    b._launch = launch
    specs = unet_conv_specs(4, 64, 3, bilinear)
    ups = [] if bilinear else [UpTSpec(f"up{i}.up", 64 * 2 ** (5 - i), 64 * 2 ** (4 - i)) for i in range(1, 5)]
    b.reset()
    for sp in backward_hook_order(specs, ups, 4):
        if isinstance(sp, (ConvSpec, UpTSpec)):  # weight gradient forked onto the side stream
            ck.wait(SIDE, MAIN)
            b.mark_ready(sp.param_names(), SIDE)
        else:  # head, BN gamma / beta: main stream
            assert isinstance(sp, BNHook) or sp.name == "outc"
            b.mark_ready(sp.param_names(), MAIN)
    return ck, len(b.buckets)


@pytest.mark.parametrize("bilinear", [True, False])
def test_stream_order_checker_on_executor_protocol(bilinear):
    ck, nb = _simulate_issue(bilinear, ordered=True)
    assert ck.launches == nb and ck.violations == []
    ck, nb = _simulate_issue(bilinear, ordered=False)  # round-3 race: issued from main behind side wgrads
    assert ck.launches == nb and ck.violations


def test_stream_order_checker_clocks():
    from robotic_discovery_platform_amd.parallel.ddp import StreamOrderChecker
    ck = StreamOrderChecker()
    ck.produced(["w"], 2)           # produced on stream 2
    ck.check_launch(["w"], 1)       # stream 1 never waited on 2
    assert len(ck.violations) == 1
    ck.wait(3, 2)                   # 3 waits on 2, 1 waits on 3: transitively ordered
    ck.wait(1, 3)
    ck.check_launch(["w"], 1)
    assert len(ck.violations) == 1
    ck.produced(["w"], 2)           # re-produced later on 2: the old wait no longer covers it
    ck.check_launch(["w"], 1)
    assert len(ck.violations) == 2
