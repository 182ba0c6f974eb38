"""Native DDP step (NativeTrainer + FlatBucketer hooks + gscale folded into Adam) with 2 ranks sharing
one GPU over gloo (RCCL refuses two ranks per device; the bucketing / hook / stream logic is
backend-agnostic: gloo's CUDA all-reduce, like RCCL, orders itself after the ISSUING stream only).

Per-shard gradients come from identical kernels on identical inputs, so the all-reduced buffer must
equal the sum of the two single-process shard gradients bit for bit.

Stream ordering (the round-3 race: buckets issued from the main stream while their conv weight
gradients were still queued on the wgrad side stream) is made deterministic by a stall: every weight
gradient kernel is preceded by a ``torch.cuda._sleep`` spin on its stream, so the side stream lags the
main stream by milliseconds per layer. The ordered step must still match bit for bit, and a negative
control that issues each bucket from the hook's current stream (no ``launch_ctx``) must NOT match --
proof that the stall exposes an unordered issue at this shape.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

STALL_CYCLES = 2_000_000  # per weight-gradient launch


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(3)
    x = torch.rand(4, 3, 64, 64, generator=g)
    t = (torch.rand(4, 1, 64, 64, generator=g) > 0.6).float()
    return x, t


def _ref(seed):
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(seed)
    return UNetRef(3, 1)


def _install_stall():
    """Spin before every weight-gradient kernel, on the stream it is issued on."""
    from robotic_discovery_platform_amd.ops import native
    C = native()
    for name in ("conv_wgrad", "wgrad_first_bn"):
        orig = getattr(C, name)

        def slow(*a, _orig=orig, **k):
            torch.cuda._sleep(STALL_CYCLES)
            return _orig(*a, **k)
        setattr(C, name, slow)


def _worker(rank, world, port, comm, stall, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from robotic_discovery_platform_amd.models.unet import UNetNative
        from robotic_discovery_platform_amd.train.engine import NativeTrainer
        dev = torch.device("cuda", 0)
        if stall:
            _install_stall()
        x, t = _data()
        sl = slice(2 * rank, 2 * rank + 2)
        res = {}
        for ordered in ([True, False] if stall else [True]):
            nat = UNetNative(3, 1, device=dev, init_from=_ref(10 + rank))  # broadcast must unify
            tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, graph=True, bucket_mb=4.0, grad_comm=comm)
            assert tr.bucketer is not None and len(tr.bucketer.buckets) > 1 and tr.graph is None
            assert tr.ex.side is not None
            if not ordered:  # negative control: issue from whatever stream the hook runs on
                tr.bucketer.launch_ctx = None
            tr.set_batch(x[sl].to(dev), t[sl].to(dev))
            tr.step()
            torch.cuda.synchronize()
            p = nat.store.flat.clone()
            ps = [torch.zeros_like(p) for _ in range(world)]
            dist.all_gather(ps, p)
            if ordered:
                assert torch.equal(ps[0], ps[1])
            res["ordered" if ordered else "unordered"] = {"grad": nat.store.grad.cpu(), "flat": p.cpu()}
        if rank == 0:
            torch.save(res, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("comm,stall", [("fp32", False), ("fp32", True), ("bf16", True)])
def test_native_ddp_two_ranks_one_gpu(tmp_path, comm, stall):
    from robotic_discovery_platform_amd.models.unet import NativeAdam, UNetNative
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), comm, stall, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    dev = torch.device("cuda")
    nat = UNetNative(3, 1, device=dev, init_from=_ref(10))
    ex = nat.executor(2, 64, 64, training=True)
    x, t = _data()
    shards = []
    for r in range(2):
        sl = slice(2 * r, 2 * r + 2)
        ex.set_input(x[sl].to(dev), t[sl].to(dev))
        ex.forward()
        ex.backward()
        shards.append(nat.store.grad.clone())
    if comm == "bf16":  # each rank narrows its bucket to bf16, the sum is rounded to bf16, then widened
        acc = (shards[0].to(torch.bfloat16) + shards[1].to(torch.bfloat16)).float()
    else:
        acc = shards[0] + shards[1]
    ok = got["ordered"]
    assert torch.equal(ok["grad"], acc.cpu()), f"max |diff| {float((ok['grad'] - acc.cpu()).abs().max()):.3g}"
    # Adam with gscale = 1/world on the summed gradient
    nat.store.grad.copy_(acc)
    NativeAdam(nat, lr=1e-3).step(gscale=0.5)
    torch.cuda.synchronize()
    assert torch.allclose(ok["flat"], nat.store.flat.cpu(), atol=1e-7, rtol=0)
    if stall:  # the stall makes an unordered issue visible: the control must have read partial gradients
        assert not torch.equal(got["unordered"]["grad"], acc.cpu())


PLAN_STEPS = 6


def _plan_worker(rank, world, port, comm, out):
    """Launch-plan mode (the default training path) with torch.distributed bucket issue: steps 3+ are
    plan replays whose bucket all-reduces are recorded host call points."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from robotic_discovery_platform_amd.models.unet import UNetNative
        from robotic_discovery_platform_amd.train.engine import NativeTrainer
        dev = torch.device("cuda", 0)
        x, t = _data()
        sl = slice(2 * rank, 2 * rank + 2)
        nat = UNetNative(3, 1, device=dev, init_from=_ref(10 + rank))
        tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, graph=False, plan=True, bucket_mb=4.0, grad_comm=comm)
        assert tr.use_plan and tr.bucketer.native_comm is None and len(tr.bucketer.buckets) > 1
        tr.set_batch(x[sl].to(dev), t[sl].to(dev))
        for _ in range(PLAN_STEPS):
            tr.step()
        torch.cuda.synchronize()
        assert tr.plan_id is not None
        if rank == 0:
            torch.save({"grad": nat.store.grad.cpu(), "flat": nat.store.flat.cpu()}, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_native_ddp_plan_replay_reduces_once(tmp_path, comm):
    """Every replayed step all-reduces each bucket exactly once (a replay used to issue every
    bucket again from finish(), doubling fp32 sums and racing the bf16 mirror). The last step's reduced
    gradient must equal the summed shard gradients bit for bit, and the weights after 6 steps must match
    a single-process replay of the same DDP arithmetic."""
    from robotic_discovery_platform_amd.models.unet import NativeAdam, UNetNative
    out = str(tmp_path / "p.pt")
    mp.spawn(_plan_worker, args=(2, _free_port(), comm, out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    dev = torch.device("cuda")
    nat = UNetNative(3, 1, device=dev, init_from=_ref(10))
    ex = nat.executor(2, 64, 64, training=True)
    adam = NativeAdam(nat, lr=1e-3)
    x, t = _data()
    for _ in range(PLAN_STEPS):
        shards = []
        for r in range(2):
            sl = slice(2 * r, 2 * r + 2)
            ex.set_input(x[sl].to(dev), t[sl].to(dev))
            ex.forward()
            ex.backward()
            shards.append(nat.store.grad.clone())
        if comm == "bf16":
            acc = (shards[0].to(torch.bfloat16) + shards[1].to(torch.bfloat16)).float()
        else:
            acc = shards[0] + shards[1]
        nat.store.grad.copy_(acc)
        adam.step(gscale=0.5)
    torch.cuda.synchronize()
    assert torch.equal(got["grad"], acc.cpu()), f"max |diff| {float((got['grad'] - acc.cpu()).abs().max()):.3g}"
    assert torch.allclose(got["flat"], nat.store.flat.cpu(), atol=1e-6, rtol=0)


def _checker_worker(rank, port, out):
    """StreamOrderChecker over the real executor's stream waits and hooks (gloo world 1, one GPU)."""
    import json
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        from robotic_discovery_platform_amd.models.unet import UNetNative
        from robotic_discovery_platform_amd.parallel.ddp import StreamOrderChecker
        from robotic_discovery_platform_amd.train.engine import NativeTrainer
        dev = torch.device("cuda", 0)
        x, t = _data()
        res = {}
        for decoder in ("bilinear", "transposed"):
            for ordered in (True, False):
                nat = UNetNative(3, 1, bilinear=decoder == "bilinear", device=dev, init_from=None)
                tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, graph=False, bucket_mb=4.0, ddp_force=True)
                if not ordered:
                    tr.bucketer.launch_ctx = None
                ck = StreamOrderChecker().install()
                tr.bucketer.checker = ck
                try:
                    tr.set_batch(x[:2].to(dev), t[:2].to(dev))
                    for _ in range(2):
                        tr.step()
                    torch.cuda.synchronize()
                finally:
                    ck.uninstall()
                res[f"{decoder}_{'ordered' if ordered else 'unordered'}"] = {
                    "launches": ck.launches, "buckets": len(tr.bucketer.buckets), "violations": ck.violations}
        json.dump(res, open(out, "w"))
    finally:
        dist.destroy_process_group()


def test_bucket_issue_is_ordered_after_every_gradient_producer(tmp_path):
    """Every bucket all-reduce is issued on a stream whose vector clock covers the producing stream of
    every gradient in it (main: BN / head / bias; side: conv weights). The unordered control (issue from
    the hook's current stream) is flagged, so the checker is not vacuous."""
    import json
    out = str(tmp_path / "ck.json")
    mp.spawn(_checker_worker, args=(_free_port(), out), nprocs=1, join=True)
    r = json.load(open(out))
    for dec in ("bilinear", "transposed"):
        good, bad = r[f"{dec}_ordered"], r[f"{dec}_unordered"]
        assert good["launches"] == 2 * good["buckets"] and good["violations"] == [], good["violations"][:5]
        assert len(bad["violations"]) > 0
