"""SyncBatchNorm in the native executor (SURVEY.md §2.5 "all_reduce BN statistics", optional).

Two ranks share one GPU over gloo, each holding half of a batch of 4 whose halves have different
statistics. With shared statistics the step must match one process on the whole batch:
  * BN running statistics equal the native single-process batch-4 run (bf16 rounding only);
  * the all-reduced (summed) gradient equals 2x the full-batch fp32 gradient, judged like
    test_unet_native_gpu.py: per-parameter cosine against the fp32 oracle, with torch's own bf16
    autocast run as the yardstick (a 64x64 U-Net's bf16 gradients are ill-conditioned: a 1e-7
    change of one BN coefficient moves them by percents, so relative-norm checks do not apply).
Control: without SyncBN the running statistics are rank-local.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data():
    g = torch.Generator().manual_seed(5)
    x = torch.rand(4, 3, 64, 64, generator=g)
    x[2:] = x[2:] * 0.5 + 0.4  # rank 1's half has different statistics: local BN would differ
    t = (torch.rand(4, 1, 64, 64, generator=g) > 0.6).float()
    return x, t


def _ref():
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(21)
    return UNetRef(3, 1)


def _running(nat):
    return {k: v.detach().cpu().clone() for k, v in nat.named_buffers() if "running" in k}


def _worker(rank, world, port, out, sync):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from robotic_discovery_platform_amd.models.unet import UNetNative
        from robotic_discovery_platform_amd.train.engine import NativeTrainer
        dev = torch.device("cuda", 0)
        nat = UNetNative(3, 1, device=dev, init_from=_ref())
        tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, graph=False, bucket_mb=4.0, sync_bn=sync)
        assert tr.ex.sync_world == (2 if sync else 1)
        x, t = _data()
        sl = slice(2 * rank, 2 * rank + 2)
        tr.set_batch(x[sl].to(dev), t[sl].to(dev))
        tr.ex.forward()
        tr.bucketer.reset()
        tr.ex.backward(grad_hook=tr._hook)
        tr.bucketer.finish()
        torch.cuda.synchronize()
        if rank == 0:
            st = nat.store
            grads = {n: st.view(n, st.grad).float().cpu().clone() for n in st.names}
            torch.save({"grads": grads, "bufs": _running(nat)}, out)
    finally:
        dist.destroy_process_group()


def _native_full_batch_running():
    from robotic_discovery_platform_amd.models.unet import UNetNative
    dev = torch.device("cuda")
    nat = UNetNative(3, 1, device=dev, init_from=_ref())
    ex = nat.executor(4, 64, 64, training=True)
    x, t = _data()
    ex.set_input(x.to(dev), t.to(dev))
    ex.forward()
    torch.cuda.synchronize()
    return _running(nat)


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _cos(a, b):
    a, b = a.reshape(-1).double(), b.reshape(-1).double()
    return float((a @ b) / (a.norm() * b.norm()).clamp_min(1e-30))


def _eager_grads(autocast: bool):
    dev = torch.device("cuda")
    m = _ref().to(dev).train()
    x, t = _data()
    x = x.to(dev).to(torch.bfloat16).float()  # the native path sees bf16 inputs too
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        o = m(x)
    F.binary_cross_entropy_with_logits(o.float(), t.to(dev)).backward()
    return {n: p.grad.detach().float().cpu() for n, p in m.named_parameters()}


def test_native_syncbn_matches_full_batch(tmp_path):
    out = str(tmp_path / "s.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, True), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    for k, v in _native_full_batch_running().items():
        assert _rel(got["bufs"][k], v) < 3e-3, (k, _rel(got["bufs"][k], v))
    g32, g16 = _eager_grads(False), _eager_grads(True)
    report = [(n, _cos(got["grads"][n], 2 * g), _cos(g16[n], g)) for n, g in g32.items()]
    print("\n".join(f"{n} {c:.4f} {c16:.4f}" for n, c, c16 in report))
    mean_c = sum(r[1] for r in report) / len(report)
    mean_c16 = sum(r[2] for r in report) / len(report)
    assert mean_c > mean_c16 - 0.02, (mean_c, mean_c16)
    for n, c, c16 in report:
        assert c > min(0.97, c16 - 0.1), (n, c, c16)


def test_native_local_bn_differs_without_sync(tmp_path):
    out = str(tmp_path / "l.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, False), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    b1 = _native_full_batch_running()
    k = "inc.double_conv.1.running_mean"
    assert _rel(got["bufs"][k], b1[k]) > 3e-2, _rel(got["bufs"][k], b1[k])
