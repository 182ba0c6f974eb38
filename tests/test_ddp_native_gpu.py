"""Native DDP step (NativeTrainer + FlatBucketer hooks + gscale folded into Adam) with 2 ranks sharing
one GPU over gloo (RCCL refuses two ranks per device; the bucketing/hook logic is backend-agnostic).

Per-shard gradients come from identical kernels on identical inputs, so the all-reduced buffer must
equal the sum of the two single-process shard gradients bit for bit.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


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


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from robotic_discovery_platform_amd.models.unet import UNetNative
        from robotic_discovery_platform_amd.train.engine import NativeTrainer
        dev = torch.device("cuda", 0)
        nat = UNetNative(3, 1, device=dev, init_from=_ref(10 + rank))  # broadcast must unify
        tr = NativeTrainer(nat, 2, 64, 64, lr=1e-3, graph=True, bucket_mb=4.0)
        assert tr.bucketer is not None and len(tr.bucketer.buckets) > 1 and tr.graph is None
        x, t = _data()
        sl = slice(2 * rank, 2 * rank + 2)
        tr.set_batch(x[sl].to(dev), t[sl].to(dev))
        tr.step()
        torch.cuda.synchronize()
        p = nat.store.flat.clone()
        ps = [torch.zeros_like(p) for _ in range(world)]
        dist.all_gather(ps, p)
        assert torch.equal(ps[0], ps[1])
        if rank == 0:
            torch.save({"grad": nat.store.grad.cpu(), "flat": p.cpu()}, out)
    finally:
        dist.destroy_process_group()


def test_native_ddp_two_ranks_one_gpu(tmp_path):
    from robotic_discovery_platform_amd.models.unet import NativeAdam, UNetNative
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    dev = torch.device("cuda")
    nat = UNetNative(3, 1, device=dev, init_from=_ref(10))
    ex = nat.executor(2, 64, 64, training=True)
    x, t = _data()
    acc = torch.zeros_like(nat.store.grad)
    for r in range(2):
        sl = slice(2 * r, 2 * r + 2)
        ex.set_input(x[sl].to(dev), t[sl].to(dev))
        ex.forward()
        ex.backward()
        acc += nat.store.grad
    assert torch.equal(got["grad"], acc.cpu())
    # Adam with gscale = 1/world on the summed gradient
    nat.store.grad.copy_(acc)
    NativeAdam(nat, lr=1e-3).step(gscale=0.5)
    torch.cuda.synchronize()
    assert torch.allclose(got["flat"], nat.store.flat.cpu(), atol=1e-7, rtol=0)
