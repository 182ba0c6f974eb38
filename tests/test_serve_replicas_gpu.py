"""Per-GPU serving replicas on real GPUs (SURVEY.md §2.4 "a replica per GPU"; reference concurrency
model: /root/reference/services/vision_analysis/server.py:172).

On a 1-GPU box two native replicas both live on cuda:0 -- the pool, session and hot-reload logic is
the same as across GPUs, and every binding now runs on the device of its tensors (csrc/bindings.cpp
``on_device``). Mixed-device calls must raise; that case needs two GPUs and is skipped otherwise.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(seed):
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(seed)
    nat = UNetNative(3, 1, device=torch.device("cuda", 0), init_from=UNetRef(3, 1)).eval()
    with torch.no_grad():
        nat.store.view("outc.conv.bias").fill_(0.0)
    nat.refresh_weights()
    return nat


def _frames(pool, scenes, rgb=False):
    out = []
    for _ in range(2):  # two streams, round-robin over the replicas
        s = pool.session()
        got = []
        for i, sc in enumerate(scenes):
            c = sc.color[..., ::-1].copy() if rgb else sc.color
            got += s.submit(c, sc.depth, tag=i, rgb=rgb)
        got += s.drain()
        out.append((s.replica, [r for _, r in got]))
    return out


def _same(a, b):
    return (np.array_equal(a.mask, b.mask) and a.coverage == b.coverage
            and a.curvature.mean_curvature == b.curvature.mean_curvature
            and a.curvature.max_curvature == b.curvature.max_curvature)


def test_engine_pool_two_native_replicas_hot_reload():
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.serve.engine import EnginePool, FramePipeline
    scenes = [make_scene(i) for i in (1, 2, 3)]
    m0 = _model(0)
    pool = EnginePool(m0, DEFAULT_K, 0.001, n=2, devices=["cuda:0", "cuda:0"], rgb=True)
    assert len(pool.replicas) == 2 and pool.replicas[1] is not m0
    # the RGB network graph and the geometry graph, captured at build
    assert all(p.graphs.keys() == {1, "geo"} for q in pool._pools.values() for p in list(q.queue))
    res = _frames(pool, scenes, rgb=True)
    assert [r for r, _ in res] == [0, 1]
    for a, b in zip(res[0][1], res[1][1]):  # the replica is a bitwise copy
        assert _same(a, b)
    # hot reload: new weights into every replica, in place; the captured graphs must serve them
    m1 = _model(1)
    sd = {k: v.detach().clone() for k, v in m1.state_dict().items()}
    with pool.exclusive() as held:
        pool.load_state_dict(sd)
        pool.refresh_weights(held)
        torch.cuda.synchronize()
    res2 = _frames(pool, scenes, rgb=True)
    fresh = FramePipeline(m1, DEFAULT_K, 0.001, graph=False)
    for i, sc in enumerate(scenes):
        ref = fresh.process(sc.color, sc.depth)
        for _, rs in res2:
            assert _same(rs[i], ref), f"frame {i}: served result differs from a fresh pipeline after reload"
    assert not all(_same(a, b) for a, b in zip(res[0][1], res2[0][1]))  # the reload changed something


def test_session_close_returns_pipelines():
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.serve.engine import EnginePool
    sc = make_scene(2)
    pool = EnginePool(_model(0), DEFAULT_K, 0.001, n=2)
    q = pool._get(0, 480, 640)
    s = pool.session()
    s.submit(sc.color, sc.depth, tag=0)
    s.submit(sc.color, sc.depth, tag=1)
    assert q.qsize() == 0 and len(s.inflight) == 2
    s.close()
    assert q.qsize() == 2 and not s.inflight
    s2 = pool.session()  # the pool still serves
    assert len(s2.submit(sc.color, sc.depth, tag=0) + s2.drain()) == 1


def test_binding_rejects_cpu_tensor_argument():
    from robotic_discovery_platform_amd.ops import native
    C = native()
    x = torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16, device="cuda")
    with pytest.raises(RuntimeError):
        C.bn_relu_apply(x, torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16), torch.zeros(256, device="cuda"), 1)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_binding_rejects_mixed_devices():
    from robotic_discovery_platform_amd.ops import native
    C = native()
    x = torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16, device="cuda:0")
    y = torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16, device="cuda:1")
    with pytest.raises(RuntimeError, match="different GPUs"):
        C.bn_relu_apply(x, y, torch.zeros(256, device="cuda:0"), 1)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_replica_on_second_gpu_matches_first():
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.serve.engine import EnginePool
    scenes = [make_scene(i) for i in (1, 2)]
    torch.cuda.set_device(0)
    pool = EnginePool(_model(0), DEFAULT_K, 0.001, n=1, devices=["cuda:0", "cuda:1"])
    assert pool.replicas[1].store.device == torch.device("cuda", 1)
    res = _frames(pool, scenes)
    for a, b in zip(res[0][1], res[1][1]):
        assert _same(a, b)
