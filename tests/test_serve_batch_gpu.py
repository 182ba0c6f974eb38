"""Cross-stream batching of the serving network (serve/engine.py BatchEngine, csrc/serve_runtime.cpp
BatchNet): frames of concurrent streams that find a network in flight join one launch of N frames
(gather inputs -> U-Net -> head + threshold -> scatter masks) instead of each running its own N = 1
network. Reference per-frame model call: /root/reference/services/vision_analysis/server.py:121-125.

Checks: (1) the batched engine's network at every N equals the N = 1 network frame by frame (masks);
(2) several threads streaming frames through pool sessions -- array and encoded (JPEG + PNG bytes)
paths -- get the same results as one frame at a time, and batches of more than one frame did form;
(3) a lone stream never batches (its frames keep their own N = 1 graph)."""
import threading

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    torch.manual_seed(0)
    return UNetNative(3, 1, device=torch.device("cuda", 0), init_from=UNetRef(3, 1)).eval()


def _close(a, b, mask_tol=2e-3):
    """Same frame through two network batch sizes: the masks differ at most on a few threshold-edge
    pixels (the convs' split-K / tile choice differs with N: bf16 rounding), everything else follows."""
    diff = np.count_nonzero(a.mask != b.mask) / a.mask.size
    assert diff <= mask_tol, diff
    assert abs(a.coverage - b.coverage) <= 100 * mask_tol
    assert a.curvature.status == b.curvature.status


def test_batched_network_matches_single_frame_network():
    from robotic_discovery_platform_amd.serve.engine import BatchEngine
    m = _model()
    dev = torch.device("cuda", 0)
    be = BatchEngine(m, dev, max_batch=4)
    g = torch.Generator().manual_seed(1)
    xs = [torch.rand(1, 3, 256, 256, generator=g) for _ in range(4)]
    ref = []
    for x in xs:  # the N = 1 executor, eager
        ex = be.ex[1]
        ex.set_input(x.to(dev))
        ex.forward(head=False, refresh_eval=False, mask_head=(m.store.view("outc.conv.weight").reshape(-1),
                                                              m.store.view("outc.conv.bias"), be.thr_logit,
                                                              be.masks[1]))
        ref.append(be.masks[1].clone())
    torch.cuda.synchronize()
    for n in (2, 3, 4):
        ex = be.ex[n]
        ex.set_input(torch.cat(xs[:n]).to(dev))
        ex.forward(head=False, refresh_eval=False, mask_head=(m.store.view("outc.conv.weight").reshape(-1),
                                                              m.store.view("outc.conv.bias"), be.thr_logit,
                                                              be.masks[n]))
        torch.cuda.synchronize()
        for i in range(n):
            got = be.masks[n][i * 65536:(i + 1) * 65536]
            assert (got != ref[i]).float().mean().item() <= 2e-3, (n, i)


def _stream(pool, scenes, frames, out, k, encoded=False):
    from robotic_discovery_platform_amd.serve.client import make_request
    s = pool.session()
    got = []
    reqs = [make_request(sc.color, sc.depth) for sc in scenes] if encoded else None
    for i in range(frames):
        j = (i + k) % len(scenes) if frames > 1 else 0
        if encoded:
            r = reqs[j]
            col, code = s.submit_encoded(r.color_image.data, r.depth_image.data, tag=j)
            assert code == 0
            got += col
        else:
            got += s.submit(scenes[j].color, scenes[j].depth, tag=j)
    got += s.drain()
    out[k] = got


@pytest.mark.parametrize("encoded", [False, True])
def test_concurrent_streams_batch_and_match(encoded):
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.serve.engine import EnginePool, WireResult
    m = _model()
    scenes = [make_scene(i) for i in range(4)]
    pool = EnginePool(m, DEFAULT_K, 0.001, n=8, graph=True, rgb=encoded, jpeg=encoded, max_batch=4)
    assert pool.batches[0] is not None
    # reference: one frame at a time through the same pool (each frame finds the GPU free: solo graph)
    solo = {}
    for k in range(len(scenes)):
        _stream(pool, scenes[k:k + 1], 1, solo, k, encoded)
    ref = [solo[k][0][1] for k in range(len(scenes))]
    assert pool.batch_sizes()[0][0] == len(scenes) and sum(pool.batch_sizes()[0][1:]) == 0
    out = {}
    ths = [threading.Thread(target=_stream, args=(pool, scenes, 24, out, k, encoded)) for k in range(4)]
    [t.start() for t in ths]
    [t.join() for t in ths]
    sizes = pool.batch_sizes()[0]
    assert sum(sizes[2:]) > 0, sizes  # some launches carried 2+ frames
    for k in range(4):
        assert len(out[k]) == 24
        for tag, r in out[k]:
            assert not isinstance(r, Exception), r
            if isinstance(r, WireResult):  # encoded path: the wire result's coverage
                assert abs(r.coverage - ref[tag].coverage) <= 0.2, (r.coverage, ref[tag].coverage)
            else:
                _close(r, ref[tag])


def test_lone_stream_keeps_single_frame_graph():
    from robotic_discovery_platform_amd.data.synthetic import DEFAULT_K, make_scene
    from robotic_discovery_platform_amd.serve.engine import EnginePool
    m = _model()
    scenes = [make_scene(i) for i in range(2)]
    pool = EnginePool(m, DEFAULT_K, 0.001, n=2, graph=True, max_batch=4)
    s = pool.session()
    for i in range(6):  # one frame at a time: every frame finds the GPU free
        s.submit(scenes[i % 2].color, scenes[i % 2].depth, tag=i)
        s.drain()
    sizes = pool.batch_sizes()[0]
    assert sizes[0] == 6 and sum(sizes[1:]) == 0, sizes
