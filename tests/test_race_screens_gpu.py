"""Race screens: every reduction-free kernel must be bitwise deterministic run-to-run.

LDS staging (LDS-DMA + s_barrier + counted vmcnt) and split-K slabs are where a missing wait or
barrier shows up as run-to-run differences; each kernel runs several times on several shapes
(odd sizes, concat inputs, split outputs) and every run must reproduce the first bit for bit.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

REPS = 5


@pytest.fixture(scope="module")
def C():
    from robotic_discovery_platform_amd.ops import native
    return native()


def _bf(shape, dev="cuda"):
    return torch.randn(*shape, device=dev).to(torch.bfloat16)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pref", [
    (4, 64, 64, 64, 0, 64, 0), (2, 33, 17, 128, 64, 128, 0), (8, 16, 16, 256, 256, 256, 0),
    (2, 32, 64, 128, 128, 64, 1), (4, 16, 16, 64, 0, 128, 1), (3, 7, 9, 64, 0, 64, 128)])
def test_conv_fwd_stats_deterministic(C, N, H, W, C1, C2, Cout, pref):
    torch.manual_seed(0)
    x1, x2 = _bf((N, H, W, C1)), (_bf((N, H, W, C2)) if C2 else None)
    w = (torch.randn(Cout, 9 * (C1 + C2), device="cuda") / math.sqrt(9 * (C1 + C2))).to(torch.bfloat16)
    rows = C.conv_stats_rows(N * H * W, Cout, 0)
    outs = []
    for _ in range(REPS):
        y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device="cuda")
        st = torch.zeros(rows * 2 * Cout, device="cuda")
        C.conv_fwd(x1, x2, w, 9, 0, y, None, st, pref, None, 0)
        outs.append((y, st))
    for y, st in outs[1:]:
        assert torch.equal(y, outs[0][0]) and torch.equal(st, outs[0][1])


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,splits", [(4, 32, 32, 64, 0, 64, 7), (2, 17, 23, 128, 128, 128, 3),
                                                     (8, 16, 16, 512, 0, 512, 16), (2, 7, 128, 64, 64, 128, 9),
                                                     (2, 64, 64, 64, 0, 64, 512)])
def test_conv_wgrad_deterministic(C, N, H, W, C1, C2, Cout, splits):
    torch.manual_seed(1)
    x1, x2 = _bf((N, H, W, C1)), (_bf((N, H, W, C2)) if C2 else None)
    dy = _bf((N, H, W, Cout))
    Cin = C1 + C2
    slab = torch.zeros(C.wgrad_slab_elems(N, H, W, Cin, Cout, 9, 0, splits), device="cuda")
    outs = []
    for _ in range(REPS):
        gw = torch.zeros(Cout * 9 * Cin, device="cuda")
        C.conv_wgrad(x1, x2, dy, 9, 0, Cin, slab, gw, 0, splits, 0)
        outs.append(gw)
    for g in outs[1:]:
        assert torch.equal(g, outs[0])


def test_native_train_step_deterministic():
    """Two identical models, same data: bitwise-identical weights after 3 graph-captured steps."""
    from robotic_discovery_platform_amd.models.unet import UNetNative
    from robotic_discovery_platform_amd.models.unet_ref import UNetRef
    from robotic_discovery_platform_amd.train.engine import NativeTrainer
    torch.manual_seed(0)
    ref = UNetRef(3, 1)
    x = torch.rand(4, 3, 64, 64, device="cuda")
    t = (torch.rand(4, 1, 64, 64, device="cuda") > 0.5).float()
    flats = []
    for _ in range(2):
        nat = UNetNative(3, 1, device=torch.device("cuda"), init_from=ref)
        tr = NativeTrainer(nat, 4, 64, 64, lr=1e-3, graph=True)
        tr.set_batch(x, t)
        for _ in range(3):
            tr.step()
        torch.cuda.synchronize()
        flats.append(nat.store.flat.clone())
    assert torch.equal(flats[0], flats[1])
