"""Numerics of every native HIP kernel vs a plain-PyTorch fp32 reference of the same op (GPU only).

Inputs are rounded to bf16 first, so the references see exactly the kernel's operands; tolerances
cover bf16 output rounding and fp32-vs-MFMA accumulation order.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from robotic_discovery_platform_amd.ops import native
    return native()


def bf(x):
    return x.to(torch.bfloat16)


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2)


def relerr(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def ohwi(w):  # [Cout,Cin,kh,kw] -> [Cout, kh*kw*Cin]
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [
    (2, 16, 16, 64, 0, 64), (1, 32, 32, 128, 0, 128), (2, 9, 13, 64, 64, 128),
    (1, 8, 8, 256, 256, 256), (3, 7, 5, 64, 0, 64), (1, 16, 16, 512, 0, 512)])
def test_conv_fwd_and_stats(C, N, H, W, C1, C2, Cout):
    torch.manual_seed(0)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    rows = C.conv_stats_rows(N * H * W, Cout, 0)
    stats = torch.zeros(rows * 2 * Cout, device=dev)
    r = C.conv_fwd(x1, x2, ohwi(w).contiguous(), 9, 0, y, None, stats, 0, None, 0)
    assert 0 < r <= rows
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.conv2d(xin, w.float(), padding=1)
    assert relerr(nchw(y), ref) < 1e-2
    yq = nchw(y).float()
    s = stats.view(rows, 2, Cout)[:r].sum(0)
    assert torch.allclose(s[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(s[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [
    (2, 8, 64, 64, 0, 64), (1, 8, 128, 64, 64, 128), (2, 16, 32, 128, 0, 64), (1, 32, 32, 128, 128, 256),
    (3, 16, 16, 64, 0, 128), (2, 32, 16, 256, 0, 64)])
def test_conv_halo_fwd_and_stats(C, N, H, W, C1, C2, Cout):
    """Halo-tile kernel (bm_pref=1) on every tile shape (64x4, 32x8, 16x16), BN=64/128, concat input."""
    torch.manual_seed(3)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    y = torch.full((N, H, W, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    rows = C.conv_stats_rows(N * H * W, Cout, 0)
    stats = torch.zeros(rows * 2 * Cout, device=dev)
    r = C.conv_fwd(x1, x2, ohwi(w).contiguous(), 9, 0, y, None, stats, 1, None, 0)
    assert 0 < r <= rows
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.conv2d(xin, w.float(), padding=1)
    assert relerr(nchw(y), ref) < 1e-2
    yq = nchw(y).float()
    s = stats.view(rows, 2, Cout)[:r].sum(0)
    assert torch.allclose(s[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(s[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    # the halo kernel and the implicit-GEMM kernel agree to bf16 rounding
    y2 = torch.empty_like(y)
    C.conv_fwd(x1, x2, ohwi(w).contiguous(), 9, 0, y2, None, None, 256, None, 0)
    assert relerr(y, y2) < 5e-3


def test_conv_halo_dgrad_split_and_eval_fold(C):
    torch.manual_seed(4)
    dev = "cuda"
    N, H, W, Cs, Cu, Cout = 2, 8, 64, 64, 64, 128
    x = torch.randn(N, Cs + Cu, H, W, device=dev, requires_grad=True)
    w = bf(torch.randn(Cout, Cs + Cu, 3, 3, device=dev) / 30)
    dy = bf(torch.randn(N, Cout, H, W, device=dev))
    F.conv2d(x, w.float(), padding=1).backward(dy.float())
    wt = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cs + Cu, 9 * Cout).contiguous()
    d1 = torch.empty(N, H, W, Cs, dtype=torch.bfloat16, device=dev)
    d2 = torch.empty(N, H, W, Cu, dtype=torch.bfloat16, device=dev)
    assert C.conv_fwd(nhwc(dy), None, wt, 9, 0, d1, d2, None, 1, None, 0) > 0
    assert relerr(torch.cat([nchw(d1), nchw(d2)], 1), x.grad) < 1e-2
    # eval BN fold + ReLU epilogue
    g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    xb = bf(torch.randn(N, H, W, Cs + Cu, device=dev))
    a = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(xb, None, ohwi(w).contiguous(), 9, 0, a, None, None, 1, coef, 1)
    ref = F.relu(F.batch_norm(F.conv2d(nchw(xb).float(), w.float(), padding=1), rm, rv, g, b, False, 0.0, 1e-5))
    assert relerr(nchw(a), ref) < 1e-2


def test_conv_fwd_asymmetric_identity(C):
    """A = I style check with an asymmetric weight: catches row/col swaps in the MFMA C-write."""
    dev = "cuda"
    N, H, W, Cin, Cout = 1, 4, 4, 64, 64
    x = torch.zeros(N, H, W, Cin, device=dev)
    for c in range(Cin):
        x[0, c // 16, (c // 4) % 4, c] = 1.0
    w = torch.zeros(Cout, Cin, 3, 3, device=dev)
    for co in range(Cout):
        for ci in range(Cin):
            w[co, ci, 1, 1] = float((co * 7 + ci * 3) % 11) - 5  # asymmetric, small ints (exact in bf16)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(bf(x), None, ohwi(bf(w)).contiguous(), 9, 0, y, None, None, 0, None, 0)
    ref = F.conv2d(nchw(x), w, padding=1)
    assert torch.equal(nchw(y).float(), ref)


def test_conv_packed_first_layer(C):
    torch.manual_seed(1)
    dev = "cuda"
    N, H, W, Cout = 2, 20, 12, 64
    x = torch.rand(N, 3, H, W, device=dev)
    x8 = torch.zeros(N, H, W, 8, dtype=torch.bfloat16, device=dev)
    x8[..., :3] = bf(nhwc(x))
    w = bf(torch.randn(Cout, 3, 3, 3, device=dev) * 0.3)
    wp = torch.zeros(Cout, 16, 8, dtype=torch.bfloat16, device=dev)
    wp[:, :9, :3] = w.permute(0, 2, 3, 1).reshape(Cout, 9, 3)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x8, None, wp.view(Cout, 128), 9, 1, y, None, None, 0, None, 0)
    ref = F.conv2d(nchw(x8[..., :3]).float(), w.float(), padding=1)
    assert relerr(nchw(y), ref) < 1e-2


@pytest.mark.parametrize("N,H,W", [(2, 20, 12), (3, 256, 256), (1, 7, 9), (5, 64, 96)])
def test_conv_first_layer_kernel(C, N, H, W):
    """conv_first.hip (bm_pref 13; auto for the packed 3-channel layer) vs the packed implicit GEMM
    (bm_pref 256) and fp32 torch: training output + BN partial sums, eval BN fold + ReLU; ragged last
    segment (M % 64 != 0) and image borders."""
    torch.manual_seed(13)
    dev = "cuda"
    Cout = 64
    x = torch.rand(N, 3, H, W, device=dev)
    x8 = torch.zeros(N, H, W, 8, dtype=torch.bfloat16, device=dev)
    x8[..., :3] = bf(nhwc(x))
    w = bf(torch.randn(Cout, 3, 3, 3, device=dev) * 0.3)
    wp = torch.zeros(Cout, 16, 8, dtype=torch.bfloat16, device=dev)
    wp[:, :9, :3] = w.permute(0, 2, 3, 1).reshape(Cout, 9, 3)
    wk = wp.view(Cout, 128)
    rows = C.conv_stats_rows(N * H * W, Cout, 0)
    ys, ss = [], []
    for pref in (256, 13):
        y = torch.full((N, H, W, Cout), 5.0, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(rows * 2 * Cout, device=dev)
        r = C.conv_fwd(x8, None, wk, 9, 1, y, None, st, pref, None, 0)
        assert 0 < r <= rows
        ys.append(y)
        ss.append(st[: r * 2 * Cout].view(r, 2, Cout).sum(0))
    ref = F.conv2d(nchw(x8[..., :3]).float(), w.float(), padding=1)
    assert relerr(nchw(ys[1]), ref) < 1e-2
    assert relerr(ys[1], ys[0]) < 1e-2
    yq = nchw(ys[1]).float()
    assert torch.allclose(ss[1][0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    assert torch.allclose(ss[1][1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-1)
    coef = torch.randn(4 * Cout, device=dev)
    a = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x8, None, wk, 9, 1, a, None, None, 13, coef, 1)
    sc, sh = coef[2 * Cout:3 * Cout].view(1, -1, 1, 1), coef[3 * Cout:].view(1, -1, 1, 1)
    assert relerr(nchw(a), torch.relu(ref * sc + sh)) < 1e-2


def test_conv_dgrad_split_output(C):
    """dgrad = conv(dy, flip(W)^T) written into two destinations (the Up-block concat split)."""
    torch.manual_seed(2)
    dev = "cuda"
    N, H, W, Cs, Cu, Cout = 2, 12, 10, 64, 64, 64
    x = torch.randn(N, Cs + Cu, H, W, device=dev, requires_grad=True)
    w = bf(torch.randn(Cout, Cs + Cu, 3, 3, device=dev) / 30)
    dy = bf(torch.randn(N, Cout, H, W, device=dev))
    y = F.conv2d(x, w.float(), padding=1)
    y.backward(dy.float())
    wt = w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cs + Cu, 9 * Cout).contiguous()  # [cin][tap'][cout]
    d1 = torch.empty(N, H, W, Cs, dtype=torch.bfloat16, device=dev)
    d2 = torch.empty(N, H, W, Cu, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(nhwc(dy), None, wt, 9, 0, d1, d2, None, 0, None, 0)
    got = torch.cat([nchw(d1), nchw(d2)], 1)
    assert relerr(got, x.grad) < 1e-2


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,splits", [
    (2, 16, 16, 64, 0, 64, 3), (1, 32, 32, 128, 0, 128, 4), (2, 9, 13, 64, 64, 128, 2), (1, 8, 8, 256, 0, 512, 1),
    # W % 64 == 0: the halo-reuse kernel (row-segment K steps, 9 taps from one staged row triple)
    (2, 5, 64, 64, 0, 64, 3), (1, 6, 128, 64, 64, 128, 4), (3, 3, 64, 128, 0, 64, 64), (1, 4, 192, 64, 128, 256, 2),
    # W | 64: multi-row segments, row-crossing taps masked on the dY side
    (2, 6, 32, 64, 0, 64, 3), (1, 8, 16, 128, 128, 128, 2), (3, 8, 8, 64, 0, 128, 5),
    # >8 splits with few elements per split: two-level slab reduction (group rows, then layout)
    (2, 64, 64, 64, 0, 64, 512), (1, 64, 128, 64, 64, 128, 512), (4, 20, 20, 64, 0, 64, 150)])
def test_conv_wgrad(C, N, H, W, C1, C2, Cout, splits):
    torch.manual_seed(3)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    dy = bf(torch.randn(N, H, W, Cout, device=dev))
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    w = torch.zeros(Cout, C1 + C2, 3, 3, device=dev, requires_grad=True)
    F.conv2d(xin, w, padding=1).backward(nchw(dy).float())
    slab = torch.zeros(C.wgrad_slab_elems(N, H, W, C1 + C2, Cout, 9, 0, splits), device=dev)
    out = torch.zeros(Cout * 9 * (C1 + C2), device=dev)
    C.conv_wgrad(x1, x2, dy, 9, 0, 0, slab, out, 0, splits, 0)
    ref = w.grad.permute(0, 2, 3, 1).reshape(-1)
    assert relerr(out, ref) < 2e-3


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [
    (2, 16, 16, 256, 0, 256), (1, 8, 8, 256, 256, 512), (2, 12, 20, 128, 0, 256), (1, 6, 128, 64, 64, 128),
    (3, 9, 13, 64, 0, 128), (2, 33, 47, 128, 0, 128), (16, 64, 64, 256, 0, 256), (64, 16, 16, 512, 0, 512)])
def test_conv_wgrad_kernels_agree(C, N, H, W, C1, C2, Cout):
    """The halo (variant 5, where it applies), generic (4) and auto (0) weight gradients vs fp32 torch;
    the same launch twice is bitwise reproducible."""
    torch.manual_seed(5)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    dy = bf(torch.randn(N, H, W, Cout, device=dev))
    # split count for the generic kernel: its fp32 slab must stay below 2 GiB (buffer-resource range)
    ncols_pad = (9 * (C1 + C2) + 255) // 256 * 256
    sp = min(512, (1 << 29) // (Cout * ncols_pad))
    slab = torch.zeros(C.wgrad_slab_elems(N, H, W, C1 + C2, Cout, 9, 0, sp), device=dev)
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    w = torch.zeros(Cout, C1 + C2, 3, 3, device=dev, requires_grad=True)
    F.conv2d(xin, w, padding=1).backward(nchw(dy).float())
    ref = w.grad.permute(0, 2, 3, 1).reshape(-1)
    halo = W % 64 == 0 or (W >= 8 and 64 % W == 0 and (H * W) % 64 == 0)
    outs = []
    for v in (0, 0, 4) + ((5,) if halo else ()):
        out = torch.full((Cout * 9 * (C1 + C2),), 3.0, device=dev)
        assert C.conv_wgrad(x1, x2, dy, 9, 0, 0, slab, out, 0, sp, v) > 0
        outs.append(out)
        assert relerr(out, ref) < 2e-3
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("N,H,W,splits", [(2, 18, 14, 5), (2, 64, 64, 300)])
def test_conv_wgrad_packed(C, N, H, W, splits):
    torch.manual_seed(4)
    dev = "cuda"
    Cout = 64
    x = bf(torch.rand(N, H, W, 3, device=dev))
    x8 = torch.zeros(N, H, W, 8, dtype=torch.bfloat16, device=dev)
    x8[..., :3] = x
    dy = bf(torch.randn(N, H, W, Cout, device=dev))
    w = torch.zeros(Cout, 3, 3, 3, device=dev, requires_grad=True)
    F.conv2d(nchw(x).float(), w, padding=1).backward(nchw(dy).float())
    slab = torch.zeros(C.wgrad_slab_elems(N, H, W, 8, Cout, 9, 1, splits), device=dev)
    out = torch.zeros(Cout * 27, device=dev)
    C.conv_wgrad(x8, None, dy, 9, 1, 3, slab, out, 0, splits, 0)
    assert relerr(out, w.grad.permute(0, 2, 3, 1).reshape(-1)) < 2e-3


@pytest.mark.parametrize("N,H,W,splits", [(2, 16, 12, 5), (2, 64, 64, 300), (3, 32, 96, 1)])
def test_wgrad_first_bn_fused(C, N, H, W, splits):
    """First layer: BN-backward apply fused into the packed wgrad (wgrad_first_bn) vs the separate
    bn_relu_bwd_apply + conv_wgrad passes (same bf16 dz, fp32 sums in another split order) and vs an
    fp32 torch reference of the whole BN-backward + weight gradient."""
    torch.manual_seed(6)
    dev = "cuda"
    Cout, M = 64, N * H * W
    x = bf(torch.rand(N, H, W, 3, device=dev))
    x8 = torch.zeros(N, H, W, 8, dtype=torch.bfloat16, device=dev)
    x8[..., :3] = x
    y = bf(torch.randn(N, H, W, Cout, device=dev) * 1.5 + 0.2)
    da = bf(torch.randn(N, H, W, Cout, device=dev))
    gamma = torch.rand(Cout, device=dev) + 0.5
    beta = torch.randn(Cout, device=dev) * 0.1
    stats = torch.stack([y.float().sum((0, 1, 2)), (y.float() ** 2).sum((0, 1, 2))]).reshape(-1).contiguous()
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_finalize(stats, 1, M, gamma, beta, None, None, None, 0.1, 1e-5, coef, None)
    part = torch.zeros(1024 * 2 * Cout, device=dev)
    T = C.bn_relu_bwd_reduce(da, y, coef, 1, part)
    coef2 = torch.zeros(3 * Cout, device=dev)
    C.bn_bwd_finalize(part, T, M, gamma, coef, None, None, coef2, torch.zeros(64 * 2 * Cout, device=dev))
    # separate passes
    dz = torch.empty_like(y)
    C.bn_relu_bwd_apply(da, y, coef, coef2, dz, 1)
    slab = torch.zeros(C.wgrad_slab_elems(N, H, W, 8, Cout, 9, 1, splits), device=dev)
    ref_sep = torch.zeros(Cout * 27, device=dev)
    C.conv_wgrad(x8, None, dz, 9, 1, 3, slab, ref_sep, 0, splits, 0)
    out = torch.full((Cout * 27,), 7.0, device=dev)
    r = C.wgrad_first_bn(x8, da, y, coef, coef2, slab, out, 3, 0, splits)
    assert r >= 1
    assert relerr(out, ref_sep) < 1e-5
    # fp32 torch: BN(train) + ReLU backward, then the conv weight gradient
    yf = nchw(y).float().requires_grad_(True)
    bn = torch.nn.functional.batch_norm(yf, None, None, gamma, beta, training=True, eps=1e-5)
    torch.relu(bn).backward(nchw(da).float())
    w = torch.zeros(Cout, 3, 3, 3, device=dev, requires_grad=True)
    F.conv2d(nchw(x).float(), w, padding=1).backward(yf.grad)
    assert relerr(out, w.grad.permute(0, 2, 3, 1).reshape(-1)) < 1e-2
    # accumulate mode adds onto out
    out2 = out.clone()
    C.wgrad_first_bn(x8, da, y, coef, coef2, slab, out2, 3, 1, splits)
    assert torch.allclose(out2, 2 * out, rtol=1e-6, atol=1e-6)


def test_bn_relu_train_fwd_bwd(C):
    torch.manual_seed(5)
    dev = "cuda"
    N, H, W, Ch = 4, 16, 16, 128
    y = bf(torch.randn(N, H, W, Ch, device=dev) * 2 + 0.5)
    gamma = torch.rand(Ch, device=dev) + 0.5
    beta = torch.randn(Ch, device=dev) * 0.1
    M = N * H * W
    stats = torch.stack([y.float().sum((0, 1, 2)), (y.float() ** 2).sum((0, 1, 2))]).reshape(-1).contiguous()
    rm, rv = torch.zeros(Ch, device=dev), torch.ones(Ch, device=dev)
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    coef = torch.zeros(4 * Ch, device=dev)
    C.bn_finalize(stats, 1, M, gamma, beta, rm, rv, nbt, 0.1, 1e-5, coef, None)
    a = torch.empty_like(y)
    C.bn_relu_apply(y, a, coef, 1)
    bn = torch.nn.BatchNorm2d(Ch).to(dev)
    with torch.no_grad():
        bn.weight.copy_(gamma); bn.bias.copy_(beta)
    yin = nchw(y).float().detach().requires_grad_(True)
    ref = torch.relu(bn(yin))
    assert relerr(nchw(a), ref) < 1e-2
    assert torch.allclose(rm, bn.running_mean, atol=1e-4) and torch.allclose(rv, bn.running_var, rtol=1e-3)
    assert nbt.item() == 1
    da = bf(torch.randn(N, H, W, Ch, device=dev))
    ref.backward(nchw(da).float())
    part = torch.zeros(1024 * 2 * Ch, device=dev)
    T = C.bn_relu_bwd_reduce(da, y, coef, 1, part)
    dg, db, coef2 = torch.zeros(Ch, device=dev), torch.zeros(Ch, device=dev), torch.zeros(3 * Ch, device=dev)
    C.bn_bwd_finalize(part, T, M, gamma, coef, dg, db, coef2, torch.zeros(64 * 2 * Ch, device=dev))
    dy = torch.empty_like(y)
    C.bn_relu_bwd_apply(da, y, coef, coef2, dy, 1)
    assert relerr(nchw(dy), yin.grad) < 2e-2
    assert relerr(dg, bn.weight.grad) < 1e-3 and relerr(db, bn.bias.grad) < 1e-3


@pytest.mark.parametrize("N,H,W,Cout", [(2, 64, 64, 64), (1, 32, 128, 64), (2, 16, 64, 128)])
def test_conv_dgrad_bnred(C, N, H, W, Cout):
    """Row-ring dgrad with the next BN's backward reduction in its epilogue: dx identical to the
    unfused dgrad; the partial sums match torch fp32 sum(g), sum(g * xhat) of the bf16 dx."""
    torch.manual_seed(17)
    dev = "cuda"
    dy = bf(torch.randn(N, H, W, 64, device=dev))
    w = bf(torch.randn(Cout, 64, 3, 3, device=dev) * 0.05)
    wk = ohwi(w).contiguous()
    y = bf(torch.randn(N, H, W, Cout, device=dev) * 2 + 0.3)
    M = N * H * W
    mean = y.float().mean((0, 1, 2))
    inv = 1.0 / (y.float().var((0, 1, 2), unbiased=False) + 1e-5).sqrt()
    scale = (torch.rand(Cout, device=dev) + 0.5) * inv
    shift = torch.randn(Cout, device=dev) * 0.1 - mean * scale
    coef = torch.cat([mean, inv, scale, shift]).contiguous()
    dx = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    part = torch.zeros(1024 * 2 * Cout, device=dev)
    rows = C.conv_dgrad_bnred(dy, wk, dx, y, coef, part)
    if Cout != 64:  # only the 64-output ring kernel has the fused variant: -1, nothing launched
        assert rows == -1
        return
    assert rows > 0
    dx_ref = torch.empty_like(dx)
    C.conv_fwd(dy, None, wk, 9, 0, dx_ref, None, None, 6, None, 0)  # same ring kernel, no fusion
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref)
    conv = F.conv2d(nchw(dy).float(), w.float(), padding=1)
    assert relerr(nchw(dx), conv) < 1e-2
    g = torch.where(y.float() * scale + shift > 0, dx.float(), torch.zeros((), device=dev))
    p = part[: rows * 2 * Cout].view(rows, 2, Cout).sum(0)
    assert relerr(p[0], g.sum((0, 1, 2))) < 1e-3
    assert relerr(p[1], (g * (y.float() - mean) * inv).sum((0, 1, 2))) < 1e-3


@pytest.mark.parametrize("N,H,W", [(2, 64, 64), (1, 32, 128), (3, 16, 64)])
def test_conv_bnin_fwd_and_wgrad(C, N, H, W):
    """Row-ring forward / weight gradient that apply the producer's BN + ReLU to the staged pre-BN rows
    (BNIN): bitwise equal to bn_relu_apply followed by the same ring kernels."""
    torch.manual_seed(23)
    dev = "cuda"
    y_pre = bf(torch.randn(N, H, W, 64, device=dev) * 1.5 + 0.2)
    mean = y_pre.float().mean((0, 1, 2))
    inv = 1.0 / (y_pre.float().var((0, 1, 2), unbiased=False) + 1e-5).sqrt()
    scale = (torch.rand(64, device=dev) + 0.5) * inv
    shift = torch.randn(64, device=dev) * 0.3 - mean * scale
    coef = torch.cat([mean, inv, scale, shift]).contiguous()
    a = torch.empty_like(y_pre)
    C.bn_relu_apply(y_pre, a, coef, 1)
    w = bf(torch.randn(64, 64, 3, 3, device=dev) * 0.05)
    wk = ohwi(w).contiguous()
    y_ref, y_out = (torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev) for _ in range(2))
    rows_cap = max(1024, C.conv_stats_rows(N * H * W, 64, 0))
    st_ref, st = (torch.zeros(rows_cap * 2 * 64, device=dev) for _ in range(2))
    rows_ref = C.conv_fwd(a, None, wk, 9, 0, y_ref, None, st_ref, 6, None, 0)  # ring kernel on a
    rows = C.conv_fwd_bnin(y_pre, wk, y_out, st, coef)
    torch.cuda.synchronize()
    assert rows == rows_ref > 0
    assert torch.equal(y_out, y_ref) and torch.equal(st[: rows * 128], st_ref[: rows * 128])
    assert relerr(nchw(y_out), F.conv2d(nchw(a).float(), w.float(), padding=1)) < 1e-2
    # with a_out: the same outputs, and the formed activation written bitwise as bn_relu_apply writes it
    a_out = torch.full_like(y_pre, 3.0)
    y_out.zero_()
    st.zero_()
    assert C.conv_fwd_bnin(y_pre, wk, y_out, st, coef, a_out) == rows
    torch.cuda.synchronize()
    assert torch.equal(y_out, y_ref) and torch.equal(st[: rows * 128], st_ref[: rows * 128])
    assert torch.equal(a_out, a)


def test_conv_bnin_not_applicable(C):
    dev = "cuda"
    y_pre = bf(torch.randn(1, 16, 48, 64, device=dev))  # W % 64 != 0: no ring kernel
    coef = torch.ones(256, device=dev)
    y = torch.empty_like(y_pre)
    wk = bf(torch.randn(64, 576, device=dev))
    assert C.conv_fwd_bnin(y_pre, wk, y, torch.zeros(1024 * 128, device=dev), coef) == -1


def test_maxpool_fwd_bwd_with_skip(C):
    torch.manual_seed(6)
    dev = "cuda"
    for (N, H, W, Ch) in [(2, 16, 16, 64), (1, 9, 7, 128)]:
        x = bf(torch.randn(N, H, W, Ch, device=dev))
        x[0, 0, 0, :8] = x[0, 0, 1, :8]  # ties: first max wins
        p = torch.empty(N, H // 2, W // 2, Ch, dtype=torch.bfloat16, device=dev)
        C.maxpool2_fwd(x, p)
        xr = nchw(x).float().requires_grad_(True)
        pr = F.max_pool2d(xr, 2)
        assert torch.equal(nchw(p).float(), pr)
        dp = bf(torch.randn_like(pr))
        ds = bf(torch.randn(N, Ch, H, W, device=dev))
        pr.backward(dp.float())
        dx = torch.empty_like(x)
        C.maxpool2_bwd(nhwc(dp), x, nhwc(ds), dx)
        assert relerr(nchw(dx), xr.grad + ds.float()) < 1e-2


@pytest.mark.parametrize("hin,win,H2,W2", [(8, 8, 16, 16), (5, 7, 11, 14), (16, 16, 32, 32), (1, 1, 2, 2)])
def test_upsample_fwd_bwd(C, hin, win, H2, W2):
    torch.manual_seed(7)
    dev = "cuda"
    N, Ch = 2, 64
    x = bf(torch.randn(N, hin, win, Ch, device=dev))
    xr = nchw(x).float().requires_grad_(True)
    up = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=True)
    dY, dX = H2 - up.shape[2], W2 - up.shape[3]
    ref = F.pad(up, [dX // 2, dX - dX // 2, dY // 2, dY - dY // 2])
    out = torch.empty(N, H2, W2, Ch, dtype=torch.bfloat16, device=dev)
    C.upsample2_fwd(x, out, dY // 2, dX // 2)
    assert relerr(nchw(out), ref) < 1e-2
    g = bf(torch.randn_like(ref))
    ref.backward(g.float())
    dx = torch.empty_like(x)
    C.upsample2_bwd(nhwc(g), dx, dY // 2, dX // 2)
    assert relerr(nchw(dx), xr.grad) < 1e-2
    # fused with the BN-backward reduction of dx's BN (dx = da of the layer with pre-BN output y)
    y = bf(torch.randn(N, hin, win, Ch, device=dev) * 2 + 0.3)
    mean, inv = torch.randn(Ch, device=dev) * 0.1, torch.rand(Ch, device=dev) + 0.5
    gamma, beta = torch.randn(Ch, device=dev), torch.randn(Ch, device=dev) * 0.2
    ss = gamma * inv
    coef = torch.cat([mean, inv, ss, beta - mean * ss]).contiguous()
    part = torch.zeros(64 * 2 * Ch, device=dev)
    dx2 = torch.empty_like(x)
    T = C.upsample2_bwd(nhwc(g), dx2, dY // 2, dX // 2, y, coef, part)
    assert 1 <= T <= 64 and torch.equal(dx2, dx)
    got = part[:T * 2 * Ch].view(T, 2, Ch).double().sum(0)
    gg = dx.float() * ((y.float() * ss + (beta - mean * ss)) > 0)
    exact = torch.stack([gg.sum((0, 1, 2)), (gg * (y.float() - mean) * inv).sum((0, 1, 2))]).double()
    assert torch.allclose(got, exact, rtol=1e-3, atol=1e-3)
    # forward fused with the producer's training BN + ReLU: identical to apply-then-upsample
    a = torch.empty_like(y)
    C.bn_relu_apply(y, a, coef, 1)
    ref_out = torch.empty_like(out)
    C.upsample2_fwd(a, ref_out, dY // 2, dX // 2)
    fused = torch.empty_like(out)
    C.upsample2_fwd(y, fused, dY // 2, dX // 2, coef)
    assert torch.equal(fused, ref_out)


@pytest.mark.parametrize("N,hin,win,H2,W2", [(16, 128, 128, 256, 256), (32, 128, 128, 256, 256),
                                              (96, 61, 64, 125, 130)])
def test_upsample_banded_large(C, N, hin, win, H2, W2):
    """Batches large enough for the banded upsample kernels (forward bands of 4-8 output rows, backward
    bands of 2-4 input-gradient rows; the small shapes above take the one-row forms): forward and
    backward against F.interpolate (align_corners) + centred pad / autograd, and the BN-fused forms
    identical to the unfused ones."""
    torch.manual_seed(17)
    dev = "cuda"
    Ch = 64
    x = bf(torch.randn(N, hin, win, Ch, device=dev))
    xr = nchw(x).float().requires_grad_(True)
    up = F.interpolate(xr, scale_factor=2, mode="bilinear", align_corners=True)
    dY, dX = H2 - up.shape[2], W2 - up.shape[3]
    ref = F.pad(up, [dX // 2, dX - dX // 2, dY // 2, dY - dY // 2])
    out = torch.empty(N, H2, W2, Ch, dtype=torch.bfloat16, device=dev)
    C.upsample2_fwd(x, out, dY // 2, dX // 2)
    assert relerr(nchw(out), ref) < 1e-2
    g = bf(torch.randn_like(ref))
    ref.backward(g.float())
    del ref, up
    dx = torch.empty_like(x)
    C.upsample2_bwd(nhwc(g), dx, dY // 2, dX // 2)
    assert relerr(nchw(dx), xr.grad) < 1e-2
    y = bf(torch.randn(N, hin, win, Ch, device=dev) * 2 + 0.3)
    mean, inv = torch.randn(Ch, device=dev) * 0.1, torch.rand(Ch, device=dev) + 0.5
    gamma, beta = torch.randn(Ch, device=dev), torch.randn(Ch, device=dev) * 0.2
    ss = gamma * inv
    coef = torch.cat([mean, inv, ss, beta - mean * ss]).contiguous()
    part = torch.zeros(4096 * 2 * Ch, device=dev)
    dx2 = torch.empty_like(x)
    T = C.upsample2_bwd(nhwc(g), dx2, dY // 2, dX // 2, y, coef, part)
    assert 1 <= T <= 4096 and torch.equal(dx2, dx)
    got = part[:T * 2 * Ch].view(T, 2, Ch).double().sum(0)
    gg = dx.float() * ((y.float() * ss + (beta - mean * ss)) > 0)
    exact = torch.stack([gg.sum((0, 1, 2)), (gg * (y.float() - mean) * inv).sum((0, 1, 2))]).double()
    assert torch.allclose(got, exact, rtol=1e-3, atol=1e-2)
    a = torch.empty_like(y)
    C.bn_relu_apply(y, a, coef, 1)
    ref_out = torch.empty_like(out)
    C.upsample2_fwd(a, ref_out, dY // 2, dX // 2)
    fused = torch.empty_like(out)
    C.upsample2_fwd(y, fused, dY // 2, dX // 2, coef)
    assert torch.equal(fused, ref_out)


@pytest.mark.parametrize("dice_w", [0.0, 1.0])
def test_head_loss(C, dice_w):
    torch.manual_seed(8)
    dev = "cuda"
    N, H, W = 2, 24, 20
    a = bf(torch.randn(N, H, W, 64, device=dev))
    wt = torch.randn(64, device=dev) * 0.1
    b = torch.randn(1, device=dev) * 0.1
    t = (torch.rand(N, 1, H, W, device=dev) > 0.5).float()
    M = N * H * W
    logits = torch.zeros(M, device=dev)
    part = torch.zeros(C.head_partial_blocks(M) * 65, device=dev)
    sums, loss = torch.zeros(4, device=dev), torch.zeros(2, device=dev)
    C.head_fwd(a, wt, b, t.reshape(-1).contiguous(), logits, part, sums, loss, dice_w, 1.0)
    ar = nchw(a).float().requires_grad_(True)
    wr = wt.clone().view(1, 64, 1, 1).requires_grad_(True)
    br = b.clone().requires_grad_(True)
    lg = F.conv2d(ar, wr, br)
    L = F.binary_cross_entropy_with_logits(lg, t)
    if dice_w:
        p = torch.sigmoid(lg)
        L = L + dice_w * (1 - (2 * (p * t).sum() + 1) / (p.sum() + t.sum() + 1))
    assert torch.allclose(logits.view_as(lg), lg, atol=1e-4)
    assert abs(loss[0].item() - L.item()) < 1e-4
    L.backward()
    da = torch.empty_like(a)
    gw, gb = torch.zeros(64, device=dev), torch.zeros(1, device=dev)
    C.head_bwd(a, wt, logits, t.reshape(-1).contiguous(), sums, da, part, gw, gb, dice_w, 1.0, 1.0)
    assert relerr(nchw(da), ar.grad) < 1e-2
    assert relerr(gw, wr.grad.view(-1)) < 1e-4 and relerr(gb, br.grad) < 1e-4


def test_adam_matches_torch(C):
    torch.manual_seed(9)
    dev = "cuda"
    n = 4096
    p0 = torch.randn(n, device=dev)
    p = p0.clone()
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    sh = torch.zeros(n, dtype=torch.bfloat16, device=dev)
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-3)
    for _ in range(5):
        g = torch.randn(n, device=dev)
        C.adam(p, g, m, v, sh, 1e-3, 0.9, 0.999, 1e-8, 0.0, 1.0, step)
        ref.grad = g.clone()
        opt.step()
    assert step.item() == 5
    assert torch.allclose(p, ref.detach(), atol=1e-6, rtol=1e-5)
    assert torch.equal(sh, p.to(torch.bfloat16))


@pytest.mark.parametrize("N,h,w,Cin,Cout,H2,W2", [(2, 8, 8, 128, 64, 16, 16), (1, 4, 5, 256, 128, 9, 11)])
def test_conv_transpose2x2(C, N, h, w, Cin, Cout, H2, W2):
    """ConvTranspose2d(k=2, s=2) as taps=1 GEMM + shuffle(+bias, zero pad), and its backward
    (unshuffle, bias colsum, role-swapped wgrad, dgrad) vs torch fp32."""
    torch.manual_seed(5)
    dev = "cuda"
    x = bf(torch.randn(N, Cin, h, w, device=dev))
    W = bf(torch.randn(Cin, Cout, 2, 2, device=dev) / math.sqrt(Cin))
    b = torch.randn(Cout, device=dev)
    oy, ox = (H2 - 2 * h) // 2, (W2 - 2 * w) // 2
    xr = x.float().requires_grad_(True)
    Wr = W.float().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    y = F.conv_transpose2d(xr, Wr, br, stride=2)
    ref = F.pad(y, [ox, W2 - 2 * w - ox, oy, H2 - 2 * h - oy])
    wphys = W.permute(0, 2, 3, 1).reshape(Cin, 4 * Cout).contiguous()  # [ci][(dh, dw, co)]
    yT = torch.empty(N, h, w, 4 * Cout, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(nhwc(x), None, wphys.t().contiguous(), 1, 0, yT, None, None, 0, None, 0)
    u = torch.full((N, H2, W2, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    C.upT_shuffle(yT, b, u, oy, ox)
    assert relerr(nchw(u), ref) < 1e-2
    # backward
    du = bf(torch.randn(N, Cout, H2, W2, device=dev))
    ref.backward(du.float())
    dyT = torch.empty_like(yT)
    C.upT_unshuffle(nhwc(du), dyT, oy, ox)
    db = torch.zeros(Cout, device=dev)
    C.colsum_bf16(dyT, 4, torch.zeros((1024 * 4 + 64) * Cout, device=dev), db, 0)
    assert torch.allclose(db, br.grad, rtol=1e-3, atol=1e-2)
    M = N * h * w
    splits = max(1, M // 64)
    slab = torch.zeros(C.wgrad_slab_elems(N, h, w, 4 * Cout, Cin, 1, 0, splits), device=dev)
    gw = torch.zeros(Cin * 4 * Cout, device=dev)
    C.conv_wgrad(dyT, None, nhwc(x), 1, 0, 4 * Cout, slab, gw, 0, splits, 0)
    assert relerr(gw.view(Cin, 2, 2, Cout).permute(0, 3, 1, 2), Wr.grad) < 1e-2
    dx = torch.empty(N, h, w, Cin, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(dyT, None, wphys, 1, 0, dx, None, None, 0, None, 0)
    assert relerr(nchw(dx), xr.grad) < 1e-2


@pytest.mark.parametrize("N,h,w,Cin,Cout,H2,W2", [(4, 64, 64, 512, 256, 128, 128), (2, 128, 128, 128, 64, 256, 256),
                                                 (4, 64, 64, 256, 256, 129, 130)])
def test_conv_upT_fwd_fused(C, N, h, w, Cin, Cout, H2, W2):
    """ConvTranspose2d(k=2, s=2) + bias with the sub-pixel scatter in the ping-pong GEMM epilogue (both
    tile widths, padded placement) vs torch fp32 and vs the unfused GEMM + upT_shuffle."""
    torch.manual_seed(7)
    dev = "cuda"
    x = bf(torch.randn(N, Cin, h, w, device=dev))
    W = bf(torch.randn(Cin, Cout, 2, 2, device=dev) / math.sqrt(Cin))
    b = torch.randn(Cout, device=dev)
    oy, ox = (H2 - 2 * h) // 2, (W2 - 2 * w) // 2
    ref = F.pad(F.conv_transpose2d(x.float(), W.float(), b, stride=2), [ox, W2 - 2 * w - ox, oy, H2 - 2 * h - oy])
    wt = W.permute(0, 2, 3, 1).reshape(Cin, 4 * Cout).t().contiguous()  # [(dh, dw, co)][ci]
    u = torch.zeros(N, H2, W2, Cout, dtype=torch.bfloat16, device=dev)
    assert C.conv_upT_fwd(nhwc(x), wt, b, u, oy, ox) == 0
    torch.cuda.synchronize()
    assert relerr(nchw(u), ref) < 1e-2
    yT = torch.empty(N, h, w, 4 * Cout, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(nhwc(x), None, wt, 1, 0, yT, None, None, 0, None, 0)
    u2 = torch.zeros_like(u)
    C.upT_shuffle(yT, b, u2, oy, ox)
    # one rounding of (acc + bias): within half a bf16 ulp of the fp32 result everywhere (the unfused path
    # rounds twice), and never further from it overall than the unfused path
    r = nhwc(ref).float()
    assert float(((u.float() - r).abs() - r.abs() * 2 ** -8).max()) < 1e-3
    assert relerr(nchw(u), ref) <= relerr(nchw(u2), ref) * 1.01
    # a grid that would not fill the chip declines (the caller runs GEMM + shuffle)
    assert C.conv_upT_fwd(nhwc(x[:1, :, :8, :8].contiguous()), wt, b, torch.zeros(1, 16, 16, Cout, dtype=torch.bfloat16,
                                                                                   device=dev), 0, 0) == -1


@pytest.mark.parametrize("N,h,w,Cin,Cout", [(8, 64, 64, 512, 256), (4, 128, 128, 128, 64), (8, 64, 64, 256, 128),
                                           (2, 8, 8, 256, 128)])
def test_conv_upT_backward_in_place(C, N, h, w, Cin, Cout):
    """ConvTranspose2d(k=2, s=2) backward read straight from du's 2x2 sub-pixels: input gradient on the
    ping-pong kernel with 4 sub-pixel taps (both tile widths; a grid too small to fill the chip
    declines), weight gradient on the generic wgrad kernel, bias as column sums -- vs torch fp32, and
    the input gradient bitwise vs unshuffle + 1x1 GEMM."""
    torch.manual_seed(8)
    dev = "cuda"
    x = bf(torch.randn(N, Cin, h, w, device=dev))
    W = bf(torch.randn(Cin, Cout, 2, 2, device=dev) / math.sqrt(Cin))
    b = torch.randn(Cout, device=dev)
    xr = x.float().requires_grad_(True)
    Wr = W.float().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    du = bf(torch.randn(N, Cout, 2 * h, 2 * w, device=dev))
    F.conv_transpose2d(xr, Wr, br, stride=2).backward(du.float())
    wd = W.permute(0, 2, 3, 1).reshape(Cin, 4 * Cout).contiguous()  # [ci][(dh, dw, co)]
    dun = nhwc(du)
    dx = torch.zeros(N, h, w, Cin, dtype=torch.bfloat16, device=dev)
    r = C.conv_upT_dgrad(dun, wd, dx, 0, 0)
    tiles = -(-N * h * w // 256) * (Cin // 128)
    assert r == (0 if tiles >= 256 else -1)
    dyT = torch.empty(N, h, w, 4 * Cout, dtype=torch.bfloat16, device=dev)
    C.upT_unshuffle(dun, dyT, 0, 0)
    dx2 = torch.empty_like(dx)
    C.conv_fwd(dyT, None, wd, 1, 0, dx2, None, None, 4 if Cin % 256 == 0 and tiles >= 512 else 5, None, 0)
    if r == 0:
        assert relerr(nchw(dx), xr.grad) < 1e-2
        assert torch.equal(dx, dx2)  # same kernel, same K order: only the A operand's addresses differ
    M = N * h * w
    splits = max(1, min(512, M // 2048))
    slab = torch.zeros(C.wgrad_slab_elems(N, h, w, 4 * Cout, Cin, 1, 0, splits), device=dev)
    gw = torch.zeros(Cin * 4 * Cout, device=dev)
    assert C.conv_wgrad_upT(dun, nhwc(x), 0, 0, slab, gw, 0, splits) > 0
    assert relerr(gw.view(Cin, 2, 2, Cout).permute(0, 3, 1, 2), Wr.grad) < 1e-2
    gw2 = torch.zeros_like(gw)
    C.conv_wgrad(dyT, None, nhwc(x), 1, 0, 4 * Cout, slab, gw2, 0, splits, 0)
    assert torch.equal(gw, gw2)
    db = torch.zeros(Cout, device=dev)
    C.colsum_bf16(dun, 1, torch.zeros((1024 * 4 + 64) * Cout, device=dev), db, 0)
    assert torch.allclose(db, br.grad, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [(1, 16, 16, 512, 0, 512), (1, 8, 8, 256, 256, 256),
                                              (2, 7, 9, 128, 0, 64), (1, 32, 32, 256, 0, 128),
                                              (1, 64, 64, 128, 0, 256), (1, 64, 64, 256, 0, 256),
                                              (1, 128, 128, 128, 128, 64)])
def test_conv_splitk(C, N, H, W, C1, C2, Cout):
    """Split-K path (small M, large K) with the stats epilogue, the BN-fold epilogue and split output;
    the slices reduce in conv_splitk_reduce_kernel."""
    _splitk_case(C, N, H, W, C1, C2, Cout)


def _splitk_case(C, N, H, W, C1, C2, Cout):
    torch.manual_seed(6)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wk = ohwi(w).contiguous()
    n_ws = C.conv_ws_elems(N, H, W, C1, C2, Cout, 9, 0, 0)
    assert n_ws > 0, "shape should take the split-K path"
    ws = torch.zeros(n_ws, device=dev)
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.conv2d(xin, w.float(), padding=1)
    rows = C.conv_stats_rows(N * H * W, Cout, 0)
    stats = torch.zeros(rows * 2 * Cout, device=dev)
    y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    r = C.conv_fwd(x1, x2, wk, 9, 0, y, None, stats, 0, None, 0, ws)
    assert 0 < r <= rows
    assert relerr(nchw(y), ref) < 1e-2
    assert torch.count_nonzero(ws[:256]) == 0  # split-K arrival counters are reset by the last arriver
    yb = torch.empty_like(y)
    C.conv_fwd(x1, x2, wk, 9, 0, yb, None, None, 0, None, 0, ws)
    assert torch.equal(yb, y)  # slices summed in split order whichever arrives last
    yq = nchw(y).float()
    s = stats.view(rows, 2, Cout)[:r].sum(0)
    assert torch.allclose(s[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(s[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    # BN fold + ReLU
    g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    a = torch.empty_like(y)
    C.conv_fwd(x1, x2, wk, 9, 0, a, None, None, 0, coef, 1, ws)
    assert relerr(nchw(a), F.relu(F.batch_norm(ref, rm, rv, g, b, False, 0.0, 1e-5))) < 1e-2
    # split destinations
    y1 = torch.empty(N, H, W, Cout // 2, dtype=torch.bfloat16, device=dev)
    y2 = torch.empty(N, H, W, Cout // 2, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x1, x2, wk, 9, 0, y1, y2, None, 0, None, 0, ws)
    assert relerr(torch.cat([nchw(y1), nchw(y2)], 1), ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [(1, 64, 64, 256, 0, 256), (1, 32, 32, 512, 0, 512),
                                              (1, 128, 128, 128, 0, 128), (2, 16, 16, 256, 256, 512),
                                              (1, 256, 256, 64, 0, 128), (1, 256, 256, 64, 0, 64),
                                              (2, 64, 128, 64, 0, 64), (1, 24, 40, 64, 0, 64),
                                              # batched serving (N = 4): split-K ping-pong + eval reduce
                                              (4, 32, 32, 512, 0, 512)])
def test_conv_eval_fused_pool(C, N, H, W, C1, C2, Cout):
    """Eval conv (BN fold + ReLU) with ``pool=``: MaxPool2d(2) fused into the split-K reduce (deep
    serving shapes), into the row-ring epilogue (64 -> 64, W % 64 == 0) or launched after the conv
    (the rest) -- bitwise the pool of the output."""
    torch.manual_seed(9)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wk = ohwi(w).contiguous()
    n_ws = C.conv_ws_elems(N, H, W, C1, C2, Cout, 9, 0, 0)
    ws = torch.zeros(n_ws, device=dev) if n_ws else None
    g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    a = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    p = torch.full((N, H // 2, W // 2, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x1, x2, wk, 9, 0, a, None, None, 0, coef, 1, ws, p)
    a2 = torch.empty_like(a)
    C.conv_fwd(x1, x2, wk, 9, 0, a2, None, None, 0, coef, 1, ws)
    assert torch.equal(a, a2)
    assert torch.equal(p, F.max_pool2d(nchw(a).float(), 2).to(torch.bfloat16).permute(0, 2, 3, 1))
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.relu(F.batch_norm(F.conv2d(xin, w.float(), padding=1), rm, rv, g, b, False, 0.0, 1e-5))
    assert relerr(nchw(a), ref) < 1e-2


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pad", [(1, 16, 16, 512, 0, 512, 0), (1, 32, 32, 512, 512, 256, 0),
                                                   (1, 64, 64, 256, 256, 128, 1), (2, 16, 16, 256, 0, 256, 1),
                                                   (1, 128, 128, 128, 128, 64, 0), (4, 32, 32, 512, 512, 512, 0)])
def test_conv_eval_fused_upsample(C, N, H, W, C1, C2, Cout, pad):
    """Eval conv (BN fold + ReLU) with ``up=``: the decoder's bilinear x2 upsample (align_corners,
    centred pad) fused into the split-K reduce (maps of <= 16^2 pixels; larger ones take the separate
    launch) == conv_fwd + upsample2_fwd (y bitwise; the upsample to within one bf16 rounding of the
    interpolation: FMA contraction may differ between the kernels)."""
    torch.manual_seed(11)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wk = ohwi(w).contiguous()
    n_ws = C.conv_ws_elems(N, H, W, C1, C2, Cout, 9, 0, 0)
    assert n_ws > 0
    ws = torch.zeros(n_ws, device=dev)
    g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    Hu, Wu = 2 * H + 2 * pad, 2 * W + 2 * pad
    a = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
    u = torch.full((N, Hu, Wu, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x1, x2, wk, 9, 0, a, None, None, 0, coef, 1, ws, None, u, pad, pad)
    a2 = torch.empty_like(a)
    C.conv_fwd(x1, x2, wk, 9, 0, a2, None, None, 0, coef, 1, ws)
    assert torch.equal(a, a2)
    u2 = torch.full_like(u, float("nan"))
    C.upsample2_fwd(a2, u2, pad, pad)
    assert not torch.isnan(u.float()).any()
    d = (u.float() - u2.float()).abs()
    assert (d <= 2 ** -7 * u2.float().abs() + 1e-6).all(), d.max()
    assert (u == u2).float().mean() > 0.99
    ref = F.interpolate(nchw(a2).float(), scale_factor=2, mode="bilinear", align_corners=True)
    assert relerr(nchw(u)[:, :, pad:pad + 2 * H, pad:pad + 2 * W], ref) < 1e-2


@pytest.mark.parametrize("N,H,W", [(1, 256, 256), (2, 64, 128), (1, 128, 64)])
def test_conv_head_mask_fused(C, N, H, W):
    """Serving: last conv (64 -> 64, BN fold + ReLU) + 1x1 head + threshold in the row-ring epilogue ==
    conv_fwd(eval) + head_mask, except pixels whose logit is within rounding of the threshold."""
    torch.manual_seed(10)
    dev = "cuda"
    x = bf(torch.randn(N, H, W, 64, device=dev))
    w = bf(torch.randn(64, 64, 3, 3, device=dev) / math.sqrt(9 * 64))
    wk = ohwi(w).contiguous()
    g, b = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.5
    rm, rv = torch.randn(64, device=dev) * 0.1, torch.rand(64, device=dev) + 0.5
    coef = torch.zeros(4 * 64, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    hw = torch.randn(64, device=dev) * 0.3
    hb = torch.randn(1, device=dev) * 0.1
    a = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x, None, wk, 9, 0, a, None, None, 0, coef, 1)
    ref = torch.full((N * H * W,), 7, dtype=torch.uint8, device=dev)
    C.head_mask(a, hw, hb, 0.0, ref)
    got = torch.full((N * H * W,), 7, dtype=torch.uint8, device=dev)
    assert C.conv_head_mask(x, wk, coef, hw, hb, 0.0, got)
    logit = a.float().reshape(-1, 64) @ hw + hb
    diff = got != ref
    assert (got <= 1).all()
    assert (logit[diff].abs() < 1e-3).all(), logit[diff].abs().max()
    assert diff.float().mean() < 1e-3
    # not applicable (W % 64 != 0): nothing launched, caller falls back
    xs = bf(torch.randn(1, 16, 24, 64, device=dev))
    assert not C.conv_head_mask(xs, wk, coef, hw, hb, 0.0, got)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pref", [(1, 64, 64, 256, 0, 256, 0), (1, 16, 16, 512, 0, 512, 0),
                                                   (4, 256, 256, 64, 0, 128, 0), (2, 33, 47, 64, 64, 64, 0),
                                                   (1, 64, 64, 128, 0, 128, 128), (1, 64, 64, 128, 0, 64, 256)])
def test_conv_tiles_and_split_reduce(C, N, H, W, C1, C2, Cout, pref):
    """The double-buffered K pipeline against fp32 torch, stats and output: covers the split-K reduce,
    persistent blocks walking several tiles (4 x 256^2) and the forced 4-wave tiles; the same launch
    twice is bitwise reproducible."""
    torch.manual_seed(8)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wk = ohwi(w).contiguous()
    n_ws = C.conv_ws_elems(N, H, W, C1, C2, Cout, 9, 0, pref)
    ws = torch.zeros(max(n_ws, 1), device=dev) if n_ws else None
    rows = C.conv_stats_rows(N * H * W, Cout, pref)
    outs = []
    for _ in range(2):
        y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(rows * 2 * Cout, device=dev)
        r = C.conv_fwd(x1, x2, wk, 9, 0, y, None, stats, pref, None, 0, ws)
        outs.append((y, stats.view(rows, 2, Cout)[:r].sum(0)))
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.conv2d(xin, w.float(), padding=1)
    assert relerr(nchw(outs[0][0]), ref) < 1e-2
    for y, s in outs[1:]:
        assert torch.equal(y, outs[0][0])
        assert torch.allclose(s, outs[0][1], rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [(2, 16, 16, 128, 0, 128), (1, 9, 13, 64, 64, 256)])
def test_conv_fwd_8wave_variant(C, N, H, W, C1, C2, Cout):
    """bm_pref=2: 128x128 tiles with 8 waves (64x32 per wave) == the 4-wave kernel's result."""
    torch.manual_seed(7)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    rows = C.conv_stats_rows(N * H * W, Cout, 0)
    outs = []
    for pref in (128, 2):
        y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(rows * 2 * Cout, device=dev)
        r = C.conv_fwd(x1, x2, ohwi(w).contiguous(), 9, 0, y, None, st, pref, None, 0)
        outs.append((y, st[: r * 2 * Cout].view(r, 2, Cout).sum(0)))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("N,H,W,Cin,Cout,pref", [(4, 32, 32, 512, 1024, 4), (3, 20, 52, 256, 512, 5),
                                                  (16, 64, 64, 64, 256, 0)])
def test_conv_pingpong_1x1(C, N, H, W, Cin, Cout, pref):
    """The ping-pong kernel on 1x1 GEMMs (the transposed decoder's ConvTranspose2d as taps=1, dgrad of
    it too): bitwise equal to the 128 x 128 kernel; pref 0 = auto (>= 256 tiles of 256 x 256)."""
    torch.manual_seed(12)
    dev = "cuda"
    x = bf(torch.randn(N, H, W, Cin, device=dev))
    w = bf(torch.randn(Cout, Cin, device=dev) / math.sqrt(Cin))
    ys = []
    for p in (128, pref):
        y = torch.empty(N, H, W, Cout, dtype=torch.bfloat16, device=dev)
        C.conv_fwd(x, None, w, 1, 0, y, None, None, p, None, 0)
        ys.append(y)
    ref = torch.einsum("nhwc,oc->nhwo", x.float(), w.float())
    assert relerr(ys[1], ref) < 1e-2
    assert torch.equal(ys[0], ys[1])


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pref", [
    (2, 32, 32, 256, 0, 256, 4), (3, 37, 29, 128, 0, 256, 4), (1, 24, 40, 128, 128, 256, 4),
    (1, 24, 40, 128, 128, 256, 5), (20, 64, 64, 64, 0, 128, 5), (5, 64, 64, 256, 0, 512, 4),
    (2, 16, 16, 512, 512, 1024, 4), (9, 32, 32, 64, 64, 128, 5)])
def test_conv_pingpong_bitwise(C, N, H, W, C1, C2, Cout, pref):
    """bm_pref 4 / 5: the ping-pong 256 x 256 / 256 x 128 kernel (one 8-wave block per CU, staggered
    wave groups, 2-3 stage ring) accumulates in the same K order as the 128 x 128 kernel: outputs
    bitwise equal, BN partial sums equal to rounding; covers persistent blocks walking several tiles
    (320 / 640 tiles), a ragged last tile (M = 3219), the concat input and 1024 couts."""
    torch.manual_seed(11)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wk = ohwi(w).contiguous()
    rows = C.conv_stats_rows(N * H * W, Cout, 0)
    outs = []
    prefs = (128, pref)
    for p in prefs:
        y = torch.full((N, H, W, Cout), 7.0, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(rows * 2 * Cout, device=dev)
        r = C.conv_fwd(x1, x2, wk, 9, 0, y, None, st, p, None, 0)
        assert 0 < r <= rows
        outs.append((y, st[: r * 2 * Cout].view(r, 2, Cout).sum(0)))
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.conv2d(xin, w.float(), padding=1)
    assert relerr(nchw(outs[1][0]), ref) < 1e-2
    for y, s in outs[1:]:
        assert torch.equal(outs[0][0], y)
        assert torch.allclose(outs[0][1], s, rtol=1e-4, atol=1e-2)
    # dgrad form: one input, output split at a concat boundary (y1 | y2)
    if C2:
        d1 = torch.zeros(N, H, W, C1, dtype=torch.bfloat16, device=dev)
        d2 = torch.zeros(N, H, W, C2, dtype=torch.bfloat16, device=dev)
        dy = bf(torch.randn(N, H, W, Cout, device=dev))
        wt = bf(torch.randn(C1 + C2, Cout * 9, device=dev) / math.sqrt(9 * Cout))
        e1, e2 = torch.empty_like(d1), torch.empty_like(d2)
        C.conv_fwd(dy, None, wt, 9, 0, e1, e2, None, 128, None, 0)
        for p in prefs[1:]:
            d1.zero_()
            d2.zero_()
            C.conv_fwd(dy, None, wt, 9, 0, d1, d2, None, p, None, 0)
            assert torch.equal(d1, e1) and torch.equal(d2, e2)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pref", [
    (4, 32, 32, 512, 512, 512, 7), (4, 32, 32, 512, 0, 512, 7), (4, 64, 64, 256, 256, 256, 7),
    (4, 32, 32, 512, 0, 512, 8), (4, 32, 32, 256, 0, 512, 0), (5, 37, 29, 256, 0, 512, 7),
    (4, 32, 32, 512, 0, 256, 0)])
def test_conv_pingpong_splitk(C, N, H, W, C1, C2, Cout, pref):
    """bm_pref 7 / 8 (and auto at the reference batch): the ping-pong kernel with K split over work
    items (fp32 partial tiles + conv_splitk_reduce_kernel) vs fp32 torch: output, BN partial sums, a
    ragged last tile (M = 5365), the concat input, split destinations (dgrad) and the eval BN fold;
    two launches bitwise equal."""
    torch.manual_seed(13)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wk = ohwi(w).contiguous()
    n_ws = C.conv_ws_elems(N, H, W, C1, C2, Cout, 9, 0, pref)
    assert n_ws > 0, "shape should have a split-K plan"
    ws = torch.full((n_ws,), float("nan"), device=dev)  # every slab element is written before it is read
    rows = C.conv_stats_rows(N * H * W, Cout, pref)
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.conv2d(xin, w.float(), padding=1)
    ys = []
    for _ in range(2):
        y = torch.full((N, H, W, Cout), 7.0, dtype=torch.bfloat16, device=dev)
        st = torch.zeros(rows * 2 * Cout, device=dev)
        r = C.conv_fwd(x1, x2, wk, 9, 0, y, None, st, pref, None, 0, ws)
        assert 0 < r <= rows
        ys.append((y, st[: r * 2 * Cout].view(r, 2, Cout).sum(0)))
    y, s = ys[0]
    assert relerr(nchw(y), ref) < 1e-2
    assert torch.equal(ys[1][0], y)
    yq = nchw(y).float()
    assert torch.allclose(s[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(s[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    # split destinations (the dgrad of a concat input)
    y1 = torch.empty(N, H, W, Cout // 2, dtype=torch.bfloat16, device=dev)
    y2 = torch.empty(N, H, W, Cout // 2, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x1, x2, wk, 9, 0, y1, y2, None, pref if pref else 7, None, 0, ws)
    assert torch.equal(torch.cat([y1, y2], 3), y)
    # eval BN fold + ReLU through the same reduce
    if pref:
        g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
        rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
        coef = torch.zeros(4 * Cout, device=dev)
        C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
        a = torch.empty_like(y)
        C.conv_fwd(x1, x2, wk, 9, 0, a, None, None, pref, coef, 1, ws)
        assert relerr(nchw(a), F.relu(F.batch_norm(ref, rm, rv, g, b, False, 0.0, 1e-5))) < 1e-2


@pytest.mark.parametrize("N,H,W", [(2, 6, 64), (1, 4, 128), (3, 2, 192), (1, 10, 64)])
def test_conv_ring_fwd_stats_eval_dgrad(C, N, H, W):
    """Row-ring kernel (64 -> 64, W % 64 == 0): forward + BN stats, eval BN fold + ReLU, and the
    dgrad use (conv of dy with the flipped transposed weight) against torch fp32; forced (pref 6)
    and via the auto dispatch, which must pick it and agree bitwise."""
    torch.manual_seed(11)
    dev = "cuda"
    x = bf(torch.randn(N, H, W, 64, device=dev))
    w = bf(torch.randn(64, 64, 3, 3, device=dev) / 24)
    ref = F.conv2d(nchw(x).float(), w.float(), padding=1)
    rows = C.conv_stats_rows(N * H * W, 64, 0)
    outs = []
    for pref in (6, 0):
        y = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(rows * 2 * 64, device=dev)
        r = C.conv_fwd(x, None, ohwi(w).contiguous(), 9, 0, y, None, stats, pref, None, 0)
        assert 0 < r <= rows
        assert relerr(nchw(y), ref) < 1e-2
        yq = nchw(y).float()
        s = stats.view(rows, 2, 64)[:r].sum(0)
        assert torch.allclose(s[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        assert torch.allclose(s[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        outs.append(y)
    assert torch.equal(outs[0], outs[1])
    # eval: BN fold + ReLU in the epilogue (affine block [mean | invstd | scale | shift])
    sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1
    aff = torch.cat([torch.zeros(64, device=dev), torch.ones(64, device=dev), sc, sh])
    ye = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x, None, ohwi(w).contiguous(), 9, 0, ye, None, None, 6, aff, 1)
    refe = torch.relu(ref * sc[None, :, None, None] + sh[None, :, None, None])
    assert relerr(nchw(ye), refe) < 1e-2
    # dgrad: dX = conv(dY, flip(W)^T)
    dy = bf(torch.randn(N, H, W, 64, device=dev))
    xr = nchw(x).float().requires_grad_(True)
    F.conv2d(xr, w.float(), padding=1).backward(nchw(dy).float())
    wt = w.flip(2, 3).permute(1, 2, 3, 0).reshape(64, 9 * 64).contiguous()
    dx = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(dy, None, wt, 9, 0, dx, None, None, 6, None, 0)
    assert relerr(nchw(dx), xr.grad) < 1e-2


@pytest.mark.parametrize("N,H,W", [(2, 6, 64), (1, 4, 128), (3, 2, 192), (1, 10, 64), (4, 64, 128)])
@pytest.mark.parametrize("form", ["concat", "one128"])
def test_conv_ring2_128_to_64(C, N, H, W, form):
    """Two-source row ring (128 -> 64, K split over wave pairs that meet in LDS): up4 conv0 on the concat
    [skip, up] (two 64-channel sources) and up3 conv1 on one 128-channel tensor (its two halves), forward +
    BN partial sums and eval BN fold + ReLU, against torch fp32; forced (pref 14) == auto dispatch where
    the grid fills the chip (>= 256 row pairs) bitwise."""
    torch.manual_seed(13)
    dev = "cuda"
    if form == "concat":
        x1, x2 = bf(torch.randn(N, H, W, 64, device=dev)), bf(torch.randn(N, H, W, 64, device=dev))
        xin = torch.cat([x1, x2], -1)
    else:
        x1, x2 = bf(torch.randn(N, H, W, 128, device=dev)), None
        xin = x1
    w = bf(torch.randn(64, 128, 3, 3, device=dev) / 34)
    wk = ohwi(w).contiguous()
    ref = F.conv2d(nchw(xin).float(), w.float(), padding=1)
    rows = C.conv_stats_rows(N * H * W, 64, 0)
    auto = N * (W // 64) * H // 2 >= 256
    outs = []
    for pref in ((14, 0) if auto else (14,)):
        y = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(rows * 2 * 64, device=dev)
        r = C.conv_fwd(x1, x2, wk, 9, 0, y, None, stats, pref, None, 0)
        assert 0 < r <= rows
        assert relerr(nchw(y), ref) < 1e-2
        yq = nchw(y).float()
        st = stats.view(rows, 2, 64)[:r].sum(0)
        assert torch.allclose(st[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        assert torch.allclose(st[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        outs.append(y)
    if auto:
        assert torch.equal(outs[0], outs[1])
    # the implicit GEMM (256 x 64 tile) computes the same conv: equal up to fp32 summation order
    yi = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x1, x2, wk, 9, 0, yi, None, torch.zeros(rows * 2 * 64, device=dev), 256, None, 0)
    assert relerr(nchw(outs[0]), nchw(yi).float()) < 1e-2
    # eval: BN fold + ReLU in the epilogue
    sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1
    aff = torch.cat([torch.zeros(64, device=dev), torch.ones(64, device=dev), sc, sh])
    ye = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x1, x2, wk, 9, 0, ye, None, None, 14, aff, 1)
    assert relerr(nchw(ye), torch.relu(ref * sc[None, :, None, None] + sh[None, :, None, None])) < 1e-2


@pytest.mark.parametrize("N,H,W,form", [(2, 8, 128, "one"), (1, 6, 64, "concat")])
def test_conv_ring2_128_to_128_halves(C, N, H, W, form):
    """128 -> 128 as two two-source-ring launches over the output-channel halves (bm_pref 15): output,
    BN partial rows ([rows][2][128], each launch filling its 64 columns) and the eval epilogue vs torch
    fp32; each half bitwise equal to the 128 -> 64 ring on that half's weights."""
    torch.manual_seed(17)
    dev = "cuda"
    if form == "concat":
        x1, x2 = bf(torch.randn(N, H, W, 64, device=dev)), bf(torch.randn(N, H, W, 64, device=dev))
        xin = torch.cat([x1, x2], -1)
    else:
        x1, x2 = bf(torch.randn(N, H, W, 128, device=dev)), None
        xin = x1
    w = bf(torch.randn(128, 128, 3, 3, device=dev) / 34)
    wk = ohwi(w).contiguous()
    ref = F.conv2d(nchw(xin).float(), w.float(), padding=1)
    rows = C.conv_stats_rows(N * H * W, 128, 0)
    y = torch.empty(N, H, W, 128, dtype=torch.bfloat16, device=dev)
    stats = torch.zeros(rows * 2 * 128, device=dev)
    r = C.conv_fwd(x1, x2, wk, 9, 0, y, None, stats, 15, None, 0)
    assert 0 < r <= rows
    assert relerr(nchw(y), ref) < 1e-2
    yq = nchw(y).float()
    st = stats.view(rows, 2, 128)[:r].sum(0)
    assert torch.allclose(st[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    for h in range(2):
        yh = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
        C.conv_fwd(x1, x2, wk[64 * h:64 * h + 64].contiguous(), 9, 0, yh, None, None, 14, None, 0)
        assert torch.equal(yh, y[..., 64 * h:64 * h + 64])
    sc, sh = torch.rand(128, device=dev) + 0.5, torch.randn(128, device=dev) * 0.1
    aff = torch.cat([torch.zeros(128, device=dev), torch.ones(128, device=dev), sc, sh])
    ye = torch.empty(N, H, W, 128, dtype=torch.bfloat16, device=dev)
    C.conv_fwd(x1, x2, wk, 9, 0, ye, None, None, 15, aff, 1)
    assert relerr(nchw(ye), torch.relu(ref * sc[None, :, None, None] + sh[None, :, None, None])) < 1e-2


@pytest.mark.parametrize("N,H,W,split", [(2, 4, 64, False), (1, 6, 128, True), (2, 2, 64, True)])
def test_conv_ring_cout128(C, N, H, W, split):
    """Row-ring kernel with 128 outputs (down1 conv0 forward; up4 conv0 dgrad into the two halves of
    the concat input) + BN stats, against torch fp32; auto dispatch picks it and agrees bitwise."""
    torch.manual_seed(12)
    dev = "cuda"
    x = bf(torch.randn(N, H, W, 64, device=dev))
    w = bf(torch.randn(128, 64, 3, 3, device=dev) / 24)
    ref = F.conv2d(nchw(x).float(), w.float(), padding=1)
    rows = C.conv_stats_rows(N * H * W, 128, 0)
    outs = []
    for pref in (6, 0):
        stats = torch.zeros(rows * 2 * 128, device=dev)
        if split:
            y1 = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
            y2 = torch.empty(N, H, W, 64, dtype=torch.bfloat16, device=dev)
            r = C.conv_fwd(x, None, ohwi(w).contiguous(), 9, 0, y1, y2, stats, pref, None, 0)
            y = torch.cat([y1, y2], -1)
        else:
            y = torch.empty(N, H, W, 128, dtype=torch.bfloat16, device=dev)
            r = C.conv_fwd(x, None, ohwi(w).contiguous(), 9, 0, y, None, stats, pref, None, 0)
        assert 0 < r <= rows
        assert relerr(nchw(y), ref) < 1e-2
        yq = nchw(y).float()
        s = stats.view(rows, 2, 128)[:r].sum(0)
        assert torch.allclose(s[0], yq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        assert torch.allclose(s[1], (yq * yq).sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
        outs.append(y)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("nbytes", [1, 15, 16, 17, 4096 + 7, 640 * 480 * 3, 640 * 480 * 2 + 3])
def test_h2d_copy_kernel(C, nbytes):
    """The serving frame upload kernel (rdp_h2d_copy): pinned host bytes -> device, 16-B chunks + tail."""
    src = torch.randint(0, 256, (nbytes,), dtype=torch.uint8).pin_memory()
    dst = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    assert C.h2d_copy(src, dst) == 0
    torch.cuda.synchronize()
    assert torch.equal(dst.cpu(), src)


@pytest.mark.parametrize("decoder", ["bilinear", "transposed"])
def test_wprep_derived_layouts(C, decoder):
    """wprep (LDS-tiled transpose) rebuilds every derived bf16 weight layout from the fp32 masters."""
    from robotic_discovery_platform_amd.models.unet import UNetNative
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    m = UNetNative(3, 1, bilinear=(decoder == "bilinear"), device=dev)
    st = m.store
    st.flat.copy_(torch.randn_like(st.flat))
    m.refresh_weights()
    torch.cuda.synchronize()
    for sp in m.specs:
        w = st.flat_slice(sp.name + ".weight", st.flat).view(sp.cout, sp.taps, -1)  # OHWI master
        if sp.packed:
            ref = torch.zeros(sp.cout, 16, 8, device=dev)
            ref[:, :sp.taps, :w.shape[2]] = w
            got = m.fwd_weight(sp).view(sp.cout, 16, 8).float()
        else:
            ref = w.flip(1).permute(2, 1, 0).reshape(sp.cin, -1)  # [cin][flipped tap][cout]
            got = m.dgrad_weight(sp).float()
        assert torch.equal(got, bf(ref).float()), sp.name
    for us in m.up_specs:
        w = st.flat_slice(us.name + ".weight", st.flat).view(us.cin, 4 * us.cout)
        assert torch.equal(m.upT_fwd_weight(us).float(), bf(w.t()).float()), us.name


@pytest.mark.parametrize("N,H,W,Ch", [(2, 16, 16, 64), (1, 9, 13, 128), (3, 8, 6, 512)])
def test_bn_relu_pool_fusions(C, N, H, W, Ch):
    """Fused BN-apply+maxpool and maxpool-bwd+BN-reduce match the separate kernels (odd sizes too)."""
    torch.manual_seed(11)
    dev = "cuda"
    y = bf(torch.randn(N, H, W, Ch, device=dev) * 2 + 0.3)
    mean, inv = torch.randn(Ch, device=dev) * 0.1, torch.rand(Ch, device=dev) + 0.5
    gamma, beta = torch.randn(Ch, device=dev), torch.randn(Ch, device=dev) * 0.2
    ss = gamma * inv
    coef = torch.cat([mean, inv, ss, beta - mean * ss]).contiguous()
    # forward: apply + pool in one pass == apply, then pool
    a_ref = torch.empty_like(y)
    p_ref = torch.empty(N, H // 2, W // 2, Ch, dtype=torch.bfloat16, device=dev)
    C.bn_relu_apply(y, a_ref, coef, 1)
    C.maxpool2_fwd(a_ref, p_ref)
    a, p = torch.empty_like(y), torch.empty_like(p_ref)
    C.bn_relu_apply_pool(y, a, p, coef)
    assert torch.equal(a, a_ref) and torch.equal(p, p_ref)
    # backward: pool bwd (+ skip grad) fused with the BN reduce == pool bwd, then reduce
    dp = bf(torch.randn(N, H // 2, W // 2, Ch, device=dev))
    dskip = bf(torch.randn(N, H, W, Ch, device=dev))
    dx_ref = torch.empty_like(y)
    C.maxpool2_bwd(dp, a_ref, dskip, dx_ref)
    part_ref = torch.zeros(1024 * 2 * Ch, device=dev)
    T_ref = C.bn_relu_bwd_reduce(dx_ref, y, coef, 1, part_ref)
    dx = torch.empty_like(y)
    part = torch.zeros(1024 * 2 * Ch, device=dev)
    T = C.maxpool2_bwd_bn_reduce(dp, a_ref, dskip, dx, y, coef, part)
    assert torch.equal(dx, dx_ref)
    got = part[:T * 2 * Ch].view(T, 2, Ch).double().sum(0)
    ref = part_ref[:T_ref * 2 * Ch].view(T_ref, 2, Ch).double().sum(0)
    # exact fp32 reference of the same sums
    g = dx_ref.float() * ((y.float() * ss + (beta - mean * ss)) > 0)
    exact = torch.stack([g.sum((0, 1, 2)), (g * (y.float() - mean) * inv).sum((0, 1, 2))]).double()
    assert torch.allclose(got, exact, rtol=1e-3, atol=1e-3)
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("N,H,Cdy,Cdx", [(4, 32, 512, 256), (4, 16, 512, 512), (2, 8, 128, 64)])
def test_dgrad_splitk_bnred_matches_separate_reduce(C, N, H, Cdy, Cdx):
    """Split-K dgrad whose reduce also writes the owner BN layer's backward partial rows
    (conv_dgrad_splitk_bnred, csrc/conv_igemm.hip conv_splitk_reduce_kernel): dx bitwise the plain dgrad,
    the row sums equal bn_relu_bwd_reduce's and the fp32 sums of the same g."""
    torch.manual_seed(12)
    dev = "cuda"
    dy = bf(torch.randn(N, H, H, Cdy, device=dev))
    w = bf(torch.randn(Cdx, 9 * Cdy, device=dev) * 0.02)
    y = bf(torch.randn(N, H, H, Cdx, device=dev) * 2 + 0.3)
    mean, inv = torch.randn(Cdx, device=dev) * 0.1, torch.rand(Cdx, device=dev) + 0.5
    gamma, beta = torch.randn(Cdx, device=dev), torch.randn(Cdx, device=dev) * 0.2
    ss = gamma * inv
    coef = torch.cat([mean, inv, ss, beta - mean * ss]).contiguous()
    n_ws = C.conv_ws_elems(N, H, H, Cdy, 0, Cdx, 9, 0, 0)
    assert n_ws > 0  # these shapes run split-K
    ws = torch.zeros(n_ws, device=dev)
    dx = torch.empty(N, H, H, Cdx, dtype=torch.bfloat16, device=dev)
    part = torch.zeros(1024 * 2 * Cdx, device=dev)
    T = C.conv_dgrad_splitk_bnred(dy, w, dx, y, coef, part, ws)
    assert T > 0
    dx_ref = torch.empty_like(dx)
    C.conv_fwd(dy, None, w, 9, 0, dx_ref, None, None, 0, None, 0, ws)
    assert torch.equal(dx, dx_ref)
    part_ref = torch.zeros(1024 * 2 * Cdx, device=dev)
    T_ref = C.bn_relu_bwd_reduce(dx_ref, y, coef, 1, part_ref)
    got = part[:T * 2 * Cdx].view(T, 2, Cdx).double().sum(0)
    ref = part_ref[:T_ref * 2 * Cdx].view(T_ref, 2, Cdx).double().sum(0)
    g = dx_ref.float() * ((y.float() * ss + (beta - mean * ss)) > 0)
    exact = torch.stack([g.sum((0, 1, 2)), (g * (y.float() - mean) * inv).sum((0, 1, 2))]).double()
    scale = exact.abs().max().item()
    assert torch.allclose(got, exact, rtol=1e-3, atol=1e-4 * scale)
    assert torch.allclose(got, ref, rtol=1e-3, atol=1e-4 * scale)


@pytest.mark.parametrize("dice_w", [0.0, 1.0])
def test_head_bn_fused(C, dice_w):
    """BN-fused head (training): forward on the pre-BN y == BN apply then head; backward partials
    and the logit-recomputed dy == head bwd -> BN reduce -> BN apply of the separate kernels."""
    torch.manual_seed(12)
    dev = "cuda"
    N, H, W, Ch = 2, 36, 28, 64
    M = N * H * W
    y = bf(torch.randn(N, H, W, Ch, device=dev) * 2 + 0.3)
    mean, inv = torch.randn(Ch, device=dev) * 0.1, torch.rand(Ch, device=dev) + 0.5
    gamma, beta = torch.randn(Ch, device=dev), torch.randn(Ch, device=dev) * 0.2
    ss = gamma * inv
    coef = torch.cat([mean, inv, ss, beta - mean * ss]).contiguous()
    wt = torch.randn(64, device=dev) * 0.1
    b = torch.randn(1, device=dev) * 0.1
    t = (torch.rand(M, device=dev) > 0.5).float()
    nb = C.head_partial_blocks(M)

    def run_fwd(src, cf):
        lg, part = torch.zeros(M, device=dev), torch.zeros(nb * 65, device=dev)
        sums, loss = torch.zeros(4, device=dev), torch.zeros(2, device=dev)
        C.head_fwd(src, wt, b, t, lg, part, sums, loss, dice_w, 1.0, cf)
        return lg, part, sums, loss

    a = torch.empty_like(y)
    C.bn_relu_apply(y, a, coef, 1)
    lg_r, part_r, sums_r, loss_r = run_fwd(a, None)
    lg, part, sums, loss = run_fwd(y, coef)
    assert torch.equal(lg, lg_r) and torch.equal(loss, loss_r)
    # backward, separate kernels
    gs = 0.5
    da = torch.empty_like(y)
    gw_r, gb_r = torch.zeros(64, device=dev), torch.zeros(1, device=dev)
    C.head_bwd(a, wt, lg_r, t, sums_r, da, part_r, gw_r, gb_r, dice_w, 1.0, gs)
    bp_r = torch.zeros(1024 * 2 * Ch, device=dev)
    T_r = C.bn_relu_bwd_reduce(da, y, coef, 1, bp_r)
    ws = torch.zeros(64 * 2 * Ch, device=dev)
    dg_r, db_r, c2_r = torch.zeros(Ch, device=dev), torch.zeros(Ch, device=dev), torch.zeros(3 * Ch, device=dev)
    C.bn_bwd_finalize(bp_r, T_r, M, gamma, coef, dg_r, db_r, c2_r, ws)
    dy_r = torch.empty_like(y)
    C.bn_relu_bwd_apply(da, y, coef, c2_r, dy_r, 1)
    # fused
    gw, gb = torch.zeros(64, device=dev), torch.zeros(1, device=dev)
    bp = torch.zeros(nb * 128, device=dev)
    T = C.head_bwd(y, wt, lg, t, sums, None, part, gw, gb, dice_w, 1.0, gs, coef, bp)
    assert T == nb
    dg, db, c2 = torch.zeros(Ch, device=dev), torch.zeros(Ch, device=dev), torch.zeros(3 * Ch, device=dev)
    C.bn_bwd_finalize(bp, T, M, gamma, coef, dg, db, c2, ws)
    dy = torch.empty_like(y)
    C.head_bn_bwd_apply(y, wt, lg, t, sums, coef, c2, dy, dice_w, 1.0, gs)
    assert relerr(gw, gw_r) < 1e-5 and relerr(gb, gb_r) < 1e-5
    assert relerr(dg, dg_r) < 1e-4 and relerr(db, db_r) < 1e-4
    assert relerr(c2, c2_r) < 1e-4
    assert relerr(dy, dy_r) < 1e-2
    # and against an fp32 torch reference of the composite (BN train backward through ReLU)
    g = da.float() * ((y.float() * ss + (beta - mean * ss)) > 0)
    xh = (y.float() - mean) * inv
    exact_db, exact_dg = g.sum((0, 1, 2)), (g * xh).sum((0, 1, 2))
    assert relerr(db, exact_db) < 1e-3 and relerr(dg, exact_dg) < 1e-3
    dy_exact = gamma * inv * (g - exact_db / M - xh * exact_dg / M)
    assert relerr(dy, dy_exact) < 1e-2
    if dice_w == 0.0:  # BCE only: the forward can emit the backward partials itself
        lg2, part2 = torch.zeros(M, device=dev), torch.zeros(nb * 65, device=dev)
        sums2, loss2 = torch.zeros(4, device=dev), torch.zeros(2, device=dev)
        gp, bp2 = torch.zeros(nb * 65, device=dev), torch.zeros(nb * 128, device=dev)
        C.head_fwd(y, wt, b, t, lg2, part2, sums2, loss2, 0.0, 1.0, coef, gp, bp2, gs)
        assert torch.equal(lg2, lg) and torch.equal(loss2, loss)
        gw2, gb2 = torch.zeros(64, device=dev), torch.zeros(1, device=dev)
        C.head_grad_finalize(gp, M, gw2, gb2)
        assert relerr(gw2, gw) < 1e-5 and relerr(gb2, gb) < 1e-5
        got = bp2.view(nb, 2, Ch).double().sum(0)
        ref = bp.view(nb, 2, Ch).double().sum(0)
        assert torch.allclose(got, ref, rtol=1e-5, atol=1e-6)


def test_conv_batch_chunks_subprocess():
    """Batches past the kernels' 2 GiB buffer-offset reach run as image slices (conv_fwd appends the BN
    partial rows, conv_wgrad accumulates, conv_dgrad_bnred defers to the chunked fallback). The bound
    is lowered with RDP_CONV_CHUNK_BYTES (read once per process) in a child process so the chunked
    path runs on small tensors; results must match the unchunked launches of this process."""
    import os
    import subprocess
    import sys
    code = r'''
import math, sys, torch
sys.path.insert(0, sys.argv[1])
from robotic_discovery_platform_amd.ops import native
C = native()
torch.manual_seed(21)
dev = "cuda"
bf = lambda t: t.to(torch.bfloat16)
N, H, W = 5, 64, 64
x1 = bf(torch.randn(N, H, W, 64, device=dev)); x2 = bf(torch.randn(N, H, W, 64, device=dev))
w = bf(torch.randn(128, 9 * 128, device=dev) / 34.0)
y = torch.empty(N, H, W, 128, dtype=torch.bfloat16, device=dev)
rows = 8 * C.conv_stats_rows(N * H * W, 128, 0)  # 5 chunked launches: 5 x the per-launch floor
st = torch.zeros(rows * 2 * 128, device=dev)
r = C.conv_fwd(x1, x2, w, 9, 0, y, None, st, 0, None, 0)
dy = bf(torch.randn(N, H, W, 128, device=dev))
slab = torch.zeros(C.wgrad_slab_elems(N, H, W, 128, 128, 9, 0, 64), device=dev)
out = torch.zeros(128 * 9 * 128, device=dev)
C.conv_wgrad(x1, x2, dy, 9, 0, 0, slab, out, 0, 64, 0)
torch.save({"y": y.cpu(), "s": st[: r * 256].view(r, 2, 128).sum(0).cpu(), "g": out.cpu()}, sys.argv[2])
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for lim in ("0", str(2 * 64 * 64 * 128 * 2 - 1)):  # unchunked / 1 image per launch (5 launches)
        path = os.path.join("/tmp", f"rdp_chunk_{lim}_{os.getpid()}.pt")
        env = dict(os.environ, RDP_CONV_CHUNK_BYTES=lim, RDP_NO_BUILD="1")
        subprocess.run([sys.executable, "-c", code, root, path], check=True, env=env, timeout=240)
        outs.append(torch.load(path, weights_only=True))
        os.unlink(path)
    assert torch.equal(outs[0]["y"], outs[1]["y"])
    assert torch.allclose(outs[0]["s"], outs[1]["s"], rtol=1e-4, atol=1e-2)
    assert relerr(outs[1]["g"], outs[0]["g"]) < 1e-5



@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pool", [
    (1, 32, 32, 256, 0, 512, False), (1, 32, 32, 512, 0, 512, True), (1, 16, 16, 512, 0, 512, False),
    (1, 16, 16, 512, 0, 512, True), (1, 32, 32, 512, 512, 512, False), (1, 32, 32, 512, 0, 256, False),
    (1, 64, 64, 128, 0, 256, False), (1, 64, 64, 256, 0, 256, True), (2, 16, 16, 256, 256, 128, True),
    (1, 64, 64, 256, 256, 256, False), (3, 16, 32, 64, 64, 96, False)])
def test_conv_rowband_eval(C, N, H, W, C1, C2, Cout, pool):
    """Row-band eval conv (bm_pref 16; auto on small maps): BN fold + ReLU, concat input, fused
    MaxPool2d(2) -- vs fp32 torch, vs the split-K implicit GEMM (bm_pref 128) at bf16 rounding, and the
    pool bitwise the 2x2 max of the output."""
    torch.manual_seed(12)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wk = ohwi(w).contiguous()
    g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    a = torch.full((N, H, W, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    p = torch.full((N, H // 2, W // 2, Cout), float("nan"), dtype=torch.bfloat16, device=dev) if pool else None
    C.conv_fwd(x1, x2, wk, 9, 0, a, None, None, 16, coef, 1, None, p)
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.relu(F.batch_norm(F.conv2d(xin, w.float(), padding=1), rm, rv, g, b, False, 0.0, 1e-5))
    assert not torch.isnan(a.float()).any()
    assert relerr(nchw(a), ref) < 1e-2
    if Cout % 128 == 0:
        n_ws = C.conv_ws_elems(N, H, W, C1, C2, Cout, 9, 0, 128)
        ws = torch.zeros(max(n_ws, 1), device=dev)
        a2 = torch.empty_like(a)
        C.conv_fwd(x1, x2, wk, 9, 0, a2, None, None, 128, coef, 1, ws)
        d = (a.float() - a2.float()).abs()
        assert (d <= 2 ** -6 * a2.float().abs() + 1e-2).all(), d.max()
    if pool:
        assert torch.equal(p, F.max_pool2d(nchw(a).float(), 2).to(torch.bfloat16).permute(0, 2, 3, 1))
    # deterministic: a second launch is bitwise identical
    a3 = torch.empty_like(a)
    C.conv_fwd(x1, x2, wk, 9, 0, a3, None, None, 16, coef, 1)
    assert torch.equal(a, a3)


@pytest.mark.parametrize("N,nl", [(1, 2), (2, 3), (1, 4)])
def test_conv_rowband_chain(C, N, nl):
    """Persistent row-band chain (one launch, row readiness counters) == the same layers as separate
    row-band launches, bitwise; no bounded wait timed out."""
    torch.manual_seed(13)
    dev = "cuda"
    H = 16
    chans = [256, 512, 256, 512, 256][: nl + 1]
    x = bf(torch.randn(N, H, H, chans[0], device=dev))
    ws, coefs, ys, refs = [], [], [], []
    for l in range(nl):
        ci, co = chans[l], chans[l + 1]
        ws.append(bf(torch.randn(co, 9 * ci, device=dev) / math.sqrt(9 * ci)))
        cf = torch.zeros(4 * co, device=dev)
        C.bn_eval_coef(torch.rand(co, device=dev) + 0.5, torch.randn(co, device=dev) * 0.1,
                       torch.randn(co, device=dev) * 0.1, torch.rand(co, device=dev) + 0.5, 1e-5, cf)
        coefs.append(cf)
        ys.append(torch.full((N, H, H, co), float("nan"), dtype=torch.bfloat16, device=dev))
        refs.append(torch.empty(N, H, H, co, dtype=torch.bfloat16, device=dev))
    inp = x
    for w, r, cf in zip(ws, refs, coefs):
        C.conv_fwd(inp, None, w, 9, 0, r, None, None, 16, cf, 1)
        inp = r
    cnt = torch.full((1 + nl * N * H,), 7, dtype=torch.int32, device=dev)  # poisoned: the launch zeroes it
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(3):
        assert C.conv_rowband_chain(x, ws, ys, coefs, cnt, err)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        for y, r in zip(ys, refs):
            assert torch.equal(y, r)


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pool", [(1, 32, 32, 256, 0, 512, False), (1, 16, 16, 512, 0, 512, True),
                                                   (2, 64, 64, 128, 128, 128, False)])
def test_conv_rowband_frag_weights(C, N, H, W, C1, C2, Cout, pool):
    """conv_rowband on fragment-major weights == on OHWI weights, bitwise (same loads, other addresses)."""
    from robotic_discovery_platform_amd.models.unet import rowband_frag_weights
    torch.manual_seed(14)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, 9 * (C1 + C2), device=dev) / math.sqrt(9 * (C1 + C2)))
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev) * 0.1,
                   torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev), 1e-5, coef)
    outs = []
    for wk, fr in ((w, 0), (rowband_frag_weights(w), 1)):
        y = torch.full((N, H, W, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
        p = torch.full((N, H // 2, W // 2, Cout), float("nan"), dtype=torch.bfloat16, device=dev) if pool else None
        assert C.conv_rowband(x1, x2, wk, y, coef, p, fr) == (1 if pool else 0)
        outs.append((y, p))
    assert torch.equal(outs[0][0], outs[1][0])
    if pool:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("N,H,W,C1,C2,Cout,pool", [
    (1, 32, 32, 256, 0, 512, False), (1, 32, 32, 512, 0, 512, True), (1, 16, 16, 512, 0, 512, True),
    (1, 32, 32, 512, 512, 512, False), (1, 64, 64, 256, 0, 256, True), (1, 64, 64, 256, 256, 256, False),
    (2, 16, 32, 256, 0, 96, True), (1, 128, 128, 128, 0, 128, True), (1, 128, 128, 64, 0, 128, False),
    (1, 64, 64, 64, 64, 64, False), (2, 32, 32, 128, 0, 256, True)])
def test_conv_rowband_staged(C, N, H, W, C1, C2, Cout, pool):
    """Activation-staged row-band conv (conv_rowband mode 2, fragment-major weights): vs fp32 torch, the
    pool bitwise the 2x2 max of the output, the unpooled call bitwise the pooled one's output, and
    deterministic."""
    from robotic_discovery_platform_amd.models.unet import rowband_frag_weights
    torch.manual_seed(15)
    dev = "cuda"
    x1 = bf(torch.randn(N, H, W, C1, device=dev))
    x2 = bf(torch.randn(N, H, W, C2, device=dev)) if C2 else None
    w = bf(torch.randn(Cout, C1 + C2, 3, 3, device=dev) / math.sqrt(9 * (C1 + C2)))
    wf = rowband_frag_weights(ohwi(w).contiguous())
    g, b = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev)
    rm, rv = torch.randn(Cout, device=dev) * 0.1, torch.rand(Cout, device=dev) + 0.5
    coef = torch.zeros(4 * Cout, device=dev)
    C.bn_eval_coef(g, b, rm, rv, 1e-5, coef)
    a = torch.full((N, H, W, Cout), float("nan"), dtype=torch.bfloat16, device=dev)
    p = torch.full((N, H // 2, W // 2, Cout), float("nan"), dtype=torch.bfloat16, device=dev) if pool else None
    assert C.conv_rowband(x1, x2, wf, a, coef, p, 2) == (1 if pool else 0)
    xin = nchw(x1).float() if x2 is None else torch.cat([nchw(x1), nchw(x2)], 1).float()
    ref = F.relu(F.batch_norm(F.conv2d(xin, w.float(), padding=1), rm, rv, g, b, False, 0.0, 1e-5))
    assert not torch.isnan(a.float()).any()
    assert relerr(nchw(a), ref) < 1e-2
    if pool:
        assert torch.equal(p, F.max_pool2d(nchw(a).float(), 2).to(torch.bfloat16).permute(0, 2, 3, 1))
    a2 = torch.empty_like(a)
    assert C.conv_rowband(x1, x2, wf, a2, coef, None, 2) == 0
    assert torch.equal(a, a2)
