"""Plain-PyTorch U-Net: the CPU/eager oracle and the reference-compatible weight layout.

Behaviour matches ``/root/reference/pkg/segmentation_model.py:24-120``:

* ``DoubleConv``  = [conv3x3 pad1 (no bias) -> BN -> ReLU] x 2 with optional mid width (``:24-40``)
* ``Down``        = MaxPool2d(2) -> DoubleConv (``:42-52``)
* ``Up``          = upsample x2 -> zero-pad to the skip's H/W -> cat([skip, up]) -> DoubleConv (``:54-76``)
* ``OutConv``     = conv1x1 with bias (``:78-84``)
* ``UNet(n_channels, n_classes, bilinear=True)`` widths 64..1024//f (``:86-120``)

State-dict keys and shapes are identical to the reference's (110 keys for ``UNet(3, 1)``), so a
reference checkpoint loads here and vice versa.

Differences (documented in SURVEY.md §0/§7.5):
  * the transposed-conv decoder (``bilinear=False``) is *fixed*: the reference builds
    ``DoubleConv(in//2, out)`` but feeds it ``in`` channels after the concat (``:63-65``), which
    crashes; we build ``DoubleConv(in, out)``.
  * ``depth`` generalises the number of Down/Up levels (reference: 4) so the tiny 2-level
    plumbing config (BASELINE.json config 1) is the same class.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


class DoubleConv(nn.Sequential):
    """Two (conv3x3 -> BN -> ReLU) stages. Registered under ``.double_conv`` for key parity."""

    def __init__(self, cin: int, cout: int, cmid: Optional[int] = None):
        super().__init__()
        cmid = cmid or cout
        layers = []
        for a, b in ((cin, cmid), (cmid, cout)):
            layers += [nn.Conv2d(a, b, 3, padding=1, bias=False), nn.BatchNorm2d(b), nn.ReLU(inplace=True)]
        # nested Sequential keeps the reference's "<block>.double_conv.<i>" key names
        self.double_conv = nn.Sequential(*layers)

    def forward(self, x):  # noqa: D401
        return self.double_conv(x)


class Down(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.maxpool_conv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(cin, cout))

    def forward(self, x):
        return self.maxpool_conv(x)


def pad_to(x: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """Zero-pad (or crop, for negative diffs) NCHW ``x`` to ``ref``'s H/W; left/top get diff//2."""
    dy = ref.shape[-2] - x.shape[-2]
    dx = ref.shape[-1] - x.shape[-1]
    if dx == 0 and dy == 0:
        return x
    return F.pad(x, [dx // 2, dx - dx // 2, dy // 2, dy - dy // 2])


class Up(nn.Module):
    def __init__(self, cin: int, cout: int, bilinear: bool = True):
        super().__init__()
        if bilinear:
            self.up = nn.Upsample(scale_factor=2, mode="bilinear", align_corners=True)
            self.conv = DoubleConv(cin, cout, cin // 2)
        else:
            self.up = nn.ConvTranspose2d(cin, cin // 2, kernel_size=2, stride=2)
            # fixed channel math: skip (cin//2) + upsampled (cin//2) = cin channels
            self.conv = DoubleConv(cin, cout)

    def forward(self, x_low, skip):
        u = pad_to(self.up(x_low), skip)
        return self.conv(torch.cat([skip, u], dim=1))


class OutConv(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, kernel_size=1)

    def forward(self, x):
        return self.conv(x)


def unet_widths(base: int, depth: int, bilinear: bool) -> List[int]:
    """Encoder output widths: [inc, down1, ..., down_depth] (last one halved when bilinear)."""
    f = 2 if bilinear else 1
    w = [base * (2 ** i) for i in range(depth + 1)]
    w[-1] = w[-1] // f
    return w


class UNetRef(nn.Module):
    """Reference-architecture U-Net in plain torch ops (NCHW or channels_last)."""

    def __init__(self, n_channels: int = 3, n_classes: int = 1, bilinear: bool = True,
                 base_width: int = 64, depth: int = 4):
        super().__init__()
        self.n_channels, self.n_classes, self.bilinear = n_channels, n_classes, bilinear
        self.base_width, self.depth = base_width, depth
        f = 2 if bilinear else 1
        enc = unet_widths(base_width, depth, bilinear)
        self.inc = DoubleConv(n_channels, enc[0])
        for i in range(1, depth + 1):
            setattr(self, f"down{i}", Down(enc[i - 1], enc[i]))
        # decoder: up_i takes (full width at level depth-i+1) channels
        for i in range(1, depth + 1):
            lvl = depth - i  # skip level
            cin = base_width * (2 ** (lvl + 1))
            cout = base_width * (2 ** lvl) // (f if i < depth else 1)
            setattr(self, f"up{i}", Up(cin, cout, bilinear))
        self.outc = OutConv(base_width, n_classes)

    def forward(self, x):
        skips = [self.inc(x)]
        for i in range(1, self.depth + 1):
            skips.append(getattr(self, f"down{i}")(skips[-1]))
        y = skips[-1]
        for i in range(1, self.depth + 1):
            y = getattr(self, f"up{i}")(y, skips[self.depth - i])
        return self.outc(y)


def UNet(n_channels: int = 3, n_classes: int = 1, bilinear: bool = True, **kw) -> UNetRef:
    """Reference-signature constructor (``pkg/segmentation_model.py:86``)."""
    return UNetRef(n_channels, n_classes, bilinear, **kw)


def conv_flops_per_image(model: nn.Module, h: int = 256, w: int = 256) -> float:
    """Forward FLOPs (2*MAC) of all conv / transposed-conv layers for one HxW image."""
    total = 0.0
    hooks = []

    def hook(mod, inp, out):
        nonlocal total
        if isinstance(mod, nn.Conv2d):
            k = mod.in_channels // mod.groups * mod.kernel_size[0] * mod.kernel_size[1]
            total += 2.0 * k * out.numel() / out.shape[0]
        elif isinstance(mod, nn.ConvTranspose2d):
            k = mod.in_channels * mod.kernel_size[0] * mod.kernel_size[1]
            total += 2.0 * k * inp[0].numel() / inp[0].shape[0] / mod.in_channels * mod.out_channels

    for m in model.modules():
        if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)):
            hooks.append(m.register_forward_hook(hook))
    with torch.no_grad():
        was = model.training
        model.eval()
        model(torch.zeros(1, model.n_channels, h, w))
        model.train(was)
    for hk in hooks:
        hk.remove()
    return total
