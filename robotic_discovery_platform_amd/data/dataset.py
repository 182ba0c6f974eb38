"""Segmentation datasets.

``SegmentationDataset`` reproduces ``/root/reference/scripts/train_segmenter.py:66-100``: images and
masks are paired by identical filename; colour is read as BGR, converted to RGB and resized with
INTER_AREA; the mask is read grayscale and resized with INTER_NEAREST; both are scaled by 1/255;
items are (float32 CHW image, float32 1HW mask).

``SyntheticSegmentationDataset`` serves procedurally generated scenes (no files needed), and
``split_dataset`` is a *seeded* random split (the reference's ``random_split`` is unseeded).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset, Subset

from .image_io import bgr2rgb, imread, imread_gray, resize_area, resize_nearest
from .synthetic import make_scene


class SegmentationDataset(Dataset):
    def __init__(self, image_dir: str, mask_dir: str, size: Tuple[int, int] = (256, 256), cache: bool = False):
        self.image_dir, self.mask_dir, self.size = image_dir, mask_dir, size
        self.ids: List[str] = sorted(f for f in os.listdir(image_dir) if os.path.isfile(os.path.join(mask_dir, f)))
        self._cache = {} if cache else None

    def __len__(self) -> int:
        return len(self.ids)

    def raw_arrays(self, idx: int) -> Tuple[np.ndarray, np.ndarray]:
        """(colour BGR u8 at file size, mask u8 at file size): input of the device-side resizes."""
        name = self.ids[idx]
        return imread(os.path.join(self.image_dir, name), color=True), imread_gray(os.path.join(self.mask_dir, name))

    def load_arrays(self, idx: int) -> Tuple[np.ndarray, np.ndarray]:
        name = self.ids[idx]
        img = imread(os.path.join(self.image_dir, name), color=True)
        img = resize_area(bgr2rgb(img), self.size)
        mask = resize_nearest(imread_gray(os.path.join(self.mask_dir, name)), self.size)
        return img, mask

    def __getitem__(self, idx: int):
        if self._cache is not None and idx in self._cache:
            return self._cache[idx]
        img, mask = self.load_arrays(idx)
        x = torch.from_numpy(img.astype(np.float32) / 255.0).permute(2, 0, 1).contiguous()
        y = torch.from_numpy(mask.astype(np.float32) / 255.0).unsqueeze(0)
        if self._cache is not None:
            self._cache[idx] = (x, y)
        return x, y


class SyntheticSegmentationDataset(Dataset):
    def __init__(self, n: int, size: Tuple[int, int] = (256, 256), seed: int = 0):
        self.n, self.size, self.seed = n, size, seed

    def __len__(self) -> int:
        return self.n

    def raw_arrays(self, idx: int) -> Tuple[np.ndarray, np.ndarray]:
        s = make_scene(self.seed + idx)
        return s.color, s.mask

    def __getitem__(self, idx: int):
        s = make_scene(self.seed + idx)
        img = resize_area(bgr2rgb(s.color), self.size)
        mask = resize_nearest(s.mask, self.size)
        x = torch.from_numpy(img.astype(np.float32) / 255.0).permute(2, 0, 1).contiguous()
        y = torch.from_numpy(mask.astype(np.float32) / 255.0).unsqueeze(0)
        return x, y


def split_dataset(ds: Dataset, val_fraction: float = 0.2, seed: int = 0) -> Tuple[Subset, Subset]:
    """random_split(ds, [n - int(n*f), int(n*f)]) with a fixed generator seed."""
    n = len(ds)
    n_val = int(n * val_fraction)
    g = torch.Generator().manual_seed(seed)
    perm = torch.randperm(n, generator=g).tolist()
    return Subset(ds, perm[: n - n_val]), Subset(ds, perm[n - n_val:])


def preload(ds: Dataset, indices: Optional[List[int]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Materialise (a subset of) a dataset as two stacked tensors (host)."""
    idx = list(range(len(ds))) if indices is None else indices
    xs, ys = zip(*(ds[i] for i in idx)) if idx else ((), ())
    if not idx:
        return torch.empty(0), torch.empty(0)
    return torch.stack(xs), torch.stack(ys)
