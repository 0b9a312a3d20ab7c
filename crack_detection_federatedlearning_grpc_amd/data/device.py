"""HBM-resident synthetic dataset rendered on the GPU (``render_cracks`` kernel, csrc/kernels/datagen.hip).

Same geometry/texture definition as ``data/synthetic.py`` (host-drawn segment table, pure per-pixel render), so the
CPU renderer is the oracle for the HIP one. The whole dataset stays on the device: batches are index vectors.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .._native_loader import hip
from .synthetic import MAX_SEG, CrackDataset, image_params, reference_split


def render_device(n: int, img: int, seed: int = 0, device="cuda"):
    segs, par = image_params(n, img, seed)
    dev = torch.device(device)
    images = torch.empty(n, img, img, 3, dtype=torch.uint8, device=dev)
    masks = torch.empty(n, img, img, dtype=torch.uint8, device=dev)
    chunk = 1024
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        sg = torch.as_tensor(segs[s:e]).to(dev)
        pr = torch.as_tensor(par[s:e]).to(dev)
        hip().render_cracks(sg, pr, images[s:e], masks[s:e], e - s, img, MAX_SEG)
    return images, masks


def make_synthetic_device(n: int, img: int, seed: int = 0, split: Optional[int] = None, shuffle_seed: int = 1337,
                          device="cuda") -> CrackDataset:
    images, masks = render_device(n, img, seed, device)
    split = n if split is None else min(split, n)
    tr, va = reference_split(n, split, shuffle_seed)
    return CrackDataset(images, masks, tr, va)
