"""Synthetic crack-segmentation data (BASELINE.json: "synthetic crack-mask data / random-init weights").

The reference trains on a folder of concrete-crack JPEGs + masks at hard-coded paths (client_fit_model.py:58-59);
no dataset is available offline, so images are synthesised with the same shapes and statistics class:
a textured concrete-like background (integer-hash value noise) with one or two random-walk crack polylines of
varying thickness; the mask is the set of pixels within the crack half-width (binary, like ``mask > 0``
at client_fit_model.py:39).

The crack geometry (segment list) is drawn on the host from a seeded NumPy RNG; rasterisation is a pure function of
(segments, image params, pixel) so the NumPy renderer here and the HIP renderer (``csrc/kernels/datagen.hip``,
``ops.datagen``) produce identical bytes.
"""
from __future__ import annotations

import math
import random
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

MAX_SEG = 48          # segments per image (padded with zero-length segments)
SEG_FIELDS = 6        # x0, y0, x1, y1, half_width, unused


def image_params(n: int, img: int, seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Returns (segments float32 [n, MAX_SEG, 6], params float32 [n, 8]) for n images of size img x img."""
    rng = np.random.default_rng(seed)
    segs = np.zeros((n, MAX_SEG, SEG_FIELDS), np.float32)
    par = np.zeros((n, 8), np.float32)
    s = img / 128.0
    for i in range(n):
        k = 0
        n_cracks = 1 if rng.random() < 0.7 else 2
        for _ in range(n_cracks):
            x, y = rng.uniform(0.05, 0.95, 2) * img
            ang = rng.uniform(0, 2 * math.pi)
            hw = rng.uniform(0.7, 2.2) * s
            steps = int(rng.integers(8, 24))
            for _ in range(steps):
                if k >= MAX_SEG:
                    break
                ln = rng.uniform(img / 24, img / 10)
                ang += rng.normal(0, 0.45)
                nx, ny = x + ln * math.cos(ang), y + ln * math.sin(ang)
                hw = float(np.clip(hw * rng.uniform(0.85, 1.15), 0.5 * s, 3.0 * s))
                segs[i, k] = (x, y, nx, ny, hw, 0)
                k += 1
                x, y = nx, ny
        bg = rng.uniform(110, 200)
        par[i] = (bg, rng.uniform(20, 60), rng.uniform(25, 80), rng.uniform(-12, 12), rng.uniform(-12, 12),
                  float(rng.integers(0, 2 ** 24)), rng.uniform(4.0, 16.0), 0)
    return segs, par


def _hash(x: np.ndarray, y: np.ndarray, seed: np.ndarray) -> np.ndarray:
    h = (x.astype(np.uint32) * np.uint32(374761393) + y.astype(np.uint32) * np.uint32(668265263)
         + seed.astype(np.uint32) * np.uint32(2246822519))
    h = (h ^ (h >> np.uint32(13))) * np.uint32(1274126177)
    return h ^ (h >> np.uint32(16))


def render_numpy(segs: np.ndarray, par: np.ndarray, img: int) -> Tuple[np.ndarray, np.ndarray]:
    """segs [n,MAX_SEG,6], par [n,8] -> (images uint8 [n,img,img,3], masks uint8 [n,img,img])."""
    n = segs.shape[0]
    ys, xs = np.meshgrid(np.arange(img, dtype=np.float32), np.arange(img, dtype=np.float32), indexing="ij")
    images = np.zeros((n, img, img, 3), np.uint8)
    masks = np.zeros((n, img, img), np.uint8)
    px, py = xs + 0.5, ys + 0.5
    xi, yi = xs.astype(np.uint32), ys.astype(np.uint32)
    with np.errstate(over="ignore"):
        for i in range(n):
            bg, noise_amp, dark, tint_r, tint_b, seed, cell, _ = par[i]
            cell_i = max(int(cell), 1)
            seed_a = np.full_like(xi, np.uint32(int(seed)))
            fine = (_hash(xi, yi, seed_a) & np.uint32(255)).astype(np.float32) / np.float32(255.0)
            coarse = (_hash(xi // np.uint32(cell_i), yi // np.uint32(cell_i), seed_a + np.uint32(7919))
                      & np.uint32(255)).astype(np.float32) / np.float32(255.0)
            v = np.float32(bg) + np.float32(noise_amp) * (np.float32(0.35) * fine + np.float32(0.65) * coarse
                                                          - np.float32(0.5))
            dmin = np.full((img, img), np.float32(1e9))
            hwmap = np.zeros((img, img), np.float32)
            for k in range(MAX_SEG):
                x0, y0, x1, y1, hw, _ = segs[i, k]
                if hw <= 0:
                    continue
                dx, dy = np.float32(x1 - x0), np.float32(y1 - y0)
                l2 = dx * dx + dy * dy
                t = ((px - np.float32(x0)) * dx + (py - np.float32(y0)) * dy) / np.float32(max(l2, 1e-12))
                t = np.clip(t, np.float32(0), np.float32(1))
                ex, ey = px - (np.float32(x0) + t * dx), py - (np.float32(y0) + t * dy)
                d = np.sqrt(ex * ex + ey * ey) / np.float32(hw)
                better = d < dmin
                dmin = np.where(better, d, dmin)
            crack = dmin < np.float32(1.0)
            shade = np.clip(np.float32(1.6) - dmin, np.float32(0), np.float32(1))
            v = v - shade * (v - np.float32(dark))
            r = np.clip(v + np.float32(tint_r), 0, 255)
            g = np.clip(v, 0, 255)
            b = np.clip(v + np.float32(tint_b), 0, 255)
            images[i] = np.stack([r, g, b], -1).astype(np.uint8)
            masks[i] = crack.astype(np.uint8)
            del hwmap
    return images, masks


@dataclass
class CrackDataset:
    """In-memory dataset with the reference's split semantics (client_fit_model.py:54-90)."""
    images: np.ndarray            # uint8 [N,H,W,3]  (or a device tensor on the GPU path)
    masks: np.ndarray             # uint8 [N,H,W]
    train_idx: np.ndarray
    val_idx: np.ndarray

    @property
    def img_size(self) -> int:
        return int(self.images.shape[1])


def reference_split(n: int, split: int, seed: int = 1337, client_first: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """Shuffle with ``random.Random(seed)`` (client_fit_model.py:77-78) then split.

    client_first=True: FIRST ``split`` are train (client_fit_model.py:79-82);
    client_first=False: LAST ``split`` are validation (test/Segmentation.py:84-90).
    """
    idx = list(range(n))
    random.Random(seed).shuffle(idx)
    idx = np.asarray(idx, np.int64)
    if client_first:
        return idx[:split], idx[split:]
    return idx[:-split], idx[-split:]


def make_synthetic(n: int, img: int, seed: int = 0, split: Optional[int] = None,
                   shuffle_seed: int = 1337) -> CrackDataset:
    segs, par = image_params(n, img, seed)
    images, masks = render_numpy(segs, par, img)
    split = n if split is None else min(split, n)
    tr, va = reference_split(n, split, shuffle_seed)
    return CrackDataset(images, masks, tr, va)
