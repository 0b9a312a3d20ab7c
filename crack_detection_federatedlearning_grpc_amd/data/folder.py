"""Folder dataset with the reference's file semantics (client_fit_model.py:19-43, 54-90).

* image paths: ``*.jpg`` in the image dir, sorted; mask paths: ``*.jpg`` not starting with '.' in the mask dir,
  sorted; both shuffled with ``random.Random(1337)`` (same permutation, equal lengths) - :61-78
* the client takes the FIRST ``val_samples`` (6213) as TRAIN and the rest as validation - :79-82
* images: decode, BGR->RGB (PIL decodes to RGB directly), resize to img x img (bilinear on the half-pixel grid,
  native ``_native.resize_bilinear``), later /255 - :34-36,43;  masks: decode, resize, ``> 0`` - :37-40
Decoding runs on a thread pool (PIL releases the GIL); the decoded uint8 arrays are loaded once and kept in memory.
On the GPU path (``device="cuda"``) the decoded images are uploaded at their own sizes and resized / binarised by ONE
HIP kernel launch per 1,024 images straight into the HBM-resident dataset (``resize_batch``, datagen.hip; equal to
the host resize when down-scaling, within 1 LSB when up-scaling) - the /255 normalisation is folded into the entry
conv.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import random
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from .._native_loader import native
from .synthetic import CrackDataset


def list_pairs(image_dir: str, mask_dir: str) -> Tuple[List[str], List[str]]:
    imgs = sorted(os.path.join(image_dir, f) for f in os.listdir(image_dir) if f.endswith(".jpg"))
    masks = sorted(os.path.join(mask_dir, f) for f in os.listdir(mask_dir)
                   if f.endswith(".jpg") and not f.startswith("."))
    return imgs, masks


def load_image(path: str, size) -> np.ndarray:
    from PIL import Image
    h, w = (size, size) if isinstance(size, int) else size
    with Image.open(path) as im:
        a = np.asarray(im.convert("RGB"), dtype=np.uint8)
    if a.shape[0] != h or a.shape[1] != w:
        a = native().resize_bilinear(np.ascontiguousarray(a), h, w, 2)
    return a


def load_mask(path: str, size) -> np.ndarray:
    from PIL import Image
    h, w = (size, size) if isinstance(size, int) else size
    with Image.open(path) as im:
        a = np.asarray(im.convert("L"), dtype=np.uint8)
    if a.shape[0] != h or a.shape[1] != w:
        a = native().resize_bilinear(np.ascontiguousarray(a), h, w, 2)
    return (a > 0).astype(np.uint8)


def decode(path: str, mode: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert(mode), dtype=np.uint8))


def resize_on_device(items: Sequence, size: int, binarize: bool, chunk: int = 1024,
                     load: Optional[Callable[[str], np.ndarray]] = None, pool=None, channels: Optional[int] = None):
    """uint8 images of any sizes -> torch uint8 [n, size, size(, c)] on the current GPU, resized by the HIP batch
    kernel (cv2.resize INTER_LINEAR grid, as the host ``_native.resize_bilinear``). ``items`` are decoded arrays,
    or paths that ``load`` decodes one ``chunk`` at a time (on ``pool`` if given), so host memory holds at most one
    chunk of source-resolution images. ``channels`` (3, or None for single-channel) shapes an empty result."""
    import torch
    from .._native_loader import hip
    C = hip()
    n = len(items)
    out = None
    for s0 in range(0, n, chunk):
        part = items[s0:s0 + chunk]
        if load is not None:
            part = list(pool.map(load, part)) if pool is not None else [load(p) for p in part]
        if out is None:
            c = part[0].shape[2] if part[0].ndim == 3 else None
            out = torch.empty((n, size, size) + ((c,) if c else ()), dtype=torch.uint8, device="cuda")
        sizes = np.array([a.size for a in part], np.int64)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        dims = np.array([a.shape[:2] for a in part], np.int32).reshape(-1)
        src = torch.from_numpy(np.concatenate([a.reshape(-1) for a in part])).to("cuda", non_blocking=False)
        C.resize_batch(src, torch.from_numpy(offs).cuda(), torch.from_numpy(dims).cuda(), out[s0:s0 + len(part)],
                       1 if binarize else 0)
    if out is None:                                       # empty folder / limit 0
        out = torch.empty((0, size, size) + ((channels,) if channels else ()), dtype=torch.uint8, device="cuda")
    return out


def load_folder_dataset(image_dir: str, mask_dir: str, img: int, split: int = 6213, seed: int = 1337,
                        workers: int = 8, limit: Optional[int] = None, device: str = "cpu") -> CrackDataset:
    imgs, masks = list_pairs(image_dir, mask_dir)
    if len(imgs) != len(masks):
        raise ValueError(f"{len(imgs)} images but {len(masks)} masks")
    random.Random(seed).shuffle(imgs)
    random.Random(seed).shuffle(masks)
    if limit:
        imgs, masks = imgs[:limit], masks[:limit]
    n = len(imgs)
    if device == "cuda":                      # decode on the host, resize + binarise on the GPU
        with cf.ThreadPoolExecutor(max_workers=workers) as ex:   # decode chunk by chunk (bounded host memory)
            X = resize_on_device(imgs, img, False, load=lambda p: decode(p, "RGB"), pool=ex, channels=3)
            Y = resize_on_device(masks, img, True, load=lambda p: decode(p, "L"), pool=ex)
        split = min(split, n)
        idx = np.arange(n)
        return CrackDataset(X, Y, idx[:split], idx[split:])
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        X = np.stack(list(ex.map(lambda p: load_image(p, img), imgs)))
        Y = np.stack(list(ex.map(lambda p: load_mask(p, img), masks)))
    split = min(split, n)
    idx = np.arange(n)
    return CrackDataset(X, Y, idx[:split], idx[split:])
