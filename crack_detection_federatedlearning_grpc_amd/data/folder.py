"""Folder dataset with the reference's file semantics (client_fit_model.py:19-43, 54-90).

* image paths: ``*.jpg`` in the image dir, sorted; mask paths: ``*.jpg`` not starting with '.' in the mask dir,
  sorted; both shuffled with ``random.Random(1337)`` (same permutation, equal lengths) - :61-78
* the client takes the FIRST ``val_samples`` (6213) as TRAIN and the rest as validation - :79-82
* images: decode, BGR->RGB (PIL decodes to RGB directly), resize to img x img (bilinear on the half-pixel grid,
  native ``_native.resize_bilinear``), later /255 - :34-36,43;  masks: decode, resize, ``> 0`` - :37-40
Decoding runs on a thread pool (PIL releases the GIL); the decoded uint8 arrays are loaded once and kept in memory
(and on the GPU path copied once into HBM).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import random
from typing import List, Optional, Tuple

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


def load_folder_dataset(image_dir: str, mask_dir: str, img: int, split: int = 6213, seed: int = 1337,
                        workers: int = 8, limit: Optional[int] = None) -> CrackDataset:
    imgs, masks = list_pairs(image_dir, mask_dir)
    if len(imgs) != len(masks):
        raise ValueError(f"{len(imgs)} images but {len(masks)} masks")
    random.Random(seed).shuffle(imgs)
    random.Random(seed).shuffle(masks)
    if limit:
        imgs, masks = imgs[:limit], masks[:limit]
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        X = np.stack(list(ex.map(lambda p: load_image(p, img), imgs)))
        Y = np.stack(list(ex.map(lambda p: load_mask(p, img), masks)))
    n = len(imgs)
    split = min(split, n)
    idx = np.arange(n)
    return CrackDataset(X, Y, idx[:split], idx[split:])
