"""Builds a client's local trainer: dataset + compute backend.

Device policy: ``device=cuda`` (or ``auto`` with a visible GPU) runs the MI355X engine (hand-written HIP kernels,
``models/engine.py``) and fails loudly if the HIP extension is missing - there is no silent eager fallback on a
GPU. ``device=cpu`` runs the fp32 reference (plumbing config / tests).
"""
from __future__ import annotations

import os
from typing import Optional

from ..config import FLConfig
from ..data.synthetic import CrackDataset, make_synthetic
from ..models.spec import ParamTable
from .local import LocalFit, RefBackend


def resolve_device(cfg: FLConfig) -> str:
    if cfg.device in ("cpu", "cuda"):
        return cfg.device
    import torch
    return "cuda" if torch.cuda.is_available() else "cpu"


def planned_batch(cfg: FLConfig, device: str) -> int:
    """batch_size=0: the HBM planner's batch for this image size (config 4, 512^2 large batch)."""
    from ..models.memplan import plan_batch
    hbm = None if device == "cuda" else 288 * 10**9
    plan = plan_batch(cfg.img_size, hbm, cfg.hbm_fraction, cfg.synthetic_samples if cfg.data == "synthetic" else 0)
    print(f"[memplan] {plan.as_dict()}", flush=True)
    return plan.batch


def make_dataset(cfg: FLConfig, rank: int = 0, device: str = "cpu") -> CrackDataset:
    if cfg.data == "folder":
        from ..data.folder import load_folder_dataset
        return load_folder_dataset(cfg.train_image_dir, cfg.train_mask_dir, cfg.img_size, cfg.val_samples,
                                   cfg.shuffle_seed, device=device)
    seed = cfg.data_seed * 7919 + rank
    if device == "cuda":
        from ..data.device import make_synthetic_device
        return make_synthetic_device(cfg.synthetic_samples, cfg.img_size, seed, cfg.val_samples, cfg.shuffle_seed)
    return make_synthetic(cfg.synthetic_samples, cfg.img_size, seed, cfg.val_samples, cfg.shuffle_seed)


def make_trainer(cfg: FLConfig, client: str = "client", rank: int = 0, table: Optional[ParamTable] = None,
                 device: Optional[str] = None) -> LocalFit:
    table = table or ParamTable()
    device = device or resolve_device(cfg)
    if cfg.batch_size <= 0:
        cfg.batch_size = planned_batch(cfg, device)
    data = make_dataset(cfg, rank, device)
    if device == "cuda":
        from ..models.engine import HipBackend
        backend = HipBackend(cfg, data, table)
    else:
        backend = RefBackend(cfg, data, table, "cpu")
    return LocalFit(cfg, data, backend, table, client)
