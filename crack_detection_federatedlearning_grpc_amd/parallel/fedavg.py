"""Host-side FedAvg (the gRPC data plane's reduction).

Reference: ``updateWeight`` fl_server.py:92-105 - unweighted mean of ALL 112 arrays (BN moving stats included),
aliasing the first client's list and never clearing ``received_parameters`` (wrong from round 2).
Here: a fresh per-round accumulator, optional n_k weighting (equal n_k reproduces the reference mean), fp64
accumulation over one flat buffer. The on-node GPU path is ``parallel/rccl.py`` (weighted RCCL all-reduce).
"""
from __future__ import annotations

from typing import Iterable, Sequence, Tuple

import numpy as np


def fedavg_flat(updates: Sequence[Tuple[np.ndarray, float]], weighted: bool = True) -> np.ndarray:
    """updates: [(flat fp32 weights, n_samples)] -> flat fp32 average."""
    if not updates:
        raise ValueError("no client updates to aggregate")
    ws = np.array([max(float(n), 0.0) for _, n in updates], np.float64)
    if not weighted or ws.sum() <= 0:
        ws = np.ones(len(updates), np.float64)
    ws = ws / ws.sum()
    acc = np.zeros_like(np.asarray(updates[0][0]), dtype=np.float64)
    for (flat, _), w in zip(updates, ws):
        acc += w * np.asarray(flat, np.float64)
    return acc.astype(np.float32)


def fedavg_lists(lists: Sequence[Sequence[np.ndarray]], weights: Iterable[float] = ()) -> list:
    """List-of-arrays form (what the reference averages)."""
    weights = list(weights) or [1.0] * len(lists)
    tot = float(sum(weights))
    out = []
    for i in range(len(lists[0])):
        acc = np.zeros(np.shape(lists[0][i]), np.float64)
        for l, w in zip(lists, weights):
            acc += (w / tot) * np.asarray(l[i], np.float64)
        out.append(acc.astype(np.float32))
    return out
