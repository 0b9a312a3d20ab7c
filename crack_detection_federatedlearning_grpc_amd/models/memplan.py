"""HBM planner for one FL client's engine (BASELINE config 4: U-Net 512^2, large batch, sized for 288 GB HBM).

The engine (``models/engine.py``) allocates every activation / gradient buffer once; their shapes are a pure
function of (batch, image size), defined HERE and consumed by ``UNetEngine._alloc`` so the plan and the allocation
cannot drift. Everything else the engine holds is batch-independent (flat fp32 params / grads / Adam moments, bf16
packed weights, BN statistics, weight-gradient slabs) or small (the split-K workspace, which only the
low-M layers use and which shrinks as the batch grows).

``plan_batch`` picks the largest per-client batch whose footprint (engine + the client's resident uint8 dataset
shard) fits a fraction of HBM. Index widths: every kernel forms ELEMENT offsets in 64 bits (``(size_t)pixel * C``;
audited over csrc/kernels for round 2), and keeps 32-bit only the pixel index (B*H*W) and the elementwise kernels'
work-item counters (pixels x channel groups of >= 4 channels, plus one grid stride) - so the index bound is
numel / 4 < 2^31 - 2^24 per tensor, which at 512^2 allows batches up to 2,040: HBM, not the index width, bounds
the 512^2 plan (58 GB at the old 2^30-element bound). The reference trains at a fixed batch 16
(client_fit_model.py:56); the planner is the MI355X-side answer to SURVEY.md §7.5 item 6.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional, Tuple

from .spec import DEC_FILTERS, ENC_FILTERS, ENTRY_FILTERS

BF16, U8, F32 = 2, 1, 4
MAX_ITEMS = 2**31 - 2**24      # 32-bit work-item counters (>= 4 channels per item) plus one grid stride
ITEM_CHANNELS = 4
MAX_ELEMS = MAX_ITEMS * ITEM_CHANNELS   # largest tensor (elements) the kernels index; element offsets are 64-bit


def _qres(k: int, Rk: int) -> int:
    return Rk if k == 0 else Rk // 2


def buffer_shapes(B: int, S: int) -> Tuple[Dict[str, Tuple[Tuple[int, ...], int]],
                                           Dict[str, Optional[Tuple[Tuple[int, ...], int]]]]:
    """(forward activations, backward buffers): name -> (shape, itemsize). NHWC; bf16 unless noted."""
    r = [S // 2, S // 4, S // 8, S // 16]
    A: Dict[str, Tuple[Tuple[int, ...], int]] = {}
    A["y0"] = ((B, r[0], r[0], ENTRY_FILTERS), BF16)
    cin = ENTRY_FILTERS
    for k, F in enumerate(ENC_FILTERS):
        H = r[k]
        A[f"e{k}_d1"] = ((B, H, H, cin), BF16)
        A[f"e{k}_y1"] = ((B, H, H, F), BF16)
        A[f"e{k}_d2"] = ((B, H, H, F), BF16)
        A[f"e{k}_y2"] = ((B, H, H, F), BF16)
        A[f"e{k}_res"] = ((B, H // 2, H // 2, F), BF16)
        A[f"e{k}_x"] = ((B, H // 2, H // 2, F), BF16)
        A[f"e{k}_am"] = ((B, H // 2, H // 2, F), U8)          # max-pool argmax
        cin = F
    for k, F in enumerate(DEC_FILTERS):
        Rk = r[3] << k
        A[f"d{k}_c1"] = ((B, Rk, Rk, F), BF16)
        A[f"d{k}_c2"] = ((B, Rk, Rk, F), BF16)
        A[f"d{k}_q"] = ((B, _qres(k, Rk), _qres(k, Rk), F), BF16)
        A[f"d{k}_xlo"] = ((B, Rk, Rk, F), BF16)
    A["h"] = ((B, r[0], r[0]), F32)                             # head logits (half resolution)
    D: Dict[str, Optional[Tuple[Tuple[int, ...], int]]] = {}
    D["dxlo3"] = ((B, r[0], r[0], DEC_FILTERS[-1]), BF16)
    for k, F in enumerate(DEC_FILTERS):
        Rk = r[3] << k
        cprev = ENC_FILTERS[-1] if k == 0 else DEC_FILTERS[k - 1]
        prevres = Rk if k == 0 else Rk // 2
        D[f"d{k}_g"] = ((B, Rk, Rk, F), BF16)
        D[f"d{k}_dc"] = ((B, Rk, Rk, F), BF16)
        D[f"d{k}_dc2"] = ((B, Rk, Rk, F), BF16)       # 2nd BN input-gradient (dc is still read by a deferred wgrad)
        D[f"d{k}_dxin"] = ((B, Rk, Rk, cprev), BF16)
        D[f"d{k}_dq"] = ((B, _qres(k, Rk), _qres(k, Rk), F), BF16)
        D[f"d{k}_dres"] = ((B, prevres, prevres, cprev), BF16)
        D[f"d{k}_dprev"] = ((B, prevres, prevres, cprev), BF16)
    cin = ENTRY_FILTERS
    for k, F in enumerate(ENC_FILTERS):
        H = r[k]
        D[f"e{k}_g"] = ((B, H, H, F), BF16)
        D[f"e{k}_dy"] = ((B, H, H, F), BF16)
        D[f"e{k}_dy2"] = ((B, H, H, F), BF16)
        D[f"e{k}_dd2"] = ((B, H, H, F), BF16)
        D[f"e{k}_dd1"] = ((B, H, H, cin), BF16)
        D[f"e{k}_dz0"] = ((B, H, H, cin), BF16)
        D[f"e{k}_dres"] = ((B, H // 2, H // 2, cin), BF16)
        D[f"e{k}_dx"] = ((B, H, H, cin), BF16) if k > 0 else None
        cin = F
    D["g0"] = ((B, r[0], r[0], ENTRY_FILTERS), BF16)
    D["dy0"] = ((B, r[0], r[0], ENTRY_FILTERS), BF16)
    return A, D


def _prod(s) -> int:
    n = 1
    for v in s:
        n *= v
    return n


def activation_bytes(B: int, S: int) -> int:
    A, D = buffer_shapes(B, S)
    return sum(_prod(s) * i for s, i in A.values()) + sum(_prod(v[0]) * v[1] for v in D.values() if v)


def largest_tensor_elems(B: int, S: int) -> int:
    A, D = buffer_shapes(B, S)
    return max(_prod(v[0]) for v in list(A.values()) + [v for v in D.values() if v])


def fixed_bytes(n_params: int = 2_058_145) -> int:
    """Batch-independent engine state: flat params, grads, Adam m/v (fp32), bf16 packed weights (fwd + dgrad
    copies), plus an allowance for BN statistics replicas, weight-gradient slabs (3x3 weight gradients keep up to
    ~512 blocks' worth of partial rows, ~40 MB per 256x256 decoder layer) and the split-K workspace. Measured on an
    MI355X at 512^2: ~400 MB of batch-independent state in total."""
    return 4 * F32 * n_params + 2 * BF16 * n_params + 512 * 2**20


def dataset_bytes(samples: int, S: int) -> int:
    return samples * S * S * 3 + samples * S * S          # uint8 RGB + uint8 mask, resident in HBM


@dataclass
class Plan:
    batch: int
    img: int
    engine_bytes: int
    dataset_bytes: int
    budget_bytes: int
    limit: str                       # "hbm" | "index" (32-bit work-item counters) | "max_batch"

    @property
    def total_bytes(self) -> int:
        return self.engine_bytes + self.dataset_bytes

    def as_dict(self) -> Dict[str, object]:
        return dict(batch=self.batch, img=self.img, engine_gb=round(self.engine_bytes / 2**30, 3),
                    dataset_gb=round(self.dataset_bytes / 2**30, 3), budget_gb=round(self.budget_bytes / 2**30, 3),
                    limit=self.limit)


def engine_bytes(B: int, S: int) -> int:
    return fixed_bytes() + activation_bytes(B, S)


def plan_batch(img: int, hbm_bytes: Optional[int] = None, fraction: float = 0.85, samples: int = 0,
               multiple: int = 8, max_batch: int = 4096) -> Plan:
    """Largest batch (a multiple of ``multiple``) with engine + dataset <= fraction * HBM and every tensor under
    the 32-bit index limit. ``hbm_bytes`` defaults to the visible device's total memory (288 GB on an MI355X)."""
    if hbm_bytes is None:
        import torch
        hbm_bytes = torch.cuda.get_device_properties(torch.cuda.current_device()).total_memory \
            if torch.cuda.is_available() else 288 * 10**9
    budget = int(hbm_bytes * fraction)
    data = dataset_bytes(samples, img)
    per = activation_bytes(1, img)
    avail = budget - data - fixed_bytes()
    if avail < per:
        raise ValueError(f"img {img}: one image needs {per / 2**30:.2f} GiB, only {avail / 2**30:.2f} GiB free")
    b_hbm = avail // per
    b_idx = MAX_ELEMS // largest_tensor_elems(1, img)
    b = min(b_hbm, b_idx, max_batch)
    limit = "hbm" if b == b_hbm else ("index" if b == b_idx else "max_batch")
    if b >= multiple:
        b -= b % multiple
    return Plan(int(b), img, engine_bytes(int(b), img), data, budget, limit)
