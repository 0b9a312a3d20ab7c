"""Training parity: the HIP engine (bf16 activations / gradients, fp32 master weights, hipGraph
steps) and the plain fp32 PyTorch oracle (models/unet_ref.py RefTrainer: Keras semantics, fp32 everywhere) trained
from the SAME init on the SAME batches, both evaluated on the same held-out images every ``every`` steps
(inference-mode BN): validation loss, pixel accuracy and crack IoU side by side.
Reference: /root/reference/client_fit_model.py:157,166 (compile + fit). Driver: tools/parity.py; pinned by
tests/test_gpu_kernels.py::test_training_parity_vs_plain_fp32.
"""
from __future__ import annotations

import json
import time
from typing import Dict, List, Optional, TextIO

import numpy as np
import torch

from ..data.device import make_synthetic_device
from ..models import unet_ref as R
from ..models.engine import UNetEngine
from ..models.spec import ParamTable
from .local import epoch_batches


def run(img: int = 128, batch: int = 16, steps: int = 800, every: int = 100, samples: int = 1024, val: int = 128,
        seed: int = 3, data_seed: int = 21, log: Optional[TextIO] = None, quiet: bool = False,
        fp8: bool = False) -> List[Dict]:
    """Train both for ``steps`` steps (reference Sequence semantics: per-epoch shuffled batch order over the train
    split of ``samples`` synthetic images); every ``every`` steps (and at the end) evaluate both on the ``val``
    held-out images. Returns one record per checkpoint: mean train losses since the last one, and per model
    val_loss / val_acc / val_iou. ``fp8``: a third model - the engine with every decoder 3x3 conv on the block-scaled
    fp8 MFMA (conv_dtype="fp8", BASELINE config 5) - trained on the same batches, reported as "engine_fp8"."""
    dev = torch.device("cuda")
    table = ParamTable()
    data = make_synthetic_device(samples, img, seed=data_seed, split=samples - val)
    flat0 = table.init_flat(seed)
    eng = UNetEngine(table, batch, img)
    eng.bind_data(data.images, data.masks)
    eng.set_flat(flat0)
    eng8 = None
    if fp8:
        eng8 = UNetEngine(table, batch, img, conv_dtype="fp8")
        eng8.bind_data(data.images, data.masks)
        eng8.set_flat(flat0)
    ref = R.RefTrainer(table, flat0, "cuda")
    nb = len(data.train_idx) // batch
    batches = np.concatenate([epoch_batches(data.train_idx, batch, nb, seed=e) for e in range((steps + nb - 1) // nb)])
    vb = epoch_batches(data.val_idx, batch, 0, 0)

    def xy(ids):
        t = torch.as_tensor(ids, dtype=torch.long, device=dev)
        return data.images[t].float() / 255.0, data.masks[t].float()[..., None]

    def evaluate():
        eng.eval_metrics.zero_()
        if eng8 is not None:
            eng8.eval_metrics.zero_()
        ev, tp, pp, tt, acc = [], 0.0, 0.0, 0.0, []
        for ids in vb:
            eng.idx.copy_(torch.as_tensor(ids, dtype=torch.int32, device=dev))
            eng.eval_step(use_graph=False)
            if eng8 is not None:
                eng8.idx.copy_(eng.idx)
                eng8.eval_step(use_graph=False)
            m = ref.evaluate(*xy(ids))
            ev.append(m["loss"])
            acc.append(m["accuracy"])
            tp, pp, tt = tp + m["tp"], pp + m["pp"], tt + m["t"]
        me = eng.read_metrics("eval")
        iou_ref = tp / (pp + tt - tp) if pp + tt - tp > 0 else 1.0
        out = {"engine": {"val_loss": me["loss"], "val_acc": me["accuracy"], "val_iou": me["iou"]},
               "fp32": {"val_loss": float(np.mean(ev)), "val_acc": float(np.mean(acc)), "val_iou": iou_ref}}
        if eng8 is not None:
            m8 = eng8.read_metrics("eval")
            out["engine_fp8"] = {"val_loss": m8["loss"], "val_acc": m8["accuracy"], "val_iou": m8["iou"]}
        return out

    out = []
    le, lr_, l8 = [], [], []
    t0 = time.perf_counter()
    for s in range(steps):
        ids = batches[s]
        eng.idx.copy_(torch.as_tensor(ids, dtype=torch.int32, device=dev))
        eng.train_step(use_graph=True)
        le.append(eng.read_metrics("train")["loss"])
        if eng8 is not None:
            eng8.idx.copy_(eng.idx)
            eng8.train_step(use_graph=True)
            l8.append(eng8.read_metrics("train")["loss"])
        lr_.append(ref.train_step(*xy(ids))["loss"])
        if (s + 1) % every == 0 or s + 1 == steps:
            rec = {"step": s + 1, "train_loss_engine": float(np.mean(le[-every:])),
                   "train_loss_fp32": float(np.mean(lr_[-every:])),
                   **({"train_loss_engine_fp8": float(np.mean(l8[-every:]))} if l8 else {}), **evaluate(),
                   "elapsed_s": round(time.perf_counter() - t0, 1)}
            out.append(rec)
            line = json.dumps(rec)
            if not quiet:
                print(line, flush=True)
            if log:
                print(line, file=log, flush=True)
    return out
