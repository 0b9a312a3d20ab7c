"""Centralized (non-FL) baseline trainer: the reference's ``test/Segmentation.py``.

What the reference script does (test/Segmentation.py:160-187): clear the Keras session (unsuffixed layer names),
build the same U-Net, compile Adam / binary cross-entropy / accuracy, ``fit`` for 60 epochs on the 1337-shuffled
split with ``ModelCheckpoint("crack_segmentation.h5", save_best_only=True)`` (monitor ``val_loss``), then
``model.save("my_model")``. Here:

  * one Adam state across all epochs (a single long ``fit``, not FL rounds);
  * per epoch: train pass (Keras Sequence semantics, shuffled batch order), validation pass, JSONL record;
  * ``save_best_only``: the full-model Keras ``.h5`` (model_config, training_config, model_weights and the Adam
    optimizer_weights) is rewritten whenever ``val_loss`` improves - written by the in-tree C++ HDF5 writer;
  * ``model.save(dir)``: TensorFlow SavedModel needs TF, so the directory holds the same full-model ``model.h5``
    plus ``weights.pickle`` (the FL hand-off layout) and ``history.json``.

The numeric work runs on the MI355X engine (``device=cuda``) or the fp32 oracle (``device=cpu``).

    python -m crack_detection_federatedlearning_grpc_amd.train.centralized --epochs 60 --img-size 256 \
        [--data folder --train-image-dir ... --train-mask-dir ...] [--checkpoint crack_segmentation.h5] \
        [--save-dir my_model]
"""
from __future__ import annotations

import argparse
import json
import os
import time
from typing import Dict, List, Optional

import numpy as np

from .. import config as _config
from ..ckpt.h5 import save_keras_h5
from ..fl import codec
from .factory import make_trainer
from .local import LocalFit, epoch_batches


class CentralizedTrainer:
    def __init__(self, cfg: _config.FLConfig, fit: Optional[LocalFit] = None):
        self.cfg = cfg
        self.fit = fit or make_trainer(cfg, "centralized")
        self.best = float("inf")
        self.history: List[Dict[str, float]] = []

    def _checkpoint(self, path: str) -> None:
        b = self.fit.backend
        opt = b.optimizer_state() if hasattr(b, "optimizer_state") else None
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        save_keras_h5(tmp, self.fit.table, b.get_flat(), self.cfg.img_size, opt, self.cfg.lr)
        os.replace(tmp, path)

    def train(self, epochs: int, checkpoint: str = "", save_best_only: bool = True) -> List[Dict[str, float]]:
        cfg, fit = self.cfg, self.fit
        fit.backend.reset_optimizer()
        data = fit.data
        for ep in range(epochs):
            seed = (cfg.data_seed * 1000003 + ep) & 0x7FFFFFFF
            batches = epoch_batches(data.train_idx, cfg.batch_size, fit.steps, seed)
            t0 = time.perf_counter()
            m = fit.backend.train_batches(batches)
            dt = time.perf_counter() - t0
            rec = {"epoch": ep + 1, "loss": m["loss"], "accuracy": m["accuracy"], "images": int(batches.size),
                   "train_s": dt, "images_per_s": batches.size / max(dt, 1e-9)}
            if len(data.val_idx) >= cfg.batch_size:
                vb = epoch_batches(data.val_idx, cfg.batch_size, 0, 0)
                v = fit.backend.eval_batches(vb)
                rec["val_loss"], rec["val_accuracy"] = v["loss"], v["accuracy"]
            monitor = rec.get("val_loss", rec["loss"])
            if checkpoint and (not save_best_only or monitor < self.best):
                self._checkpoint(checkpoint)
                rec["checkpoint"] = checkpoint
            self.best = min(self.best, monitor)
            fit._log(dict(rec, mode="centralized"))
            self.history.append(rec)
        return self.history

    def save(self, directory: str) -> None:
        """``model.save("my_model")`` (test/Segmentation.py:187) without TensorFlow: full-model h5 + pickle."""
        os.makedirs(directory, exist_ok=True)
        self._checkpoint(os.path.join(directory, "model.h5"))
        codec.save_weight_file(os.path.join(directory, "weights.pickle"), self.fit.get_weights())
        with open(os.path.join(directory, "history.json"), "w") as f:
            json.dump(self.history, f, indent=1)


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    _config.add_arguments(ap)
    ap.add_argument("--checkpoint", default="crack_segmentation.h5")
    ap.add_argument("--save-dir", default="my_model")
    ap.add_argument("--no-save-best-only", action="store_true")
    args = ap.parse_args(argv)
    extra = {k: getattr(args, k) for k in ("checkpoint", "save_dir", "no_save_best_only")}
    cfg = _config.from_args(args)
    preset = args.preset or os.environ.get("FL_PRESET", "")
    if args.epochs is None and "FL_EPOCHS" not in os.environ and "epochs" not in _config.PRESETS.get(preset, {}):
        cfg.epochs = 60                                   # test/Segmentation.py:186
    tr = CentralizedTrainer(cfg)
    tr.train(cfg.epochs, extra["checkpoint"], not extra["no_save_best_only"])
    if extra["save_dir"]:
        tr.save(extra["save_dir"])
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
