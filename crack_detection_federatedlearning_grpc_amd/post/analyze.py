"""Offline inference / crack analysis tool: the reference's ``test/Segmentation2.py`` plus the
``Predict`` step of ``client_fit_model.py:176-223``.

The reference loads ``my_model`` (Keras SavedModel), predicts on the validation split, writes the prediction as
``pred2.png``, then runs ``contour()`` (test/Segmentation2.py:114-141: threshold 127, contours, area / perimeter /
approxPolyDP at 1 % and 10 %) and draws the contours to ``contour/img{1,2,3}.jpg``. Here:

  * weights come from a full-model or weights-only Keras ``.h5`` (C++ HDF5 reader), a ``my_model`` directory
    written by ``train/centralized.py``, or a ``weights.pickle`` FL hand-off file (pickle is only ever read from
    files this framework wrote);
  * prediction runs on the MI355X engine (``device=cuda``) or the fp32 oracle (``device=cpu``);
  * every analysed image gets ``pred{i}.png`` (probability * 255), ``contour/img{i}.png`` (the input with the
    crack contours drawn in red) and one record of crack metrics in ``analysis.json``.

    python -m crack_detection_federatedlearning_grpc_amd.post.analyze --weights my_model --out analysis/ \
        --count 4 [--img-size 256 --data folder --train-image-dir ... --train-mask-dir ...]
"""
from __future__ import annotations

import argparse
import json
import os
from typing import Dict, List, Optional

import numpy as np

from .. import config as _config
from ..ckpt.h5 import load_weights_h5
from ..fl import codec
from ..models.spec import ParamTable
from .contour import crack_metrics, find_contours


def load_weights(path: str, table: ParamTable) -> np.ndarray:
    """Flat fp32 parameters from an .h5 file, a centralized ``save`` directory, or a weights.pickle file."""
    if os.path.isdir(path):
        h5 = os.path.join(path, "model.h5")
        return load_weights_h5(h5, table) if os.path.exists(h5) else \
            table.from_list(codec.load_weight_file(os.path.join(path, "weights.pickle")))
    if path.endswith((".h5", ".hdf5", ".keras")):
        return load_weights_h5(path, table)
    return table.from_list(codec.load_weight_file(path))


def draw_contours(rgb: np.ndarray, prob_u8: np.ndarray, thresh: int = 127) -> np.ndarray:
    """cv2.drawContours(img, contours, -1, (255, 0, 0)) equivalent: contour points painted red on a copy."""
    out = np.array(rgb, np.uint8, copy=True)
    cs, _ = find_contours(prob_u8, thresh, simple=False)
    for c in cs:
        pts = np.asarray(c, np.int64).reshape(-1, 2)
        out[pts[:, 1], pts[:, 0]] = (255, 0, 0)
    return out


def _save_png(path: str, arr: np.ndarray) -> None:
    from PIL import Image
    Image.fromarray(np.asarray(arr, np.uint8)).save(path)


def analyze(cfg: _config.FLConfig, weights: str, out_dir: str, count: int = 3, trainer=None) -> List[Dict]:
    from ..train.factory import make_trainer
    fit = trainer or make_trainer(cfg, "analyze")
    fit.backend.set_flat(load_weights(weights, fit.table))
    data = fit.data
    idx = np.asarray(data.val_idx[:count] if len(data.val_idx) else data.train_idx[:count])
    probs = fit.backend.predict(idx)
    os.makedirs(os.path.join(out_dir, "contour"), exist_ok=True)
    images = data.images.cpu().numpy() if hasattr(data.images, "cpu") else np.asarray(data.images)
    masks = data.masks.cpu().numpy() if hasattr(data.masks, "cpu") else np.asarray(data.masks)
    recs = []
    for i, (k, p) in enumerate(zip(idx, probs)):
        pu8 = (np.clip(p, 0.0, 1.0) * 255.0 + 0.5).astype(np.uint8)
        _save_png(os.path.join(out_dir, f"pred{i + 1}.png"), pu8)
        _save_png(os.path.join(out_dir, "contour", f"img{i + 1}.png"), draw_contours(images[k], pu8))
        m = crack_metrics(pu8)
        truth = masks[k] > 0
        pred = pu8 > 127
        inter, union = float((truth & pred).sum()), float((truth | pred).sum())
        m.update(index=int(k), iou=inter / union if union else 1.0,
                 dice=2 * inter / float(truth.sum() + pred.sum()) if truth.sum() + pred.sum() else 1.0)
        recs.append(m)
    with open(os.path.join(out_dir, "analysis.json"), "w") as f:
        json.dump(recs, f, indent=1)
    return recs


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    _config.add_arguments(ap)
    ap.add_argument("--weights", default="my_model")
    ap.add_argument("--out", default="analysis")
    ap.add_argument("--count", type=int, default=3)
    args = ap.parse_args(argv)
    cfg = _config.from_args(args)
    for r in analyze(cfg, args.weights, args.out, args.count):
        print(json.dumps(r))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
