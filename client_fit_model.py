"""Compat module for the reference's local trainer (/root/reference/client_fit_model.py).

Same public names: ``Generator`` (data Sequence, :19-43), ``learning_fit(mt, ec, bs, pr, cr)`` (:46-240) with
``gen_train_val_data`` / ``change_model_layers`` / ``train_model_tosave`` / ``Predict`` / ``manage_train``, and the
``contour`` post-processing the reference calls but never defines. The numeric work runs on the
framework's engines (MI355X HIP kernels on a GPU, fp32 reference on CPU).
"""
from __future__ import annotations

import pickle
from typing import List, Optional, Sequence

import numpy as np

from crack_detection_federatedlearning_grpc_amd import config as _config
from crack_detection_federatedlearning_grpc_amd.fl import codec
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable, build_layers
from crack_detection_federatedlearning_grpc_amd.post.contour import crack_metrics


class Generator:
    """client_fit_model.py:19-43: ``len = n // batch``; item = (x / 255, mask > 0) batches.

    Accepts image/mask path lists (decoded with PIL + the native bilinear resize) or in-memory uint8 arrays.
    """

    def __init__(self, input_img_paths, target_img_paths, batch_size, img_size):
        self.x, self.y = input_img_paths, target_img_paths
        self.batch_size, self.img_size = batch_size, img_size

    def __len__(self):
        return len(self.y) // self.batch_size

    def __getitem__(self, idx):
        from crack_detection_federatedlearning_grpc_amd.data.folder import load_image, load_mask
        sl = slice(idx * self.batch_size, (idx + 1) * self.batch_size)
        bx, by = self.x[sl], self.y[sl]
        if isinstance(self.x, np.ndarray):
            return bx / 255, (by > 0).astype(np.uint8)[..., None] / 1
        xs = np.stack([load_image(p, self.img_size) for p in bx])
        ys = np.stack([load_mask(p, self.img_size) for p in by])[..., None]
        return xs / 255, ys / 1


def contour(img) -> dict:
    """test/Segmentation2.py:114-141 - returns the crack metrics instead of printing/writing images."""
    return crack_metrics(np.asarray(img))


class learning_fit(object):
    """client_fit_model.py:46-240. ``pr`` is the (pickled or flat-encoded) initial global weights."""

    def __init__(self, mt, ec, bs, pr, cr, cfg: Optional[_config.FLConfig] = None):
        self.model_type, self.epochs, self.batch_size = mt, ec, bs
        self.params = codec.decode(pr)[0] if pr else []
        self.round = cr
        self.cfg = cfg or _config.FLConfig()
        self.table = ParamTable()
        self._fit = None

    def _trainer(self):
        if self._fit is None:
            from crack_detection_federatedlearning_grpc_amd.train.factory import make_trainer
            self._fit = make_trainer(self.cfg, "learning_fit", table=self.table)
        return self._fit

    def gen_train_val_data(self):
        d = self._trainer().data
        return (Generator(np.asarray(d.images)[d.train_idx], np.asarray(d.masks)[d.train_idx], self.cfg.batch_size,
                          (self.cfg.img_size, self.cfg.img_size)),
                Generator(np.asarray(d.images)[d.val_idx], np.asarray(d.masks)[d.val_idx], self.cfg.batch_size,
                          (self.cfg.img_size, self.cfg.img_size)))

    def change_model_layers(self):
        """:92-150 - the U-Net; returned as the Keras-ordered layer table."""
        return build_layers(self.cfg.img_size)

    def train_model_tosave(self, params):
        fit = self._trainer()
        fit.set_weights(params if params is not None else self.params)
        fit.train_round(self.round)
        return fit

    def Predict(self, model) -> List[dict]:
        """:176-223 with the index bug fixed."""
        d = model.data
        return model.predict_and_analyze(d.val_idx[:min(16, len(d.val_idx))])

    def manage_train(self, params=None, cr=None):
        """:225-240: train one round, write ./saved_weight/weights.pickle, return the weights."""
        print(f"### Model Training - Round: {cr} ###")
        if self.params == [] and params is None:
            return []
        if cr is not None:
            self.round = cr
        if params is not None and isinstance(params, (bytes, bytearray)):
            params = codec.decode(params)[0]
        fit = self.train_model_tosave(params)
        weights = fit.get_weights()
        print("### Save model weight to ./saved_weight/ ###")
        codec.save_weight_file(self.cfg.client_weight_file, weights)
        return weights
