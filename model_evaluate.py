"""Server-side global model (missing from the reference snapshot; used at fl_server.py:12,24,31,230-231).

Interface reconstructed in SURVEY.md §2.1 C6: ``evaluate_LocalModel(bs, img, labels)`` with ``buildGlobalModel``,
``get_weights`` (bytes for ``buffer_chunk``), ``train_model_tosave`` (evaluation -> {'loss','accuracy'}) and
``saved_model``. The reference advertises mobilenet_v2/224; here the global model IS the U-Net the
clients train, so ``set_weights`` always matches.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from crack_detection_federatedlearning_grpc_amd import config as _config
from crack_detection_federatedlearning_grpc_amd.ckpt.h5 import save_keras_h5
from crack_detection_federatedlearning_grpc_amd.fl import codec
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable


class evaluate_LocalModel:
    def __init__(self, bs: int = 16, img: int = 128, labels=None, cfg: Optional[_config.FLConfig] = None):
        self.bs, self.img, self.labels = bs, img, labels
        self.cfg = cfg or _config.FLConfig(batch_size=bs)
        self.table = ParamTable()
        self._eval = None

    def buildGlobalModel(self, ch: int = 3, lr: float = 1e-3) -> np.ndarray:
        return self.table.init_flat(self.cfg.seed)

    def get_weights(self, model: np.ndarray) -> bytes:
        """Bytes for ``buffer_chunk``: the reference client ``pickle.loads`` them (client_fit_model.py:51)."""
        return codec.encode(self.table.to_list(model), "pickle")

    def train_model_tosave(self, model: np.ndarray, max_batches: int = 0) -> Dict[str, float]:
        """fl_server.py:31 expects {'loss','accuracy'} of the global model.

        With a visible GPU the global model is evaluated by the MI355X engine at the clients' resolution
        (``cfg.img_size``) over the SAME held-out split the clients validate on (inference-mode BN, the same
        validation path they run): the folder dataset's reference split, or - synthetic data - client rank 0's shard
        (same seed, sample count and split), so the server's numbers are comparable to that client's ``val_*``;
        ``max_batches`` bounds the pass. On a CPU-only server the fp32 oracle evaluates a small (<= 64^2) shard."""
        if self._eval is None:
            import dataclasses
            from crack_detection_federatedlearning_grpc_amd.train.factory import make_trainer, resolve_device
            dev = resolve_device(self.cfg)
            if dev == "cuda":
                cfg = dataclasses.replace(self.cfg, device="cuda", batch_size=self.bs)
            else:
                cfg = dataclasses.replace(self.cfg, device="cpu", synthetic_samples=max(2 * self.bs, 32),
                                          val_samples=self.bs, img_size=min(self.cfg.img_size, 64),
                                          batch_size=self.bs)
            self._eval = make_trainer(cfg, "server-eval", rank=0, table=self.table, device=dev)
        self._eval.backend.set_flat(model)
        from crack_detection_federatedlearning_grpc_amd.train.local import epoch_batches
        vb = epoch_batches(self._eval.data.val_idx, self.bs, 0, 0)
        return self._eval.backend.eval_batches(vb[:max_batches] if max_batches else vb)

    def saved_model(self, model: np.ndarray, path: str = "global_model.h5") -> str:
        save_keras_h5(path, self.table, model, self.img)
        return path


def server_evaluator(cfg: _config.FLConfig):
    """Evaluation hook for the server (enabled with FL_SERVER_EVAL=1)."""
    import os
    if os.environ.get("FL_SERVER_EVAL", "0") != "1":
        return None
    ev = evaluate_LocalModel(cfg.batch_size, cfg.img_size, cfg=cfg)
    return ev.train_model_tosave
