"""Local fit loop of one FL client (the reference's ``learning_fit``, client_fit_model.py:46-240).

Per round (``train_round``), as the reference does at client_fit_model.py:152-174, 225-240:
  * fresh Adam state (the reference rebuilds + recompiles the model every round, :155-157)
  * ``epochs`` passes over the training split, Keras Sequence semantics: ``len = n // batch`` (remainder dropped,
    :27-28) and batch order shuffled every epoch (Keras ``fit(shuffle=True)`` on a Sequence)
  * validation pass per epoch (``validation_data=val_gen``, :166)
  * at ``predict_round`` run prediction + crack contour analysis (:235-237; fixed)
The numeric work is delegated to a backend: ``HipBackend`` (models/engine.py, MI355X) or ``RefBackend`` (fp32
PyTorch oracle, CPU plumbing config).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Protocol

import numpy as np

from ..config import FLConfig
from ..data.synthetic import CrackDataset
from ..models.spec import ParamTable
from ..utils.trace import phase


class StepBackend(Protocol):
    def set_flat(self, flat: np.ndarray) -> None: ...

    def get_flat(self) -> np.ndarray: ...

    def reset_optimizer(self) -> None: ...

    def train_batches(self, batches: np.ndarray) -> Dict[str, float]: ...

    def eval_batches(self, batches: np.ndarray) -> Dict[str, float]: ...

    def predict(self, idx: np.ndarray) -> np.ndarray: ...


def epoch_batches(idx: np.ndarray, batch: int, steps: int, seed: int) -> np.ndarray:
    """[steps, batch] dataset indices; Sequence.__len__ = n // batch, batch order shuffled per epoch."""
    nb = len(idx) // batch
    if nb == 0:
        raise ValueError(f"split of {len(idx)} samples is smaller than one batch of {batch}")
    order = np.random.default_rng(seed).permutation(nb)
    if steps and steps > nb:
        order = np.concatenate([order] * (-(-steps // nb)))
    if steps:
        order = order[:steps]
    return np.stack([idx[b * batch:(b + 1) * batch] for b in order])


class RefBackend:
    """fp32 PyTorch reference backend (CPU path)."""

    def __init__(self, cfg: FLConfig, data: CrackDataset, table: ParamTable, device: str = "cpu"):
        import torch
        from ..models.unet_ref import RefTrainer
        self.torch = torch
        self.data = data
        self.table = table
        self.tr = RefTrainer(table, table.init_flat(cfg.seed), device, cfg.lr, cfg.beta1, cfg.beta2, cfg.adam_eps,
                             cfg.bn_momentum, cfg.bn_eps, cfg.loss)
        self.device = device

    def _batch(self, ids):
        t = self.torch
        x = t.from_numpy(self.data.images[ids].astype(np.float32) / 255.0).to(self.device)
        y = t.from_numpy(self.data.masks[ids].astype(np.float32)[..., None]).to(self.device)
        return x, y

    def set_flat(self, flat):
        self.tr.flat = self.torch.as_tensor(np.asarray(flat, np.float32), device=self.device).clone()

    def get_flat(self):
        return self.tr.flat.detach().cpu().numpy().copy()

    def reset_optimizer(self):
        self.tr.reset_optimizer()

    def optimizer_state(self):
        o = self.tr.opt
        return o.t, o.m.detach().cpu().numpy().copy(), o.v.detach().cpu().numpy().copy()

    def train_batches(self, batches):
        ls, acc = [], []
        for ids in batches:
            m = self.tr.train_step(*self._batch(ids))
            ls.append(m["loss"])
            acc.append(m["accuracy"])
        return {"loss": float(np.mean(ls)), "accuracy": float(np.mean(acc))}

    def eval_batches(self, batches):
        ls, acc = [], []
        tp = pp = t = 0.0
        for ids in batches:
            m = self.tr.evaluate(*self._batch(ids))
            ls.append(m["loss"])
            acc.append(m["accuracy"])
            tp, pp, t = tp + m["tp"], pp + m["pp"], t + m["t"]
        return {"loss": float(np.mean(ls)), "accuracy": float(np.mean(acc)),
                "iou": tp / (pp + t - tp) if pp + t - tp > 0 else 1.0,
                "dice": 2.0 * tp / (pp + t) if pp + t > 0 else 1.0}

    def predict(self, idx):
        x, _ = self._batch(idx)
        return self.tr.predict(x)[..., 0].cpu().numpy()


class LocalFit:
    def __init__(self, cfg: FLConfig, data: CrackDataset, backend: StepBackend, table: Optional[ParamTable] = None,
                 client: str = "client"):
        self.cfg = cfg
        self.data = data
        self.backend = backend
        self.table = table or ParamTable()
        self.client = client
        self.n_samples = int(len(data.train_idx))
        self.steps = cfg.steps_per_epoch or (len(data.train_idx) // cfg.batch_size)
        self.metrics_path = cfg.metrics_file
        self.last: Dict[str, float] = {}

    def set_weights(self, arrays: List[np.ndarray]) -> None:
        self.backend.set_flat(self.table.from_list(arrays))

    def get_weights(self) -> List[np.ndarray]:
        return self.table.to_list(self.backend.get_flat())

    def fedavg_device_async(self, aggregator, n_local: float):
        """Device-resident FedAvg (RCCL data plane) without a host wait: the engine's flat fp32 parameter buffer is
        reduced in place, bucketed on a side stream (first bucket = the encoder's parameters) with each bucket's
        layers repacked to bf16 there; the next round's first step waits per bucket on the device
        (``defer_until``) and records its stalls (``stall_log``) for the exposed-time split. Returns the
        ``PendingFedAvg`` (its watchdog owns the deadline), or None when the backend holds no device buffer. A failure
        while issuing was rolled back by the aggregator; the bf16 copies are rebuilt and the error raised."""
        eng = getattr(self.backend, "eng", None)
        if eng is None or eng.flat.device.type != "cuda" or not hasattr(aggregator, "fedavg_device_async"):
            return None
        eng.stall_log = []
        pending = aggregator.fedavg_device_async(eng.flat, n_local, on_bucket=eng.pack_bucket,
                                                 first_bucket=eng.split_at)
        if pending.error is not None:
            eng.stall_log = None
            eng.defer_until([])
            eng.pack()
            raise pending.error
        pending.engine = eng
        eng.defer_until(pending.events)
        return pending

    def fedavg_device(self, aggregator, n_local: float) -> bool:
        """Blocking form (the last round's synchronous report): issue, wait for the watchdog's verdict; on failure
        the local parameters are restored (after the side stream drained) and the bf16 copies, which the side
        stream may have partly repacked, rebuilt before the error propagates (the client then uploads its local
        model over gRPC). False when the backend holds no device buffer."""
        pending = self.fedavg_device_async(aggregator, n_local)
        if pending is None:
            return False
        self.settle_fedavg(pending)
        return True

    def settle_fedavg(self, pending) -> bool:
        """Wait for ``pending``; on failure roll the local model back (pre-FedAvg copy) and raise."""
        eng = pending.engine
        if pending.wait(rollback=True):
            return True
        if eng is not None:
            eng.defer_until([])
            eng.stall_log = None
            eng.pack()
        raise pending.error

    def restore_flat(self, flat: "np.ndarray | object") -> None:
        """Replace the local model by a device or host flat buffer (e.g. the round's average kept by a
        ``PendingFedAvg`` when the server ends the run while the next round was already training)."""
        eng = getattr(self.backend, "eng", None)
        if eng is not None and not isinstance(flat, np.ndarray):
            eng.defer_until([])
            eng.flat.copy_(flat)
            eng.pack()
        else:
            self.backend.set_flat(np.asarray(flat))

    def _log(self, rec: Dict) -> None:
        line = json.dumps(rec)
        print(line)
        if self.metrics_path:
            os.makedirs(os.path.dirname(os.path.abspath(self.metrics_path)), exist_ok=True)
            with open(self.metrics_path, "a") as f:
                f.write(line + "\n")

    def train_round(self, current_round: int) -> Dict[str, float]:
        cfg = self.cfg
        print(f"### Model Training - Round: {current_round} ###")
        self.backend.reset_optimizer()
        out: Dict[str, float] = {}
        tb = None
        if cfg.tensorboard:
            from ..utils.tfevents import KerasTensorBoard
            tb = KerasTensorBoard(cfg.log_dir, current_round, cfg.histogram_freq)
        # a device backend issues every epoch without a host sync and the records are read after the loop (one sync
        # per round instead of several per epoch: an epoch boundary left the GPU idle while the host read metrics and
        # uploaded the next batch table); TensorBoard histograms need the weights per epoch, so they keep the
        # per-epoch reads
        deferred = tb is None and hasattr(self.backend, "train_batches_deferred")
        issued = []
        for ep in range(cfg.epochs):
            seed = (cfg.data_seed * 1000003 + current_round * 1009 + ep) & 0x7FFFFFFF
            batches = epoch_batches(self.data.train_idx, cfg.batch_size, self.steps, seed)
            vbs = None
            if cfg.validate and len(self.data.val_idx) >= cfg.batch_size:
                vb = epoch_batches(self.data.val_idx, cfg.batch_size, 0, 0)
                vbs = vb[:max(1, min(len(vb), self.steps))]
            if deferred:
                with phase("fl/train_epoch"):
                    hm = self.backend.train_batches_deferred(batches)
                with phase("fl/validate"):
                    hv = self.backend.eval_batches_deferred(vbs) if vbs is not None else None
                issued.append((ep, int(batches.size), hm, hv))
                continue
            t0 = time.perf_counter()
            with phase("fl/train_epoch"):
                m = self.backend.train_batches(batches)
            dt = time.perf_counter() - t0
            rec = self._epoch_record(current_round, ep, int(batches.size), m, dt)
            if vbs is not None:
                with phase("fl/validate"):
                    self._val_record(rec, self.backend.eval_batches(vbs))
            self._log(rec)
            if tb is not None:
                ws = None
                if cfg.histogram_freq and ep % cfg.histogram_freq == 0:
                    flat = self.backend.get_flat()
                    ws = [(e.keras_name, flat[e.offset:e.offset + e.size]) for e in self.table.entries]
                tb.on_epoch_end(ep, rec, ws)
            out = rec
        for ep, n_img, hm, hv in issued:                      # one sync: the round's records, in epoch order
            rec = self._epoch_record(current_round, ep, n_img, hm.result(), hm.seconds())
            if hv is not None:
                self._val_record(rec, hv.result())
            self._log(rec)
            out = rec
        if tb is not None:
            tb.close()
        if current_round == cfg.predict_round and len(self.data.val_idx):
            out["predict"] = self.predict_and_analyze(self.data.val_idx[:min(4, len(self.data.val_idx))])
        self.last = out
        return out

    def _epoch_record(self, current_round: int, ep: int, n_img: int, m: Dict[str, float], dt: float) -> Dict:
        return {"client": self.client, "round": current_round, "epoch": ep + 1, "loss": m["loss"],
                "accuracy": m["accuracy"], "images": n_img, "train_s": dt, "images_per_s": n_img / max(dt, 1e-9)}

    @staticmethod
    def _val_record(rec: Dict, v: Dict[str, float]) -> None:
        rec["val_loss"], rec["val_accuracy"] = v["loss"], v["accuracy"]
        if "iou" in v:
            rec["val_iou"], rec["val_dice"] = v["iou"], v["dice"]

    def predict_and_analyze(self, idx: np.ndarray) -> List[Dict[str, float]]:
        """client_fit_model.py:176-223 + test/Segmentation2.py:114-141: predict, threshold, crack contours."""
        from ..post.contour import crack_metrics
        probs = self.backend.predict(idx)
        res = []
        for p in probs:
            res.append(crack_metrics((np.clip(p, 0, 1) * 255).astype(np.uint8)))
        print(f"### predict done ### {res}")
        return res
