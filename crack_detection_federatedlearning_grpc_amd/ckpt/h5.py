"""Keras-layout ``.h5`` checkpoints over the native HDF5 writer/reader (``csrc/native/h5lite.cpp``).

Two layouts, as TF2 Keras writes them:
* full model (``model.save('x.h5')`` / ``ModelCheckpoint('crack_segmentation.h5')``, test/Segmentation.py:177-178):
  root attrs ``backend``, ``keras_version``, ``model_config``, ``training_config``; group ``model_weights`` (attrs
  ``layer_names``, ``backend``, ``keras_version``) with one group per layer (attr ``weight_names``) holding
  ``<layer>/<weight>:0`` datasets; group ``optimizer_weights`` (attr ``weight_names``) with Adam ``iter``/``m``/``v``.
* weights only (``model.save_weights('x.h5')``): the ``model_weights`` content at the root.
``load_weights_h5`` accepts both; like Keras ``load_weights`` without ``by_name`` it falls back to positional
matching of weighted layers when names differ (non-clean-session names such as ``conv2d_9``).
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Tuple

import numpy as np

from .._native_loader import native
from ..models.keras_config import KERAS_VERSION, model_config, training_config
from ..models.spec import ParamTable


def _layer_tree(table: ParamTable, flat: np.ndarray) -> Dict:
    groups = {}
    flat = np.asarray(flat, np.float32)
    for ly in table.layers:
        ents = [table.entry(ly.name, w) for w, _, _ in ly.weights]
        g = {"attrs": {"weight_names": [e.keras_name.encode() for e in ents]}, "groups": {}, "datasets": {}}
        if ents:
            g["groups"][ly.name] = {"attrs": {}, "groups": {}, "datasets": {
                f"{e.wname}:0": np.ascontiguousarray(flat[e.offset:e.offset + e.size].reshape(e.shape))
                for e in ents}}
        groups[ly.name] = g
    return {"attrs": {"layer_names": [ly.name.encode() for ly in table.layers], "backend": "tensorflow",
                      "keras_version": KERAS_VERSION}, "groups": groups, "datasets": {}}


def save_weights_h5(path: str, table: ParamTable, flat: np.ndarray) -> None:
    native().h5lite.write_file(path, _layer_tree(table, flat))


def save_keras_h5(path: str, table: ParamTable, flat: np.ndarray, img_size: int = 128,
                  optimizer: Optional[Tuple[int, np.ndarray, np.ndarray]] = None, lr: float = 1e-3) -> None:
    """Full-model Keras HDF5. ``optimizer`` = (iterations, m_flat, v_flat) over the same flat layout."""
    mw = _layer_tree(table, flat)
    tree = {"attrs": {"backend": "tensorflow", "keras_version": KERAS_VERSION,
                      "model_config": json.dumps(model_config(img_size)),
                      "training_config": json.dumps(training_config(lr))},
            "groups": {"model_weights": mw}, "datasets": {}}
    if optimizer is not None:
        it, m, v = optimizer
        names = [b"Adam/iter:0"]
        adam: Dict = {"attrs": {}, "groups": {}, "datasets": {"iter:0": np.asarray(it, np.int64)}}
        for kind, buf in (("m", m), ("v", v)):
            for e in table.entries:
                if not e.trainable:
                    continue
                names.append(f"Adam/{e.layer}/{e.wname}/{kind}:0".encode())
                lg = adam["groups"].setdefault(e.layer, {"attrs": {}, "groups": {}, "datasets": {}})
                wg = lg["groups"].setdefault(e.wname, {"attrs": {}, "groups": {}, "datasets": {}})
                wg["datasets"][f"{kind}:0"] = np.ascontiguousarray(
                    np.asarray(buf, np.float32)[e.offset:e.offset + e.size].reshape(e.shape))
        tree["groups"]["optimizer_weights"] = {"attrs": {"weight_names": names}, "groups": {"Adam": adam},
                                               "datasets": {}}
    native().h5lite.write_file(path, tree)


def _s(v) -> str:
    return v.decode() if isinstance(v, (bytes, bytearray)) else str(v)


def _get(node: Dict, path: str):
    cur = node
    parts = path.split("/")
    for i, p in enumerate(parts):
        if i == len(parts) - 1 and p in cur.get("datasets", {}):
            return cur["datasets"][p]["data"]
        cur = cur["groups"][p]
    return cur


def read_h5(path: str) -> Dict:
    return native().h5lite.read_file(path)


def load_weights_h5(path: str, table: ParamTable) -> np.ndarray:
    tree = read_h5(path)
    root = tree["groups"]["model_weights"] if "model_weights" in tree["groups"] else tree
    names = [_s(n) for n in root["attrs"].get("layer_names", [])] or sorted(root["groups"])
    flat = np.zeros(table.total, np.float32)
    file_layers: List[Tuple[str, List[str]]] = []
    for n in names:
        g = root["groups"].get(n)
        if g is None:
            continue
        wn = [_s(w) for w in g["attrs"].get("weight_names", [])]
        if wn:
            file_layers.append((n, wn))
    ours = table.weighted_layers()
    if len(file_layers) != len(ours):
        raise ValueError(f"{path}: {len(file_layers)} weighted layers in file, model has {len(ours)}")
    for ly, (fname, wnames) in zip(ours, file_layers):
        if len(wnames) != len(ly.weights):
            raise ValueError(f"{path}: layer {fname} has {len(wnames)} weights, {ly.name} expects {len(ly.weights)}")
        g = root["groups"][fname]
        for (wname, shape, _), fw in zip(ly.weights, wnames):
            arr = np.asarray(_get(g, fw), np.float32)
            if tuple(arr.shape) != tuple(shape):
                raise ValueError(f"{path}: {fw} has shape {arr.shape}, expected {shape}")
            e = table.entry(ly.name, wname)
            flat[e.offset:e.offset + e.size] = arr.reshape(-1)
    return flat


def load_optimizer_h5(path: str, table: ParamTable) -> Optional[Tuple[int, np.ndarray, np.ndarray]]:
    tree = read_h5(path)
    ow = tree["groups"].get("optimizer_weights")
    if ow is None:
        return None
    adam = ow["groups"]["Adam"]
    it = int(np.asarray(adam["datasets"]["iter:0"]["data"]))
    m = np.zeros(table.total, np.float32)
    v = np.zeros(table.total, np.float32)
    for e in table.entries:
        if not e.trainable:
            continue
        g = adam["groups"][e.layer]["groups"][e.wname]["datasets"]
        m[e.offset:e.offset + e.size] = np.asarray(g["m:0"]["data"]).reshape(-1)
        v[e.offset:e.offset + e.size] = np.asarray(g["v:0"]["data"]).reshape(-1)
    return it, m, v
