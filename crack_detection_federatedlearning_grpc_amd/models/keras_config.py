"""Keras ``model_config`` / ``training_config`` JSON for the U-Net (what ``model.save('x.h5')`` stores).

Mirrors the functional-model config TF2 Keras writes for the graph built at
/root/reference/client_fit_model.py:92-150 (and test/Segmentation.py:102-159, saved at :177-178), so a
``.h5`` written by this framework carries the same root attributes as a Keras checkpoint.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional

from .spec import Layer, build_layers

KERAS_VERSION = "2.8.0"


def _init(name: str) -> Dict:
    return {"class_name": name, "config": {"seed": None} if name == "GlorotUniform" else {}}


def _conv_common(ly: Layer) -> Dict:
    return {"name": ly.name, "trainable": True, "dtype": "float32", "filters": ly.cout,
            "kernel_size": [ly.ksize, ly.ksize], "strides": [ly.stride, ly.stride], "padding": "same",
            "data_format": "channels_last", "dilation_rate": [1, 1], "groups": 1, "activation": ly.activation,
            "use_bias": True, "kernel_initializer": _init("GlorotUniform"), "bias_initializer": _init("Zeros"),
            "kernel_regularizer": None, "bias_regularizer": None, "activity_regularizer": None,
            "kernel_constraint": None, "bias_constraint": None}


def layer_config(ly: Layer, img_size: int) -> Dict:
    if ly.kind == "input":
        return {"class_name": "InputLayer", "config": {"batch_input_shape": [None, img_size, img_size, 3],
                                                        "dtype": "float32", "sparse": False, "ragged": False,
                                                        "name": ly.name}}
    if ly.kind == "conv":
        return {"class_name": "Conv2D", "config": _conv_common(ly)}
    if ly.kind == "sepconv":
        c = _conv_common(ly)
        c.pop("groups")
        c.pop("kernel_initializer")
        c.pop("kernel_regularizer")
        c.pop("kernel_constraint")
        c.update({"depth_multiplier": 1, "depthwise_initializer": _init("GlorotUniform"),
                  "pointwise_initializer": _init("GlorotUniform"), "depthwise_regularizer": None,
                  "pointwise_regularizer": None, "depthwise_constraint": None, "pointwise_constraint": None})
        return {"class_name": "SeparableConv2D", "config": c}
    if ly.kind == "convt":
        c = _conv_common(ly)
        c.pop("groups")
        c["output_padding"] = None
        return {"class_name": "Conv2DTranspose", "config": c}
    if ly.kind == "bn":
        return {"class_name": "BatchNormalization", "config": {
            "name": ly.name, "trainable": True, "dtype": "float32", "axis": [3], "momentum": 0.99, "epsilon": 0.001,
            "center": True, "scale": True, "beta_initializer": _init("Zeros"), "gamma_initializer": _init("Ones"),
            "moving_mean_initializer": _init("Zeros"), "moving_variance_initializer": _init("Ones"),
            "beta_regularizer": None, "gamma_regularizer": None, "beta_constraint": None, "gamma_constraint": None}}
    if ly.kind == "act":
        return {"class_name": "Activation", "config": {"name": ly.name, "trainable": True, "dtype": "float32",
                                                       "activation": "relu"}}
    if ly.kind == "pool":
        return {"class_name": "MaxPooling2D", "config": {"name": ly.name, "trainable": True, "dtype": "float32",
                                                         "pool_size": [3, 3], "padding": "same", "strides": [2, 2],
                                                         "data_format": "channels_last"}}
    if ly.kind == "up":
        return {"class_name": "UpSampling2D", "config": {"name": ly.name, "trainable": True, "dtype": "float32",
                                                         "size": [2, 2], "data_format": "channels_last",
                                                         "interpolation": "nearest"}}
    if ly.kind == "add":
        return {"class_name": "Add", "config": {"name": ly.name, "trainable": True, "dtype": "float32"}}
    raise ValueError(ly.kind)


def model_config(img_size: int = 128, layers: Optional[List[Layer]] = None) -> Dict:
    layers = layers or build_layers(img_size)
    out = []
    for ly in layers:
        d = layer_config(ly, img_size)
        d["name"] = ly.name
        d["inbound_nodes"] = [] if not ly.inbound else [[[src, 0, 0, {}] for src in ly.inbound]]
        out.append(d)
    return {"class_name": "Functional", "config": {"name": "model", "layers": out,
                                                  "input_layers": [[layers[0].name, 0, 0]],
                                                  "output_layers": [[layers[-1].name, 0, 0]]},
            "keras_version": KERAS_VERSION, "backend": "tensorflow"}


def training_config(lr: float = 1e-3, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-7) -> Dict:
    """compile(optimizer="Adam", loss="binary_crossentropy", metrics=['accuracy']) - client_fit_model.py:157."""
    return {"loss": "binary_crossentropy", "metrics": [[{"class_name": "MeanMetricWrapper", "config": {
        "name": "accuracy", "dtype": "float32", "fn": "binary_accuracy"}}]], "weighted_metrics": None,
            "loss_weights": None, "optimizer_config": {"class_name": "Adam", "config": {
                "name": "Adam", "learning_rate": lr, "decay": 0.0, "beta_1": beta1, "beta_2": beta2,
                "epsilon": eps, "amsgrad": False}}}


def model_config_json(img_size: int = 128) -> str:
    return json.dumps(model_config(img_size))
