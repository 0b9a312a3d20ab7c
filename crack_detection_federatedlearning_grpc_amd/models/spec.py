"""U-Net layer/parameter table with Keras-exact names, shapes and ``get_weights()`` order.

The architecture is the Keras-example "U-Net-like" (Xception-style) network built at
/root/reference/client_fit_model.py:92-150 (duplicate: test/Segmentation.py:102-159):

  entry   Conv2D(32,3,s2,same) -> BN -> ReLU                                   :100-102
  enc x3  [ReLU, SepConv(F,3), BN, ReLU, SepConv(F,3), BN, MaxPool(3,s2)]
          + Conv2D(F,1,s2)(prev) residual, add                        F=64,128,256  :107-123
  dec x4  [ReLU, ConvT(F,3), BN, ReLU, ConvT(F,3), BN, UpSample(2)]
          + Conv2D(F,1)(UpSample(prev)) residual, add            F=256,128,64,32  :127-142
  head    Conv2D(1,1,sigmoid)                                                   :145

Weight arrays: 112 arrays, 82 trainable, 2,058,145 parameters; names are the clean-session
auto-names (test/Segmentation.py:163 calls clear_session) so the ``.h5`` layout matches a Keras checkpoint.
Layouts: Conv2D kernel (kh,kw,Cin,Cout); SeparableConv2D depthwise (3,3,C,1), pointwise (1,1,C,F);
Conv2DTranspose kernel (kh,kw,Cout,Cin); BatchNormalization gamma, beta, moving_mean, moving_variance.

All arrays live in ONE flat fp32 buffer (``ParamTable.offsets``) so that FedAvg, Adam and the wire codec touch a
single contiguous allocation (one RCCL all-reduce, one multi-tensor Adam launch).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

ENC_FILTERS = (64, 128, 256)
DEC_FILTERS = (256, 128, 64, 32)
ENTRY_FILTERS = 32


@dataclass
class Layer:
    name: str                      # Keras auto-name (clean session)
    kind: str                      # conv | sepconv | convt | bn | input | act | pool | add | up
    cin: int = 0
    cout: int = 0
    ksize: int = 0
    stride: int = 1
    activation: str = "linear"
    inbound: List[str] = field(default_factory=list)
    weights: List[Tuple[str, Tuple[int, ...], bool]] = field(default_factory=list)  # (wname, shape, trainable)


class _Namer:
    def __init__(self) -> None:
        self.counts: Dict[str, int] = {}

    def __call__(self, base: str) -> str:
        n = self.counts.get(base, 0)
        self.counts[base] = n + 1
        return base if n == 0 else f"{base}_{n}"


def build_layers(img_size: int = 128) -> List[Layer]:
    """Every Keras layer (weighted or not) in creation order, with inbound-layer names."""
    nm = _Namer()
    L: List[Layer] = []

    def add(layer: Layer) -> str:
        L.append(layer)
        return layer.name

    def conv(cin, cout, k, s, src, act="linear"):
        n = nm("conv2d")
        return add(Layer(n, "conv", cin, cout, k, s, act, [src],
                         [("kernel", (k, k, cin, cout), True), ("bias", (cout,), True)]))

    def sep(cin, cout, src):
        n = nm("separable_conv2d")
        return add(Layer(n, "sepconv", cin, cout, 3, 1, "linear", [src],
                         [("depthwise_kernel", (3, 3, cin, 1), True), ("pointwise_kernel", (1, 1, cin, cout), True),
                          ("bias", (cout,), True)]))

    def convt(cin, cout, src):
        n = nm("conv2d_transpose")
        return add(Layer(n, "convt", cin, cout, 3, 1, "linear", [src],
                         [("kernel", (3, 3, cout, cin), True), ("bias", (cout,), True)]))

    def bn(c, src):
        n = nm("batch_normalization")
        return add(Layer(n, "bn", c, c, inbound=[src],
                         weights=[("gamma", (c,), True), ("beta", (c,), True),
                                  ("moving_mean", (c,), False), ("moving_variance", (c,), False)]))

    def relu(src):
        return add(Layer(nm("activation"), "act", activation="relu", inbound=[src]))

    def pool(src):
        return add(Layer(nm("max_pooling2d"), "pool", ksize=3, stride=2, inbound=[src]))

    def up(src):
        return add(Layer(nm("up_sampling2d"), "up", stride=2, inbound=[src]))

    def addl(a, b):
        return add(Layer(nm("add"), "add", inbound=[a, b]))

    x = add(Layer(nm("input_1"), "input", 3, 3, inbound=[]))
    x = conv(3, ENTRY_FILTERS, 3, 2, x)
    x = bn(ENTRY_FILTERS, x)
    x = relu(x)
    prev, cprev = x, ENTRY_FILTERS
    c = ENTRY_FILTERS
    for f in ENC_FILTERS:
        x = relu(x)
        x = sep(c, f, x)
        x = bn(f, x)
        x = relu(x)
        x = sep(f, f, x)
        x = bn(f, x)
        x = pool(x)
        r = conv(cprev, f, 1, 2, prev)
        x = addl(x, r)
        prev, cprev, c = x, f, f
    for f in DEC_FILTERS:
        x = relu(x)
        x = convt(c, f, x)
        x = bn(f, x)
        x = relu(x)
        x = convt(f, f, x)
        x = bn(f, x)
        x = up(x)
        r = up(prev)
        r = conv(cprev, f, 1, 1, r)
        x = addl(x, r)
        prev, cprev, c = x, f, f
    conv(c, 1, 1, 1, x, act="sigmoid")
    return L


@dataclass
class ParamEntry:
    layer: str
    wname: str
    shape: Tuple[int, ...]
    trainable: bool
    offset: int
    size: int

    @property
    def keras_name(self) -> str:      # e.g. "conv2d/kernel:0" (TF2 variable name)
        return f"{self.layer}/{self.wname}:0"


class ParamTable:
    """Keras-ordered table of the 112 weight arrays over one flat fp32 buffer."""

    def __init__(self, layers: Optional[Sequence[Layer]] = None, align: int = 64):
        self.layers = list(layers) if layers is not None else build_layers()
        self.entries: List[ParamEntry] = []
        off = 0
        for ly in self.layers:
            for wname, shape, tr in ly.weights:
                size = int(np.prod(shape))
                self.entries.append(ParamEntry(ly.name, wname, tuple(shape), tr, off, size))
                # align every array to `align` floats (256 B) so vectorised kernels never straddle arrays
                off += (size + align - 1) // align * align
        self.total = off
        self.by_key: Dict[Tuple[str, str], ParamEntry] = {(e.layer, e.wname): e for e in self.entries}

    # -- queries ----------------------------------------------------------------------------
    @property
    def num_params(self) -> int:
        return sum(e.size for e in self.entries)

    @property
    def num_trainable(self) -> int:
        return sum(e.size for e in self.entries if e.trainable)

    def __len__(self) -> int:
        return len(self.entries)

    def entry(self, layer: str, wname: str) -> ParamEntry:
        return self.by_key[(layer, wname)]

    def weighted_layers(self) -> List[Layer]:
        return [ly for ly in self.layers if ly.weights]

    def layer(self, name: str) -> Layer:
        for ly in self.layers:
            if ly.name == name:
                return ly
        raise KeyError(name)

    def trainable_mask(self) -> np.ndarray:
        m = np.zeros(self.total, np.float32)
        for e in self.entries:
            if e.trainable:
                m[e.offset:e.offset + e.size] = 1.0
        return m

    # -- flat <-> list[np.ndarray] (Keras get_weights / set_weights) ---------------------------
    def to_list(self, flat: np.ndarray) -> List[np.ndarray]:
        flat = np.asarray(flat, dtype=np.float32)
        return [flat[e.offset:e.offset + e.size].reshape(e.shape).copy() for e in self.entries]

    def from_list(self, arrays: Sequence[np.ndarray]) -> np.ndarray:
        if len(arrays) != len(self.entries):
            raise ValueError(f"expected {len(self.entries)} weight arrays, got {len(arrays)}")
        flat = np.zeros(self.total, np.float32)
        for e, a in zip(self.entries, arrays):
            a = np.asarray(a, dtype=np.float32)
            if tuple(a.shape) != e.shape:
                raise ValueError(f"{e.keras_name}: expected shape {e.shape}, got {tuple(a.shape)}")
            flat[e.offset:e.offset + e.size] = a.reshape(-1)
        return flat

    def init_flat(self, seed: int = 0) -> np.ndarray:
        """Keras default initialisers: glorot_uniform kernels, zero bias, BN (1, 0, 0, 1)."""
        rng = np.random.default_rng(seed)
        flat = np.zeros(self.total, np.float32)
        for e in self.entries:
            if e.wname in ("kernel", "depthwise_kernel", "pointwise_kernel"):
                fan_in, fan_out = _glorot_fans(e.shape)
                lim = math.sqrt(6.0 / (fan_in + fan_out))
                v = rng.uniform(-lim, lim, e.size).astype(np.float32)
            elif e.wname in ("gamma", "moving_variance"):
                v = np.ones(e.size, np.float32)
            else:
                v = np.zeros(e.size, np.float32)
            flat[e.offset:e.offset + e.size] = v
        return flat


def _glorot_fans(shape: Tuple[int, ...]) -> Tuple[int, int]:
    # keras.initializers._compute_fans: receptive field * (shape[-2], shape[-1])
    rf = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    return shape[-2] * rf, shape[-1] * rf


def forward_flops_per_image(img: int) -> float:
    """Dense forward FLOPs (2*MAC) of one image at img x img (1.25 G @128)."""
    L = build_layers(img)
    fl = 0.0
    r = img
    res = {"input_1": img}
    for ly in L:
        if ly.kind == "input":
            continue
        src = res[ly.inbound[0]]
        if ly.kind == "conv":
            out = -(-src // ly.stride)
            fl += 2.0 * out * out * ly.ksize * ly.ksize * ly.cin * ly.cout
        elif ly.kind == "sepconv":
            out = src
            fl += 2.0 * out * out * (9 * ly.cin + ly.cin * ly.cout)
        elif ly.kind == "convt":
            out = src
            fl += 2.0 * out * out * 9 * ly.cin * ly.cout
        elif ly.kind == "pool":
            out = -(-src // 2)
        elif ly.kind == "up":
            out = src * 2
        else:
            out = src
        res[ly.name] = out
    return fl
