"""fp32 PyTorch reference of the U-Net with Keras-exact semantics (CPU path and numerics oracle).

This is NOT the GPU compute path (that is ``models/engine.py`` on hand-written HIP kernels); it is the
correctness oracle every HIP kernel is tested against, and the device-agnostic path used by the CPU plumbing
config (BASELINE config 1). Keras semantics reproduced here:

* Conv2D stride 2 ``same``: TF pads the whole deficit bottom/right (pad_top = 0)      client_fit_model.py:100
* Conv2D 1x1 stride 2 ``same``: samples the even pixels                                client_fit_model.py:119
* SeparableConv2D: depthwise 3x3 (dm=1) then pointwise 1x1 + bias                      client_fit_model.py:109
* Conv2DTranspose 3x3 s1 ``same``: kernel (kh,kw,out,in), i.e. correlation with the flipped kernel   :129
* BatchNormalization: batch stats (biased var) for normalisation, eps 1e-3, momentum 0.99, unbiased
  variance into moving_variance (TF fused-BN convention)                                :101
* MaxPooling2D(3, s2, same): pad bottom/right with -inf                                 :116
* UpSampling2D(2): nearest                                                              :136
* sigmoid head + binary_crossentropy: TF2 Keras computes BCE from the logits            :145, :157
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from .spec import DEC_FILTERS, ENC_FILTERS, ParamTable


def _p(flat: torch.Tensor, table: ParamTable, layer: str, w: str) -> torch.Tensor:
    e = table.entry(layer, w)
    return flat[e.offset:e.offset + e.size].view(e.shape)


def tf_same_pad(size: int, k: int, s: int) -> Tuple[int, int]:
    out = -(-size // s)
    total = max((out - 1) * s + k - size, 0)
    return total // 2, total - total // 2


def conv2d_same(x: torch.Tensor, kernel_hwio: torch.Tensor, bias: Optional[torch.Tensor], stride: int) -> torch.Tensor:
    k = kernel_hwio.shape[0]
    pt, pb = tf_same_pad(x.shape[2], k, stride)
    pl, pr = tf_same_pad(x.shape[3], k, stride)
    if pt or pb or pl or pr:
        x = F.pad(x, (pl, pr, pt, pb))
    return F.conv2d(x, kernel_hwio.permute(3, 2, 0, 1), bias, stride=stride)


def sepconv_same(x, dw, pw, bias):
    c = x.shape[1]
    y = F.conv2d(F.pad(x, (1, 1, 1, 1)), dw.permute(2, 3, 0, 1), None, groups=c)
    return F.conv2d(y, pw.permute(3, 2, 0, 1), bias)


def convt_same(x, kernel_hwoi, bias):
    # TF conv2d_transpose(filter[kh,kw,out,in]) == torch conv_transpose2d(weight[in,out,kh,kw])
    return F.conv_transpose2d(x, kernel_hwoi.permute(3, 2, 0, 1), bias, padding=1)


def maxpool_same(x):
    x = F.pad(x, (0, 1, 0, 1), value=float("-inf"))
    return F.max_pool2d(x, 3, 2)


def batchnorm_train(x, gamma, beta, mm, mv, momentum: float, eps: float, training: bool = True):
    """Returns (y, new_moving_mean, new_moving_var)."""
    if not training:
        y = (x - mm.view(1, -1, 1, 1)) * torch.rsqrt(mv.view(1, -1, 1, 1) + eps) * gamma.view(1, -1, 1, 1) \
            + beta.view(1, -1, 1, 1)
        return y, mm, mv
    n = x.shape[0] * x.shape[2] * x.shape[3]
    mean = x.mean(dim=(0, 2, 3))
    var = x.var(dim=(0, 2, 3), unbiased=False)
    y = (x - mean.view(1, -1, 1, 1)) * torch.rsqrt(var.view(1, -1, 1, 1) + eps) * gamma.view(1, -1, 1, 1) \
        + beta.view(1, -1, 1, 1)
    unbiased = var.detach() * (n / max(n - 1, 1))
    new_mm = mm * momentum + mean.detach() * (1.0 - momentum)
    new_mv = mv * momentum + unbiased * (1.0 - momentum)
    return y, new_mm, new_mv


def upsample2(x):
    return x.repeat_interleave(2, dim=2).repeat_interleave(2, dim=3)


def _bf16_st(t: torch.Tensor) -> torch.Tensor:
    """bf16 rounding with a straight-through gradient (emulates bf16 activation storage)."""
    return t + (t.to(torch.bfloat16).float() - t).detach()


def unet_forward(flat: torch.Tensor, x_nhwc: torch.Tensor, table: Optional[ParamTable] = None,
                 training: bool = True, momentum: float = 0.99, eps: float = 1e-3, emulate_bf16: bool = False
                 ) -> Tuple[torch.Tensor, Dict[str, Tuple[torch.Tensor, torch.Tensor]]]:
    """x_nhwc: (B,H,W,3) float in [0,1]. Returns (logits NHWC (B,H,W,1), {bn_layer: (new_mm, new_mv)}).

    ``emulate_bf16``: round to bf16 at exactly the points where the MI355X engine stores activations or feeds bf16
    MFMA operands (conv outputs, depthwise outputs, residual joins, MFMA-packed weights, transformed MFMA inputs);
    gradients pass straight through. Used to separate dataflow bugs from bf16 storage error in the GPU tests.
    """
    table = table or ParamTable()
    r = _bf16_st if emulate_bf16 else (lambda t: t)
    P = lambda l, w: _p(flat, table, l, w)  # noqa: E731
    bn_updates: Dict[str, Tuple[torch.Tensor, torch.Tensor]] = {}

    def bn(x, name):
        y, nm, nv = batchnorm_train(x, P(name, "gamma"), P(name, "beta"), P(name, "moving_mean"),
                                    P(name, "moving_variance"), momentum, eps, training)
        bn_updates[name] = (nm, nv)
        return y

    def sep(x, s):
        c = x.shape[1]
        # the depthwise kernels stage the transformed (BN-apply + ReLU) input in LDS as bf16
        d = r(F.conv2d(F.pad(r(x), (1, 1, 1, 1)), P(s, "depthwise_kernel").permute(2, 3, 0, 1), None, groups=c))
        return r(F.conv2d(d, r(P(s, "pointwise_kernel")).permute(3, 2, 0, 1), P(s, "bias")))

    names = iter([ly.name for ly in table.weighted_layers()])
    x = x_nhwc.permute(0, 3, 1, 2)
    n = next(names)
    x = r(conv2d_same(x, r(P(n, "kernel")), P(n, "bias"), 2))    # entry MFMA kernel: bf16 weights
    x = F.relu(bn(x, next(names)))
    prev = x
    for _f in ENC_FILTERS:
        s1, b1, s2, b2, rc = next(names), next(names), next(names), next(names), next(names)
        x = F.relu(x)
        x = bn(sep(x, s1), b1)
        x = F.relu(x)
        x = bn(sep(x, s2), b2)
        x = maxpool_same(x)
        x = r(x + r(conv2d_same(r(prev), r(P(rc, "kernel")), P(rc, "bias"), 2)))
        prev = x
    for _f in DEC_FILTERS:
        t1, b1, t2, b2, rc = next(names), next(names), next(names), next(names), next(names)
        x = F.relu(x)
        x = bn(r(convt_same(x, r(P(t1, "kernel")), P(t1, "bias"))), b1)
        x = r(F.relu(x))
        x = bn(r(convt_same(x, r(P(t2, "kernel")), P(t2, "bias"))), b2)
        x = upsample2(x)
        x = r(x + r(conv2d_same(upsample2(prev), r(P(rc, "kernel")), P(rc, "bias"), 1)))
        prev = x
    h = next(names)
    logits = conv2d_same(x, P(h, "kernel"), P(h, "bias"), 1)
    return logits.permute(0, 2, 3, 1), bn_updates


def bce_with_logits_mean(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    # Keras binary_crossentropy on a Sigmoid output uses sigmoid_cross_entropy_with_logits, mean over pixels
    return (logits.clamp(min=0) - logits * target + torch.log1p(torch.exp(-logits.abs()))).mean()


def dice_loss(logits: torch.Tensor, target: torch.Tensor, smooth: float = 1.0) -> torch.Tensor:
    p = torch.sigmoid(logits)
    inter = (p * target).sum()
    return 1.0 - (2.0 * inter + smooth) / (p.sum() + target.sum() + smooth)


def seg_loss(logits, target, kind: str = "bce"):
    loss = bce_with_logits_mean(logits, target)
    if kind == "bce_dice":
        loss = loss + dice_loss(logits, target)
    return loss


def binary_accuracy(logits: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    return ((logits > 0).to(target.dtype) == target).float().mean()


class KerasAdam:
    """Keras OptimizerV2 Adam (ResourceApplyAdam): lr_t = lr*sqrt(1-b2^t)/(1-b1^t); eps NOT bias-corrected."""

    def __init__(self, numel: int, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7, device="cpu"):
        self.m = torch.zeros(numel, device=device)
        self.v = torch.zeros(numel, device=device)
        self.t = 0
        self.lr, self.b1, self.b2, self.eps = lr, beta1, beta2, eps

    def step(self, flat: torch.Tensor, grad: torch.Tensor, mask: torch.Tensor) -> None:
        self.t += 1
        lr_t = self.lr * (1 - self.b2 ** self.t) ** 0.5 / (1 - self.b1 ** self.t)
        self.m.mul_(self.b1).add_(grad * (1 - self.b1))
        self.v.mul_(self.b2).add_(grad * grad * (1 - self.b2))
        upd = lr_t * self.m / (self.v.sqrt() + self.eps)
        flat.sub_(upd * mask)


class RefTrainer:
    """Plain fp32 train step on the reference model (CPU plumbing path / oracle)."""

    def __init__(self, table: ParamTable, flat0, device="cpu", lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-7,
                 momentum=0.99, bn_eps=1e-3, loss="bce"):
        self.table = table
        self.device = torch.device(device)
        self.flat = torch.as_tensor(flat0, dtype=torch.float32, device=self.device).clone()
        self.mask = torch.as_tensor(table.trainable_mask(), device=self.device)
        self.opt = KerasAdam(table.total, lr, beta1, beta2, eps, self.device)
        self.momentum, self.bn_eps, self.loss_kind = momentum, bn_eps, loss

    def reset_optimizer(self) -> None:
        self.opt = KerasAdam(self.table.total, self.opt.lr, self.opt.b1, self.opt.b2, self.opt.eps, self.device)

    def train_step(self, x: torch.Tensor, y: torch.Tensor) -> Dict[str, float]:
        p = self.flat.detach().requires_grad_(True)
        logits, bnu = unet_forward(p, x, self.table, True, self.momentum, self.bn_eps)
        loss = seg_loss(logits, y, self.loss_kind)
        g, = torch.autograd.grad(loss, p)
        with torch.no_grad():
            self.opt.step(self.flat, g, self.mask)
            for name, (nm, nv) in bnu.items():
                e1 = self.table.entry(name, "moving_mean")
                e2 = self.table.entry(name, "moving_variance")
                self.flat[e1.offset:e1.offset + e1.size] = nm
                self.flat[e2.offset:e2.offset + e2.size] = nv
        return {"loss": float(loss.detach()), "accuracy": float(binary_accuracy(logits.detach(), y))}

    @torch.no_grad()
    def evaluate(self, x: torch.Tensor, y: torch.Tensor) -> Dict[str, float]:
        """Loss / accuracy of the batch plus the crack-class counts (tp, pp, t) for IoU / Dice over a pass."""
        logits, _ = unet_forward(self.flat, x, self.table, False, self.momentum, self.bn_eps)
        pred = logits > 0
        tgt = y > 0.5
        return {"loss": float(seg_loss(logits, y, self.loss_kind)), "accuracy": float(binary_accuracy(logits, y)),
                "tp": float((pred & tgt).sum()), "pp": float(pred.sum()), "t": float(tgt.sum())}

    @torch.no_grad()
    def predict(self, x: torch.Tensor) -> torch.Tensor:
        logits, _ = unet_forward(self.flat, x, self.table, False, self.momentum, self.bn_eps)
        return torch.sigmoid(logits)
