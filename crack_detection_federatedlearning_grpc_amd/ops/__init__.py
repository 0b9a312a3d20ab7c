"""PyTorch autograd ops over the gfx950 kernels, for models other than the fused U-Net engine.

The engine (``models/engine.py``) schedules the whole U-Net step itself; these ops expose the same kernels one layer
at a time so a user can compose a different NHWC network with ``torch.autograd``. Tensors are NHWC; activations
are bf16 (``torch.bfloat16``); weights are fp32 in the Keras layouts the reference uses (Conv2D HWIO
``(kh, kw, in, out)``, Conv2DTranspose ``(kh, kw, out, in)``, depthwise ``(3, 3, C, 1)``) and are packed to bf16
``[N][K]`` on every call (cheap: the pack kernel). Padding is TF "same".

    y = conv2d(x, w, b)                   # 3x3 / 1x1, stride 1, Conv2D        (kernel: conv3x3.hip / conv_igemm.hip)
    y = conv2d_transpose(x, w, b)         # 3x3, stride 1, Conv2DTranspose     (kernel: conv3x3.hip, flip in pack)
    y = depthwise3x3(x, w)                # SeparableConv2D first stage        (kernel: dwconv.hip)

Backward: data gradient with the dgrad-packed weights through the same forward kernels, weight gradient through
conv_wgrad / conv3x3_wgrad / dw_wgrad (fp32 accumulation). Shapes the kernels do not cover raise.
"""
from __future__ import annotations

from typing import Optional

import torch

from .._native_loader import hip

PK_CONV, PK_CONV_DGRAD1x1, PK_CONVT, PK_CONVT_DGRAD, PK_PW, PK_PW_DGRAD = range(6)


def _bits(t: torch.Tensor) -> torch.Tensor:
    if t.dtype != torch.bfloat16:
        raise TypeError("activations must be torch.bfloat16 NHWC")
    return t.contiguous().view(torch.int16)


def _pack(w: torch.Tensor, kind: int, ks: int, cin: int, cout: int) -> torch.Tensor:
    C = hip()
    flat = w.detach().reshape(-1).float().contiguous()
    out = torch.empty(ks * ks * cin * cout, dtype=torch.int16, device=w.device)
    table = C.make_pack_table([(kind, 0, 0, ks, cin, cout)], flat)
    C.pack_weights(flat, out, table, 1, out.numel())
    return out


def _conv_fwd(xb: torch.Tensor, wp: torch.Tensor, bias: Optional[torch.Tensor], B: int, H: int, W: int, Cin: int,
              N: int, ks: int) -> torch.Tensor:
    C = hip()
    pad = (ks - 1) // 2
    y = torch.empty(B, H, W, N, dtype=torch.int16, device=xb.device)
    splits = C.conv_splits(B, H, W, N, ks, 1, pad, Cin)
    ws = torch.empty(splits * B * H * W * N, dtype=torch.float32, device=xb.device) if splits > 1 else None
    C.conv_igemm(xb, wp, bias, y, None, None, 0, B, H, W, Cin, 0, H, W, N, ks, 1, pad, pad, ws)
    return y


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, transpose: bool):
        B, H, W, Cin = x.shape
        ks = w.shape[0]
        N = w.shape[2] if transpose else w.shape[3]
        if ks not in (1, 3) or w.shape[1] != ks or (transpose and ks != 3):
            raise ValueError("supported: 3x3 (Conv2D / Conv2DTranspose) and 1x1 Conv2D, stride 1")
        if Cin % 32 or N % 32:
            raise ValueError("channel counts must be multiples of 32")
        xb = _bits(x)
        kind = PK_CONVT if transpose else PK_PW            # 3x3 Conv2D arrives here as its ConvT equivalent
        y = _conv_fwd(xb, _pack(w, kind, ks, Cin, N), None if b is None else b.detach().float().contiguous(),
                      B, H, W, Cin, N, ks)
        ctx.save_for_backward(x, w)
        ctx.meta = (B, H, W, Cin, N, ks, transpose, b is not None)
        return y.view(torch.bfloat16)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        B, H, W, Cin, N, ks, transpose, has_b = ctx.meta
        C = hip()
        gb = _bits(gy)
        gx = gw = gbias = None
        if ctx.needs_input_grad[0]:
            # dgrad of a stride-1 "same" conv = the same kernel run on dy with the dgrad-packed weights (3x3: the
            # flipped, in/out-swapped kernel; the pack kernel owns the permutation)
            wd = _pack(w, PK_CONVT_DGRAD, 3, Cin, N) if ks == 3 else _pack(w, PK_PW_DGRAD, 1, Cin, N)
            gx = _conv_fwd(gb, wd, None, B, H, W, N, Cin, ks).view(torch.bfloat16)
        if ctx.needs_input_grad[1]:
            gw = torch.zeros(ks * ks * Cin * N, dtype=torch.float32, device=x.device)
            pad = (ks - 1) // 2
            C.conv_wgrad(_bits(x), gb, gw, None, 0, B, H, W, Cin, 0, H, W, N, ks, 1, pad, pad,
                         1 if transpose else 0, 0)
            gw = gw.view(w.shape)
        if has_b and ctx.needs_input_grad[2]:
            gbias = gy.float().sum(dim=(0, 1, 2))
        return gx, gw, gbias, None


def conv2d(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Keras Conv2D (stride 1, same) on NHWC bf16; w: (kh, kw, in, out) fp32."""
    if w.shape[0] == 3:
        # a 3x3 Conv2D with kernel W[ky][kx][c][n] IS a Conv2DTranspose whose (kh,kw,out,in) kernel is the
        # spatially flipped W with in/out swapped - express it that way so one packing path serves both
        wt = w.flip(0, 1).permute(0, 1, 3, 2)
        y = _Conv.apply(x, wt, b, True)
        return y
    return _Conv.apply(x, w, b, False)


def conv2d_transpose(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Keras Conv2DTranspose (3x3, stride 1, same) on NHWC bf16; w: (kh, kw, out, in) fp32."""
    return _Conv.apply(x, w, b, True)


class _Depthwise(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        B, H, W, Cc = x.shape
        if tuple(w.shape) != (3, 3, Cc, 1):
            raise ValueError("depthwise kernel must be (3, 3, C, 1)")
        C = hip()
        y = torch.empty(B, H, W, Cc, dtype=torch.int16, device=x.device)
        wf = w.detach().reshape(-1).float().contiguous()
        C.dw_fwd(_bits(x), wf, y, None, 0, B, H, W, Cc)
        ctx.save_for_backward(x, w)
        return y.view(torch.bfloat16)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        B, H, W, Cc = x.shape
        C = hip()
        gb = _bits(gy)
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty(B, H, W, Cc, dtype=torch.int16, device=x.device)
            C.dw_dgrad(gb, w.detach().reshape(-1).float().contiguous(), gx, B, H, W, Cc)
            gx = gx.view(torch.bfloat16)
        if ctx.needs_input_grad[1]:
            gw = torch.zeros(9 * Cc, dtype=torch.float32, device=x.device)
            C.dw_wgrad(_bits(x), gb, gw, None, 0, B, H, W, Cc)
            gw = gw.view(3, 3, Cc, 1)
        return gx, gw


def depthwise3x3(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """Keras DepthwiseConv2D 3x3 (depth multiplier 1, same) on NHWC bf16; w: (3, 3, C, 1) fp32."""
    return _Depthwise.apply(x, w)


__all__ = ["conv2d", "conv2d_transpose", "depthwise3x3"]
