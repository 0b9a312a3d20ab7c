"""Stock-framework comparator: the same U-Net (client_fit_model.py:92-150) as an idiomatic PyTorch-ROCm nn.Module
(nn.Conv2d / BatchNorm2d / ConvTranspose2d via MIOpen, channels_last, bf16 autocast, torch.optim.Adam) trained on
the bench shapes. This is what a user gets by porting the reference's TF/Keras trainer to stock PyTorch on an
MI355X; ``bench.py`` numbers are compared against it (the reference itself publishes none).

Not part of the framework's compute path - a measurement tool only.

    python tools/bench_torch_stock.py --img 256 --batch 16 --iters 200 [--graph]
"""
from __future__ import annotations

import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F

ENC = (64, 128, 256)
DEC = (256, 128, 64, 32)


class SamePadConv(nn.Conv2d):
    """TF 'same' for stride 2 on even inputs: all padding bottom/right (client_fit_model.py:100)."""

    def forward(self, x):
        if self.stride[0] == 2 and self.kernel_size[0] == 3:
            x = F.pad(x, (0, 1, 0, 1))
        return super().forward(x)


class SepConv(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.dw = nn.Conv2d(cin, cin, 3, padding=1, groups=cin, bias=False)
        self.pw = nn.Conv2d(cin, cout, 1)

    def forward(self, x):
        return self.pw(self.dw(x))


class StockUNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.entry = SamePadConv(3, 32, 3, stride=2)
        self.bn0 = nn.BatchNorm2d(32, eps=1e-3, momentum=0.01)
        self.enc = nn.ModuleList()
        cin = 32
        for f in ENC:
            self.enc.append(nn.ModuleDict(dict(
                s1=SepConv(cin, f), b1=nn.BatchNorm2d(f, eps=1e-3, momentum=0.01),
                s2=SepConv(f, f), b2=nn.BatchNorm2d(f, eps=1e-3, momentum=0.01),
                res=nn.Conv2d(cin, f, 1, stride=2))))
            cin = f
        self.dec = nn.ModuleList()
        for f in DEC:
            self.dec.append(nn.ModuleDict(dict(
                t1=nn.ConvTranspose2d(cin, f, 3, padding=1), b1=nn.BatchNorm2d(f, eps=1e-3, momentum=0.01),
                t2=nn.ConvTranspose2d(f, f, 3, padding=1), b2=nn.BatchNorm2d(f, eps=1e-3, momentum=0.01),
                res=nn.Conv2d(cin, f, 1))))
            cin = f
        self.head = nn.Conv2d(cin, 1, 1)

    def forward(self, x):
        x = F.relu(self.bn0(self.entry(x)))
        prev = x
        for b in self.enc:
            x = F.relu(x)
            x = b["b1"](b["s1"](x))
            x = F.relu(x)
            x = b["b2"](b["s2"](x))
            x = F.max_pool2d(F.pad(x, (0, 1, 0, 1), value=float("-inf")), 3, 2)
            x = x + b["res"](prev)
            prev = x
        for b in self.dec:
            x = F.relu(x)
            x = b["b1"](b["t1"](x))
            x = F.relu(x)
            x = b["b2"](b["t2"](x))
            x = F.interpolate(x, scale_factor=2, mode="nearest")
            x = x + b["res"](F.interpolate(prev, scale_factor=2, mode="nearest"))
            prev = x
        return self.head(x)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--graph", action="store_true", help="capture fwd+bwd+Adam in a CUDA(HIP) graph")
    ap.add_argument("--fp32", action="store_true", help="fp32 (the reference's precision) instead of bf16 autocast")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.backends.cudnn.benchmark = True
    model = StockUNet().to(dev).to(memory_format=torch.channels_last)
    n_params = sum(p.numel() for p in model.parameters()) + sum(b.numel() for n, b in model.named_buffers()
                                                                 if "running" in n)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, eps=1e-7, capturable=args.graph)
    B, S = args.batch, args.img
    x = torch.rand(B, 3, S, S, device=dev).to(memory_format=torch.channels_last)
    y = (torch.rand(B, 1, S, S, device=dev) > 0.9).float()
    dt = torch.float32 if args.fp32 else torch.bfloat16

    def step():
        opt.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=dt, enabled=not args.fp32):
            logits = model(x)
        loss = F.binary_cross_entropy_with_logits(logits.float(), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    run = step
    if args.graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        run = g.replay
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        run()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / args.iters
    print(json.dumps({"stack": "pytorch-rocm stock (MIOpen, channels_last, " + ("fp32" if args.fp32 else "bf16 autocast")
                      + (", hipGraph" if args.graph else ", eager") + ")",
                      "img": S, "batch": B, "params": n_params, "ms_per_iteration": round(ms, 4),
                      "images_per_s": round(B * 1000 / ms, 1)}), flush=True)


if __name__ == "__main__":
    main()
