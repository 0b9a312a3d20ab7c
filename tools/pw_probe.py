"""Time the 1x1 (pointwise / dgrad) conv shapes of the 256^2 / batch-16 step under launch variants (isolated calls
between HIP events), plus a plain copy of the same bytes as the streaming reference.

    python tools/pw_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd._native_loader import hip  # noqa: E402

C = hip()
dev = torch.device("cuda")


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def case(B, H, Cin, N):
    M = B * H * H
    x = torch.randn(M * Cin, device=dev).to(torch.bfloat16).view(torch.int16)
    wt = (torch.randn(N * Cin, device=dev) * 0.05).to(torch.bfloat16).view(torch.int16)
    y = torch.zeros(M * N, dtype=torch.int16, device=dev)
    stats = torch.zeros(32 * 2 * N, device=dev)
    ab = torch.rand(4 * Cin, device=dev) + 0.5
    bias = torch.zeros(N, device=dev)
    out = {}
    src = torch.empty(M * Cin, dtype=torch.int16, device=dev)
    dst = torch.empty(M * N, dtype=torch.int16, device=dev)
    out["copy"] = f"{timeit(lambda: dst[:M * Cin].copy_(src) if N >= Cin else dst.copy_(src[:M * N])):6.1f}"
    st, pl = dict(stats=stats, ab=None, relu=0), dict(stats=None, ab=None, relu=0)
    D, BL = C.TUNE_PW_DEPTH, C.TUNE_PW_BLOCKS
    for name, kw, tune in [("igemm-stats", st, {C.TUNE_PW: 1}), ("igemm-plain", pl, {C.TUNE_PW: 1}),
                           ("pw-stats", st, {}), ("pw-plain", pl, {}), ("d1", st, {D: 1}), ("d2", st, {D: 2}),
                           ("d4", st, {D: 4}), ("b256", st, {BL: 256}), ("b768", st, {BL: 768}),
                           ("b1024", st, {BL: 1024}), ("d1b1024", st, {D: 1, BL: 1024})]:
        for k, v in tune.items():
            C.set_tune(k, v)
        try:
            t = timeit(lambda: C.conv_igemm(x, wt, bias, y, kw["stats"], kw["ab"], kw["relu"], B, H, H, Cin, 0,
                                            H, H, N, 1, 1, 0, 0, None, 0))
            out[name] = f"{t:6.1f}"
        except RuntimeError:
            out[name] = "  n/a"
        for k in tune:
            C.set_tune(k, 0)
    mb = M * (Cin + N) * 2 / 1e6
    print(f"B{B} {H:3d}^2 {Cin:3d}->{N:3d} ({mb:5.1f} MB): " + "  ".join(f"{k} {v}" for k, v in out.items()),
          flush=True)


for args in [(16, 128, 32, 64), (16, 128, 64, 64), (16, 128, 64, 32), (16, 64, 64, 128), (16, 64, 128, 128),
             (16, 64, 128, 64), (16, 32, 128, 256), (16, 32, 256, 256), (16, 32, 256, 128)]:
    case(*args)
