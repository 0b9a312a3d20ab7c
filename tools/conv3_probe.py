"""Time one 3x3 conv call shape under launch variants (isolated replays between HIP events).

    python tools/conv3_probe.py            # the 256^2 / batch-16 decoder shapes
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


def case(B, H, Cin, N, up=0):
    Hin = H >> up
    x = torch.randn(B * Hin * Hin * Cin, device=dev).to(torch.bfloat16).view(torch.int16)
    wt = (torch.randn(N * 9 * Cin, device=dev) * 0.05).to(torch.bfloat16).view(torch.int16)
    y = torch.zeros(B * H * H * N, dtype=torch.int16, device=dev)
    stats = torch.zeros(32 * 2 * N, device=dev)
    ab = torch.rand(4 * Cin, device=dev) + 0.5
    bias = torch.zeros(N, device=dev)
    out = {}
    std = dict(stats=stats, ab=ab, relu=1)
    variants = [("default", std, {}), ("no-sk", std, {C.TUNE_CONV3_SK: 1})]
    variants += [(f"sk{c}", std, {C.TUNE_CONV3_SK: 2, C.TUNE_CONV3_SK_CFG: c}) for c in (1, 2, 3, 4)]
    variants += [("sk-plain", dict(stats=stats, ab=None, relu=0), {C.TUNE_CONV3_SK: 2})]
    if not os.environ.get("PROBE_SK_ONLY"):
        variants += [("no-stats", dict(stats=None, ab=ab, relu=1), {C.TUNE_CONV3_SK: 1}),
                     ("no-xform", dict(stats=stats, ab=None, relu=0), {C.TUNE_CONV3_SK: 1}),
                     ("BN32", std, {C.TUNE_CONV3_SK: 1, C.TUNE_CONV3_BN: 32}),
                     ("ws", std, {C.TUNE_CONV3_WS: 2}),
                     ("small", std, {C.TUNE_CONV3_SMALL: 2}),
                     ("deep", std, {C.TUNE_CONV3_DEEP: 2}),
                     ("8x16x64", std, {C.TUNE_CONV3_SK: 1, C.TUNE_CONV3_SMALL: 1}),
                     ("generic", dict(std, algo=1), {})]
    for name, kw, tune in variants:
        for k, v in tune.items():
            C.set_tune(k, v)
        algo = kw.get("algo", 0)
        try:
            t = timeit(lambda: C.conv_igemm(x, wt, bias, y, kw["stats"], kw["ab"], kw["relu"], B, Hin, Hin, Cin, up,
                                            H, H, N, 3, 1, 1, 1, None, algo))
            out[name] = f"{t:6.1f}"
        except RuntimeError:
            out[name] = "  n/a"
        for k in tune:
            C.set_tune(k, 0)
    print(f"B{B} {H:3d}^2 {Cin:3d}->{N:3d} up{up}: " + "  ".join(f"{k} {v}" for k, v in out.items()), flush=True)


SHAPES = [(16, 64, 64, 64), (16, 64, 128, 64, 1), (16, 64, 64, 128), (16, 32, 128, 128), (16, 32, 256, 128, 1),
          (16, 32, 128, 256), (16, 16, 256, 256), (16, 128, 32, 32), (16, 128, 64, 32, 1)]
if len(sys.argv) > 1:                       # e.g. "16" -> only the shapes at that output resolution
    SHAPES = [s for s in SHAPES if s[1] in [int(a) for a in sys.argv[1:]]]
for args in SHAPES:
    case(*args)
