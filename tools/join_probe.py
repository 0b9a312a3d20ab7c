"""Time the residual 1x1 join convs (conv_igemm JOIN_POOL / JOIN_ADD / JOIN_ADD_UP, the engine's shapes at 256^2 /
batch 16) under launch variants, isolated replays between HIP events:
  join    - the engine's call (consumer-side finalize of the join BN)
  nojfin  - the join BN's coefficients read final (no consumer-side finalize from replica sums)
  plain   - the same conv without the join epilogue (generic tiles, TUNE_PW = 1)
  floor   - a 1-element torch kernel (launch + event overhead)

    python tools/join_probe.py
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


def bf(*shape):
    return torch.randn(*shape, device=dev).to(torch.bfloat16).view(torch.int16)


def case(name, B, Hx, Cin, N, stride, mode, H, use_ab):
    Ho = (Hx + 1) // 2 if stride == 2 else Hx
    x = bf(B, Hx, Hx, Cin)
    wt = (torch.randn(N * Cin, device=dev) * 0.05).to(torch.bfloat16).view(torch.int16)
    bias = torch.zeros(N, device=dev)
    ab = torch.rand(4 * Cin, device=dev) + 0.5 if use_ab else None
    yj = bf(B, H, H, N)
    out = torch.zeros(B, H if mode != C.JOIN_POOL else Ho, H if mode != C.JOIN_POOL else Ho, N, dtype=torch.int16,
                      device=dev)
    am = torch.zeros(B, Ho, Ho, N, dtype=torch.uint8, device=dev) if mode == C.JOIN_POOL else None
    jab = torch.rand(4 * N, device=dev) + 0.5
    R = C.STAT_REPLICAS
    st = torch.rand(R * 2 * N, device=dev) * 100
    gam, bet = torch.rand(N, device=dev) + 0.5, torch.zeros(N, device=dev)
    jfin = dict(jfin_stats=st, jfin_gamma=gam, jfin_beta=bet, jfin_count=float(B * H * H), jfin_eps=1e-3)
    r = torch.zeros(B, Ho, Ho, N, dtype=torch.int16, device=dev)
    res = {}

    def run(join, fin):
        kw = dict(join_mode=mode, join_y=yj, join_ab=jab, join_out=out, join_H=H, join_W=H) if join else {}
        if join and am is not None:
            kw["join_argmax"] = am
        if join and fin:
            kw.update(jfin)
        return lambda: C.conv_igemm(x, wt, bias, r, None, ab, 1 if use_ab else 0, B, Hx, Hx, Cin, 0, Ho, Ho, N, 1,
                                    stride, 0, 0, None, 0, **kw)

    res["join"] = timeit(run(True, True))
    res["nojfin"] = timeit(run(True, False))
    C.set_tune(C.TUNE_PW, 1)
    res["plain"] = timeit(run(False, False))
    C.set_tune(C.TUNE_PW, 0)
    t = torch.zeros(1, device=dev)
    res["floor"] = timeit(lambda: t.add_(1.0))
    print(f"{name:4s} B{B} {Hx:3d}^2 {Cin:3d}->{N:3d} s{stride}: " + "  ".join(f"{k} {v:6.1f}" for k, v in res.items()),
          flush=True)


if __name__ == "__main__":
    B = 16
    case("e0", B, 128, 32, 64, 2, C.JOIN_POOL, 128, True)
    case("e1", B, 64, 64, 128, 2, C.JOIN_POOL, 64, False)
    case("e2", B, 32, 128, 256, 2, C.JOIN_POOL, 32, False)
    case("d0", B, 16, 256, 256, 1, C.JOIN_ADD, 16, False)
    case("d1", B, 16, 256, 128, 1, C.JOIN_ADD_UP, 32, False)
    case("d2", B, 32, 128, 64, 1, C.JOIN_ADD_UP, 64, False)
    case("d3", B, 64, 64, 32, 1, C.JOIN_ADD_UP, 128, False)
