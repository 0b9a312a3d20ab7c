"""pw_bwd.hip probe: launch time, block timeline and in-kernel phases (cfl_ts_phase) vs grid size per shape, next to
the two-pass kernels it replaces (pw.hip dgrad with the BN fold + conv_wgrad).

    python tools/pwb_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd._native_loader import hip  # noqa: E402

C = hip()
DEV = torch.device("cuda")


def timed(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def stamps(f):
    buf = torch.zeros(1 << 16, 2, dtype=torch.int64, device=DEV)
    f()
    torch.cuda.synchronize()
    C.set_ts(buf)
    f()
    torch.cuda.synchronize()
    C.set_ts(None)
    t = buf.cpu().numpy()
    ph = t[1 << 15:]
    t = t[:1 << 15]
    keep = t[:, 0] != 0
    t, ph = t[keep], ph[keep]
    s, e = t[:, 0] / 100.0, t[:, 1] / 100.0
    d = e - s
    out = f"span {e.max() - s.min():6.1f} disp {s.max() - s.min():5.1f} blk med {np.median(d):5.1f} max {d.max():5.1f}"
    if (ph[:, 0] != 0).all():
        p0, p1 = ph[:, 0] / 100.0, ph[:, 1] / 100.0
        out += (f" | prologue med {np.median(p0 - s):5.1f} loop med {np.median(p1 - p0):5.1f}"
                f" epilogue med {np.median(e - p1):5.1f}")
    return out


B = 16
for (H, K, N) in [(128, 64, 32), (128, 64, 64)]:
    M = B * H * H
    r = lambda *s: torch.randint(-2000, 2000, s, dtype=torch.int16, device=DEV) // 8 + 16256   # bf16 ~ 1.0
    g, y, d = r(M, K), r(M, K), r(M, N)
    w = r(N * K)
    ab = torch.rand(4 * K, device=DEV) + 0.5
    sums = torch.randn(16 * 2 * K, device=DEV)
    dd = torch.zeros(M, N, dtype=torch.int16, device=DEV)
    dy = torch.zeros(M, K, dtype=torch.int16, device=DEV)
    rows = C.conv_wgrad_slabs(B, H, H, N, 0, H, H, K, 1, 1, 0, 0)[0]
    slab = torch.zeros(rows * N * K, device=DEV)
    dg, db = torch.zeros(K, device=DEV), torch.zeros(K, device=DEV)
    print(f"== H {H} K {K} N {N} M {M}: HBM floor g+y+d+dd {M * (2 * K + 2 * N) * 2 / 8e6:.1f} us at 8 TB/s", flush=True)
    two = lambda: (C.conv_igemm(g, w, None, dd, None, None, 0, B, H, H, K, 0, H, H, N, 1, 1, 0, 0, None, bwd_y=y,
                                bwd_ab=ab, bwd_sums=sums, bwd_reps=16, bwd_dx=dy, bwd_dgamma=dg, bwd_dbeta=db))
    wg = lambda: C.conv_wgrad(d, dy, slab, None, 0, B, H, H, N, 0, H, H, K, 1, 1, 0, 0, 0, 0, 0, rows)
    print(f"  pw.hip dgrad(bwd) {timed(two):6.1f} us   conv_wgrad {timed(wg):6.1f} us", flush=True)
    for blocks in (128, 256, 384, 512, 768):
        C.set_tune(C.TUNE_PWB_BLOCKS, blocks)
        f = lambda: C.pw_bwd(g, y, ab, sums, 16, w, d, dd, slab, rows, dg, db, B, H, H, K, N)
        print(f"  pw_bwd blocks {blocks:5d}: {timed(f):6.1f} us   {stamps(f)}", flush=True)
    C.set_tune(C.TUNE_PWB_BLOCKS, 0)
