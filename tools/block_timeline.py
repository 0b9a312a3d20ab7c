"""Block timelines of every extension call of one training step (256^2, batch 16), each replayed in isolation with the
block stamp buffer installed (common.h CflTsGuard: per block the s_memrealtime stamps, 100 MHz, of its dispatch and of
wave 0's exit).

Per call: blocks, kernel span (first dispatch -> last exit), dispatch spread (first -> last dispatch: > 0 when
blocks wait for a slot), block duration median / max, and the tail (last exit - 90th-percentile exit). A span close
to one block's duration means the launch is one round of blocks bound by the per-block critical path; a large
dispatch spread with short blocks means a slot-bound launch.

    python tools/block_timeline.py [--img 256] [--batch 16] [--ops conv_igemm,conv_wgrad_batch]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd.data.device import make_synthetic_device  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.engine import UNetEngine  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable  # noqa: E402

SKIP = {"conv_splits", "conv_wgrad_slabs", "make_pack_table", "make_bn_moving_table", "make_grad_finish_table",
        "make_zero_table", "adam_step_done", "sep_fwd_supported", "pw_bwd_supported", "set_ts", "set_tune", "get_tune",
        "det"}
CAP = 1 << 16


class Recorder:
    def __init__(self, C):
        self._C = C
        self.calls = []

    def __getattr__(self, name):
        f = getattr(self._C, name)
        if not callable(f) or name in SKIP or name.startswith("make_"):
            return f

        def wrap(*a, **k):
            self.calls.append((name, a, k))
            return f(*a, **k)
        return wrap


def shape_key(name, a, k):
    ints = [x for x in a if isinstance(x, int) and not isinstance(x, bool)]
    if name.endswith("_batch") and a and isinstance(a[0], (list, tuple)):
        return f"{name}[{len(a[0])} items]"
    return f"{name}{tuple(ints)}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--ops", default="")
    ap.add_argument("--reps", type=int, default=5, help="timed replays per call (stamps of the last one)")
    a = ap.parse_args()
    table = ParamTable()
    data = make_synthetic_device(max(64, a.batch), a.img, seed=0)
    eng = UNetEngine(table, a.batch, a.img)
    eng.bind_data(data.images, data.masks)
    eng.set_flat(table.init_flat(0))
    eng.idx.copy_(torch.arange(a.batch, dtype=torch.int32, device=eng.dev))
    eng.train_step_eager()
    torch.cuda.synchronize()
    C = eng.C
    rec = Recorder(C)
    eng.C = rec
    eng.train_step_eager()
    eng.C = C
    torch.cuda.synchronize()
    buf = torch.zeros(CAP, 2, dtype=torch.int64, device=eng.dev)
    want = set(a.ops.split(",")) if a.ops else None
    print(f"{'span':>7} {'disp':>6} {'med':>6} {'max':>6} {'tail':>6} {'blocks':>6}  call   (us; 100 MHz stamps)")
    tot = 0.0
    for name, args, kw in rec.calls:
        if want and name not in want:
            continue
        f = getattr(C, name)
        for _ in range(2):
            f(*args, **kw)
        torch.cuda.synchronize()
        buf.zero_()
        C.set_ts(buf)
        f(*args, **kw)
        torch.cuda.synchronize()
        C.set_ts(None)
        full = buf.cpu().numpy()
        t, ph = full[:CAP // 2], full[CAP // 2:]   # the upper half holds in-kernel phase stamps (cfl_ts_phase)
        keep = t[:, 0] != 0
        t, ph = t[keep], ph[keep]
        if len(t) == 0:
            continue
        s, e = t[:, 0].astype(np.float64) / 100.0, t[:, 1].astype(np.float64) / 100.0   # us
        d = e - s
        span = e.max() - s.min()
        tot += span
        extra = ""
        if len(ph) and (ph[:, 0] != 0).all() and (ph[:, 1] != 0).all():   # phases: prologue | loop | epilogue
            p0, p1 = ph[:, 0] / 100.0, ph[:, 1] / 100.0
            extra = (f"   [phases: prologue {np.median(p0 - s):.1f}, loop {np.median(p1 - p0):.1f}, "
                     f"epilogue {np.median(e - p1):.1f}]")
        print(f"{span:7.1f} {s.max() - s.min():6.1f} {np.median(d):6.1f} {d.max():6.1f} "
              f"{e.max() - np.percentile(e, 90):6.1f} {len(t):6d}  {shape_key(name, args, kw)}{extra}", flush=True)
    print(f"{tot:7.1f} total span (us)")


if __name__ == "__main__":
    main()
