"""Per-op micro-benchmark of the HIP engine at the bench shapes.

Records every extension call made by one eager training step (exact shapes and buffers), then replays each call in
isolation N times between CUDA events. Replays only rewrite the op's own outputs (gradient atomics just keep
accumulating), so the numbers are pure kernel time at the real shapes. Variants (e.g. the weight-gradient algo)
are timed side by side.

    python tools/kbench.py [--img 256] [--batch 16] [--reps 20] [--ops conv_wgrad,node_bwd] [--variants]
"""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd.data.device import make_synthetic_device  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.engine import UNetEngine  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable  # noqa: E402

SKIP = {"conv_splits", "conv_wgrad_slabs", "make_pack_table", "make_bn_moving_table", "make_grad_finish_table",
        "make_zero_table", "adam_step_done", "sep_fwd_supported"}


class Recorder:
    def __init__(self, C):
        self._C = C
        self.calls = []

    def __getattr__(self, name):
        f = getattr(self._C, name)
        if not callable(f) or name in SKIP:
            return f

        def wrap(*a, **k):
            if name in ("conv_wgrad_batch", "dw_wgrad_batch"):   # deferred weight gradients: time each one alone
                for c in a[0]:
                    self.calls.append((name[:-len("_batch")], tuple(c), {}))
            else:
                self.calls.append((name, a, k))
            return f(*a, **k)
        return wrap


def shape_key(name, a, k):
    ints = [x for x in a if isinstance(x, int) and not isinstance(x, bool)]
    return f"{name}{tuple(ints)}"


def time_call(C, name, a, k, reps):
    f = getattr(C, name)
    f(*a, **k)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        f(*a, **k)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ops", default="")
    ap.add_argument("--variants", action="store_true", help="also time algo variants of conv_wgrad / conv_igemm")
    ap.add_argument("--tune", default="", help="launch knobs, e.g. 3=256,4=2 (see TuneKey in launch.h)")
    ap.add_argument("--quiet", action="store_true", help="totals only")
    ap.add_argument("--roofline", action="store_true",
                    help="per call: minimum HBM bytes (every tensor argument read or written once), MFMA flops, "
                         "achieved GB/s / TF/s and the roofline floor max(bytes / 6.3 TB/s, flops / 2.5 PF/s)")
    args = ap.parse_args()
    table = ParamTable()
    # at least one image per batch slot: the step's batch indices (0..batch-1) address the resident dataset
    data = make_synthetic_device(max(64, args.batch), args.img, seed=0)
    eng = UNetEngine(table, args.batch, args.img)
    eng.bind_data(data.images, data.masks)
    eng.set_flat(table.init_flat(0))
    eng.idx.copy_(torch.arange(args.batch, dtype=torch.int32, device=eng.dev))
    eng.train_step_eager()
    torch.cuda.synchronize()
    rec = Recorder(eng.C)
    C = eng.C
    eng.C = rec
    eng.train_step_eager()
    eng.C = C
    torch.cuda.synchronize()
    # knobs apply to the timed replays only (the recorded step ran with the defaults, which size the slabs)
    for kv in filter(None, args.tune.split(",")):
        kk, v = kv.split("=")
        C.set_tune(int(kk), int(v))
    want = set(args.ops.split(",")) if args.ops else None
    roof = defaultdict(float)
    if args.roofline:
        print(f"{'us':>8}  {'floor':>7} {'eff':>5}   {'min bytes':>11} {'achieved':>10}  {'MFMA':>12}  op(shape ints)")
    tot = defaultdict(float)
    n = defaultdict(int)
    print(f"{'us':>8}  op(shape ints)")
    for name, a, k in rec.calls:
        if want and name not in want:
            continue
        try:
            t = time_call(C, name, a, k, args.reps)
        except RuntimeError as ex:      # e.g. a forced tile config that does not divide this shape
            print(f"     n/a  {shape_key(name, a, k)}  ({str(ex)[:60]})", flush=True)
            continue
        tot[name] += t
        n[name] += 1
        line = f"{t:8.1f}  {shape_key(name, a, k)}"
        if args.roofline:
            by, fl = min_bytes(eng, name, a, k), conv_flops(name, a)
            floor = max(by / HBM_BPS, fl / MFMA_FPS) * 1e6
            roof["bytes"] += by
            roof["flops"] += fl
            roof["floor"] += floor
            roof["time"] += t
            line = (f"{t:8.1f}  {floor:7.1f} {100 * floor / max(t, 1e-9):5.0f}%  {by / 1e6:8.2f} MB {by / t / 1e6:6.2f} "
                    f"TB/s  {fl / t / 1e6:7.1f} TF/s  {shape_key(name, a, k)}")
        if args.variants and name in ("conv_wgrad", "conv_igemm", "dw_fwd", "dw_dgrad", "dw_wgrad"):
            for algo in (1, 0):
                a2, kk = list(a), dict(k)
                if name == "conv_wgrad":      # (..., dst_mode, m_chunk, algo, slabs): direct atomics variant
                    a2[-2], a2[-1] = algo, 0
                elif name == "dw_dgrad" and len(a2) > 7:      # algo passed positionally (node epilogue call)
                    a2[7] = algo
                else:
                    kk["algo"] = algo
                try:
                    line += f"  algo{algo}={time_call(C, name, a2, kk, args.reps):.1f}"
                except Exception as ex:  # noqa: BLE001 - unsupported variant for this shape
                    line += f"  algo{algo}=n/a({str(ex)[:30]})"
        if not args.quiet:
            print(line, flush=True)
    print("\nper-op totals (us per step):")
    for name in sorted(tot, key=lambda x: -tot[x]):
        print(f"{tot[name]:9.1f}  {n[name]:3d} calls  {name}")
    print(f"{sum(tot.values()):9.1f}  total")
    if args.roofline and roof["time"]:
        print(f"\nwhole step (isolated replays, L2/Infinity-Cache warm): {roof['time']:.1f} us measured, minimum "
              f"{roof['bytes'] / 1e6:.1f} MB + {roof['flops'] / 1e9:.1f} GFLOP -> roofline floor {roof['floor']:.1f} us "
              f"({100 * roof['floor'] / roof['time']:.0f}% of measured; {roof['bytes'] / roof['time'] / 1e6:.2f} TB/s "
              f"average over the step)")


HBM_BPS = 6.3e12          # achievable HBM3E streaming rate on MI355X (MI355X_MICROARCH.md: 8 TB/s spec, ~6.3 achievable)
MFMA_FPS = 2.5e15         # dense bf16 MFMA peak


def min_bytes(eng, name, a, k):
    """Bytes the call must move at least: every tensor argument read or written once (the dataset arguments count
    only the batch's images / masks; packed weights and tables are small)."""
    tot = 0
    scratch = [eng.ws, eng.gws] + list(eng._wslabs.values())   # split-K workspace / weight-gradient slab rows: design
    spans = [(t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()) for t in scratch if t.numel()]
    for x in list(a) + list(k.values()):
        if not isinstance(x, torch.Tensor) or x.device.type != "cuda":
            continue
        if any(lo <= x.data_ptr() < hi for lo, hi in spans):
            continue                     # scratch of this design, not a minimum (the weight gradient itself is small)
        if eng.images is not None and x.data_ptr() == eng.images.data_ptr():
            tot += eng.B * eng.S * eng.S * 3
        elif eng.masks is not None and x.data_ptr() == eng.masks.data_ptr():
            tot += eng.B * eng.S * eng.S
        else:
            tot += x.numel() * x.element_size()
    return tot


def conv_flops(name, a):
    """2*M*N*K of the conv_igemm / conv_wgrad calls (positional ints: B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, ...)."""
    if name not in ("conv_igemm", "conv_wgrad"):
        return 0.0
    ints = [x for x in a if isinstance(x, int) and not isinstance(x, bool)]
    i0 = 1    # relu flag precedes B
    try:
        B, Hin, Win, Cin, up, Ho, Wo, N, ks = ints[i0:i0 + 9]
    except ValueError:
        return 0.0
    return 2.0 * B * Ho * Wo * N * ks * ks * Cin


if __name__ == "__main__":
    main()
