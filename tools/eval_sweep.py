"""Validation (inference forward) cost per image vs the evaluator's batch, at the bench's shapes.

    python tools/eval_sweep.py [--img 256] [--batches 48,96,128,...] [--reps 12]

Every evaluator shares the training engine's weights (UNetEngine.evaluator); each batch size is timed over ``reps``
graph replays between HIP events after one warm-up replay (capture included there).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd.data.device import make_synthetic_device  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.engine import UNetEngine  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--batches", default="48,64,96,128,160,192,256,384,592")
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--samples", type=int, default=2000)
    a = ap.parse_args()
    table = ParamTable()
    data = make_synthetic_device(a.samples, a.img, seed=3)
    eng = UNetEngine(table, 16, a.img, "cuda")
    eng.bind_data(data.images, data.masks)
    eng.set_flat(table.init_flat(0))
    for B in [int(b) for b in a.batches.split(",")]:
        ev = eng.evaluator(B)
        ev.idx.copy_(torch.arange(B, dtype=torch.int32, device=eng.dev) % a.samples)
        ev.eval_step(True)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.reps):
            ev.eval_step(True)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / a.reps
        print(json.dumps({"eval_batch": B, "ms_per_launch": round(ms, 4), "us_per_image": round(1e3 * ms / B, 3),
                          "peak_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)}), flush=True)
        eng._evaluators.clear()
        del ev
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
