"""Run-to-run spread of the engine's first-step loss and gradient (fresh engines, same data and weights): the noise
band the engine-switch tests compare variants against. Prints one JSON line per engine switch setting.

    python tools/loss_noise.py [--runs 6] [--S 128] [--B 4] [--vars CFL_BNB_FOLD_ENTRY=0,CFL_SEP_FUSE=0]
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


def one(S, B, seed):
    table = ParamTable()
    data = make_synthetic_device(max(8, B), S, seed=seed)   # idx 0..B-1 must be bound images
    eng = UNetEngine(table, B, S)
    eng.bind_data(data.images, data.masks)
    eng.set_flat(table.init_flat(seed))
    eng.idx.copy_(torch.arange(B, dtype=torch.int32, device=eng.dev))
    eng._zero_step()
    eng.forward(True)
    eng.backward()
    torch.cuda.synchronize()
    return eng.read_metrics("train")["loss"], eng.grad.cpu()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=6)
    ap.add_argument("--S", type=int, default=128)
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--vars", default="")
    a = ap.parse_args()
    for setting in [""] + [v for v in a.vars.split(",") if v]:
        if setting:
            k, v = setting.split("=")
            os.environ[k] = v
        losses, grads = [], []
        for _ in range(a.runs):
            lo, g = one(a.S, a.B, a.seed)
            losses.append(lo)
            grads.append(g)
        if setting:
            os.environ.pop(k)
        ref = grads[0]
        rels = [float((g - ref).norm() / ref.norm()) for g in grads[1:]]
        print(json.dumps({"setting": setting or "default", "losses": [round(x, 7) for x in losses],
                          "loss_spread": max(losses) - min(losses), "grad_rel_vs_first": [round(r, 5) for r in rels]}),
              flush=True)


if __name__ == "__main__":
    main()
