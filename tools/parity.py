"""Training parity run (crack_detection_federatedlearning_grpc_amd/train/parity.py): engine vs plain fp32 oracle
from the same init on the same batches, validation loss / accuracy / IoU every --every steps. One JSON line per
checkpoint plus a summary line.

    python tools/parity.py --img 128 --batch 16 --steps 1200 --every 100 [--samples 1024 --val 128] [--out f.jsonl]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd.train.parity import run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--img", type=int, default=128)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=1200)
    ap.add_argument("--every", type=int, default=100)
    ap.add_argument("--samples", type=int, default=1024)
    ap.add_argument("--val", type=int, default=128)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    log = open(a.out, "w") if a.out else None
    recs = run(a.img, a.batch, a.steps, a.every, a.samples, a.val, log=log)
    last = recs[-1]
    summ = {"summary": True, "img": a.img, "batch": a.batch, "steps": a.steps,
            "d_iou": last["engine"]["val_iou"] - last["fp32"]["val_iou"],
            "d_val_loss_rel": (last["engine"]["val_loss"] - last["fp32"]["val_loss"]) / last["fp32"]["val_loss"]}
    print(json.dumps(summ), flush=True)
    if log:
        print(json.dumps(summ), file=log, flush=True)


if __name__ == "__main__":
    main()
