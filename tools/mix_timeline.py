"""Per-item block timeline of the mixed weight-gradient launch (conv_wgrad.hip wgrad_mix_kernel) of one training step
(256^2, batch 16): the launch replayed once with the block stamp buffer installed (common.h CflTsGuard), each
block mapped to its item through the launch's XCD grouping (the item table from TUNE_WGRAD_MIX_LIST), then per item:
blocks, summed block-time (the slot time the item costs the slot-bound launch), median / max block duration and
first dispatch / last exit relative to the launch start.

    python tools/mix_timeline.py [img] [batch]      (env CFL_MIX_TUNE="KEY=V,..." sets launch knobs first)
"""
import os
import re
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd.data.device import make_synthetic_device  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.engine import UNetEngine  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable  # noqa: E402


def xcd_swizzle(b, n):
    q, r = n >> 3, n & 7
    x, i = b & 7, b >> 3
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + i


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    if os.environ.get("CFL_MIX_TUNE"):                   # launch knobs, "KEY=V,..." (launch.h names without TUNE_)
        from crack_detection_federatedlearning_grpc_amd._native_loader import hip
        for kv in os.environ["CFL_MIX_TUNE"].split(","):
            k, v = kv.split("=")
            hip().set_tune(getattr(hip(), "TUNE_" + k.strip().upper()), int(v))
    table = ParamTable()
    data = make_synthetic_device(max(64, B), S, seed=0)
    eng = UNetEngine(table, B, S)
    eng.bind_data(data.images, data.masks)
    eng.set_flat(table.init_flat(0))
    eng.idx.copy_(torch.arange(B, dtype=torch.int32, device=eng.dev))
    C = eng.C
    eng.train_step(use_graph=False)
    captured = []

    class Shim:
        def __getattr__(self, k):
            return getattr(C, k)

        def conv_wgrad_batch(self, wq):
            captured.append(list(wq))
            C.conv_wgrad_batch(wq)
    eng.C = Shim()
    eng.train_step(use_graph=False)
    eng.C = C
    torch.cuda.synchronize()
    wq = captured[-1]
    # the item table: the launcher prints it to stderr once per process (TUNE_WGRAD_MIX_LIST)
    with tempfile.TemporaryFile(mode="w+") as tf:
        fd = os.dup(2)
        os.dup2(tf.fileno(), 2)
        try:
            C.set_tune(C.TUNE_WGRAD_MIX_LIST, 1)
            C.conv_wgrad_batch(wq)
            torch.cuda.synchronize()
        finally:
            os.dup2(fd, 2)
            os.close(fd)
            C.set_tune(C.TUNE_WGRAD_MIX_LIST, 0)
        tf.seek(0)
        lines = [ln for ln in tf.read().splitlines() if ln.startswith("[wgrad_mix]")]
    items = []
    for ln in lines:
        m = re.search(r"item\s+(\d+) kind\s+(\d+) (.*): (\d+) blocks", ln)
        items.append((int(m.group(1)), int(m.group(2)), m.group(3), int(m.group(4))))
    total = sum(it[3] for it in items)
    buf = torch.zeros(total + 64, 2, dtype=torch.int64, device=eng.dev)
    for _ in range(2):
        C.conv_wgrad_batch(wq)
    torch.cuda.synchronize()
    C.set_ts(buf)
    C.conv_wgrad_batch(wq)
    torch.cuda.synchronize()
    C.set_ts(None)
    t = buf.cpu().numpy()[:total].astype(np.float64) / 100.0        # us
    t0 = t[:, 0].min()
    # physical block -> logical (XCD-grouped within 64-block windows) -> item
    bounds = np.cumsum([0] + [it[3] for it in items])
    owner = np.zeros(total, dtype=np.int64)
    for b in range(total):
        base = b & ~63
        span = min(64, total - base)
        vb = base + xcd_swizzle(b & 63, span)
        owner[b] = np.searchsorted(bounds, vb, side="right") - 1
    d = t[:, 1] - t[:, 0]
    span_all = t[:, 1].max() - t0
    print(f"mixed launch: {total} blocks, span {span_all:.1f} us, summed block time {d.sum():.0f} us "
          f"(= {d.sum() / span_all:.0f} busy slots on average)")
    print(f"{'item':>4} {'kind':>4} {'blocks':>6} {'blk-us':>8} {'share':>6} {'med':>6} {'max':>6} {'first':>6} "
          f"{'last':>6}  shape")
    for k, (idx, kind, shape, nb) in enumerate(items):
        sel = owner == k
        dk = d[sel]
        print(f"{idx:4d} {kind:4d} {nb:6d} {dk.sum():8.0f} {100 * dk.sum() / d.sum():5.1f}% {np.median(dk):6.1f} "
              f"{dk.max():6.1f} {t[sel, 0].min() - t0:6.1f} {t[sel, 1].max() - t0:6.1f}  {shape}")


if __name__ == "__main__":
    main()
