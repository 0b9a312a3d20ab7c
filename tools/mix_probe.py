"""Time the mixed weight-gradient launch (conv_wgrad.hip wgrad_mix_kernel) of the bench step and each of its items:
the deferred wgrad list of one eager training step (256^2, batch 16) is captured and replayed between HIP events
as a whole, with only item k (TUNE_WGRAD_MIX_ONLY) and without item k (TUNE_WGRAD_MIX_SKIP). Timing only: the
restricted launches leave the other items' slabs stale.

    python tools/mix_probe.py [img] [batch]

Env: CFL_MIX_TUNE="KEY=V,..." sets launch knobs (launch.h TuneKey names without TUNE_) before the engine is built (e.g.
WGRAD3_WIDE=2 for the 64-channel halo blocks); MIX_ORDER_ONLY=1 stops after the whole-launch timings; MIX_ALONE_ONLY=1
times each item alone but skips the "mix without it" runs.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd.data.device import make_synthetic_device  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.engine import UNetEngine  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.spec import ParamTable  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda")
if os.environ.get("CFL_MIX_TUNE"):
    from crack_detection_federatedlearning_grpc_amd._native_loader import hip
    for kv in os.environ["CFL_MIX_TUNE"].split(","):
        k, v = kv.split("=")
        hip().set_tune(getattr(hip(), "TUNE_" + k.strip().upper()), int(v))
table = ParamTable()
data = make_synthetic_device(max(64, B), S, seed=0)   # every index of the probe batch must be a bound image
eng = UNetEngine(table, B, S, dev)
eng.bind_data(data.images, data.masks)
eng.set_flat(table.init_flat(0))
assert data.images.shape[0] >= B, "the batch indexes images 0..B-1"
eng.idx.copy_(torch.arange(B, dtype=torch.int32, device=dev))
C = eng.C
eng.train_step(use_graph=False)                     # allocates the slabs
captured = []
real = C.conv_wgrad_batch


class Shim:
    def __getattr__(self, k):
        return getattr(C, k)

    def conv_wgrad_batch(self, wq):
        captured.append(list(wq))
        real(wq)


eng.C = Shim()
eng.train_step(use_graph=False)
eng.C = C
torch.cuda.synchronize()
wq = captured[-1]


def timeit(reps=30):
    for _ in range(3):
        real(wq)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        real(wq)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


C.set_tune(C.TUNE_WGRAD_MIX_LIST, 1)
full = timeit()
C.set_tune(C.TUNE_WGRAD_MIX_LIST, 0)
print(f"whole mixed launch: {full:.1f} us ({len(wq)} deferred wgrads)", flush=True)
for mode in (1, 3):                                  # other item orders (TUNE_WGRAD_MIX_ORDER; default 2)
    C.set_tune(C.TUNE_WGRAD_MIX_ORDER, mode)
    print(f"  item order {mode}: {timeit():.1f} us", flush=True)
C.set_tune(C.TUNE_WGRAD_MIX_ORDER, 0)
if os.environ.get("MIX_ORDER_ONLY"):
    sys.exit(0)
n = len(wq)
for k in range(n):
    C.set_tune(C.TUNE_WGRAD_MIX_ONLY, k + 1)
    alone = timeit()
    C.set_tune(C.TUNE_WGRAD_MIX_ONLY, 0)
    if os.environ.get("MIX_ALONE_ONLY"):
        print(f"item {k:2d}: alone {alone:6.1f} us", flush=True)
        continue
    C.set_tune(C.TUNE_WGRAD_MIX_SKIP, 1 << k)
    without = timeit()
    C.set_tune(C.TUNE_WGRAD_MIX_SKIP, 0)
    print(f"item {k:2d}: alone {alone:6.1f} us   mix without it {without:6.1f} us ({without - full:+.1f})", flush=True)
