"""List the grad_finish entries (optim.hip) of the bench step: per entry the gradient it finishes, its element count,
row count, mode and the bytes the launch moves for it (row reads, re-zeroing writes, the destination update), plus
the opt_step item mix. Sizes the end-of-backward tail (grad_finish + opt_step) against its HBM floor.

    python tools/finish_table.py [img] [batch]
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
table = ParamTable()
data = make_synthetic_device(max(64, B), S, seed=0)
eng = UNetEngine(table, B, S, dev)
eng.bind_data(data.images, data.masks)
eng.set_flat(table.init_flat(0))
eng.idx.copy_(torch.arange(B, dtype=torch.int32, device=dev))
eng.train_step(use_graph=False)                     # allocates the weight-gradient slabs
torch.cuda.synchronize()
C = eng.C
names = {C.GF_REDUCE: "reduce", C.GF_COPY: "copy", C.GF_SUM: "sum"}
base = eng.grad.data_ptr()
owner = {}
for e in table.entries:
    owner[e.offset] = f"{e.layer}/{e.wname}"
tot = 0
rows_hist = {}
print(f"{'dst':46s} {'n':>9s} {'rows':>5s} {'mode':>7s} {'MB':>7s}")
for src, dst, n, rows, mode in eng._finish_static + eng._finish_dyn:
    off = (dst.data_ptr() - base) // 4
    r = 1 if mode == C.GF_COPY else rows
    # reads of every row + the destination read-modify-write (+ re-zeroing writes of atomic replica rows)
    b = 4 * n * (r + 2 + (r if mode == C.GF_REDUCE else 0))
    tot += b
    rows_hist[r] = rows_hist.get(r, 0) + n
    print(f"{owner.get(off, hex(off)):46s} {n:9d} {r:5d} {names.get(mode, mode):>7s} {b / 1e6:7.2f}")
print(f"grad_finish: {len(eng._finish_static) + len(eng._finish_dyn)} entries, {eng.finish_work} blocks, "
      f"{tot / 1e6:.1f} MB -> {tot / 6.3e12 * 1e6:.1f} us at 6.3 TB/s")
print("elements by row count:", dict(sorted(rows_hist.items())))
print(f"opt_step: {eng.n_opt} items; params {table.total:,}; trainable {int(eng.trainable.sum()):,}; "
      f"minimum bytes ~{(int(eng.trainable.sum()) * 32) / 1e6:.1f} MB")
