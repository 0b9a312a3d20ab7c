"""MI355X training engine for the crack U-Net: a static forward/backward schedule over hand-written HIP kernels.

No autograd and no tracing compiler: the network is fixed (client_fit_model.py:92-150), so the engine lays out every
activation, gradient and statistics buffer once (sized for the batch; 288 GB of HBM is never the constraint) and
issues a fixed launch sequence that is captured into ONE hipGraph per train step (forward, backward, Adam, BN
moving-stat update, weight repack). Per step the host only copies the batch's dataset indices and replays.

Folds that keep the high-resolution tensors from ever being written:
* BatchNorm apply + ReLU are applied when the NEXT kernel loads the raw conv output (``InXform``);
* every decoder UpSampling2D commutes with the residual add and with the 1x1 convs, so each decoder block's
  output is kept at half resolution (``x_lo``) and the upsample is folded into the consumers' indexing; the head's
  logits are computed at 128^2 for a 256^2 image and each one scores a 2x2 block of the target mask;
* batch assembly, /255 normalisation and mask lookup are folded into the entry conv and the head (dataset resident
  in HBM, indexed by a batch index vector).

Layouts: activations NHWC bf16; master weights, grads, Adam moments fp32 in one flat buffer (Keras order,
``models/spec.py``); GEMM operands repacked to bf16 [N][K] by one ``pack_weights`` launch per step.
"""
from __future__ import annotations

import contextlib
import gc
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .._native_loader import hip
from .memplan import buffer_shapes
from .spec import DEC_FILTERS, ENC_FILTERS, ENTRY_FILTERS, ParamTable

PK_CONV, PK_CONV_DGRAD1x1, PK_CONVT, PK_CONVT_DGRAD, PK_PW, PK_PW_DGRAD = range(6)
GM_NONE, GM_SAME, GM_SCATTER2, GM_SUM2X2, GM_MAXPOOL = range(5)


@contextlib.contextmanager
def _no_gc():
    """Collect garbage now and keep the collector off for the block: a hipGraph capture (global capture mode) must not
    run a destructor of an unreachable object from an earlier engine - a CUDAGraph's private pool release or a
    pinned-block event query is a prohibited call during capture and aborts the process (seen in the GPU test suite
    after the FL tests: an engine cycle collected mid-capture)."""
    was = gc.isenabled()
    gc.collect()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


@dataclass
class Lazy:
    """A tensor as seen by its consumers: stored raw values + optional BN coefficients + ReLU."""
    t: torch.Tensor
    ab: Optional[torch.Tensor]
    relu: int
    H: int
    C: int


class UNetEngine:
    def __init__(self, table: ParamTable, batch: int, img: int, device="cuda", loss: str = "bce",
                 lr: float = 1e-3, beta1: float = 0.9, beta2: float = 0.999, adam_eps: float = 1e-7,
                 bn_momentum: float = 0.99, bn_eps: float = 1e-3, share: Optional["UNetEngine"] = None,
                 deterministic: Optional[bool] = None, conv_dtype: Optional[str] = None):
        """``share``: an inference-only engine (see ``evaluator``) reading another engine's parameters and packed
        weights in place (no copy, no repack).

        ``deterministic`` (default: env CFL_DETERMINISTIC=1): every cross-block reduction of the step (BN batch
        statistics, BN-backward sums, weight-gradient replica rows, the head's dW / db) accumulates 64-bit
        fixed-point integers instead of float atomics (csrc/kernels/common.h), so replays of the same step are
        bitwise equal. The mode is per PROCESS (each kernel module's constant flag): an engine refuses to step when
        the process mode differs from its own (its reduction buffers are laid out for one of the two).

        ``conv_dtype`` (default: env CFL_CONV_DTYPE, else "bf16"): "fp8" runs every decoder 3x3 convolution - each
        Conv2DTranspose forward and data gradient - on the block-scaled fp8 MFMA (csrc/kernels/fp8.hip: e4m3 operands,
        one e8m0 scale per 32 channels of a pixel / weight row, fp32 accumulation; BASELINE config 5). The bf16
        packed weights stay the source of truth (fp32 master + Adam unchanged): one quant_w8 launch at the start of
        every step (and of every inference forward) re-quantises the ConvT views."""
        if img % 16:
            raise ValueError("image size must be a multiple of 16")
        self.C = hip()
        if deterministic is None:
            deterministic = share.det if share is not None else os.environ.get("CFL_DETERMINISTIC", "0") == "1"
        self.det = bool(deterministic)
        if conv_dtype is None:
            conv_dtype = share.conv_dtype if share is not None else os.environ.get("CFL_CONV_DTYPE", "bf16")
        if conv_dtype not in ("bf16", "fp8"):
            raise ValueError(f"conv_dtype must be bf16 or fp8, got {conv_dtype!r}")
        self.conv_dtype = conv_dtype
        self.C.set_det(1 if self.det else 0)
        self._w = 2 if self.det else 1       # float slots per reduction-buffer element (int64 in the mode)
        self._pending: List[tuple] = []
        self.table = table
        self.B, self.S = batch, img
        self.dev = torch.device(device)
        if self.dev.type == "cuda" and self.dev.index is None:
            self.dev = torch.device("cuda", torch.cuda.current_device())
        self.dice = 1 if loss == "bce_dice" else 0
        self.lr, self.b1, self.b2, self.adam_eps = lr, beta1, beta2, adam_eps
        self.momentum, self.bn_eps = bn_momentum, bn_eps
        self.names = [ly.name for ly in table.weighted_layers()]
        dev = self.dev
        f32 = dict(dtype=torch.float32, device=dev)
        # ---- parameters / optimizer state (flat fp32) ----
        self._share = share
        self.flat = share.flat if share is not None else torch.zeros(table.total, **f32)
        self.grad = torch.zeros(table.total, **f32)
        self.m = torch.zeros(table.total, **f32)
        self.v = torch.zeros(table.total, **f32)
        self.trainable = torch.as_tensor(table.trainable_mask().astype(np.uint8), device=dev)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=dev)
        self.metrics = torch.zeros(10, dtype=torch.float64, device=dev)        # head.hip metrics layout
        self.eval_metrics = torch.zeros(10, dtype=torch.float64, device=dev)
        self.idx = torch.zeros(batch, dtype=torch.int32, device=dev)
        # optional device batch table (bind_batches): the step's first kernel selects idx = table[cursor % nb] and
        # advances the cursor, so replayed steps need no host-issued index copy
        self.batch_table: Optional[torch.Tensor] = None
        self.batch_cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self.lr_buf = torch.zeros(1, dtype=torch.float32, device=dev)    # the step's Adam rate (_zero_step)
        self.ws = torch.zeros(0, dtype=torch.float32, device=dev)     # split-K workspace
        self._build_pack()
        self._build_fp8()
        self._alloc()
        # the optimizer tail (Adam + BN moving statistics + bf16 repack + step / cursor advance) as ONE opt_step
        # launch (training engines only)
        if share is None:
            self._build_opt()
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        # the same step as TWO graphs split after the encoder forward (capture()): replayed right after a FedAvg,
        # so the encoder - whose parameters form the first all-reduce bucket - runs while the later buckets reduce
        self.graph_pre: Optional[torch.cuda.CUDAGraph] = None
        self.graph_post: Optional[torch.cuda.CUDAGraph] = None
        self._mid_hook = None
        self.split_at = self.table.entry(self.names[17], "kernel").offset   # flat end of the encoder parameters
        self.stall_log: Optional[List[tuple]] = None   # (before, after) event pairs of post-FedAvg waits (bench)
        self.eval_graph: Optional[torch.cuda.CUDAGraph] = None
        self._retired: List[torch.Tensor] = []   # replaced workspaces a captured graph may still reference
        self._evaluators: Dict[int, "UNetEngine"] = {}
        self._eval_batch_memo: Dict[Tuple[int, int], int] = {}   # eval_batch_for's choices
        self.images: Optional[torch.Tensor] = None
        self.masks: Optional[torch.Tensor] = None

    # ------------------------------------------------------------------------------------------------ params
    def P(self, layer: str, w: str) -> torch.Tensor:
        e = self.table.entry(layer, w)
        if self._pending:
            self._await_range(e.offset + e.size)
        return self.flat[e.offset:e.offset + e.size]

    # ---- overlapped aggregation (parallel/rccl.py FedAvgAllReduce.average_async) ----
    def defer_until(self, bucket_events) -> None:
        """Register per-bucket completion events of an in-flight FedAvg all-reduce (+ bucket repack). The eager
        step waits per layer - each parameter read waits only for the bucket holding it, so the first layers
        start while later buckets are still reducing; a graph replay (no per-layer hooks) waits for all."""
        self._pending = [(sl.start, sl.stop, ev) for sl, ev in bucket_events]

    def _await_range(self, end: int) -> None:
        cur = torch.cuda.current_stream(self.dev)
        while self._pending and self._pending[0][0] < end:
            _, _, ev = self._pending.pop(0)
            cur.wait_event(ev)

    def _await_all(self) -> None:
        if self._pending:
            self._await_range(self.table.total + 1)

    def pack_bucket(self, sl: slice) -> None:
        """bf16 repack of the views whose source range ENDS inside this bucket (buckets complete in order, so the
        earlier part of a view that straddles a boundary is already reduced)."""
        key = (sl.start, sl.stop)
        if key not in self._bucket_packs:
            sub = [v for v in self._views if sl.start < v[1] + v[3] * v[3] * v[4] * v[5] <= sl.stop]
            self._bucket_packs[key] = (self.C.make_pack_table(sub, self.flat), len(sub),
                                       max([v[3] * v[3] * v[4] * v[5] for v in sub], default=0)) if sub else None
        t = self._bucket_packs[key]
        if t is not None:
            self.C.pack_weights(self.flat, self.packed, t[0], t[1], t[2])

    def G(self, layer: str, w: str) -> torch.Tensor:
        e = self.table.entry(layer, w)
        return self.grad[e.offset:e.offset + e.size]

    def _build_pack(self) -> None:
        views, self.packed_at = [], {}
        off, max_el = 0, 0

        def add(kind, layer, wname, ks, cin, cout):
            nonlocal off, max_el
            e = self.table.entry(layer, wname)
            n = ks * ks * cin * cout
            views.append((kind, e.offset, off, ks, cin, cout))
            self.packed_at[(layer, kind)] = (off, n)
            off += (n + 63) // 64 * 64
            max_el = max(max_el, n)

        for ly in self.table.weighted_layers():
            if ly.kind == "sepconv":
                add(PK_PW, ly.name, "pointwise_kernel", 1, ly.cin, ly.cout)
                add(PK_PW_DGRAD, ly.name, "pointwise_kernel", 1, ly.cin, ly.cout)
            elif ly.kind == "convt":
                add(PK_CONVT, ly.name, "kernel", 3, ly.cin, ly.cout)
                add(PK_CONVT_DGRAD, ly.name, "kernel", 3, ly.cin, ly.cout)
            elif ly.kind == "conv" and ly.ksize == 1 and ly.cout > 1:
                add(PK_CONV, ly.name, "kernel", 1, ly.cin, ly.cout)
                add(PK_CONV_DGRAD1x1, ly.name, "kernel", 1, ly.cin, ly.cout)
        self.packed = self._share.packed if self._share is not None else torch.zeros(off, dtype=torch.int16,
                                                                                     device=self.dev)
        self.pack_table = self.C.make_pack_table(views, self.flat)
        self._views = views
        self._view_src = {(v[0], ly): v for ly, v in zip([k[0] for k in self.packed_at], views)}
        self._bucket_packs: Dict[Tuple[int, int], object] = {}
        self.n_views, self.max_pack = len(views), max_el

    def _build_fp8(self) -> None:
        """fp8 mode: e4m3 copies (+ e8m0 scales per 32 K-elements) of every ConvT's two packed views (PK_CONVT for the
        forward, PK_CONVT_DGRAD for the data gradient), rewritten from the bf16 packs by one quant_w8 launch."""
        self.w8: Dict[Tuple[str, int], Tuple[torch.Tensor, torch.Tensor]] = {}
        self._q8 = []
        if self.conv_dtype != "fp8":
            return
        if self._share is not None and getattr(self._share, "w8", None):
            self.w8, self._q8 = self._share.w8, self._share._q8
            return
        for (layer, kind), (off, n) in self.packed_at.items():
            if kind in (PK_CONVT, PK_CONVT_DGRAD):
                w8 = torch.zeros(n, dtype=torch.uint8, device=self.dev)
                s8 = torch.zeros(n // 32, dtype=torch.uint8, device=self.dev)
                self.w8[(layer, kind)] = (w8, s8)
                self._q8.append((self.packed[off:off + n], w8, s8))

    def _quant_fp8(self) -> None:
        if self._q8:
            self.C.quant_w8(self._q8)

    def _f8(self, layer: str, kind: int) -> Dict[str, torch.Tensor]:
        """conv_igemm kwargs of a ConvT view's fp8 operands (empty in bf16 mode)."""
        if not self.w8:
            return {}
        w8, s8 = self.w8[(layer, kind)]
        return {"wt8": w8, "ws8": s8}

    def _build_opt(self) -> None:
        """Work items of opt_step (launch.h): 64x64 Adam tiles of every GEMM weight, each writing both bf16 views of
        its tile (the same layouts pack_weights writes), 1024-element Adam items over the other trainable arrays,
        one moving-statistics item per BN layer."""
        C = self.C
        items, tiled = [], set()
        for ly in self.table.weighted_layers():
            if ly.kind == "sepconv":         # (1,1,C,F) as [C][F]: PK_PW = transpose, PK_PW_DGRAD = copy
                wn, kt, kc, rows, cols = "pointwise_kernel", PK_PW, PK_PW_DGRAD, ly.cin, ly.cout
                rmap = (rows, cols, 0, 0)
            elif ly.kind == "convt":         # (3,3,out,in) as [9 out][in]: PK_CONVT_DGRAD = transpose, PK_CONVT = flip
                wn, kt, kc, rows, cols = "kernel", PK_CONVT_DGRAD, PK_CONVT, 9 * ly.cout, ly.cin
                rmap = (ly.cout, 9 * ly.cin, -ly.cin, 8 * ly.cin)
            elif ly.kind == "conv" and ly.ksize == 1 and ly.cout > 1:   # [cin][cout]: PK_CONV = transpose
                wn, kt, kc, rows, cols = "kernel", PK_CONV, PK_CONV_DGRAD1x1, ly.cin, ly.cout
                rmap = (rows, cols, 0, 0)
            else:
                continue
            e = self.table.entry(ly.name, wn)
            if not e.trainable or e.size != rows * cols:
                raise RuntimeError(f"opt table: {ly.name}/{wn} is not a trainable [{rows}][{cols}] weight")
            dt, dc = self.packed_at[(ly.name, kt)][0], self.packed_at[(ly.name, kc)][0]
            for r0 in range(0, rows, 64):
                for c0 in range(0, cols, 64):
                    items.append((C.OI_TILE, 0, r0, c0, rows, cols) + rmap + (e.offset, dt, dc))
            tiled.add((ly.name, wn))
        for e in self.table.entries:
            if e.trainable and (e.layer, e.wname) not in tiled:
                for i in range(0, e.size, 1024):
                    items.append((C.OI_FLAT, min(1024, e.size - i), 0, 0, 0, 0, 0, 0, 0, 0, e.offset + i, 0, 0))
        moving = [(self.bn[n]["stats"], self.P(n, "moving_mean"), self.P(n, "moving_variance"), self.bn[n]["C"],
                   float(self.bn_count(n))) for n in self.bn_names]
        self.opt_table = C.make_opt_table(items, moving, self.flat)
        self.n_opt = len(items) + len(moving)
        self.opt_ticket = torch.zeros(1, dtype=torch.int32, device=self.dev)

    def W(self, layer: str, kind: int) -> torch.Tensor:
        off, n = self.packed_at[(layer, kind)]
        if self._pending:
            v = self._view_src[(kind, layer)]
            self._await_range(v[1] + v[3] * v[3] * v[4] * v[5])
        return self.packed[off:off + n]

    # ------------------------------------------------------------------------------------------------ buffers
    def _t(self, *shape, dtype=torch.int16):
        return torch.zeros(*shape, dtype=dtype, device=self.dev)

    def _alloc(self) -> None:
        B, S = self.B, self.S
        r = [S // 2, S // 4, S // 8, S // 16]
        self.r = r
        t = self._t
        R = self.C.STAT_REPLICAS
        bn_layers = [ly for ly in self.table.weighted_layers() if ly.kind == "bn"]
        self.bn_names = [ly.name for ly in bn_layers]
        tot_c = sum(ly.cout for ly in bn_layers)
        RS = self.RS = int(os.environ.get("CFL_SUM_REPLICAS", self.C.SUM_REPLICAS))
        w = self._w                          # deterministic mode: int64 elements at the same indices
        self.stats_all = torch.zeros(w * R * 2 * tot_c, dtype=torch.float32, device=self.dev)
        self.sums_all = torch.zeros(w * RS * 2 * tot_c, dtype=torch.float32, device=self.dev)
        self.ab_all = torch.zeros(4 * tot_c, dtype=torch.float32, device=self.dev)
        self.bn: Dict[str, Dict[str, torch.Tensor]] = {}
        so = 0
        for ly in bn_layers:
            c = ly.cout
            self.bn[ly.name] = dict(C=c, stats=self.stats_all[w * R * 2 * so:w * R * 2 * (so + c)],
                                    sums=self.sums_all[w * RS * 2 * so:w * RS * 2 * (so + c)],
                                    ab=self.ab_all[4 * so:4 * (so + c)])
            so += c
        # forward activations (raw bf16) and backward buffers: shapes from models/memplan.py (the HBM planner
        # prices exactly these)
        shapes_a, shapes_d = buffer_shapes(B, S)
        dt = {2: torch.int16, 1: torch.uint8, 4: torch.float32}
        self.act = {n: t(*shp, dtype=dt[isz]) for n, (shp, isz) in shapes_a.items() if n != "h"}
        self.h = t(*shapes_a["h"][0], dtype=torch.float32)
        # inference-only engines (evaluator) never run backward: no gradient buffers (33.5 of 55 MB per 256^2 image)
        self.dg = {n: (t(*v[0], dtype=dt[v[1]]) if v and self._share is None else None) for n, v in shapes_d.items()}
        # replica rows for the small weight gradients every block adds into (depthwise kernels, entry conv):
        # [R][n] slabs summed into the flat gradient by ONE grad_finish launch at the end of backward, which
        # also applies the gradient copies (residual-conv bias grad == its BN's beta grad)
        names = self.names
        slabs = [(names[0], "kernel", 27 * ENTRY_FILTERS)]
        cin = ENTRY_FILTERS
        for k, F in enumerate(ENC_FILTERS):
            s1, s2 = names[2 + 5 * k], names[2 + 5 * k + 2]
            slabs += [(s1, "depthwise_kernel", 9 * cin), (s2, "depthwise_kernel", 9 * F)]
            cin = F
        tot = sum((n + 63) // 64 * 64 for _, _, n in slabs)
        self.gws = torch.zeros(self._w * R * tot, dtype=torch.float32, device=self.dev)
        self.gslab: Dict[Tuple[str, str], torch.Tensor] = {}
        entries, off = [], 0
        for ly, wn, n in slabs:
            sl = self.gws[self._w * off:self._w * (off + R * n)]
            self.gslab[(ly, wn)] = sl
            entries.append((sl, self.G(ly, wn), n, R, self.C.GF_REDUCE))
            off += R * ((n + 63) // 64 * 64)
        for k in range(len(ENC_FILTERS)):
            entries.append((self.G(names[2 + 5 * k + 3], "beta"), self.G(names[2 + 5 * k + 4], "bias"),
                            ENC_FILTERS[k], 1, self.C.GF_COPY))
        for k in range(len(DEC_FILTERS)):
            base = 17 + 5 * k
            entries.append((self.G(names[base + 3], "beta"), self.G(names[base + 4], "bias"), DEC_FILTERS[k], 1,
                            self.C.GF_COPY))
        # deterministic mode: the head's dW / db accumulate as int64 fixed point here (head_bwd), converted into the
        # flat gradient by two GF_FIXED entries
        cin = DEC_FILTERS[-1]
        self.head_fx = torch.zeros(2 * (cin + 1) + 62, dtype=torch.float32, device=self.dev) if self.det else None
        if self.det:
            hl = names[-1]
            entries.append((self.head_fx, self.G(hl, "kernel"), cin, 1, self.C.GF_FIXED))
            entries.append((self.head_fx[2 * cin:], self.G(hl, "bias"), 1, 1, self.C.GF_FIXED))
        self._finish_static = entries
        self._finish_dyn: List[tuple] = []
        self._wslabs: Dict[str, torch.Tensor] = {}
        self._build_finish()
        # The schedule's folds were each kept by a whole-bench A/B on the GPU (profiles/README.md; round 4 retired
        # their env switches and off-branches):
        # * weight gradients deferred to the end of backward and issued as ONE grouped batch (conv_wgrad_batch);
        # * BN-backward apply folded into the encoder's pointwise dgrads (pw.hip) and the entry wgrad's dy load;
        # * decoder residual-conv gradient dq = 2x2 sums of dxlo formed in its 1x1 dgrad's operand load;
        # * depthwise dgrad + wgrad (+ the BN node) of a layer in one fused pass (dw_bwd);
        # * decoder node join in the convT1 dgrad's epilogue; BN finalize in each BN layer's first consumer;
        # * SeparableConv forward in one pass (sepconv.hip); streaming BN-backward passes co-launched with the
        #   residual convs' 1x1 dgrads (launch.h SideJob); residual joins in the residual conv's epilogue.
        # Training head: forward + backward in ONE pass over x_lo (head.hip FWD) whenever the loss has no
        # whole-batch term (the Dice gradient needs the forward's sums first).
        self.fuse_head = self.dice == 0
        self._wq: Optional[List[tuple]] = None
        self._dwq: Optional[List[tuple]] = None
        # per-step zeroing of gradients / statistics in one launch
        spans = [self.grad, self.stats_all, self.sums_all, self.metrics[4:10]]
        self.zero_table = self.C.make_zero_table(spans)
        self.n_zero, self.max_zero = len(spans), max(t.numel() * t.element_size() for t in spans)
        # inference BN coefficients of every layer (one launch per eval forward)
        self.eval_table = self.C.make_bn_eval_table([
            (self.P(n, "gamma"), self.P(n, "beta"), self.P(n, "moving_mean"), self.P(n, "moving_variance"),
             self.bn[n]["ab"], self.bn[n]["C"]) for n in self.bn_names], self.bn_eps)
        # BN moving-stat table
        self.moving_table = self.C.make_bn_moving_table([
            (self.bn[n]["stats"], self.P(n, "moving_mean"), self.P(n, "moving_variance"), self.bn[n]["C"],
             float(self.bn_count(n))) for n in self.bn_names])

    def _build_finish(self) -> None:
        entries = self._finish_static + self._finish_dyn
        self.finish_table, self.finish_work = self.C.make_grad_finish_table(entries)
        self.n_finish = len(entries)
        self._finish_dirty = False

    def _wgrad(self, x, dy, layer, ab, relu, B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, stride, pad_t, pad_l,
               dst_mode) -> None:
        """Weight gradient into a slab of partial rows (plain-stored pixel splits for the 3x3 halo kernel, atomic
        replica rows otherwise) that grad_finish sums into the flat gradient at the end of backward. ``layer`` is
        a layer name (weight "kernel") or a (layer, weight) pair. Slabs are allocated on the eager warm-up pass,
        before graph capture."""
        key = layer if isinstance(layer, tuple) else (layer, "kernel")
        rows, plain = self.C.conv_wgrad_slabs(B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, stride, pad_t, pad_l)
        slab = self._wslab(key, rows, plain, ks * ks * Cin * N)
        args = (x, dy, slab, ab, relu, B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, stride, pad_t, pad_l, dst_mode, 0, 0,
                rows)
        if self._wq is not None:
            self._wq.append(args)          # deferred: issued as one batch at the end of backward
        else:
            self.C.conv_wgrad(*args)

    def _wslab(self, key, rows: int, plain: bool, n: int) -> torch.Tensor:
        """The partial-row slab of weight ``key`` (``rows`` rows of ``n``; int64 pairs for atomic rows in the
        deterministic mode) registered with grad_finish; (re)allocated on the eager warm-up pass only."""
        slab = self._wslabs.get(key)
        if slab is None or slab.numel() != rows * n * (1 if plain else self._w):
            if self.dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("weight-gradient slabs must be allocated before graph capture")
            if key in self._wslabs:
                self._retired.append(self._wslabs[key])
            dst = self.G(*key)
            self._finish_dyn = [e for e in self._finish_dyn if e[1].data_ptr() != dst.data_ptr()]
            if rows == 1 and plain:
                # one plainly-stored row (the 16^2 decoder layers) IS the gradient: stored in place, no finish pass
                slab = dst
            else:       # atomic replica rows hold int64 fixed point in the deterministic mode (plain rows: floats)
                slab = torch.zeros(rows * n * (1 if plain else self._w), dtype=torch.float32, device=self.dev)
                self._finish_dyn.append((slab, dst, n, rows, self.C.GF_SUM if plain else self.C.GF_REDUCE))
            self._wslabs[key] = slab
            self._finish_dirty = True
        return slab

    def _pw_bwd(self, g, y, bname, d, dd, dy, layer, B, H, K, N) -> None:
        """Backward of an encoder pointwise conv (K = its output channels, N = its input channels) whose output
        feeds BN ``bname``: dd = W^T BN_bwd(g, y) and the pointwise weight gradient. One fused streaming pass
        (pw_bwd.hip) where it supports the shape and TUNE_PWB is 0; otherwise pw.hip's dgrad with the BN backward
        folded into its operand load (it also stores dy) and the weight gradient from (d, dy)."""
        C = self.C
        if C.get_tune(C.TUNE_PWB) == 0 and C.pw_bwd_supported(B, H, H, K, N):
            rows = C.conv_wgrad_slabs(B, H, H, N, 0, H, H, K, 1, 1, 0, 0)[0]
            slab = self._wslab((layer, "pointwise_kernel"), rows, False, N * K)
            bb = self.bn[bname]
            C.pw_bwd(g, y, bb["ab"], bb["sums"], self.RS, self.W(layer, PK_PW_DGRAD), d, dd, slab, rows,
                     self.G(bname, "gamma"), self.G(bname, "beta"), B, H, H, K, N)
            return
        self._igemm(g, self.W(layer, PK_PW_DGRAD), None, dd, None, None, 0, B, H, H, K, 0, H, H, N, 1, 1, 0, 0,
                    bwd=(y, bname, dy))
        self._wgrad(d, dy, (layer, "pointwise_kernel"), None, 0, B, H, H, N, 0, H, H, K, 1, 1, 0, 0, 0)

    def bn_count(self, name: str) -> int:
        """Pixels per channel in the batch statistics of a BN layer."""
        i = self.bn_names.index(name)
        B, r = self.B, self.r
        if i == 0:
            return B * r[0] * r[0]
        if i <= 6:
            k = (i - 1) // 2
            return B * r[k] * r[k]
        k = (i - 7) // 2
        Rk = r[3] << k
        return B * Rk * Rk

    def nbytes(self) -> int:
        tot = 0
        for d in (self.act, self.dg):
            tot += sum(v.numel() * v.element_size() for v in d.values() if v is not None)
        return tot

    # ------------------------------------------------------------------------------------------------ data
    def bind_data(self, images: torch.Tensor, masks: torch.Tensor) -> None:
        if images.device != self.dev or images.dtype != torch.uint8 or images.shape[1:] != (self.S, self.S, 3):
            raise ValueError(f"images must be uint8 [N,{self.S},{self.S},3] on {self.dev}")
        if masks.shape[1:] != (self.S, self.S) or masks.dtype != torch.uint8:
            raise ValueError("masks must be uint8 [N,S,S]")
        self.images, self.masks = images.contiguous(), masks.contiguous()
        self.n_data = images.shape[0]
        for ev in self._evaluators.values():
            ev.bind_data(self.images, self.masks)

    # ------------------------------------------------------------------------------------------------ schedule
    def _xfin(self, name: str, train: bool) -> Dict[str, object]:
        """Consumer-side BN finalize kwargs: the consumer computes layer ``name``'s coefficients from its replica
        sums (and writes its ab rows) instead of a bn_finalize launch (empty: ab is final already)."""
        if not train:
            return {}
        return dict(xfin_stats=self.bn[name]["stats"], xfin_gamma=self.P(name, "gamma"),
                    xfin_beta=self.P(name, "beta"), xfin_count=float(self.bn_count(name)), xfin_eps=self.bn_eps)

    def _jfin(self, name: str, train: bool) -> Dict[str, object]:
        """_xfin for a residual conv's join epilogue (the join BN's first consumer)."""
        return {"j" + k[1:]: v for k, v in self._xfin(name, train).items()}

    def _bn_final(self, name: str) -> torch.Tensor:
        """ab of BN layer ``name``: in training its next consumer finalizes it from the batch statistics (_xfin),
        in inference forward()'s bn_eval_coefs wrote it - nothing is launched here."""
        return self.bn[name]["ab"]

    def _igemm(self, x, wt, bias, y, stats, ab, relu, B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, stride, pad_t,
               pad_l, node: Optional[Tuple[torch.Tensor, Dict[str, torch.Tensor], int]] = None,
               join: Optional[Dict[str, object]] = None,
               bwd: Optional[Tuple[torch.Tensor, str, torch.Tensor]] = None, **extra) -> None:
        """conv_igemm with the shared split-K workspace (grown on the eager warm-up pass, before graph capture).

        ``node`` = (y, bn, relu): the output is the incoming gradient of that BN node; the kernel's epilogue writes
        the masked node gradient and accumulates the BN-backward sums (fused node_bwd).
        ``bwd`` = (y, bn name, dx): x is the gradient w.r.t. that BN layer's output and the conv's operand is the
        BN-backward apply of it (the kernel folds bn_bwd_apply into its operand load and also stores dx, for the
        weight gradient, and the layer's dgamma / dbeta)."""
        need = self.C.conv_splits(B, Ho, Wo, N, ks, stride, pad_t, Cin)
        if need > 1 and need * B * Ho * Wo * N > self.ws.numel():
            if self.dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("split-K workspace must be sized before graph capture")
            self._retired.append(self.ws)
            self.ws = torch.empty(need * B * Ho * Wo * N, dtype=torch.float32, device=self.dev)
        kw = {}
        if node is not None:
            ny, bn, nrelu = node
            kw = dict(node_y=ny, node_ab=bn["ab"], node_sums=bn["sums"], node_reps=self.RS, node_relu=nrelu)
        if join:
            kw.update(join)
        kw.update(extra)
        if bwd is not None:
            by, bname, bdx = bwd
            bb = self.bn[bname]
            kw.update(bwd_y=by, bwd_ab=bb["ab"], bwd_sums=bb["sums"], bwd_reps=self.RS, bwd_dx=bdx,
                      bwd_dgamma=self.G(bname, "gamma"), bwd_dbeta=self.G(bname, "beta"))
        self.C.conv_igemm(x, wt, bias, y, stats, ab, relu, B, Hin, Win, Cin, up_in, Ho, Wo, N, ks, stride, pad_t,
                          pad_l, self.ws if need > 1 else None, **kw)

    def _conv(self, x: Lazy, layer: str, kind: int, y: torch.Tensor, N: int, ks: int, stride: int, up_in: int,
              Ho: int, bias: Optional[torch.Tensor], stats: Optional[torch.Tensor],
              join: Optional[Dict[str, object]] = None, **extra) -> None:
        pad = (ks - 1) // 2 if stride == 1 else 0
        B = self.B
        self._igemm(x.t, self.W(layer, kind), bias, y, stats, x.ab, x.relu, B, x.H, x.H, x.C, up_in, Ho, Ho,
                    N, ks, stride, pad, pad, join=join, **extra)

    def forward(self, train: bool = True) -> None:
        C, B, r, A = self.C, self.B, self.r, self.act
        if not train:                          # every BN's inference coefficients in one launch
            if self._pending:
                self._await_all()
            C.bn_eval_coefs(self.eval_table, len(self.bn_names))
            self._quant_fp8()
        n = iter(self.names)
        e_conv, e_bn = next(n), next(n)
        st = self.bn[e_bn]["stats"] if train else None
        C.entry_fwd(self.images, self.idx, self.P(e_conv, "kernel"), self.P(e_conv, "bias"), A["y0"], st, B, self.S,
                    ENTRY_FILTERS)
        ab0 = self._bn_final(e_bn)
        x = Lazy(A["y0"], ab0, 1, r[0], ENTRY_FILTERS)     # a0 = relu(BN0(y0))
        for k, F in enumerate(ENC_FILTERS):
            s1, b1, s2, b2, rc = (next(n) for _ in range(5))
            H = r[k]
            # SeparableConv 1: the depthwise conv is the first consumer of BN0 (k = 0): it finalizes it
            self._sepconv(x.t, x.ab, s1, A[f"e{k}_d1"], A[f"e{k}_y1"], b1, H, x.C, F, train,
                          self._xfin(e_bn, train) if k == 0 else {})
            ab1 = self._bn_final(b1)
            self._sepconv(A[f"e{k}_y1"], ab1, s2, A[f"e{k}_d2"], A[f"e{k}_y2"], b2, H, F, F, train,
                          self._xfin(b1, train))
            ab2 = self._bn_final(b2)
            # residual 1x1/s2 conv whose epilogue does max-pool(BN(y2)) + add + argmax
            self._conv(x, rc, PK_CONV, A[f"e{k}_res"], F, 1, 2, 0, H // 2, self.P(rc, "bias"), None,
                       join=dict(join_mode=C.JOIN_POOL, join_y=A[f"e{k}_y2"], join_ab=ab2,
                                 join_out=A[f"e{k}_x"], join_argmax=A[f"e{k}_am"], join_H=H, join_W=H,
                                 **self._jfin(b2, train)))
            x = Lazy(A[f"e{k}_x"], None, 0, H // 2, F)
        if self._mid_hook is not None:                       # split-graph capture: the encoder graph ends here
            self._mid_hook()
        if train and self._q8:
            # fp8 mode: quantise the ConvT views of this step's weights HERE, in the decoder part of the step - after
            # a FedAvg the encoder graph replays once only the encoder bucket landed, while the decoder buckets may
            # still be reducing / repacking on the side stream; the post graph runs after every bucket, and an eager
            # step waits for all of them first (the quantisation reads the whole packed buffer, not one layer)
            if self._pending:
                self._await_all()
            self._quant_fp8()
        prev = x                                             # x3 at r[3]
        for k, F in enumerate(DEC_FILTERS):
            t1, b1, t2, b2, rc = (next(n) for _ in range(5))
            Rk = r[3] << k
            up = 0 if k == 0 else 1
            self._convt(Lazy(prev.t, None, 1, prev.H, prev.C), t1, A[f"d{k}_c1"], F, up, Rk,
                        self.P(t1, "bias"), self.bn[b1]["stats"] if train else None)
            abA = self._bn_final(b1)                             # finalized by the convT2 forward below
            self._convt(Lazy(A[f"d{k}_c1"], abA, 1, Rk, F), t2, A[f"d{k}_c2"], F, 0, Rk,
                        self.P(t2, "bias"), self.bn[b2]["stats"] if train else None,
                        **self._xfin(b1, train))
            abB = self._bn_final(b2)
            # residual 1x1 conv whose epilogue adds BN_B(c2) (4 pixels per q pixel when up)
            self._conv(prev, rc, PK_CONV, A[f"d{k}_q"], F, 1, 1, 0, prev.H, self.P(rc, "bias"), None,
                       join=dict(join_mode=C.JOIN_ADD_UP if up else C.JOIN_ADD, join_y=A[f"d{k}_c2"],
                                 join_ab=abB, join_out=A[f"d{k}_xlo"], join_H=Rk, join_W=Rk,
                                 **self._jfin(b2, train)))
            prev = Lazy(A[f"d{k}_xlo"], None, 0, Rk, F)
        hl = next(n)
        if train and self.fuse_head:             # the training step's head forward runs inside head_bwd (backward)
            return
        C.head_fwd(prev.t, self.P(hl, "kernel"), self.P(hl, "bias"), self.masks, self.idx, self.h,
                   self.metrics if train else self.eval_metrics, B, r[0], DEC_FILTERS[-1], self.dice)

    def _sepconv(self, x: torch.Tensor, ab: Optional[torch.Tensor], layer: str, d: torch.Tensor, y: torch.Tensor,
                 bn: str, H: int, K: int, N: int, train: bool, xfin: Dict[str, object]) -> None:
        """SeparableConv2D forward on relu(BN(x)) (client_fit_model.py:109,113): d = depthwise 3x3, y = pointwise(d)
        + bias with BN ``bn``'s batch statistics. One fused launch (sepconv.hip: the depthwise output formed in the
        pointwise MFMA's operand registers, d side-stored for the weight gradient) where the kernel covers the shape,
        else dw_fwd + the streaming pointwise conv."""
        C, B = self.C, self.B
        stats = self.bn[bn]["stats"] if train else None
        if C.sep_fwd_supported(B, H, H, K, N):
            C.sep_fwd(x, ab, 1, self.P(layer, "depthwise_kernel"), self.W(layer, PK_PW), self.P(layer, "bias"), d, y,
                      stats, B, H, H, K, N, **xfin)
            return
        C.dw_fwd(x, self.P(layer, "depthwise_kernel"), d, ab, 1, B, H, H, K, **xfin)
        self._conv(Lazy(d, None, 0, H, K), layer, PK_PW, y, N, 1, 1, 0, H, self.P(layer, "bias"), stats)

    def _dw_wgrad(self, *args) -> None:
        """Depthwise weight gradient: deferred with the conv weight gradients (its inputs - a forward activation and
        the depthwise dgrad's incoming gradient - are not rewritten later in backward) and issued in one grouped
        launch with the other depthwise layers' (dw_wgrad_batch)."""
        if self._dwq is not None:
            self._dwq.append(args + (0,))
        else:
            self.C.dw_wgrad(*args)

    def backward(self) -> None:
        self._wq = []
        self._dwq = []
        try:
            self._backward()
        finally:
            wq, self._wq = self._wq, None
            dwq, self._dwq = self._dwq, None
        if dwq:
            self.C.dw_wgrad_batch(dwq)
        if wq:
            self.C.conv_wgrad_batch(wq)
        if self._finish_dirty:
            if self.dev.type == "cuda" and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("grad_finish table changed during graph capture")
            self._build_finish()
        self.C.grad_finish(self.finish_table, self.n_finish, self.finish_work)

    def _backward(self) -> None:
        C, B, r, A, D = self.C, self.B, self.r, self.act, self.dg
        names = self.names
        hl = names[-1]
        # the head's input gradient is also the gradient of the last BN_B node (x_lo = BN_B(c2) + q, no ReLU): its
        # BN-backward sums are accumulated in head_bwd's epilogue (no separate node pass over dxlo3)
        bn_last = self.bn[names[17 + 5 * 3 + 3]]
        C.head_bwd(A["d3_xlo"], self.P(hl, "kernel"), self.P(hl, "bias"), self.masks, self.idx, self.h,
                   self.metrics, D["dxlo3"], self.G(hl, "kernel"), self.G(hl, "bias"), B, r[0], DEC_FILTERS[-1],
                   self.dice, node_y=A["d3_c2"], node_ab=bn_last["ab"], node_sums=bn_last["sums"], node_reps=self.RS,
                   fused=1 if self.fuse_head else 0, dwfx=self.head_fx)
        dxlo = D["dxlo3"]
        for k in range(3, -1, -1):
            F = DEC_FILTERS[k]
            base = 17 + 5 * k
            t1, b1, t2, b2, rc = names[base:base + 5]
            Rk = r[3] << k
            cprev = ENC_FILTERS[-1] if k == 0 else DEC_FILTERS[k - 1]
            prev_t = A["e2_x"] if k == 0 else A[f"d{k - 1}_xlo"]
            prevres = Rk if k == 0 else Rk // 2
            up = 0 if k == 0 else 1
            bnB, bnA = self.bn[b2], self.bn[b1]
            # BN_B node: x_lo = BN_B(c2) + up?(q)  (no ReLU) -> its gradient IS dxlo. Its BN-backward sums were
            # accumulated by the pass that produced dxlo: head_bwd (k = 3) or the convT1 dgrad join of level k+1.
            # The BN-backward applies of the decoder run as streaming passes (folded into the latency-bound 3x3
            # dgrads' operand loads they measured slower twice, profiles/README.md); this one is independent of the
            # residual conv's dgrad below, which reads the same dxlo: it runs as that launch's side job
            bba_B = (dxlo, A[f"d{k}_c2"], bnB["ab"], bnB["sums"], D[f"d{k}_dc"], self.G(b2, "gamma"),
                     self.G(b2, "beta"), B * Rk * Rk, F, self.RS)
            # residual 1x1 conv R_k on prev: q = R(prev) at prevres, dq = dxlo (k=0) or sum2x2(dxlo) (k > 0: the
            # 2x2 sum is formed by the dgrad's operand load, which also stores dq for the weight gradient)
            dq = dxlo if k == 0 else D[f"d{k}_dq"]
            # bias grad of R_k: sum(dq) == sum(g_B) == dbeta_B (the BN_B node has no ReLU) -> grad_finish copy
            self._igemm(dq, self.W(rc, PK_CONV_DGRAD1x1), None, D[f"d{k}_dres"], None, None, 0, B, prevres,
                        prevres, F, 0, prevres, prevres, cprev, 1, 1, 0, 0, **({"sum2x2": dxlo} if k > 0 else {}),
                        side_bba=bba_B)
            self._wgrad(prev_t, dq, rc, None, 0, B, prevres, prevres, cprev, 0, prevres, prevres,
                        F, 1, 1, 0, 0, 0)
            # dgrad of convT2 with the BN_A node (ReLU mask + sums) fused into its epilogue
            self._igemm(D[f"d{k}_dc"], self.W(t2, PK_CONVT_DGRAD), None, D[f"d{k}_g"], None, None,
                        0, B, Rk, Rk, F, 0, Rk, Rk, F, 3, 1, 1, 1, node=(A[f"d{k}_c1"], bnA, 1),
                        **self._f8(t2, PK_CONVT_DGRAD))
            # convT2: input relu(BN_A(c1))
            self._wgrad(A[f"d{k}_c1"], D[f"d{k}_dc"], t2, bnA["ab"], 1, B, Rk, Rk, F, 0, Rk, Rk,
                        F, 3, 1, 1, 1, 1)
            C.bn_bwd_apply(D[f"d{k}_g"], A[f"d{k}_c1"], bnA["ab"], bnA["sums"], D[f"d{k}_dc2"],
                           self.G(b1, "gamma"), self.G(b1, "beta"), B * Rk * Rk, F, self.RS)
            # grad of prev (x_lo_{k-1} or x3): relu-masked main path (2x2 summed when upsampled) + residual path;
            # for k > 0 this gradient is also BN_B(k-1)'s node gradient (its BN-backward sums accumulate here) -
            # the join runs in the convT1 dgrad's epilogue at half resolution (dxin is never stored)
            pjkw = {}
            if k > 0:
                bprev = self.bn[names[17 + 5 * (k - 1) + 3]]
                pjkw = dict(pj_v=prev_t, pj_add=D[f"d{k}_dres"], pj_out=D[f"d{k}_dprev"], pj_sy=A[f"d{k - 1}_c2"],
                            pj_sab=bprev["ab"], pj_sums=bprev["sums"], pj_reps=self.RS)
            self._igemm(D[f"d{k}_dc2"], self.W(t1, PK_CONVT_DGRAD), None,
                        D[f"d{k}_dxin"], None, None, 0, B, Rk, Rk, F, 0, Rk, Rk, cprev, 3, 1, 1, 1, **pjkw,
                        **self._f8(t1, PK_CONVT_DGRAD))
            # convT1: input relu(up?(prev))
            self._wgrad(prev_t, D[f"d{k}_dc2"], t1, None, 1, B, prevres, prevres, cprev, up, Rk,
                        Rk, F, 3, 1, 1, 1, 1)
            if k == 0:          # x3 = the encoder output: relu-masked main path + residual path
                C.node_bwd(D[f"d{k}_dxin"], GM_SAME, 1, D[f"d{k}_dres"], GM_SAME, 0, None,
                           prev_t, None, 0, D[f"d{k}_dprev"], None, B, prevres, prevres, cprev)
            dxlo = D[f"d{k}_dprev"]
        # encoder
        dx_out = dxlo                                         # grad of x3
        for k in range(2, -1, -1):
            F = ENC_FILTERS[k]
            base = 2 + 5 * k
            s1, b1, s2, b2, rc = names[base:base + 5]
            H = r[k]
            cin = ENTRY_FILTERS if k == 0 else ENC_FILTERS[k - 1]
            if k == 0:
                xin = Lazy(A["y0"], self.bn[names[1]]["ab"], 1, H, cin)
            else:
                xin = Lazy(A[f"e{k - 1}_x"], None, 0, H, cin)
            bnb, bna = self.bn[b2], self.bn[b1]
            # BN_b node: routed through the max-pool (no ReLU); independent of the residual 1x1 stride-2 conv's
            # dgrad on x_in (dres = W^T dx_out, read only by the last depthwise backward of this level), which reads
            # the same dx_out: the routing pass runs as that launch's side job
            pool_b = (dx_out, A[f"e{k}_am"], A[f"e{k}_y2"], bnb["ab"], D[f"e{k}_g"], bnb["sums"], B, H, H, F, self.RS)
            # bias grad: sum(dx_out) == sum(g_b) == dbeta_b (max-pool routing keeps sums) -> grad_finish copy
            self._igemm(dx_out, self.W(rc, PK_CONV_DGRAD1x1), None, D[f"e{k}_dres"], None, None, 0, B, H // 2,
                        H // 2, F, 0, H // 2, H // 2, cin, 1, 1, 0, 0, side_pool=pool_b)
            # pointwise 2 with BN_b's backward folded in (dgrad + weight gradient)
            self._pw_bwd(D[f"e{k}_g"], A[f"e{k}_y2"], b2, A[f"e{k}_d2"], D[f"e{k}_dd2"], D[f"e{k}_dy"], s2, B, H, F,
                         F)
            # depthwise 2 on relu(BN_a(y1)): dgrad with the BN_a node (ReLU mask + sums) fused into its epilogue
            # and the weight gradient from the same dy rows, one pass
            C.dw_bwd(A[f"e{k}_y1"], bna["ab"], 1, D[f"e{k}_dd2"], self.P(s2, "depthwise_kernel"), D[f"e{k}_g"],
                     self.gslab[(s2, "depthwise_kernel")], self.C.STAT_REPLICAS, B, H, H, F,
                     node_y=A[f"e{k}_y1"], node_ab=bna["ab"], node_sums=bna["sums"], node_reps=self.RS,
                     node_relu=1)
            # pointwise 1 with BN_a's backward folded in
            self._pw_bwd(D[f"e{k}_g"], A[f"e{k}_y1"], b1, A[f"e{k}_d1"], D[f"e{k}_dd1"], D[f"e{k}_dy2"], s1, B, H, F,
                         cin)
            # residual 1x1 stride-2 conv on x_in (dres = dx_out)
            self._wgrad(xin.t, dx_out, rc, xin.ab, xin.relu, B, H, H, cin, 0, H // 2, H // 2, F,
                        1, 2, 0, 0, 0)
            # depthwise 1 on relu(x_in), and the gradient of x_in itself: the depthwise branch (ReLU-masked) plus the
            # stride-2 scatter of dres, in one pass (dgrad + wgrad + the node join in the dgrad's epilogue); for
            # k = 0 x_in is relu(BN0(y0)), a BN node (mask + sums)
            bn0 = self.bn[names[1]]
            out = D[f"e{k}_dx"] if k > 0 else D["g0"]
            nkw = dict(node_y=A["y0"], node_ab=bn0["ab"], node_sums=bn0["sums"], node_reps=self.RS,
                       node_relu=1) if k == 0 else dict(mask_x=1)
            C.dw_bwd(xin.t, xin.ab, 1, D[f"e{k}_dd1"], self.P(s1, "depthwise_kernel"), out,
                     self.gslab[(s1, "depthwise_kernel")], self.C.STAT_REPLICAS, B, H, H, cin,
                     add_half=D[f"e{k}_dres"], **nkw)
            if k > 0:
                dx_out = out
            else:          # the entry BN's backward apply folded into the entry wgrad's dy load
                C.entry_wgrad(self.images, self.idx, D["g0"], self.gslab[(names[0], "kernel")], B, self.S,
                              ENTRY_FILTERS, self.C.STAT_REPLICAS, bwd_y=A["y0"], bwd_ab=bn0["ab"],
                              bwd_sums=bn0["sums"], bwd_reps=self.RS, bwd_dx=D["dy0"],
                              bwd_dgamma=self.G(names[1], "gamma"), bwd_dbeta=self.G(names[1], "beta"))

    def optimizer_step(self, advanced: bool = False) -> None:
        """The fused optimizer tail (opt_step). ``advanced``: the step's zero_spans launch already advanced the
        step / cursor and left the Adam rate in ``lr_buf`` (the training step's form: no end-of-launch ticket);
        otherwise opt_step advances them itself (its last block, by ticket)."""
        self._await_all()
        if self._share is not None:
            raise RuntimeError("optimizer_step on an inference-only engine")
        if advanced:
            self.C.opt_step(self.opt_table, self.n_opt, self.flat, self.grad, self.m, self.v, self.trainable,
                            self.packed, self.lr, self.b1, self.b2, self.adam_eps, self.momentum, None, None, None,
                            self.lr_buf)
            return
        cursor = self.batch_cursor if self.batch_table is not None else None
        self.C.opt_step(self.opt_table, self.n_opt, self.flat, self.grad, self.m, self.v, self.trainable, self.packed,
                        self.lr, self.b1, self.b2, self.adam_eps, self.momentum, self.step_t, cursor, self.opt_ticket)

    def bind_batches(self, batches: torch.Tensor, checked: bool = False) -> None:
        """Device batch table [nb, B] (int32 dataset indices): every training step takes its batch from row
        ``cursor % nb`` (selected and the cursor advanced by the step's zero_spans launch) instead of
        a host copy into ``idx``. After graph capture the table buffer is fixed (the graph holds its address and
        row count): a table of the same row count is copied in; a smaller one whose row count divides the bound
        one is tiled into it, so ``cursor % nb`` still wraps onto the NEW rows; anything else is refused.
        Every index is checked against the bound dataset (the kernels read images / masks through them) - on the
        device (two host syncs), unless the caller already ``checked`` the host copy it uploaded."""
        batches = batches.to(device=self.dev, dtype=torch.int32).contiguous()
        if batches.dim() != 2 or batches.shape[1] != self.B:
            raise ValueError(f"bind_batches: expected [nb, {self.B}], got {tuple(batches.shape)}")
        if self.images is not None and batches.numel() and not checked:
            lo, hi = int(batches.min()), int(batches.max())
            if lo < 0 or hi >= self.n_data:
                raise ValueError(f"bind_batches: indices [{lo}, {hi}] outside the bound dataset of {self.n_data}")
        nb = batches.shape[0]
        if self.batch_table is None and self.graph is not None:
            raise RuntimeError("bind_batches: the step graph was captured without a batch table (it reads idx); "
                               "bind a batch table before the first graph capture")
        if self.batch_table is not None and nb == self.batch_table.shape[0]:
            self.batch_table.copy_(batches)
            return
        if self.graph is None:
            self.batch_table = batches.clone()
            return
        bound = self.batch_table.shape[0]
        if nb > bound or bound % nb:
            raise RuntimeError(f"bind_batches: {nb} rows after graph capture of a {bound}-row table (must divide it)")
        self.batch_table.copy_(batches.repeat(bound // nb, 1))

    def set_batch_cursor(self, i: int = 0) -> None:
        self.batch_cursor.fill_(i)

    def pack(self, step: bool = False) -> None:
        cursor = self.batch_cursor if step and self.batch_table is not None else None
        self.C.pack_weights(self.flat, self.packed, self.pack_table, self.n_views, self.max_pack,
                            self.step_t if step else None, cursor)

    def _convt(self, x: "Lazy", layer: str, y: torch.Tensor, N: int, up_in: int, Ho: int,
               bias: torch.Tensor, stats: Optional[torch.Tensor], **extra) -> None:
        """Decoder Conv2DTranspose forward (client_fit_model.py:129,133) on the bf16 3x3 kernels. ``extra``:
        consumer-side finalize kwargs of the input's BN. (Round 4 removed the fp8 e4m3 forward path: on the
        non-scaled fp8 MFMA, which issues at the bf16 rate on gfx950, it measured slower at 256^2 and 512^2 -
        profiles/README.md.)"""
        self._conv(x, layer, PK_CONVT, y, N, 3, 1, up_in, Ho, bias, stats, **extra, **self._f8(layer, PK_CONVT))

    def _zero_step(self) -> None:
        """The step's first launch: zero the gradient / statistics spans, select the batch from the bound table,
        and advance the Adam step (rate into ``lr_buf``) and batch cursor for this step's optimizer_step."""
        adv = dict(step=self.step_t, lr_buf=self.lr_buf, lr=self.lr, b1=self.b1, b2=self.b2)
        if self.batch_table is not None:
            self.C.zero_spans(self.zero_table, self.n_zero, self.max_zero, self.batch_table, self.batch_cursor,
                              self.idx, **adv)
        else:
            self.C.zero_spans(self.zero_table, self.n_zero, self.max_zero, **adv)

    def _check_idx(self) -> None:
        """Host-side range check of a directly written ``idx`` (eager steps / before capture; bound batch tables are
        checked in bind_batches): the kernels gather images and masks through it, so an index past the bound
        dataset is an out-of-range device read (a GPU memory fault), not an error."""
        if self.images is None or self.batch_table is not None:
            return
        lo, hi = int(self.idx.min()), int(self.idx.max())
        if lo < 0 or hi >= self.n_data:
            raise ValueError(f"idx holds [{lo}, {hi}] but the bound dataset has {self.n_data} images")

    def check_fixed_point(self) -> None:
        """Deterministic mode: raise if any fixed-point reduction add was clamped (a partial sum beyond the
        documented bounds of common.h red_add, or a NaN) since the mode was set - the totals are then wrong."""
        if self.det and self.C.fx_overflow():
            raise FloatingPointError("deterministic-mode fixed-point reduction overflowed (clamped at 2^62): the "
                                     "step's statistics / gradients exceed the int64 range at their scale")

    def _check_det(self) -> None:
        if self.C.det() != int(self.det):
            raise RuntimeError(f"engine built for deterministic={self.det} but the process mode is "
                               f"{bool(self.C.det())} (another engine switched it; the mode is per process)")

    def train_step_eager(self) -> None:
        self._check_det()
        self._zero_step()
        self.forward(True)                   # (fp8 mode: quantises the ConvT views at the decoder's start)
        self.backward()
        self.optimizer_step(advanced=True)

    # ------------------------------------------------------------------------------------------------ graph
    def capture(self) -> None:
        self._await_all()
        s = torch.cuda.Stream(device=self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(s):
            # warm-up launch outside capture (module load, lazy init) on a scratch copy of the state
            state = (self.flat, self.m, self.v, self.step_t, self.metrics, self.batch_cursor)
            saved = [t.clone() for t in state]
            self.train_step_eager()
            for t, c in zip(state, saved):
                t.copy_(c)
            self.pack()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with _no_gc(), torch.cuda.graph(g):
            self.train_step_eager()
        self.graph = g
        # the same launch sequence split after the encoder forward into two graphs sharing the step's buffers (the
        # engine allocates nothing during capture): replayed only for the first step after a FedAvg
        pre, post = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        torch.cuda.synchronize(self.dev)
        with _no_gc(), torch.cuda.stream(s):
            pre.capture_begin()

            def split():
                pre.capture_end()
                post.capture_begin(pool=pre.pool())
            self._mid_hook = split
            try:
                self.train_step_eager()
            finally:
                self._mid_hook = None
            post.capture_end()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        self.graph_pre, self.graph_post = pre, post

    def _stall_wait(self, end: Optional[int]) -> None:
        """Make the stream wait for the FedAvg buckets up to flat offset ``end`` (None: all); with ``stall_log``
        set, bracket the wait with timing events (their elapsed time = how long the compute stream stalled)."""
        if self.stall_log is None:
            self._await_all() if end is None else self._await_range(end)
            return
        cur = torch.cuda.current_stream(self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(cur)
        self._await_all() if end is None else self._await_range(end)
        e1.record(cur)
        self.stall_log.append((e0, e1))

    def train_step(self, use_graph: bool = True) -> None:
        """One training iteration: a replay of the captured hipGraph. After an overlapped FedAvg (``defer_until``)
        the step replays as its two split graphs: the encoder graph waits (device-side event waits, no host sync)
        only for the buckets holding the encoder's parameters and their repack, the rest of the step for every
        bucket - so the later buckets' all-reduce runs under the encoder forward."""
        if use_graph:
            self._check_det()
        if use_graph and self.graph is None:
            self._check_idx()
            self.capture()
        if not use_graph:
            self._check_idx()
            self.train_step_eager()
        elif self._pending:
            self._stall_wait(self.split_at)
            self.graph_pre.replay()
            self._stall_wait(None)
            self.graph_post.replay()
        else:
            self.graph.replay()

    def eval_step(self, use_graph: bool = True) -> None:
        """Inference-mode forward (moving BN statistics) of the batch in ``idx``; loss / accuracy accumulate into
        ``eval_metrics``. Replayed from its own hipGraph (captured after an eager warm-up)."""
        if self._share is not None:
            self._share._await_all()                   # the parameters are the parent's (FedAvg buckets in flight)
        if not use_graph:
            self._check_idx()
            self.forward(False)
            return
        self._await_all()
        if self.eval_graph is None:
            self._check_idx()
            s = torch.cuda.Stream(device=self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            with torch.cuda.stream(s):
                saved = self.eval_metrics.clone()
                self.forward(False)
                self.eval_metrics.copy_(saved)
            torch.cuda.current_stream(self.dev).wait_stream(s)
            torch.cuda.synchronize(self.dev)
            g = torch.cuda.CUDAGraph()
            with _no_gc(), torch.cuda.graph(g):
                self.forward(False)
            self.eval_graph = g
        self.eval_graph.replay()

    # ------------------------------------------------------------------------------------------------ state
    def set_flat(self, flat: np.ndarray) -> None:
        self._await_all()
        self.flat.copy_(torch.as_tensor(np.asarray(flat, np.float32)).to(self.dev))
        self.pack()

    def get_flat(self) -> np.ndarray:
        self._await_all()
        return self.flat.detach().cpu().numpy().copy()

    def reset_optimizer(self) -> None:
        self.m.zero_()
        self.v.zero_()
        self.step_t.zero_()

    def read_metrics(self, which: str = "train", reset: bool = True) -> Dict[str, float]:
        mt = self.metrics if which == "train" else self.eval_metrics
        v = mt.cpu().numpy()
        if reset:
            mt.zero_()
        return self.metrics_dict(v, which)

    @staticmethod
    def metrics_dict(v: np.ndarray, which: str = "train") -> Dict[str, float]:
        """The metric record of a metrics vector (``metrics`` / ``eval_metrics`` layout) read to the host."""
        n = max(v[2], 1.0)
        out = {"loss": float(v[0] / n) * 1.0, "bce_sum": float(v[0]), "accuracy": float(v[1] / n),
               "pixels": float(v[2]), "dice_sum": float(v[3])}
        if which != "train":       # crack-class overlap over the whole pass (train zeroes these every step)
            tp, pp, t = float(v[7]), float(v[8]), float(v[6])
            out["iou"] = tp / (pp + t - tp) if pp + t - tp > 0 else 1.0
            out["dice"] = 2.0 * tp / (pp + t) if pp + t > 0 else 1.0
        return out

    def evaluator(self, batch: int, snapshot: bool = False) -> "UNetEngine":
        """An inference-only engine of batch ``batch`` over THIS engine's parameters, packed weights and dataset.
        Validation loss / accuracy are per-pixel means over the whole held-out split (head.hip sums, normalised by
        the pixel count), so evaluating the same images in larger batches gives the same numbers - and larger
        batches fill the GPU (the 16-image eval forward is launch/latency-bound). Not used with the per-batch Dice term.

        ``snapshot``: the evaluator reads its OWN copy of the fp32 parameters and packed weights (``ParamSnapshot``,
        refreshed from this engine by ``snap.refresh()``), so a validation pass can run on another stream while the
        next epoch trains (``overlapped_validation``)."""
        if (batch == self.B and not snapshot) or self.dice:
            return self
        key = (batch, snapshot)
        ev = self._evaluators.get(key)
        if ev is None:
            share = ParamSnapshot(self) if snapshot else self
            ev = UNetEngine(self.table, batch, self.S, self.dev, "bce", self.lr, self.b1, self.b2, self.adam_eps,
                            self.momentum, self.bn_eps, share=share, deterministic=self.det,
                            conv_dtype=self.conv_dtype)
            ev.snap = share if snapshot else None
            if self.images is not None:
                ev.bind_data(self.images, self.masks)
            self._evaluators[key] = ev
        return ev

    def overlapped_validation(self, ev: "UNetEngine", batches: torch.Tensor, stream: torch.cuda.Stream,
                              use_graph: bool = True) -> torch.cuda.Event:
        """Validation of the CURRENT parameters on ``stream``, concurrent with whatever the caller issues next on
        the current (training) stream: the snapshot evaluator ``ev`` copies the parameters first (the training
        stream waits only for that 12 MB copy), then replays its inference graph over ``batches`` [n, ev.B].
        Keras semantics hold: the pass sees exactly the epoch-end weights. Returns the event marking the pass's
        end (join it before reading ``ev.eval_metrics``)."""
        main = torch.cuda.current_stream(self.dev)
        stream.wait_stream(main)
        with torch.cuda.stream(stream):
            ev.snap.refresh()
            copied = torch.cuda.Event()
            copied.record(stream)
            for v in range(batches.shape[0]):
                ev.idx.copy_(batches[v])
                ev.eval_step(use_graph)
            done = torch.cuda.Event()
            done.record(stream)
        main.wait_event(copied)                 # training may overwrite the parameters once they are copied
        return done

    def eval_batch_for(self, n_images: int, cap: int = 0) -> int:
        """Largest eval batch <= cap that is a multiple of B and divides ``n_images`` (a whole number of the
        reference's batches), so every held-out image is evaluated exactly once. Default cap (CFL_EVAL_CAP): 1024
        images, further bounded to a quarter of the device's free HBM at ~21.7 MB of forward activations per 256^2
        image (scaled by resolution) - several clients may share one device in a rehearsal. Round 4's 2048 cap (the
        bench's 1,776-image split in ONE launch) measured 12,754 / 12,688 img/s and 40.6 GB peak HBM per client
        against 12,859 / 12,812 img/s and 15.5 GB for three 592-image launches (profiles/r5_evalcap, one box).

        The choice is made ONCE per (n_images, cap) and remembered: free HBM shrinks once the first evaluator and its
        graph exist, and re-deciding every pass would pick a smaller batch and build (and capture) another evaluator
        each round (advisor r5)."""
        key = (n_images, cap)
        memo = self._eval_batch_memo
        if key in memo:
            return memo[key]
        if cap <= 0:
            cap = int(os.environ.get("CFL_EVAL_CAP", "1024"))
            if self.dev.type == "cuda":
                free, _total = torch.cuda.mem_get_info(self.dev)
                per_img = 21.7e6 * (self.S / 256.0) ** 2
                cap = max(self.B, min(cap, int(free / 4 / per_img)))
        nb = n_images // self.B
        best = 1
        for k in range(1, nb + 1):
            if nb % k == 0 and k * self.B <= cap:
                best = k
        memo[key] = best * self.B
        return memo[key]

    def predict_probs(self) -> torch.Tensor:
        """Sigmoid probabilities at full resolution for the current ``idx`` batch (eval-mode BN)."""
        self.forward(False)
        p = torch.sigmoid(self.h)
        return p.repeat_interleave(2, 1).repeat_interleave(2, 2)


class ParamSnapshot:
    """The parameter-side view an inference engine shares (``UNetEngine(share=...)``): private copies of a training
    engine's fp32 flat buffer and bf16 packed weights, refreshed on demand (the evaluator's BN tables point at these
    copies, so the training engine may keep updating its own while a validation pass runs)."""

    def __init__(self, parent: "UNetEngine"):
        self.parent = parent
        self.flat = parent.flat.clone()
        self.packed = parent.packed.clone()

    def refresh(self) -> None:
        self.parent._await_all()
        self.flat.copy_(self.parent.flat)
        self.packed.copy_(self.parent.packed)

    def _await_all(self) -> None:
        pass


class DeferredMetrics:
    """An epoch's metrics snapshot on the device plus the HIP events around its launches; ``result()`` reads it (the
    first call synchronises on the snapshot), ``seconds()`` is the GPU time between the events."""

    def __init__(self, snap: torch.Tensor, t0, t1, finish):
        self.snap, self.t0, self.t1, self.finish = snap, t0, t1, finish
        self._res: Optional[Dict[str, float]] = None

    def result(self) -> Dict[str, float]:
        if self._res is None:
            self._res = self.finish(self.snap.cpu().numpy())
        return self._res

    def seconds(self) -> float:
        self.t1.synchronize()
        return self.t0.elapsed_time(self.t1) / 1e3


class HipBackend:
    """``train.local.StepBackend`` on the MI355X engine."""

    def __init__(self, cfg, data, table: ParamTable):
        self.cfg = cfg
        self.table = table
        self.eng = UNetEngine(table, cfg.batch_size, data.img_size, "cuda", cfg.loss, cfg.lr, cfg.beta1, cfg.beta2,
                              cfg.adam_eps, cfg.bn_momentum, cfg.bn_eps,
                              deterministic=True if getattr(cfg, "deterministic", False) else None,
                              conv_dtype=getattr(cfg, "conv_dtype", None) or None)
        images = data.images if isinstance(data.images, torch.Tensor) else torch.as_tensor(data.images)
        masks = data.masks if isinstance(data.masks, torch.Tensor) else torch.as_tensor(data.masks)
        self.eng.bind_data(images.to(self.eng.dev), masks.to(self.eng.dev))
        self.eng.set_flat(table.init_flat(cfg.seed))
        self.use_graph = cfg.use_graph

    def set_flat(self, flat):
        self.eng.set_flat(flat)

    def get_flat(self):
        return self.eng.get_flat()

    def reset_optimizer(self):
        self.eng.reset_optimizer()

    def optimizer_state(self):
        e = self.eng
        return int(e.step_t.item()), e.m.cpu().numpy().copy(), e.v.cpu().numpy().copy()

    def _upload_indices(self, idx: np.ndarray) -> torch.Tensor:
        """Dataset indices to the device without a host sync: range-checked here on the host (the kernels gather
        images / masks through them), then an asynchronous copy from pinned memory (a pageable copy would wait for
        the stream to drain)."""
        e = self.eng
        idx = np.ascontiguousarray(idx, np.int32)
        if idx.size and (int(idx.min()) < 0 or int(idx.max()) >= e.n_data):
            raise ValueError(f"indices [{int(idx.min())}, {int(idx.max())}] outside the bound dataset of {e.n_data}")
        h = torch.from_numpy(idx)
        if e.dev.type == "cuda":
            h = h.pin_memory()
        return h.to(e.dev, non_blocking=True)

    def train_batches_deferred(self, batches: np.ndarray) -> "DeferredMetrics":
        """One epoch of training steps, issued without any host sync: the batch table goes up asynchronously
        (range-checked on the host), and the epoch's metrics are snapshotted on the device (stream-ordered clone)
        between two timing events. ``DeferredMetrics.result()`` reads them later - the FL client resolves a whole
        round's epochs at once, so the GPU never idles at an epoch boundary waiting for the host (train.local)."""
        e = self.eng
        dev_b = self._upload_indices(np.asarray(batches, np.int32))
        e.metrics.zero_()
        e.bind_batches(dev_b, checked=True)    # the steps select their batches on the device (no per-step copy)
        e.set_batch_cursor(0)
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(dev_b.shape[0]):
            e.train_step(self.use_graph)
        snap = e.metrics.clone()
        t1 = torch.cuda.Event(enable_timing=True)
        t1.record()
        nb = max(1, len(batches))

        def finish(v: np.ndarray) -> Dict[str, float]:
            e.check_fixed_point()
            m = UNetEngine.metrics_dict(v, "train")
            if e.dice:
                m["loss"] = m["loss"] + m["dice_sum"] / nb
            return m
        return DeferredMetrics(snap, t0, t1, finish)

    def eval_batches_deferred(self, batches: np.ndarray) -> "DeferredMetrics":
        """Validation over the images of ``batches`` (the reference's 16-image batches), evaluated in the largest
        multiple of them up to the eval cap per launch (eval_batch_for / evaluator: same per-pixel means, fewer and
        fuller launches); issued without a host sync, like ``train_batches_deferred``."""
        e = self.eng
        idx = np.asarray(batches, np.int32).reshape(-1)
        ev = e.evaluator(e.eval_batch_for(len(idx)))
        e._await_all()
        dev_b = self._upload_indices(idx.reshape(-1, ev.B))
        ev.eval_metrics.zero_()
        t0 = torch.cuda.Event(enable_timing=True)
        t0.record()
        for s in range(dev_b.shape[0]):
            ev.idx.copy_(dev_b[s])
            ev.eval_step(self.use_graph)
        snap = ev.eval_metrics.clone()
        t1 = torch.cuda.Event(enable_timing=True)
        t1.record()
        return DeferredMetrics(snap, t0, t1, lambda v: UNetEngine.metrics_dict(v, "eval"))

    def train_batches(self, batches: np.ndarray) -> Dict[str, float]:
        return self.train_batches_deferred(batches).result()

    def eval_batches(self, batches: np.ndarray) -> Dict[str, float]:
        return self.eval_batches_deferred(batches).result()

    def predict(self, idx: np.ndarray) -> np.ndarray:
        e = self.eng
        out = []
        idx = np.asarray(idx, np.int32)
        for s in range(0, len(idx), e.B):
            chunk = idx[s:s + e.B]
            pad = np.concatenate([chunk, np.repeat(chunk[-1:], e.B - len(chunk))])
            e.idx.copy_(torch.as_tensor(pad).to(e.dev))
            out.append(e.predict_probs()[:len(chunk)].cpu().numpy())
        return np.concatenate(out)
