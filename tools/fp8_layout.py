"""Operand lane maps of gfx950's block-scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4 / _32x32x64_), checked
with exact small-integer data against a host GEMM through the ``mfma_scale_probe`` binding (csrc/kernels/fp8.hip).

Measured maps (FP8_DISCOVER=1 prints the experiments that found them): lane l holds 32 bytes of ONE row of A (one
column of B) in two 16-element halves from DIFFERENT 32-element K-blocks, and its scale word's byte 0 (opsel 0) is
the e8m0 exponent (2^(e - 127)) of the block with its lane group's index:
  16x16x128: row / col = l & 15, g = l >> 4: bytes 0-15 = k 16 g .. 16 g + 15, bytes 16-31 = k 64 + 16 g .. ;
             scale = block g (k 32 g .. 32 g + 31)
  32x32x64:  row / col = l & 31, h = l >> 5: bytes 0-15 = k 16 h .. 16 h + 15, bytes 16-31 = k 32 + 16 h .. ;
             scale = block h
i.e. K-block b is the first (b even: ...) halves of two lane groups - a block of 32 is never one lane's 32 bytes.
C/D: 16x16: col = l & 15, row = 4 (l >> 4) + r;  32x32: col = l & 31, row = (r & 3) + 8 (r >> 2) + 4 (l >> 5).
Prints one line per check; exits non-zero if a check fails.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd._native_loader import hip  # noqa: E402


def e4m3_bytes(x: np.ndarray) -> np.ndarray:
    return torch.from_numpy(x.astype(np.float32)).to(torch.float8_e4m3fn).view(torch.uint8).numpy()


def run(shape: int, A: np.ndarray, B: np.ndarray, sa_blk: np.ndarray, sb_blk: np.ndarray, byte: int = 0):
    """A [M][K], B [K][N] exact e4m3 values; sa_blk [M][K/32], sb_blk [N][K/32] e8m0 exponents."""
    M = N = shape
    K = 128 if shape == 16 else 64
    grp = 16 if shape == 16 else 32
    a = np.zeros((64, 32), np.uint8)
    b = np.zeros((64, 32), np.uint8)
    sa = np.zeros(64, np.int64)
    sb = np.zeros(64, np.int64)
    ab, bb = e4m3_bytes(A), e4m3_bytes(B.T)
    half = K // 2                                   # k offset of a lane's second 16-byte half
    for l in range(64):
        r, g = l % grp, l // grp
        a[l, :16], a[l, 16:] = ab[r, 16 * g:16 * g + 16], ab[r, half + 16 * g:half + 16 * g + 16]
        b[l, :16], b[l, 16:] = bb[r, 16 * g:16 * g + 16], bb[r, half + 16 * g:half + 16 * g + 16]
        sa[l] = int(sa_blk[r, g]) << (8 * byte)
        sb[l] = int(sb_blk[r, g]) << (8 * byte)
    dev = "cuda"
    ta = torch.from_numpy(a.view(np.int32).copy()).to(dev)
    tb = torch.from_numpy(b.view(np.int32).copy()).to(dev)
    tsa = torch.from_numpy(sa.astype(np.int64).astype(np.uint32).view(np.int32)).to(dev)
    tsb = torch.from_numpy(sb.astype(np.int64).astype(np.uint32).view(np.int32)).to(dev)
    d = hip().mfma_scale_probe(ta, tb, tsa, tsb, shape).cpu().numpy()
    D = np.zeros((M, N), np.float64)
    for l in range(64):
        for r in range(d.shape[1]):
            if shape == 16:
                row, col = 4 * (l // 16) + r, l % 16
            else:
                row, col = (r & 3) + 8 * (r >> 2) + 4 * (l // 32), l % 32
            D[row, col] = d[l, r]
    As = A * np.repeat(2.0 ** (sa_blk - 127.0), 32, axis=1)
    Bs = B * np.repeat(2.0 ** (sb_blk - 127.0), 32, axis=1).T
    return D, As @ Bs


def discover(shape: int) -> None:
    """Which (row, 32-block) each lane's A scale and which (col, block) each lane's B scale governs: all-ones data,
    every scale 2^0 except ONE lane's at 2^1; the doubled blocks show up as +32 in the affected D rows / cols."""
    K = 128 if shape == 16 else 64
    grp = 16 if shape == 16 else 32
    ones = np.ones((shape, K))
    for which in ("A", "B"):
        out = []
        for l in range(64):
            a = np.zeros((64, 32), np.uint8)
            b = np.zeros((64, 32), np.uint8)
            a[:] = e4m3_bytes(np.ones((1, 32)))[0]
            b[:] = a
            sa = np.full(64, 127, np.int64)
            sb = np.full(64, 127, np.int64)
            (sa if which == "A" else sb)[l] = 128
            dev = "cuda"
            d = hip().mfma_scale_probe(torch.from_numpy(a.view(np.int32).copy()).to(dev),
                                       torch.from_numpy(b.view(np.int32).copy()).to(dev),
                                       torch.from_numpy(sa.astype(np.int32)).to(dev),
                                       torch.from_numpy(sb.astype(np.int32)).to(dev), shape).cpu().numpy()
            D = np.zeros((shape, shape))
            for ll in range(64):
                for r in range(d.shape[1]):
                    if shape == 16:
                        row, col = 4 * (ll // 16) + r, ll % 16
                    else:
                        row, col = (r & 3) + 8 * (r >> 2) + 4 * (ll // 32), ll % 32
                    D[row, col] = d[ll, r]
            diff = D - K
            if which == "A":
                rows = [int(i) for i in np.nonzero(np.abs(diff).sum(1))[0]]
                inc = sorted(set(float(x) for x in diff[rows].ravel())) if rows else []
                out.append(f"l{l}:rows{rows}+{inc}")
            else:
                cols = [int(i) for i in np.nonzero(np.abs(diff).sum(0))[0]]
                inc = sorted(set(float(x) for x in diff[:, cols].ravel())) if cols else []
                out.append(f"l{l}:cols{cols}+{inc}")
        print(f"{shape}x{shape} {which} scale lanes: " + " ".join(out), flush=True)


def discover_blocks(shape: int) -> None:
    """Which DATA lane group's 32-element block each SCALE lane group governs: lane group g's data = g + 1 (all
    32 bytes), the other operand all ones; doubling the scale of one lane of scale group h adds 32 (g + 1) to its
    row / column, where g is the data group whose block that scale covers."""
    K = 128 if shape == 16 else 64
    grp = 16 if shape == 16 else 32
    ng = 64 // grp
    for which in ("A", "B"):
        res = []
        for h in range(ng):
            a = np.zeros((64, 32), np.uint8)
            b = np.zeros((64, 32), np.uint8)
            for l in range(64):
                v = float(l // grp + 1)
                (a if which == "A" else b)[l] = e4m3_bytes(np.full((1, 32), v))[0]
                (b if which == "A" else a)[l] = e4m3_bytes(np.ones((1, 32)))[0]
            sa = np.full(64, 127, np.int64)
            sb = np.full(64, 127, np.int64)
            (sa if which == "A" else sb)[h * grp] = 128
            dev = "cuda"
            d = hip().mfma_scale_probe(torch.from_numpy(a.view(np.int32).copy()).to(dev),
                                       torch.from_numpy(b.view(np.int32).copy()).to(dev),
                                       torch.from_numpy(sa.astype(np.int32)).to(dev),
                                       torch.from_numpy(sb.astype(np.int32)).to(dev), shape).cpu().numpy()
            base = 32 * sum(range(1, ng + 1))
            inc = sorted(set(float(x) - base for x in d.ravel()) - {0.0})
            res.append(f"scale group {h} -> +{inc} (data group {[int(i / 32) - 1 for i in inc]})")
        print(f"{shape}x{shape} {which}: " + "; ".join(res), flush=True)


def main() -> int:
    if os.environ.get("FP8_DISCOVER"):
        for shape in (16, 32):
            discover_blocks(shape)
        return 0
    if os.environ.get("FP8_DISCOVER_ROWS"):
        for shape in (16, 32):
            discover(shape)
        return 0
    rng = np.random.default_rng(0)
    bad = 0
    for shape in (16, 32):
        K = 128 if shape == 16 else 64
        A = rng.integers(-4, 5, (shape, K)).astype(np.float64)
        B = rng.integers(-4, 5, (K, shape)).astype(np.float64)
        one = np.full((shape, K // 32), 127)
        D, ref = run(shape, A, B, one, one)
        ok = np.array_equal(D, ref)
        print(f"{shape}x{shape}: unscaled integer GEMM {'OK' if ok else 'MISMATCH'} (max |d| {np.abs(D - ref).max()})")
        bad += not ok
        sa = rng.integers(124, 131, (shape, K // 32))
        sb = rng.integers(124, 131, (shape, K // 32))
        D, ref = run(shape, A, B, sa, sb)
        ok = np.allclose(D, ref, rtol=0, atol=0)
        print(f"{shape}x{shape}: per-32 block scales {'OK' if ok else 'MISMATCH'} (max |d| {np.abs(D - ref).max()})")
        bad += not ok
        for byte in (1, 2, 3):
            D, _ = run(shape, A, B, sa, sb, byte=byte)
            _, ref0 = run(shape, A, B, np.zeros_like(sa), np.zeros_like(sb))   # a zero byte 0 (2^-127)
            print(f"{shape}x{shape}: scale in byte {byte} with opsel 0 -> matches 2^-127 scales: "
                  f"{np.allclose(D, ref0)}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
