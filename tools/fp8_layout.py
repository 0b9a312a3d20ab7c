"""Operand lane maps of gfx950's block-scaled fp8 MFMA (v_mfma_scale_f32_16x16x128_f8f6f4 / _32x32x64_), checked
with exact small-integer data against a host GEMM through the ``mfma_scale_probe`` binding (csrc/kernels/fp8.hip).

Hypothesis (the maps the fp8 kernels use): lane l holds 32 consecutive k of ONE row of A (and of one column of B):
  16x16x128: row / col = l & 15, k = 32 (l >> 4) + j;   32x32x64: row / col = l & 31, k = 32 (l >> 5) + j
and its scale word's byte 0 (opsel 0) is the e8m0 exponent (2^(e - 127)) of exactly that 32-element block.
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
    for l in range(64):
        r, kb = l % grp, l // grp
        a[l] = ab[r, 32 * kb:32 * kb + 32]
        b[l] = bb[r, 32 * kb:32 * kb + 32]
        sa[l] = int(sa_blk[r, kb]) << (8 * byte)
        sb[l] = int(sb_blk[r, kb]) << (8 * byte)
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


def main() -> int:
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
