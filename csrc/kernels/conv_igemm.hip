// Implicit-GEMM convolution (forward and data-gradient) on gfx950 MFMA (v_mfma_f32_16x16x32_bf16).
//
// Covers every Conv2D / SeparableConv2D-pointwise / Conv2DTranspose of the U-Net
// (/root/reference/client_fit_model.py:100-145) except the 3-channel entry conv (csrc/kernels/entry.hip):
//   GEMM  M = B*Ho*Wo (pixels),  N = Cout,  K = ks*ks*Cin  (NHWC: a K-slice of 32 is 32 channels of one tap)
//   * TF "same" padding with explicit top/left pads (stride-2 convs pad bottom/right only);
//   * logical input may be the nearest-2x upsample of the stored tensor (UpSampling2D folded into indexing);
//   * the producer's BatchNorm apply + ReLU is applied on load (no normalised activation is ever stored);
//   * epilogue: + bias, bf16 store, per-channel sum / sum-of-squares for the NEXT BatchNorm (batch stats).
// Conv2DTranspose (stride 1, same) is a correlation with the spatially flipped, in/out-transposed kernel: that
// permutation lives in the packed weight matrix (csrc/kernels/optim.hip, pack kernel), so the same kernel serves
// the transposed conv and every data-gradient (dgrad = forward conv of dy with the dgrad-packed weights).
//
// Tiling: block 128(M) x BN(N), K-step 32, 256 threads = 4 waves (WM x WN), each wave (128/WM) x (BN/WN) of
// 16x16 MFMA fragments. Operands are register-staged (global_load_dwordx4 -> transform -> ds_write_b128) into two
// LDS buffers; the next K-tile's global loads are issued before the current tile's MFMAs (one barrier per K-step).
// LDS rows are padded to 40 bf16 (80 B) so the 16 row-reads of a ds_read_b128 lane group hit distinct bank slots.
#include "common.h"
#include "launch.h"

namespace {

constexpr int BM = 128;
constexpr int BK = 32;
constexpr int LDK = BK + 8;   // padded LDS row (bf16 elements)
constexpr int NT = 256;

template <int BN_, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void conv_igemm_kernel(ConvParams p) {
  static_assert(WM * WN == 4, "4 waves");
  constexpr int TM = BM / WM, TN = BN_ / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int B_CHUNKS = BN_ * BK / 8;                 // 16-byte chunks in one B tile
  constexpr int B_PER_T = (B_CHUNKS + NT - 1) / NT;

  __shared__ __attribute__((aligned(16))) bf16_t sA[2][BM][LDK];
  __shared__ __attribute__((aligned(16))) bf16_t sB[2][BN_][LDK];
  __shared__ float sred[2][WM][BN_];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int mBlock = blockIdx.x * BM, nBlock = blockIdx.y * BN_;
  const int HWo = p.Ho * p.Wo;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;

  // ---- per-thread A rows (fixed over the K loop) ----
  const int kq = tid & 3;
  int a_b[2], a_ih[2], a_iw[2];
  bool a_ok[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = mBlock + (tid >> 2) + i * 64;
    a_ok[i] = m < p.M;
    const int mm = a_ok[i] ? m : 0;
    const int b = mm / HWo, r = mm - b * HWo;
    const int oh = r / p.Wo, ow = r - oh * p.Wo;
    a_b[i] = b;
    a_ih[i] = oh * p.stride - p.pad_t;
    a_iw[i] = ow * p.stride - p.pad_l;
  }

  uint4 ra[2], rb[B_PER_T];
  const int KT = p.K / BK;

  auto load_tiles = [&](int kt) {
    const int k0 = kt * BK + kq * 8;
    const int tap = k0 / p.Cin, c = k0 - tap * p.Cin;
    const int ky = tap / p.ks, kx = tap - ky * p.ks;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ih = a_ih[i] + ky, iw = a_iw[i] + kx;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_ok[i] && ih >= 0 && ih < Hl && iw >= 0 && iw < Wl) {
        const size_t off = (((size_t)a_b[i] * p.Hin + (ih >> p.up_in)) * p.Win + (iw >> p.up_in)) * p.Cin + c;
        v = *reinterpret_cast<const uint4*>(p.x + off);
        if (p.xf.ab || p.xf.relu) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = xform1(f[j], p.xf, c + j);
          v = pack8(f);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int ch = tid + i * NT;
      if (ch < B_CHUNKS) {
        const int n = ch >> 2, q = ch & 3;
        rb[i] = *reinterpret_cast<const uint4*>(p.wt + (size_t)(nBlock + n) * p.K + kt * BK + q * 8);
      }
    }
  };

  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *reinterpret_cast<uint4*>(&sA[buf][(tid >> 2) + i * 64][kq * 8]) = ra[i];
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int ch = tid + i * NT;
      if (ch < B_CHUNKS) *reinterpret_cast<uint4*>(&sB[buf][ch >> 2][(ch & 3) * 8]) = rb[i];
    }
  };

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  load_tiles(0);
  store_tiles(0);
  __syncthreads();

  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load_tiles(kt + 1);
    s8v af[FM], bfg[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const s8v*>(&sA[cur][wm * TM + i * 16 + fr][fk]);
#pragma unroll
    for (int j = 0; j < FN; ++j) bfg[j] = *reinterpret_cast<const s8v*>(&sB[cur][wn * TN + j * 16 + fr][fk]);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    if (kt + 1 < KT) store_tiles(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + r ----
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = nBlock + wn * TN + j * 16 + (lane & 15);
    const float bias = p.bias ? p.bias[n] : 0.f;
    float s = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mBlock + wm * TM + i * 16 + (lane >> 4) * 4 + r;
        if (m < p.M) {
          const bf16_t yb = f2bf(acc[i][j][r] + bias);
          p.y[(size_t)m * p.N + n] = yb;
          const float yv = bf2f(yb);
          s += yv;
          s2 += yv * yv;
        }
      }
    }
    if (p.stats) {
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lane < 16) {
        sred[0][wm][wn * TN + j * 16 + lane] = s;
        sred[1][wm][wn * TN + j * 16 + lane] = s2;
      }
    }
  }
  if (p.stats) {
    // combine the WM wave rows, then one atomic per (stat, column) into this block's replica row
    __syncthreads();
    float* rep = p.stats + (size_t)(blockIdx.x % STAT_REPLICAS) * 2 * p.N;
    for (int e = tid; e < 2 * BN_; e += NT) {
      const int st = e / BN_, c = e - st * BN_;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) v += sred[st][w][c];
      atomicAdd(&rep[st * p.N + nBlock + c], v);
    }
  }
}

}  // namespace

int conv_igemm(const ConvParams& p, hipStream_t st) {
  if (p.Cin % 32 != 0 || p.K % BK != 0 || p.K != p.ks * p.ks * p.Cin) return 1;
  dim3 blk(NT);
  if (p.N % 128 == 0 && p.N >= 128) {
    dim3 grid((p.M + BM - 1) / BM, p.N / 128);
    hipLaunchKernelGGL((conv_igemm_kernel<128, 2, 2>), grid, blk, 0, st, p);
  } else if (p.N % 64 == 0) {
    dim3 grid((p.M + BM - 1) / BM, p.N / 64);
    hipLaunchKernelGGL((conv_igemm_kernel<64, 2, 2>), grid, blk, 0, st, p);
  } else if (p.N % 32 == 0) {
    dim3 grid((p.M + BM - 1) / BM, p.N / 32);
    hipLaunchKernelGGL((conv_igemm_kernel<32, 4, 1>), grid, blk, 0, st, p);
  } else {
    return 2;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
