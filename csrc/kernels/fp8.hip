// Block-scaled fp8 (OCP e4m3) MFMA on gfx950: v_mfma_scale_f32_32x32x64_f8f6f4 with per-32-element e8m0 block
// scales - BASELINE config 5's fp8 Conv2D MFMA path, for the decoder's 3x3 convolutions (every Conv2DTranspose
// forward and data gradient, /root/reference/client_fit_model.py:129,133; 66 % of the network's FLOPs).
//
// Why block-scaled. gfx950's non-scaled fp8 MFMA (16x16x32 / 32x32x16 fp8) issues at the bf16 form's rate; the
// scaled f8f6f4 forms take twice the bf16 cycles for four times the K, i.e. 2x the bf16 MFMA rate (MI355X_MICROARCH.md
// matrix-core table). Round 2-3's non-scaled fp8 path was slower than bf16 and was removed in round 4.
//
// Numerics. A K-block is 32 consecutive input channels of ONE tap (K order tap * Cin + c, Cin % 32 == 0): the
// activations get one e8m0 scale per (halo pixel, 32-channel chunk), the weights one per (output channel, tap, chunk);
// scale 2^e with e = ceil(log2(amax / 448)), so every block's largest element maps to <= 448 (e4m3's max) and is
// rounded to 3 mantissa bits. Products accumulate in fp32 (the MFMA's C); the epilogue is the bf16 kernels'.
//
// Kernel (conv3x3_f8_kernel): the whole-chunk structure of conv3x3.hip's WB path - a block owns a TH x TW pixel tile
// x BN output channels; per 32-channel chunk it stages the (TH+2) x (TW+2) halo (producer BN-apply + ReLU and the
// nearest-2x upsample folded into the load, then quantised: 4 lanes hold a pixel's 32 channels, their amax meets by
// two lane shuffles) and the chunk's 9-tap fp8 weight tile with its scales, next chunk prefetched in registers during
// the current chunk's MFMAs. One 32x32x64 MFMA covers TWO taps of a chunk (k-half h = lane >> 5 of the fragment =
// tap 2s + h), so a chunk is 5 k-steps (the 10th tap slot has zero weights): 10 % padding against the 2x rate.
// LDS rows are 32 bytes (a pixel's chunk or a weight row's chunk) with the two 16-byte halves swapped in every other
// group of 8 rows, plus one scale byte per row. Fragment rows are PERMUTED (f8_perm): a ds_read_b128 serves its 64
// lanes in four 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31}, + 32), so fragment row rho of lane l & 31
// holds pixel / output channel f8_perm(rho), which gives every group 16 CONSECUTIVE rows - with the 8-row half swap,
// all 64 banks for any start row (tap shifts move it). The first build (natural order, 4-row swap) measured 20-32 %
// LDS bank conflicts (profiles/r5_fp8/pmc_compare.txt).
//
// mfma_scale_probe: one wave runs ONE scaled MFMA on caller-supplied lane registers (32 fp8 bytes of A and of B per
// lane, one int32 scale word each) and returns the raw accumulator registers - the operand lane maps are checked
// against a host GEMM with exact small-integer data (tools/fp8_layout.py, tests/test_gpu_kernels.py).
#include "common.h"
#include "launch.h"

namespace {

typedef int i8v __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(64) void mfma_scale_probe_kernel(const int* __restrict__ a, const int* __restrict__ b,
                                                              const int* __restrict__ sa, const int* __restrict__ sb,
                                                              float* __restrict__ d, int shape) {
  CFL_TS_GUARD;
  const int l = threadIdx.x;
  i8v av, bv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a[l * 8 + j];
    bv[j] = b[l * 8 + j];
  }
  if (shape == 16) {
    f4v c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, sa[l], 0, sb[l]);
#pragma unroll
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
  } else {
    f16v c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c, 0, 0, 0, sa[l], 0, sb[l]);
#pragma unroll
    for (int r = 0; r < 16; ++r) d[l * 16 + r] = c[r];
  }
}

// ---------------------------------------------------------------- quantisation helpers
// e8m0 exponent byte of a 32-element block with largest magnitude amax: e = ceil(log2(amax / 448)) (so that
// amax * 2^-e <= 448), clamped to [-127, 126]; byte = e + 127 (2^(byte - 127) is the MFMA's block scale)
CFL_DEVICE int f8_block_exp(float amax) {
  const uint32_t u = __float_as_uint(amax * (1.0f / 448.0f));
  int e = (int)((u >> 23) & 0xff) - 127 + ((u & 0x7fffff) != 0 ? 1 : 0);
  return imin(imax(e, -127), 126);
}
CFL_DEVICE float f8_inv_scale(int e) { return __uint_as_float((uint32_t)(127 - e) << 23); }   // 2^-e
// 8 floats (already scaled into e4m3 range) -> 8 e4m3 bytes
CFL_DEVICE uint2 f8_pack8(const float* f) {
  int lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return make_uint2((uint32_t)lo, (uint32_t)hi);
}

// ---------------------------------------------------------------- weight quantisation (one launch per step)
// item: a packed bf16 [N][K] weight view -> e4m3 [N][K] + e8m0 scales [N][K / 32]; one thread per 32-element block
constexpr int Q8_MAX = 24;
struct Q8Item {
  const bf16_t* src;
  uint8_t* dst;
  uint8_t* sc;
  int nblk, blk0;
};
struct Q8Table {
  Q8Item it[Q8_MAX];
  int n, total;
};

__global__ __launch_bounds__(256) void quant_w8_kernel(const Q8Table t) {
  CFL_TS_GUARD;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < t.total; g += gridDim.x * 256) {
    int k = 0;
    while (k + 1 < t.n && t.it[k + 1].blk0 <= g) ++k;
    const Q8Item& I = t.it[k];
    const int blk = g - I.blk0;
    const uint4* src = reinterpret_cast<const uint4*>(I.src + (size_t)blk * 32);
    float f[32];
#pragma unroll
    for (int i = 0; i < 4; ++i) unpack8(src[i], f + 8 * i);
    float amax = 0.f;
#pragma unroll
    for (int j = 0; j < 32; ++j) amax = fmaxf(amax, fabsf(f[j]));
    const int e = f8_block_exp(amax);
    const float inv = f8_inv_scale(e);
#pragma unroll
    for (int j = 0; j < 32; ++j) f[j] *= inv;
    uint2* dst = reinterpret_cast<uint2*>(I.dst + (size_t)blk * 32);
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i] = f8_pack8(f + 8 * i);
    I.sc[blk] = (uint8_t)(e + 127);
  }
}

// ---------------------------------------------------------------- 3x3 / stride-1 / same conv, fp8 operands
constexpr int F8_NT = 256;
constexpr int F8_BK = 32;
// byte offset of 16-byte half h of LDS row r (32-byte rows; halves swapped in every other group of 8 rows)
CFL_DEVICE int f8_off(int r, int h) { return r * 32 + ((h ^ ((r >> 3) & 1)) << 4); }
// fragment row rho (0..31) -> pixel / channel index within the 32-row fragment: the ds_read_b128 lane group
// {0-3, 12-15, 20-27} gets rows 0..15, {4-11, 16-19, 28-31} rows 16..31
CFL_DEVICE int f8_perm(int rho) {
  return rho < 4 ? rho : rho < 12 ? rho + 12 : rho < 16 ? rho - 8 : rho < 20 ? rho + 8 : rho < 28 ? rho - 12 : rho;
}

template <int TH, int TW, int BN_, int WM, int WN, bool PJ, bool XFIN>
__global__ __launch_bounds__(F8_NT, 2) void conv3x3_f8_kernel(ConvParams p) {
  CFL_TS_GUARD;
  constexpr int NT = F8_NT, BK = F8_BK;
  constexpr int BM = TH * TW;
  constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;
  constexpr int TM = BM / WM, TN = BN_ / WN, FM = TM / 32, FN = TN / 32;
  constexpr int HALO_PIECES = HP * 4, H_PER_T = (HALO_PIECES + NT - 1) / NT;      // 8-channel pieces
  constexpr int WROWS = 9 * BN_;                                                  // (tap, n) weight rows
  constexpr int W_PIECES = WROWS * 2, W_PER_T = (W_PIECES + NT - 1) / NT;       // 16-byte pieces
  constexpr int S_PER_T = (WROWS + NT - 1) / NT;                                  // scale bytes
  constexpr int LDC = BN_ + 8;
  constexpr int STAGE = HP * 32 + WROWS * 32;                                     // fp8 bytes
  constexpr int SCALES = ((HP + WROWS) + 15) / 16 * 16;
  constexpr int CBYTES = BM * LDC * 2;
  constexpr int SMEM = STAGE + SCALES > CBYTES ? STAGE + SCALES : CBYTES;
  static_assert(WM * WN == 4 && TM % 32 == 0 && TN % 32 == 0, "wave tiling");

  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];
  __shared__ float sred[2][4][BN_];
  __shared__ float sxab[XFIN ? 2 * 256 : 1];
  uint8_t* sH = smem;                        // [HP][32] fp8 halo of the chunk
  uint8_t* sW = smem + HP * 32;              // [9 * BN_][32] fp8 weights of the chunk
  uint8_t* sHs = smem + STAGE;               // [HP] halo scales
  uint8_t* sWs = smem + STAGE + HP;          // [9 * BN_] weight scales

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_w = (p.Wo + TW - 1) / TW, tiles_h = (p.Ho + TH - 1) / TH;
  const int lin = xcd_block_linear();
  const int bn_idx = lin % gridDim.y;
  int t = lin / gridDim.y;
  const int tile_id = t;
  const int b = t / (tiles_w * tiles_h);
  t -= b * tiles_w * tiles_h;
  const int ty0 = (t / tiles_w) * TH, tx0 = (t % tiles_w) * TW;
  const int nBlock = bn_idx * BN_;
  const int chunks = p.Cin / BK;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;
  const int kblocks = p.K / BK;              // scale bytes per weight row

  // ---- halo: piece e -> halo pixel e / 4, 8-channel quarter e % 4 (= tid & 3 for every piece of a thread) ----
  uint4 rh[H_PER_T];
  uint32_t hvalid = 0;
  float ha[8], hb[8];
  auto load_coefs = [&](int ch) {
    const int c8 = ch * BK + (tid & 3) * 8;
    if constexpr (XFIN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ha[j] = sxab[c8 + j];
        hb[j] = sxab[256 + c8 + j];
      }
    } else {
      load_f8_or(p.xf.ab + c8, has_ab, 1.f, ha);
      load_f8_or(p.xf.ab + p.xf.C + c8, has_ab, 0.f, hb);
    }
  };
  auto load_halo = [&](int ch) {
    uint32_t hv = 0;
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < HALO_PIECES) {
        const int hp = e >> 2, q = e & 3;
        const int hy = hp / HW, hx = hp - hy * HW;
        const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
        if (iy >= 0 && iy < Hl && ix >= 0 && ix < Wl) {
          v = *reinterpret_cast<const uint4*>(
              p.x + (((size_t)b * p.Hin + (iy >> p.up_in)) * p.Win + (ix >> p.up_in)) * p.Cin + ch * BK + q * 8);
          hv |= 1u << i;
        }
      }
      rh[i] = v;
    }
    hvalid = hv;
  };
  // transform (BN-apply + ReLU; padding stays 0) + quantise + LDS store of the chunk's halo
  auto store_halo = [&]() {
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      float f[8];
      unpack8(rh[i], f);
      const bool ok = (hvalid >> i) & 1u;
      float amax = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = has_ab ? fmaf(ha[j], f[j], hb[j]) : f[j];
        if (relu) v = fmaxf(v, 0.f);
        f[j] = ok ? v : 0.f;
        amax = fmaxf(amax, fabsf(f[j]));
      }
      // the pixel's 32 channels are held by 4 consecutive lanes (e = tid + i NT, NT % 4 == 0)
      amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
      amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
      const int ex = f8_block_exp(amax);
      const float inv = f8_inv_scale(ex);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= inv;
      const uint2 q8 = f8_pack8(f);
      if (e < HALO_PIECES) {
        const int hp = e >> 2, q = e & 3;
        *reinterpret_cast<uint2*>(sH + f8_off(hp, q >> 1) + (q & 1) * 8) = q8;
        if (q == 0) sHs[hp] = (uint8_t)(ex + 127);
      }
    }
  };
  // ---- weights: piece e -> row e / 2 (= tap * BN_ + n), 16-byte half e % 2; scale byte per row ----
  uint4 rw[W_PER_T];
  uint32_t rs[S_PER_T];
  auto load_w = [&](int ch) {
#pragma unroll
    for (int i = 0; i < W_PER_T; ++i) {
      const int e = tid + i * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (W_PIECES % NT == 0 || e < W_PIECES) {
        const int row = e >> 1, h = e & 1, tap = row / BN_, n = row - tap * BN_;
        v = *reinterpret_cast<const uint4*>(p.wt8 + (size_t)(nBlock + n) * p.K + (size_t)tap * p.Cin + ch * BK +
                                            h * 16);
      }
      rw[i] = v;
    }
#pragma unroll
    for (int i = 0; i < S_PER_T; ++i) {
      const int row = tid + i * NT;
      uint32_t v = 127;
      if (WROWS % NT == 0 || row < WROWS) {
        const int tap = row / BN_, n = row - tap * BN_;
        v = p.ws8[(size_t)(nBlock + n) * kblocks + tap * chunks + ch];
      }
      rs[i] = v;
    }
  };
  auto store_w = [&]() {
#pragma unroll
    for (int i = 0; i < W_PER_T; ++i) {
      const int e = tid + i * NT;
      if (W_PIECES % NT == 0 || e < W_PIECES) *reinterpret_cast<uint4*>(sW + f8_off(e >> 1, e & 1)) = rw[i];
    }
#pragma unroll
    for (int i = 0; i < S_PER_T; ++i) {
      const int row = tid + i * NT;
      if (WROWS % NT == 0 || row < WROWS) sWs[row] = (uint8_t)rs[i];
    }
  };

  // fragment rows: A = pixel (lane & 31) of fragment i, B = output channel (lane & 31) of fragment j; the lane's
  // k-half kh = lane >> 5 is tap 2 s + kh of k-step s
  const int prow = f8_perm(lane & 31);
  int fhp[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pp = wm * TM + i * 32 + prow;
    fhp[i] = (pp / TW) * HW + pp % TW;
  }
  const int kh = lane >> 5;
  const int bcol = wn * TN + prow;

  // decoder node join: this thread's half-resolution pixel (loads in flight during the K loop)
  uint4 pjv = make_uint4(0, 0, 0, 0), pja = pjv, pjy = pjv;
  size_t pjoff = 0;
  bool pjok = false;
  if constexpr (PJ) {
    constexpr int CGp = BN_ / 8, HTW = TW / 2, HB = BM / 4;
    static_assert(HB <= NT / CGp, "one half-resolution pixel per thread");
    const int hr = tid / CGp, hy = hr / HTW, hx = hr % HTW;
    const int oy = ty0 + 2 * hy, ox = tx0 + 2 * hx;
    pjok = hr < HB && oy < p.Ho && ox < p.Wo;
    pjoff = (((size_t)b * (p.Ho >> 1) + (oy >> 1)) * (p.Wo >> 1) + (ox >> 1)) * p.N + nBlock + (tid % CGp) * 8;
    if (pjok) {
      pjv = *reinterpret_cast<const uint4*>(p.pj.v + pjoff);
      if (p.pj.add) pja = *reinterpret_cast<const uint4*>(p.pj.add + pjoff);
      if (p.pj.sy) pjy = *reinterpret_cast<const uint4*>(p.pj.sy + pjoff);
    }
  }

  f16v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load_halo(0);
  load_w(0);
  if constexpr (XFIN) {            // consumer-side BN finalize while the first chunk's loads are in flight
    if (tid < p.Cin) {
      float a, bb, mean, rstd;
      bn_coef_from_stats(p.xfin, p.Cin, tid, a, bb, mean, rstd);
      sxab[tid] = a;
      sxab[256 + tid] = bb;
      if ((blockIdx.x | blockIdx.y | blockIdx.z) == 0) {
        float* ab = const_cast<float*>(p.xf.ab);
        ab[tid] = a;
        ab[p.Cin + tid] = bb;
        ab[2 * p.Cin + tid] = mean;
        ab[3 * p.Cin + tid] = rstd;
      }
    }
    __syncthreads();
  }
  load_coefs(0);
  store_halo();
  store_w();
  __syncthreads();
  for (int ch = 0; ch < chunks; ++ch) {
    const bool next = ch + 1 < chunks;
    if (next) {                                             // in flight during this chunk's MFMAs
      load_halo(ch + 1);
      load_w(ch + 1);
    }
#pragma unroll 1
    for (int s = 0; s < 5; ++s) {               // (not unrolled: all five steps' fragments in flight spill)
      const int t0 = 2 * s, t1 = t0 + 1;                  // K-block 0 / 1 of this step
      const bool live1 = t1 < 9;                          // the 10th tap slot: zero weights
      const int t1c = live1 ? t1 : t0;
      const int ky0 = (t0 * 11) >> 5, kx0 = t0 - 3 * ky0, ky1 = (t1c * 11) >> 5, kx1 = t1c - 3 * ky1;
      i8v af[FM], bw[FN];
      int sa[FM], sb[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int r0 = fhp[i] + ky0 * HW + kx0, r1 = fhp[i] + ky1 * HW + kx1;
        const uint4 lo = *reinterpret_cast<const uint4*>(sH + f8_off(r0, kh));
        const uint4 hi = *reinterpret_cast<const uint4*>(sH + f8_off(r1, kh));
        af[i] = i8v{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
        sa[i] = sHs[kh ? r1 : r0];
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = bcol + j * 32, w0 = t0 * BN_ + n, w1 = t1c * BN_ + n;
        const uint4 lo = *reinterpret_cast<const uint4*>(sW + f8_off(w0, kh));
        uint4 hi = *reinterpret_cast<const uint4*>(sW + f8_off(w1, kh));
        if (!live1) hi = make_uint4(0, 0, 0, 0);
        bw[j] = i8v{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
        sb[j] = sWs[kh ? w1 : w0];
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(af[i], bw[j], acc[i][j], 0, 0, 0, sa[i], 0,
                                                                     sb[j]);
    }
    __syncthreads();
    if (next) {
      load_coefs(ch + 1);
      store_halo();
      store_w();
      __syncthreads();
    }
  }

  // ---- epilogue (conv3x3.hip): C map of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  //      (fragment rows / cols in f8_perm order)
  auto out_m = [&](int row, int& m) -> bool {
    const int py = row / TW, px = row % TW;
    const int oy = ty0 + py, ox = tx0 + px;
    m = (b * p.Ho + oy) * p.Wo + ox;
    return oy < p.Ho && ox < p.Wo;
  };
  bf16_t (*sC)[LDC] = reinterpret_cast<bf16_t (*)[LDC]>(smem);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int cl = wn * TN + j * 32 + prow;
    const float bias = p.bias ? p.bias[nBlock + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sC[wm * TM + i * 32 + f8_perm((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5))][cl] = f2bf(acc[i][j][r] + bias);
  }
  __syncthreads();
  constexpr int CG = BN_ / 8, ROWS_PER_PASS = NT / CG;
  const int cg = tid % CG;
  const bool node = p.node.y != nullptr;
  NodeCoef nk;
  if (node) node_coef_load(p.node.ab, p.N, nBlock + cg * 8, nk);
  float s2[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s2[0][q] = s2[1][q] = 0.f;
  if constexpr (PJ) {
    float pm[8], pr[8];
    load_f8_or(p.pj.sab + 2 * p.N + nBlock + cg * 8, p.pj.sy != nullptr, 0.f, pm);
    load_f8_or(p.pj.sab + 3 * p.N + nBlock + cg * 8, p.pj.sy != nullptr, 0.f, pr);
    constexpr int HTW = TW / 2;
    if (pjok) {
      const int hr = tid / CG, hy = hr / HTW, hx = hr % HTW;
      uint4 o4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        o4[q] = *reinterpret_cast<const uint4*>(&sC[(2 * hy + (q >> 1)) * TW + 2 * hx + (q & 1)][cg * 8]);
      *reinterpret_cast<uint4*>(p.pj.out + pjoff) = pool_join8(o4, pjv, pja, pjy, p.pj.add != nullptr,
                                                               p.pj.sy != nullptr, pm, pr, s2[0], s2[1]);
    }
  } else {
#pragma unroll
    for (int r0 = 0; r0 < BM; r0 += ROWS_PER_PASS) {
      const int row = r0 + tid / CG;
      int m;
      if (out_m(row, m)) {
        const size_t off = (size_t)m * p.N + nBlock + cg * 8;
        uint4 v = *reinterpret_cast<const uint4*>(&sC[row][cg * 8]);
        if (node) {
          v = node_epi(v, p.node.y + off, nk, p.node.relu, s2[0], s2[1]);
        } else {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            s2[0][q] += f[q];
            s2[1][q] += f[q] * f[q];
          }
        }
        *reinterpret_cast<uint4*>(p.y + off) = v;
      }
    }
  }
  if (p.stats || node || (PJ && p.pj.sums)) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int o = CG; o < 64; o <<= 1) {
        s2[0][q] = xor_add(s2[0][q], o);
        s2[1][q] = xor_add(s2[1][q], o);
      }
    if (lane < CG) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        sred[0][wid][cg * 8 + q] = s2[0][q];
        sred[1][wid][cg * 8 + q] = s2[1][q];
      }
    }
    __syncthreads();
    float* rep = PJ ? p.pj.sums : node ? p.node.sums : p.stats;
    const int nrep = PJ ? (p.pj.reps > 1 ? p.pj.reps : 1) : node ? (p.node.reps > 1 ? p.node.reps : 1) : STAT_REPLICAS;
    const size_t ro = (size_t)(tile_id % nrep) * 2 * p.N;
    for (int e = tid; e < 2 * BN_; e += NT) {
      const int st = e / BN_, cc = e - st * BN_;
      red_add(rep, ro + st * p.N + nBlock + cc, sred[st][0][cc] + sred[st][1][cc] + sred[st][2][cc] + sred[st][3][cc],
              red_scale(!PJ && !node, st));
    }
  }
}

template <int TH, int TW, int BN_, int WM, int WN>
int launch_f8(const ConvParams& p, hipStream_t st) {
  const dim3 grid(((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * p.B, p.N / BN_, 1);
  if (p.xfin.stats)
    hipLaunchKernelGGL((conv3x3_f8_kernel<TH, TW, BN_, WM, WN, false, true>), grid, dim3(F8_NT), 0, st, p);
  else if (p.pj.v) {
    if constexpr (TH * TW / 4 <= F8_NT / (BN_ / 8))    // one half-resolution pixel per thread
      hipLaunchKernelGGL((conv3x3_f8_kernel<TH, TW, BN_, WM, WN, true, false>), grid, dim3(F8_NT), 0, st, p);
    else
      return 8;
  }
  else
    hipLaunchKernelGGL((conv3x3_f8_kernel<TH, TW, BN_, WM, WN, false, false>), grid, dim3(F8_NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

// fp8 3x3 conv: ConvParams with wt8 / ws8 (quant_w8 of the packed bf16 weights) - 3x3 / stride 1 / same, Cin and N
// multiples of 32, Cin <= 256, no BN-backward fold, no split-K (the whole K per block)
bool conv3x3_f8_supported(const ConvParams& p) {
  return p.wt8 && p.ws8 && p.ks == 3 && p.stride == 1 && p.pad_t == 1 && p.pad_l == 1 && p.Cin % F8_BK == 0 &&
         p.Cin <= 256 && p.N % 32 == 0 && p.K == 9 * p.Cin && !p.bwd.y && !(p.xfin.stats && p.pj.v) &&
         !(p.pj.v && (p.Ho % 2 || p.Wo % 2));
}

int conv3x3_f8(const ConvParams& p, hipStream_t st) {
  if (!conv3x3_f8_supported(p)) return 1;
  const bool bn64 = p.N % 64 == 0;
  // 16 x 16 pixel tiles from 1M output pixels (as the bf16 whole-chunk path's TUNE_CONV3_BIG), on a 4 x 1 wave grid
  // (64 px x 64 ch per wave: 4 instead of 5 fragment reads per 4 MFMAs), else 8 x 16 / 16 x 8
  if ((int64_t)p.B * p.Ho * p.Wo >= (1 << 20) && p.Ho % 16 == 0 && p.Wo % 16 == 0 && !p.pj.v)
    return bn64 ? launch_f8<16, 16, 64, 4, 1>(p, st) : launch_f8<16, 16, 32, 4, 1>(p, st);
  if (p.Wo >= 16) return bn64 ? launch_f8<8, 16, 64, 2, 2>(p, st) : launch_f8<8, 16, 32, 4, 1>(p, st);
  return bn64 ? launch_f8<16, 8, 64, 2, 2>(p, st) : launch_f8<16, 8, 32, 4, 1>(p, st);
}

// one launch over every view of the table: (src bf16 [N][K], dst e4m3 [N][K], scales e8m0 [N][K/32], N * K / 32)
int quant_w8(const bf16_t* const* src, uint8_t* const* dst, uint8_t* const* sc, const int* nblk, int n, hipStream_t st) {
  if (n < 1 || n > Q8_MAX) return 1;
  Q8Table t{};
  int tot = 0;
  for (int i = 0; i < n; ++i) {
    t.it[i] = Q8Item{src[i], dst[i], sc[i], nblk[i], tot};
    tot += nblk[i];
  }
  t.n = n;
  t.total = tot;
  const int blocks = (tot + 255) / 256 < 2048 ? (tot + 255) / 256 : 2048;
  hipLaunchKernelGGL(quant_w8_kernel, dim3(blocks), dim3(256), 0, st, t);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int mfma_scale_probe(const int* a, const int* b, const int* sa, const int* sb, float* d, int shape, hipStream_t st) {
  if (shape != 16 && shape != 32) return 1;
  hipLaunchKernelGGL(mfma_scale_probe_kernel, dim3(1), dim3(64), 0, st, a, b, sa, sb, d, shape);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_fp8(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_fp8(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
