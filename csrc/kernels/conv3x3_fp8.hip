// fp8 (e4m3) forward 3x3 / stride-1 convolution for the decoder Conv2DTranspose layers (BASELINE config 5:
// "fp8 Conv2D MFMA path"; /root/reference/client_fit_model.py:129,133 are the layers). gfx950 MFMA
// v_mfma_f32_16x16x32_fp8_fp8: same fragment geometry as the bf16 16x16x32 op with 8-byte operands, so the LDS
// halo and weight tiles are half the bytes of conv3x3.hip's.
//
// Scaling (fp32 accumulate, fp32 dequantisation in the epilogue):
//   * weights: per OUTPUT channel, scale_w[n] = amax(W[n, :]) / FP8_MAX, quantised once per optimizer step by
//     pack_fp8 (below) from the fp32 master weights;
//   * activations: per tensor, DELAYED scaling - the halo loader quantises with amax[0], the amax recorded for this
//     conv's input by the previous step(s), and records this step's amax into amax[1] with one atomicMax per block
//     (non-negative floats order like their bit patterns); pack_fp8, which runs once per optimizer step after every
//     forward conv, folds amax[1] into amax[0]. Values beyond the delayed range saturate at +-FP8_MAX. The engine
//     seeds amax with a calibration forward before the first step.
//   out = acc * scale_a * scale_w[n] + bias  -> bf16, BN batch statistics as in conv3x3.hip.
// Structure: whole-chunk weight staging (all 9 taps of a 32-channel chunk), halo per chunk with BN-apply + ReLU +
// nearest-2x upsample folded into the load, next chunk register-prefetched, two barriers per chunk.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr int BK = 32;             // channels per chunk (K-step of one tap)
constexpr int LDH8 = BK + 16;      // halo pixel pitch in BYTES (16 lanes x 48 B spread over distinct banks)
constexpr int LDB8 = BK + 16;
constexpr float FP8_MAX = 240.f;   // stays inside the e4m3 range of both the OCP and the FNUZ encodings

CFL_DEVICE uint32_t q4(float a, float b, float c, float d) {
  int w = 0;
  w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, w, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

CFL_DEVICE float clampq(float v) { return fminf(fmaxf(v, -FP8_MAX), FP8_MAX); }

template <int TH, int TW, int BN_, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void conv3x3_fp8_kernel(Conv8Params p, int chunks_per_split) {
  const ConvParams& c = p.c;
  constexpr int BM = TH * TW;
  constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;
  constexpr int TM = BM / WM, TN = BN_ / WN, FM = TM / 16, FN = TN / 16;
  constexpr int HALO_CHUNKS = HP * (BK / 8);                   // 8-channel pieces per halo tile
  constexpr int H_PER_T = (HALO_CHUNKS + NT - 1) / NT;
  constexpr int B_PIECES = 9 * BN_ * (BK / 16);                // 16-byte fp8 pieces of a chunk's 9 weight tiles
  constexpr int B_PER_T = (B_PIECES + NT - 1) / NT;
  constexpr int SH = HP * LDH8, SB = 9 * BN_ * LDB8;
  constexpr int LDC = BN_ + 8;
  __shared__ __attribute__((aligned(16))) uint8_t smem[SH + SB > BM * LDC * 2 ? SH + SB : BM * LDC * 2];
  __shared__ float sred[2][4][BN_];
  __shared__ float samax[4];
  uint8_t* sH = smem;
  uint8_t* sB = smem + SH;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_w = (c.Wo + TW - 1) / TW, tiles_h = (c.Ho + TH - 1) / TH;
  const int lin = xcd_block_linear();
  const int bn_idx = lin % gridDim.y, rest = lin / gridDim.y;
  const int bz = rest % gridDim.z;
  int t = rest / gridDim.z;
  const int tile_id = t;
  const int b = t / (tiles_w * tiles_h);
  t -= b * tiles_w * tiles_h;
  const int ty0 = (t / tiles_w) * TH, tx0 = (t % tiles_w) * TW;
  const int nBlock = bn_idx * BN_;
  const int chunks = c.Cin / BK;
  const int ch0 = bz * chunks_per_split;
  const int ch1 = imin(chunks, ch0 + chunks_per_split);
  const int Hl = c.Hin << c.up_in, Wl = c.Win << c.up_in;
  const bool has_ab = c.xf.ab != nullptr;
  const int relu = c.xf.relu;
  const float amax_prev = fmaxf(p.amax[0], 1e-12f);
  const float inv_sa = FP8_MAX / amax_prev, sa = amax_prev / FP8_MAX;
  float lmax = 0.f;

  // ---- halo: transformed values quantised to fp8 on the way to LDS ----
  uint2 rh[H_PER_T];
  auto load_halo = [&](int chunk) {
    const int cbase = chunk * BK;
    float a8[8], b8[8];
    load_f8_or(c.xf.ab + cbase + (tid & 3) * 8, has_ab, 1.f, a8);
    load_f8_or(c.xf.ab + c.xf.C + cbase + (tid & 3) * 8, has_ab, 0.f, b8);
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      const int hp = e >> 2, q = e & 3;
      const int hy = hp / HW, hx = hp - hy * HW;
      const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
      const bool valid = e < HALO_CHUNKS && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl;   // else: zero padding
      uint4 v = make_uint4(0, 0, 0, 0);
      if (valid)
        v = *reinterpret_cast<const uint4*>(
            c.x + (((size_t)b * c.Hin + (iy >> c.up_in)) * c.Win + (ix >> c.up_in)) * c.Cin + cbase + q * 8);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = fmaf(a8[j], f[j], b8[j]);
        if (relu) t = fmaxf(t, 0.f);
        t = valid ? t : 0.f;
        lmax = fmaxf(lmax, fabsf(t));
        f[j] = clampq(t * inv_sa);
      }
      rh[i] = make_uint2(q4(f[0], f[1], f[2], f[3]), q4(f[4], f[5], f[6], f[7]));
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < HALO_CHUNKS) *reinterpret_cast<uint2*>(sH + (e >> 2) * LDH8 + (e & 3) * 8) = rh[i];
    }
  };
  // ---- fp8 weights [N][K] (K = tap*Cin + c): piece e -> tap, row n, 16-byte half ----
  uint4 rb[B_PER_T];
  auto load_b = [&](int chunk) {
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int e = tid + i * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (B_PIECES % NT == 0 || e < B_PIECES) {
        const int tap = e / (BN_ * 2), w = e - tap * BN_ * 2;
        v = *reinterpret_cast<const uint4*>(p.wt8 + (size_t)(nBlock + (w >> 1)) * c.K + (size_t)tap * c.Cin +
                                            chunk * BK + (w & 1) * 16);
      }
      rb[i] = v;
    }
  };
  auto store_b = [&]() {
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int e = tid + i * NT;
      if (B_PIECES % NT == 0 || e < B_PIECES) {
        const int tap = e / (BN_ * 2), w = e - tap * BN_ * 2;
        *reinterpret_cast<uint4*>(sB + ((size_t)tap * BN_ + (w >> 1)) * LDB8 + (w & 1) * 16) = rb[i];
      }
    }
  };

  int fpy[FM], fpx[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pp = wm * TM + i * 16 + (lane & 15);
    fpy[i] = pp / TW;
    fpx[i] = pp % TW;
  }
  const int fk = (lane >> 4) * 8;      // byte offset of this lane's 8 k-values

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  if (ch0 < ch1) {
    load_halo(ch0);
    load_b(ch0);
    store_halo();
    store_b();
  }
  __syncthreads();
  for (int ch = ch0; ch < ch1; ++ch) {
    const bool next_chunk = ch + 1 < ch1;
    if (next_chunk) {
      load_halo(ch + 1);
      load_b(ch + 1);
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - ky * 3;
      long af[FM], bfg[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const long*>(sH + ((fpy[i] + ky) * HW + fpx[i] + kx) * LDH8 + fk);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfg[j] = *reinterpret_cast<const long*>(sB + ((size_t)tap * BN_ + wn * TN + j * 16 + (lane & 15)) * LDB8 + fk);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
    if (next_chunk) {
      store_halo();
      store_b();
      __syncthreads();
    }
  }

  // ---- this step's input amax -> the other parity slot (read by the next step) ----
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lmax = fmaxf(lmax, __shfl_xor(lmax, o, 64));
  if (lane == 0) samax[wid] = lmax;

  auto out_m = [&](int row, int& m) -> bool {
    const int py = row / TW, px = row % TW;
    const int oy = ty0 + py, ox = tx0 + px;
    m = (b * c.Ho + oy) * c.Wo + ox;
    return oy < c.Ho && ox < c.Wo;
  };

  // dequantise: activation scale x per-output-channel weight scale
  float swj[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) swj[j] = sa * p.wscale[nBlock + wn * TN + j * 16 + (lane & 15)];

  if (c.ws != nullptr && gridDim.z > 1) {            // split-K partials (fp32, dequantised)
    float* dst = c.ws + (size_t)bz * c.M * c.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = nBlock + wn * TN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int m;
          if (out_m(wm * TM + i * 16 + (lane >> 4) * 4 + r, m)) dst[(size_t)m * c.N + n] = acc[i][j][r] * swj[j];
        }
      }
    __syncthreads();
    if (tid == 0) {
      const float bm = fmaxf(fmaxf(samax[0], samax[1]), fmaxf(samax[2], samax[3]));
      atomicMax(reinterpret_cast<unsigned int*>(&p.amax[1]), __float_as_uint(bm));
    }
    return;
  }

  bf16_t (*sC)[LDC] = reinterpret_cast<bf16_t (*)[LDC]>(smem);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int cl = wn * TN + j * 16 + (lane & 15);
    const float bias = c.bias ? c.bias[nBlock + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sC[wm * TM + i * 16 + (lane >> 4) * 4 + r][cl] = f2bf(acc[i][j][r] * swj[j] + bias);
  }
  __syncthreads();
  if (tid == 0) {
    const float bm = fmaxf(fmaxf(samax[0], samax[1]), fmaxf(samax[2], samax[3]));
    atomicMax(reinterpret_cast<unsigned int*>(&p.amax[1]), __float_as_uint(bm));
  }
  constexpr int CG = BN_ / 8, ROWS_PER_PASS = NT / CG;
  const int cg = tid % CG;
  float s[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[0][q] = s[1][q] = 0.f;
#pragma unroll
  for (int r0 = 0; r0 < BM; r0 += ROWS_PER_PASS) {
    const int row = r0 + tid / CG;
    int m;
    if (out_m(row, m)) {
      const uint4 v = *reinterpret_cast<const uint4*>(&sC[row][cg * 8]);
      *reinterpret_cast<uint4*>(c.y + (size_t)m * c.N + nBlock + cg * 8) = v;
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        s[0][q] += f[q];
        s[1][q] += f[q] * f[q];
      }
    }
  }
  if (c.stats) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      for (int o = CG; o < 64; o <<= 1) {
        s[0][q] += __shfl_xor(s[0][q], o, 64);
        s[1][q] += __shfl_xor(s[1][q], o, 64);
      }
    if (lane < CG) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        sred[0][wid][cg * 8 + q] = s[0][q];
        sred[1][wid][cg * 8 + q] = s[1][q];
      }
    }
    __syncthreads();
    float* rep = c.stats + (size_t)(tile_id % STAT_REPLICAS) * 2 * c.N;
    for (int e = tid; e < 2 * BN_; e += NT) {
      const int st = e / BN_, cc = e - st * BN_;
      atomicAdd(&rep[st * c.N + nBlock + cc], sred[st][0][cc] + sred[st][1][cc] + sred[st][2][cc] + sred[st][3][cc]);
    }
  }
}

// per-output-row amax -> scale, quantise: one block per (row n, view)
__global__ __launch_bounds__(NT) void pack_fp8_kernel(const float* flat, uint8_t* packed8, float* scales,
                                                     const PackView* views, float* amax, int n_amax) {
  __shared__ float red[NT / 64];
  if (amax != nullptr && blockIdx.x == 0 && blockIdx.y == 0) {
    // delayed activation scaling: this step's recorded amax becomes the next step's scale
    for (int i = threadIdx.x; i < n_amax; i += NT) {
      if (amax[2 * i + 1] > 0.f) amax[2 * i] = amax[2 * i + 1];
      amax[2 * i + 1] = 0.f;
    }
  }
  const PackView v = views[blockIdx.y];
  const int n = blockIdx.x;
  if (n >= v.cout) return;                                   // PK_CONVT: N = cout, K = 9 * cin
  const int K = 9 * v.cin;
  const float* src = flat + v.src;
  auto at = [&](int k) {                                     // (3,3,out,in) flipped, as pack_kernel's PK_CONVT
    const int tap = k / v.cin, cc = k - tap * v.cin;
    return src[((8 - tap) * v.cout + n) * v.cin + cc];
  };
  float m = 0.f;
  for (int k = threadIdx.x; k < K; k += NT) m = fmaxf(m, fabsf(at(k)));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  const float wmax = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float sc = wmax > 0.f ? wmax / FP8_MAX : 1.f, inv = 1.f / sc;
  if (threadIdx.x == 0) scales[v.dst_scale + n] = sc;
  uint8_t* dst = packed8 + v.dst + (size_t)n * K;
  for (int k4 = threadIdx.x * 4; k4 < K; k4 += NT * 4) {
    *reinterpret_cast<uint32_t*>(dst + k4) =
        q4(clampq(at(k4) * inv), clampq(at(k4 + 1) * inv), clampq(at(k4 + 2) * inv), clampq(at(k4 + 3) * inv));
  }
}

template <int TH, int TW, int BN_, int WM, int WN>
int launch(const Conv8Params& p, int splits, hipStream_t st) {
  const ConvParams& c = p.c;
  const int chunks = c.Cin / BK;
  const int per = (chunks + splits - 1) / splits;
  splits = (chunks + per - 1) / per;
  const int tiles = ((c.Ho + TH - 1) / TH) * ((c.Wo + TW - 1) / TW) * c.B;
  dim3 grid(tiles, c.N / BN_, splits);
  hipLaunchKernelGGL((conv3x3_fp8_kernel<TH, TW, BN_, WM, WN>), grid, dim3(NT), 0, st, p, per);
  return splits;
}

}  // namespace

bool conv3x3_fp8_supported(const ConvParams& c) {
  return c.ks == 3 && c.stride == 1 && c.pad_t == 1 && c.pad_l == 1 && c.Cin % BK == 0 && c.N % 32 == 0 &&
         c.Ho >= 8 && c.Wo >= 8 && c.K == 9 * c.Cin;
}

int conv3x3_fp8(const Conv8Params& p, hipStream_t st) {
  const ConvParams& c = p.c;
  if (!conv3x3_fp8_supported(c) || !p.wt8 || !p.wscale || !p.amax) return 1;
  int splits = conv3x3_split_k(c);
  if (splits > 1 && (c.ws == nullptr || c.ws_elems < (int64_t)splits * c.M * c.N)) splits = 1;
  Conv8Params q = p;
  if (splits == 1) q.c.ws = nullptr;
  const bool w16 = c.Wo >= 16;
  if (c.N % 64 == 0) splits = w16 ? launch<8, 16, 64, 2, 2>(q, splits, st) : launch<16, 8, 64, 2, 2>(q, splits, st);
  else splits = w16 ? launch<8, 16, 32, 4, 1>(q, splits, st) : launch<16, 8, 32, 4, 1>(q, splits, st);
  if (hipGetLastError() != hipSuccess) return 3;
  return splits > 1 ? -splits : 0;    // negative: caller runs the split-K epilogue (conv_igemm.hip) on c.ws
}

int pack_fp8(const float* flat, uint8_t* packed8, float* scales, const PackView* d_views, int n_views, int max_rows,
             hipStream_t st, float* amax, int n_amax) {
  if (n_views <= 0) return 0;
  hipLaunchKernelGGL(pack_fp8_kernel, dim3(max_rows, n_views), dim3(NT), 0, st, flat, packed8, scales, d_views, amax,
                     n_amax);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
