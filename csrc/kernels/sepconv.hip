// Fused SeparableConv2D forward (/root/reference/client_fit_model.py:109,113): depthwise 3x3 (depth_multiplier 1,
// "same") of the producer's BN-apply + ReLU, then the pointwise 1x1 conv + bias, with the next BatchNorm's batch
// statistics - one pass instead of dw_stream_kernel (dwconv.hip) writing the depthwise output d and pw_kernel
// (pw.hip) reading it back.
//
// A block owns a TW-pixel column strip of one image and a segment of rows, and walks down it RS output rows per
// step (4 waves, TPW 16-pixel tiles each: RS rows of input in flight per step - with one tile per wave and 2-row
// steps the block held too few bytes in flight to cover HBM latency). The transformed input rows live in an LDS ring (row-streaming as in
// dwconv.hip: each input row fetched once per segment, the next step's rows in flight in registers during the
// current step's compute, one barrier per step). Per 16-pixel tile a lane (r16, q) forms the depthwise output of
// pixel r16, channels s*32 + 8q .. +7 of every 32-channel k-step s - exactly the B-fragment layout of pw.hip's
// swapped-operand MFMA (D = W * X^T) - from 9 shifted 16-byte LDS reads, rounds it to bf16 (the bits dw_fwd
// stores), side-stores it (the pointwise weight gradient reads d later) and feeds it straight to the MFMAs against
// the block-resident pointwise weights. The epilogue (bias, bf16, lane-pair swap for 64-byte stores, statistics
// held in registers, one atomic per channel per block) is pw.hip's.
// Arithmetic = dw_fwd then pw_conv: the depthwise fmaf chain runs over the taps in the same order from the same bf16
// transformed inputs, and the MFMA k-steps in the same order, so d and y are bit-identical to the two-pass form
// (tests/test_gpu_kernels.py); only the statistics' float-atomic order differs.
// Consumer-side BN finalize (p.xfin, the dw layer's input BN): the block turns the producer's replica sums into its
// channels' (a, b) (the first block also writes the ab rows), while its first rows are in flight.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

CFL_DEVICE int wswz(int n, int q) { return n * 32 + ((q ^ ((n >> 1) & 3)) << 3); }   // pw.hip's weight swizzle

template <int K, int N, int TW>
struct Sep {
  static constexpr int WT = TW / 16;                  // wave tiles per row
  static constexpr int TPW = N <= 64 ? 2 : 1;         // tiles per wave per step (N = 128: registers)
  static constexpr int RS = 4 * TPW / WT;             // output rows per step
  static constexpr int NRING = 2 * RS + 2;            // rows read by a step + rows prefetched for the next
  static constexpr int HWp = TW + 2;                  // halo pixels per row
  static constexpr int CQ = K / 8;                    // 16-byte channel pieces per pixel
  static constexpr int PIECES = HWp * CQ;             // per row
  static constexpr int KS = K / 32, NF = N / 16;
  static constexpr int RING = NRING * HWp * K;        // bf16 elements
  static_assert(NT % CQ == 0, "a thread's pieces share one channel group");
};

// Rows [row0, row0 + R) of strip (b, x0) into registers: raw bf16, zeros outside the image
template <int K, int N, int TW, int R>
CFL_DEVICE void sep_fetch(const SepParams& p, const bf16_t* img, int x0, int row0, bool on,
                          uint4 (&v)[(R * Sep<K, N, TW>::PIECES + NT - 1) / NT], uint32_t& okm) {
  using S = Sep<K, N, TW>;
  constexpr int PPT = (R * S::PIECES + NT - 1) / NT;
  const int tid = threadIdx.x, cq = tid % S::CQ;
  okm = 0;
  // buffer loads from the image's resource, padding / rows past the segment at the out-of-range offset (read as 0):
  // no per-lane branch around a load, no 64-bit address math
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(img, (uint32_t)p.H * p.W * K * 2u);
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int e = tid + i * NT;
    const int r = e / S::PIECES, px = (e - r * S::PIECES) / S::CQ;
    const int iy = row0 + r, ix = x0 - 1 + px;
    const bool ok = on && e < R * S::PIECES && (unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W;
    v[i] = buf_load16(rs, ok ? ((uint32_t)iy * p.W + ix) * (K * 2u) + cq * 16u : CFL_OOB, 0);
    okm |= (uint32_t)ok << i;
  }
}

// Ring layout: [row slot][32-channel plane][pixel][32 channels], 64 B per pixel per plane with conv3x3.hip's XOR
// swizzle of the four 16-byte quarters (quarter q of pixel r at q ^ ((r >> 1) & 2)): a B-fragment read - 16
// consecutive pixels x 4 quarters, any start pixel - then covers all 64 banks (a padded [pixel][K] row left 2-way
// conflicts in the ds_read_b128 lane groups).
CFL_DEVICE int sep_off(int slot_plane, int hwp, int px, int q) {
  return (slot_plane * hwp + px) * 32 + ((q ^ ((px >> 1) & 2)) << 3);
}

// ... and into their ring slots, with the producer transform (padding stays zero: TF SAME pads the conv input)
template <int K, int N, int TW, int R>
CFL_DEVICE void sep_put(bf16_t* ring, const uint4 (&v)[(R * Sep<K, N, TW>::PIECES + NT - 1) / NT], uint32_t okm,
                        int row0, bool xform, const float* a8, const float* b8, int relu) {
  using S = Sep<K, N, TW>;
  constexpr int PPT = (R * S::PIECES + NT - 1) / NT;
  const int tid = threadIdx.x, cq = tid % S::CQ;
#pragma unroll
  for (int i = 0; i < PPT; ++i) {
    const int e = tid + i * NT;
    if (e >= R * S::PIECES) continue;
    const int r = e / S::PIECES, px = (e - r * S::PIECES) / S::CQ;
    uint4 t = v[i];
    if (xform) t = xform8(t, a8, b8, relu ? 0u : 0x80008000u, ((okm >> i) & 1u) ? 0xffffffffu : 0u);   // common.h
    const int slot = (row0 + r + S::NRING) % S::NRING;      // row0 >= -1
    *reinterpret_cast<uint4*>(ring + sep_off(slot * S::KS + (cq >> 2), S::HWp, px, cq & 3)) = t;
  }
}

template <int K, int N, int TW, bool XFIN>
__global__ __launch_bounds__(NT, 2) void sep_fwd_kernel(const SepParams p, int seg_rows) {
  CFL_TS_GUARD;
  using S = Sep<K, N, TW>;
  constexpr int KS = S::KS, NF = S::NF, RS = S::RS;
  constexpr int P0 = (RS + 2) * S::PIECES, PPT0 = (P0 + NT - 1) / NT;
  constexpr int PPT = (RS * S::PIECES + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) bf16_t ring[S::RING];
  __shared__ __attribute__((aligned(16))) bf16_t sW[KS * N * 32];      // pointwise weights [N][K], swizzled
  __shared__ __attribute__((aligned(16))) float sWd[9 * K];            // depthwise taps [tap][K]
  __shared__ __attribute__((aligned(16))) float sBias[N];
  __shared__ float sAB[XFIN ? 2 * K : 1];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int tiles_w = p.W / TW, nseg = (p.H + seg_rows - 1) / seg_rows;
  int lin = xcd_swizzle(blockIdx.x, gridDim.x);
  const int tw = lin % tiles_w;
  lin /= tiles_w;
  const int sg = lin % nseg, b = lin / nseg;
  const int x0 = tw * TW, ybeg = sg * seg_rows, yend = imin(p.H, ybeg + seg_rows);
  const int nsteps = (yend - ybeg + RS - 1) / RS;
  const bf16_t* img = p.x + (size_t)b * p.H * p.W * K;

  uint4 v0[PPT0];
  uint32_t ok0;
  sep_fetch<K, N, TW, RS + 2>(p, img, x0, ybeg - 1, true, v0, ok0);
  // the block's weights, depthwise taps and bias issued with the first rows: the prologue waits one round trip
  // (a strided weight-copy loop after the ring fill waited one per iteration: 4-5 us per block before the loop)
  Stage16<NT, N * K / 8> wst;
  wst.load([&](int c) { const int n = c / (K / 8), kc = c - n * (K / 8); return p.wpw + (size_t)n * K + kc * 8; });
  const float bias_v = p.bias ? p.bias[imin(tid, N - 1)] : 0.f;
  constexpr int WDT = (9 * K + NT - 1) / NT;
  float wd[WDT];
#pragma unroll
  for (int i = 0; i < WDT; ++i) wd[i] = p.wdw[imin(tid + i * NT, 9 * K - 1)];

  // this thread's channel group (fixed: NT % CQ == 0) and its transform coefficients
  const int cq = tid % S::CQ;
  const bool has_ab = p.xf.ab != nullptr || XFIN;
  float a8[8], b8[8];
  if constexpr (XFIN) {
    if (tid < K) {
      float a, bb, mean, rstd;
      bn_coef_from_stats(p.xfin, K, tid, a, bb, mean, rstd);
      sAB[tid] = a;
      sAB[K + tid] = bb;
      if (blockIdx.x == 0) {                              // the layer's later consumers read the ab rows
        float* ab = const_cast<float*>(p.xf.ab);
        ab[tid] = a;
        ab[K + tid] = bb;
        ab[2 * K + tid] = mean;
        ab[3 * K + tid] = rstd;
      }
    }
    __syncthreads();
    load_f8(&sAB[cq * 8], a8);
    load_f8(&sAB[K + cq * 8], b8);
  } else {
    load_f8_or(p.xf.ab + cq * 8, has_ab, 1.f, a8);
    load_f8_or(p.xf.ab + K + cq * 8, has_ab, 0.f, b8);
  }
  const int relu = p.xf.relu;
  sep_put<K, N, TW, RS + 2>(ring, v0, ok0, ybeg - 1, has_ab || relu, a8, b8, relu);
  wst.store([&](int c) { const int n = c / (K / 8), kc = c - n * (K / 8); return sW + (kc >> 2) * N * 32 + wswz(n, kc & 3); });
#pragma unroll
  for (int i = 0; i < WDT; ++i)
    if (tid + i * NT < 9 * K) sWd[tid + i * NT] = wd[i];
  if (tid < N) sBias[tid] = bias_v;
  __syncthreads();

  const bool stats = p.stats != nullptr;
  float s1[NF][4], s2[NF][4];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[nf][r] = s2[nf][r] = 0.f;

  const int px0 = (wid % S::WT) * 16;                        // this wave's tile column
  uint4 vn[PPT];
  uint32_t okn = 0;
  cfl_ts_phase(0);
  for (int s = 0; s < nsteps; ++s) {
    const int a = ybeg + s * RS;
    const bool more = s + 1 < nsteps;
    sep_fetch<K, N, TW, RS>(p, img, x0, a + RS + 1, more, vn, okn);
#pragma unroll 1
    for (int ti = 0; ti < S::TPW; ++ti) {
    const int oy = a + (wid + 4 * ti) / S::WT;                 // tile wid + 4 ti of the step's RS x WT tiles
    if (oy < yend) {
      const int ox = x0 + px0 + r16;
      const size_t m = ((size_t)b * p.H + oy) * p.W + ox;
      // opaque zero: keeps the loop-invariant LDS weight reads inside the loop (hoisted they would stay live)
      int wo = 0;
      asm volatile("" : "+v"(wo));
      s8v d[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int c0 = ks * 32 + q * 8;
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
          const int slot = (oy - 1 + ky + S::NRING) % S::NRING;
          const int sp = slot * KS + ks;
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            float f[8], w[8];
            unpack8(*reinterpret_cast<const uint4*>(ring + sep_off(sp, S::HWp, px0 + r16 + kx, q)), f);
            load_f8(&sWd[(ky * 3 + kx) * K + c0 + wo], w);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = fmaf(f[j], w[j], acc[j]);
          }
          __builtin_amdgcn_sched_barrier(0);   // one input row's reads in flight at a time (register pressure)
        }
        const uint4 dv = pack8(acc);
        *reinterpret_cast<uint4*>(p.d + m * K + c0) = dv;           // the pointwise weight gradient's input
        d[ks] = *reinterpret_cast<const s8v*>(&dv);
      }
      f4v acc[NF];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf) acc[nf] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const s8v w = *reinterpret_cast<const s8v*>(sW + wo + ks * N * 32 + wswz(nf * 16 + r16, q));
          acc[nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, d[ks], acc[nf], 0, 0, 0);
        }
      // lane (r16, q) holds channels nf*16 + 4q .. +3 of pixel r16: pair fragments 2h, 2h+1 (pw.hip epilogue)
      const bool odd = q & 1;
#pragma unroll
      for (int h = 0; h < NF / 2; ++h) {
        const float4 b0 = *reinterpret_cast<const float4*>(&sBias[(2 * h) * 16 + q * 4]);
        const float4 b1 = *reinterpret_cast<const float4*>(&sBias[(2 * h + 1) * 16 + q * 4]);
        const f4v c0 = acc[2 * h], c1 = acc[2 * h + 1];
        const uint2 u0 = make_uint2(pack2bf(c0[0] + b0.x, c0[1] + b0.y), pack2bf(c0[2] + b0.z, c0[3] + b0.w));
        const uint2 u1 = make_uint2(pack2bf(c1[0] + b1.x, c1[1] + b1.y), pack2bf(c1[2] + b1.z, c1[3] + b1.w));
        const uint2 give = odd ? u0 : u1;
        const uint2 got = make_uint2(xor16_get(give.x), xor16_get(give.y));
        const uint4 v = odd ? make_uint4(got.x, got.y, u1.x, u1.y) : make_uint4(u0.x, u0.y, got.x, got.y);
        *reinterpret_cast<uint4*>(p.y + m * N + (2 * h + odd) * 16 + (q >> 1) * 8) = v;
        if (stats) {
          const uint32_t w[4] = {u0.x, u0.y, u1.x, u1.y};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = __uint_as_float(w[e] << 16), hi = __uint_as_float(w[e] & 0xffff0000u);
            const int nf = 2 * h + (e >> 1), r = (e & 1) * 2;
            s1[nf][r] += lo;
            s2[nf][r] = fmaf(lo, lo, s2[nf][r]);
            s1[nf][r + 1] += hi;
            s2[nf][r + 1] = fmaf(hi, hi, s2[nf][r + 1]);
          }
        }
      }
    }
    }
    if (more) sep_put<K, N, TW, RS>(ring, vn, okn, a + RS + 1, has_ab || relu, a8, b8, relu);
    __syncthreads();
  }

  cfl_ts_phase(1);
  if (!stats) return;
  float (*sred)[NT / 64][N] = reinterpret_cast<float (*)[NT / 64][N]>(ring);   // the loop ended on a barrier
  static_assert(2 * (NT / 64) * N * 4 <= S::RING * 2, "statistics staging fits the ring");
#pragma unroll
  for (int nf = 0; nf < NF; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[nf][r] = xor_add(s1[nf][r], o);
        s2[nf][r] = xor_add(s2[nf][r], o);
      }
  if (r16 == 0) {
#pragma unroll
    for (int nf = 0; nf < NF; ++nf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sred[0][wid][nf * 16 + q * 4 + r] = s1[nf][r];
        sred[1][wid][nf * 16 + q * 4 + r] = s2[nf][r];
      }
  }
  __syncthreads();
  const size_t ro = (size_t)(blockIdx.x % STAT_REPLICAS) * 2 * N;
  for (int e = tid; e < 2 * N; e += NT) {
    const int st = e / N, cc = e - st * N;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) v += sred[st][w][cc];
    red_add(p.stats, ro + st * N + cc, v, red_scale(true, st));
  }
}

template <int K, int N, int TW>
int launch(const SepParams& p, hipStream_t st) {
  using S = Sep<K, N, TW>;
  const int steps = (p.H + S::RS - 1) / S::RS;
  const int strips = p.B * (p.W / TW);
  // one round of resident blocks: 3 per CU at K = 32 (155 VGPRs, 27 KB LDS), else 2 (LDS / VGPRs)
  int target = cfl_tune(TUNE_SEP_BLOCKS) > 0 ? cfl_tune(TUNE_SEP_BLOCKS) : (K == 32 ? 768 : 512);
  int nseg = (target + strips - 1) / strips;
  nseg = nseg < 1 ? 1 : (nseg > steps ? steps : nseg);
  const int seg_rows = ((steps + nseg - 1) / nseg) * S::RS;
  nseg = (p.H + seg_rows - 1) / seg_rows;
  const int blocks = strips * nseg;
  if (p.xfin.stats) hipLaunchKernelGGL((sep_fwd_kernel<K, N, TW, true>), dim3(blocks), dim3(NT), 0, st, p, seg_rows);
  else hipLaunchKernelGGL((sep_fwd_kernel<K, N, TW, false>), dim3(blocks), dim3(NT), 0, st, p, seg_rows);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

bool sep_fwd_supported(const SepParams& p) {
  if (cfl_tune(TUNE_SEP) == 1 || p.W % 32 || p.H < 1 || p.B < 1) return false;
  if ((int64_t)p.H * p.W * p.K * 2 >= (1ll << 31)) return false;   // one image per buffer resource (sep_fetch)
  return (p.K == 32 && p.N == 64) || (p.K == 64 && (p.N == 64 || p.N == 128));
}

int sep_fwd(const SepParams& p, hipStream_t st) {
  if (!sep_fwd_supported(p)) return 1;
  if (p.xfin.stats && p.xf.ab == nullptr) return 2;          // the finalize writes the ab rows
  if (p.K == 32) return launch<32, 64, 32>(p, st);
  if (p.N == 64) return launch<64, 64, 32>(p, st);
  return launch<64, 128, 32>(p, st);
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_sepconv(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_sepconv(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
