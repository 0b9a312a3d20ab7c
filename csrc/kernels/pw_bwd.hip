// Fused backward of a SeparableConv's pointwise (1x1) conv with its output BatchNorm's backward folded in - the
// encoder's pw dgrad AND pw wgrad in ONE streaming pass (/root/reference/client_fit_model.py:109,113).
//
// Per pixel m the incoming gradient g = dL/d BN(y) and the BN input y give the pointwise output gradient
//   dy[m] = bnb_apply(g[m], y[m])                               (common.h, the bn_bwd_apply arithmetic)
// from which the layer needs
//   dgrad  dd[m][c] = sum_f dy[m][f] * W[c][f]                 (the depthwise conv's incoming gradient)
//   wgrad  dW[c][f] = sum_m d[m][c] * dy[m][f]                 (d = the pointwise input, the depthwise output)
// Until round 5 they were two passes: pw.hip's BWD form formed dy on load, wrote dd AND a side copy of dy, and the
// mixed weight-gradient launch read d and dy back (at 128^2 / 64 channels: 67 MB of the dy write + read per layer,
// and the mixed launch's largest streaming item, tools/mix_timeline.py). Here a block streams 64-pixel tiles:
//   * g, y (K = pw output channels) and d (N = pw input channels) of the tile are loaded into registers one tile
//     ahead; dy is formed on the way into LDS (bf16) and d is staged beside it;
//   * dgrad: wave w owns a pair of 16-channel output fragments for the whole launch, their weights held in
//     registers (loaded once from HBM), against NF / 2 of the tile's 16-pixel fragments - pw.hip's swapped-operand
//     MFMA (D = W * dy^T), all the wave's pixel fragments per k-step (NF independent accumulator chains: one
//     fragment at a time left the MFMA pipe waiting on its own results). Only dy is read from LDS;
//   * a thread's channel group is the same for every piece it loads (tid % (K / 8)): its BN-backward apply is two
//     packed FMAs per channel pair from three per-channel coefficients held in registers for the launch,
//       dy = A g + (Bc y + Cc),  A = a,  Bc = -a k2 rstd,  Cc = a (k2 rstd mean - k1)
//     (bnb_apply's a (g - k1 - (y - mean) rstd k2) regrouped: the same value to fp32 rounding, a third of the VALU
//     work - the apply was the largest phase of a tile; dd therefore matches pw.hip's to bf16 rounding, not bit
//     for bit);
//   * wgrad: the tile's 64 pixels are the MFMA reduction, read with the transposing ds_read_b64_tr_b16 from the two
//     staged tiles (conv_wgrad.hip's operand scheme); each wave owns a fixed part of dW in registers for the whole
//     launch, added once per block into a replica row (WGRAD_REPLICAS rows, summed by grad_finish);
//   * block 0 writes dgamma / dbeta (bnb_prologue), as pw.hip's BWD form does.
// HBM bytes per layer: g + y + d read, dd written (pw.hip's dgrad alone moved the same with dy instead of d).
// Shapes: the encoder's 128^2 level (K = 64 output channels, N = 32 or 64 input channels; pw_bwd_supported).
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr int TP = 64;                 // pixels per tile

typedef short s4v_lds __attribute__((ext_vector_type(4)));
CFL_DEVICE s4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4v_lds __attribute__((address_space(3)))*)(p));
}

template <int K, int N>
struct Pwb {
  static constexpr int KS = K / 32, KF = K / 16, NF = N / 16;
  // tile rows of 32 x odd bytes: a transposing read's 8 consecutive pixel rows x 32 bytes cover all 64 banks
  static constexpr int LDY = K + 16, LDX = N + 16;
  static constexpr int GPT = TP * K / 8 / NT, XPT = TP * N / 8 / NT;        // 16-byte pieces per thread per tile
  // the wave's share of dW [N (c) x K (f)] fragments: NF >= 4 -> NF / 4 c-fragments x all f; NF = 2 -> one c-fragment
  // x half the f-fragments
  static constexpr int CW = NF >= 4 ? NF / 4 : 1;
  static constexpr int FW = NF >= 4 ? KF : KF / 2;
  // dgrad: NG = NF / 2 channel-fragment pairs; wave w takes pair w % NG and pixel fragments w / NG + j (4 / NG)
  static constexpr int NG = NF / 2, PS = 4 / NG;
  static_assert(TP * K / 8 % NT == 0 && TP * N / 8 % NT == 0 && NF % 2 == 0 && (NF >= 4 || NF == 2) && NG <= 4 &&
                TP == 64 && NT % (K / 8) == 0, "tiling");
  // LDS: dy tile | d tile, overlaid at the end by the block's dW partial [N][K + 16] floats
  static constexpr int OFF_Y = 0, OFF_X = OFF_Y + 2 * TP * LDY, TILES = OFF_X + 2 * TP * LDX;
  static constexpr int LDD = K + 16;
  static constexpr int BYTES = TILES > 4 * N * LDD ? TILES : 4 * N * LDD;
};

template <int K, int N>
__global__ __launch_bounds__(NT, 2) void pw_bwd_kernel(const PwBwdParams p) {
  CFL_TS_GUARD;
  using S = Pwb<K, N>;
  constexpr int KS = S::KS, NF = S::NF, GPT = S::GPT, XPT = S::XPT, CW = S::CW, FW = S::FW, NG = S::NG, PS = S::PS;
  __shared__ __attribute__((aligned(16))) char smem[S::BYTES];
  bf16_t* const sY = reinterpret_cast<bf16_t*>(smem + S::OFF_Y);         // dy tile [px][K]
  bf16_t* const sX = reinterpret_cast<bf16_t*>(smem + S::OFF_X);         // d tile [px][N]
  __shared__ __attribute__((aligned(16))) float sco[5 * K + NT];         // BN-backward coefficients (bnb_prologue)

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  const int tiles = p.M / TP;

  // ---- one tile's g / y / d pieces into registers (piece e = tid + i NT: pixel e / (C/8), channels (e % (C/8)) * 8)
  uint4 rg[GPT], ry[GPT];
  u4v rx[XPT];                  // a native vector: a uint4 struct copied whole into LDS kept rx in scratch
  auto load = [&](int t) __attribute__((always_inline)) {
    const size_t m0 = (size_t)t * TP;
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int e = tid + i * NT;
      const size_t off = (m0 + e / (K / 8)) * K + (e % (K / 8)) * 8;
      rg[i] = *reinterpret_cast<const uint4*>(p.g + off);
      ry[i] = *reinterpret_cast<const uint4*>(p.y + off);
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int e = tid + i * NT;
      rx[i] = *reinterpret_cast<const u4v*>(p.d + (m0 + e / (N / 8)) * N + (e % (N / 8)) * 8);
    }
  };
  // ---- prologue in ONE memory round trip: the wave's dgrad weight fragments (registers, for the whole launch), the
  //      first tile and the BN-backward coefficients' replica rows are all issued before bnb_prologue's wait (block
  //      0 writes dgamma / dbeta). Lane (r16, q) of fragment h, k-step s: row n = (2 cg + h) 16 + r16, k = 32 s + 8 q.
  const int cg = wid % NG, pf0 = wid / NG;
  s8v wa[2][KS];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      wa[h][s] = *reinterpret_cast<const s8v*>(p.w + (size_t)((2 * cg + h) * 16 + r16) * K + s * 32 + q * 8);
  int t = blockIdx.x;
  load(imin(t, tiles - 1));
  bnb_prologue<NT>(p.bwd, K, sco, sco + 5 * K, blockIdx.x == 0);       // ends with a barrier
  const int cq = (tid % (K / 8)) * 8;                       // this thread's channel group of every g / y piece
  f32x2_t ca[4], cb[4], cc[4];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cq + j;
    const float a = sco[c], mean = sco[K + c], rstd = sco[2 * K + c], k1 = sco[3 * K + c], k2 = sco[4 * K + c];
    const float kr = k2 * rstd;
    ca[j >> 1][j & 1] = a;
    cb[j >> 1][j & 1] = -a * kr;
    cc[j >> 1][j & 1] = a * (kr * mean - k1);
  }
  // dy of 8 channels from one 16-byte g piece and one y piece
  auto apply8 = [&](const uint4& gv, const uint4& yv) __attribute__((always_inline)) {
    const uint32_t gw[4] = {gv.x, gv.y, gv.z, gv.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w};
    uint32_t o[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const f32x2_t g2 = {__uint_as_float(gw[u] << 16), __uint_as_float(gw[u] & 0xffff0000u)};
      const f32x2_t y2 = {__uint_as_float(yw[u] << 16), __uint_as_float(yw[u] & 0xffff0000u)};
      const f32x2_t d2 = __builtin_elementwise_fma(ca[u], g2, __builtin_elementwise_fma(cb[u], y2, cc[u]));
      o[u] = pack2bf(d2[0], d2[1]);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
  };
  cfl_ts_phase(0);

  f4v accw[CW][FW];
#pragma unroll
  for (int i = 0; i < CW; ++i)
#pragma unroll
    for (int j = 0; j < FW; ++j) accw[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  const int cf0 = NF >= 4 ? wid * CW : (wid & 1);          // the wave's first c-fragment of dW
  const int ff0 = NF >= 4 ? 0 : (wid >> 1) * FW;           // ... and first f-fragment
  const int g4 = lane >> 4, q4 = (lane & 15) >> 2, pq = lane & 3;

  for (; t < tiles; t += gridDim.x) {
    // dy = BN-backward apply of (g, y) into the dy tile; d beside it
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int px = (tid + i * NT) / (K / 8);
      *reinterpret_cast<uint4*>(&sY[px * S::LDY + cq]) = apply8(rg[i], ry[i]);
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int e = tid + i * NT;
      *reinterpret_cast<u4v*>(&sX[(e / (N / 8)) * S::LDX + (e % (N / 8)) * 8]) = rx[i];
    }
    __syncthreads();
    const int m0 = t * TP;
    // the next tile, in flight during this tile's MFMAs and stores (unconditional - clamped to the last tile - so the
    // registers stay registers: a conditional refill made hipcc keep them in scratch and wait for every load)
    load(imin(t + (int)gridDim.x, tiles - 1));

    // ---- dgrad: channel fragments 2 cg, 2 cg + 1 x pixel fragments pf0 + j PS, D = W * dy^T (pw.hip's operand order)
    {
      f4v c0[NG], c1[NG];
#pragma unroll
      for (int j = 0; j < NG; ++j) c0[j] = c1[j] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s8v b[NG];
#pragma unroll
        for (int j = 0; j < NG; ++j)
          b[j] = *reinterpret_cast<const s8v*>(&sY[((pf0 + j * PS) * 16 + r16) * S::LDY + s * 32 + q * 8]);
#pragma unroll
        for (int j = 0; j < NG; ++j) {
          c0[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[0][s], b[j], c0[j], 0, 0, 0);
          c1[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[1][s], b[j], c1[j], 0, 0, 0);
        }
      }
      // lane (r16, q) holds channels (2 cg + h) 16 + 4q .. +3 of pixel px: the pair is exchanged across lane halves so
      // every lane stores 8 consecutive channels (64 contiguous bytes per pixel per store instruction, pw.hip)
      const bool odd = q & 1;
#pragma unroll
      for (int j = 0; j < NG; ++j) {
        const size_t m = (size_t)m0 + (pf0 + j * PS) * 16 + r16;
        const f4v x0 = c0[j], x1 = c1[j];
        const uint2 u0 = make_uint2(pack2bf(x0[0], x0[1]), pack2bf(x0[2], x0[3]));
        const uint2 u1 = make_uint2(pack2bf(x1[0], x1[1]), pack2bf(x1[2], x1[3]));
        const uint2 give = odd ? u0 : u1;
        const uint2 got = make_uint2(xor16_get(give.x), xor16_get(give.y));
        const uint4 v = odd ? make_uint4(got.x, got.y, u1.x, u1.y) : make_uint4(u0.x, u0.y, got.x, got.y);
        *reinterpret_cast<uint4*>(p.dd + m * N + (2 * cg + odd) * 16 + (q >> 1) * 8) = v;
      }
    }
    // ---- wgrad: dW[c][f] += sum over the tile's pixels of d[px][c] * dy[px][f] (two 32-pixel k-steps)
#pragma unroll
    for (int ks = 0; ks < TP / 32; ++ks) {
      const int r0 = 32 * ks + 4 * g4 + q4;                 // this lane's pixel rows r0 (elements 0-3), r0 + 16 (4-7)
      s8v af[CW], bf[FW];
#pragma unroll
      for (int i = 0; i < CW; ++i) {
        const int cc = (cf0 + i) * 16 + 4 * pq;
        const s4v lo = tr_read(&sX[r0 * S::LDX + cc]);
        const s4v hi = tr_read(&sX[(r0 + 16) * S::LDX + cc]);
        af[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < FW; ++j) {
        const int fc = (ff0 + j) * 16 + 4 * pq;
        const s4v lo = tr_read(&sY[r0 * S::LDY + fc]);
        const s4v hi = tr_read(&sY[(r0 + 16) * S::LDY + fc]);
        bf[j] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < CW; ++i)
#pragma unroll
        for (int j = 0; j < FW; ++j)
          accw[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], accw[i][j], 0, 0, 0);
    }
    __syncthreads();                                          // tiles read: the next tile may overwrite them
  }

  // ---- dW partial -> this block's replica row, Keras (1,1,Cin=N,Cout=K) layout [c][f]. The MFMA layout (col f =
  //      lane & 15, row c = (lane >> 4) * 4 + r) puts each wave instruction's lanes on 4 rows x 64 bytes; the
  //      memory-side atomics run at full rate on 256 contiguous bytes per instruction (optim.hip grad_finish), so the
  //      partial goes through LDS (rows padded by 16 floats: the 4 rows of a write land on disjoint banks) and is
  //      added back in element order. (an element offset, not a pointer: red_add indexes int64 elements in the
  //      deterministic mode)
  cfl_ts_phase(1);
  float* const sD = reinterpret_cast<float*>(smem);          // the tile loop ended with a barrier
#pragma unroll
  for (int i = 0; i < CW; ++i)
#pragma unroll
    for (int j = 0; j < FW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sD[((cf0 + i) * 16 + (lane >> 4) * 4 + r) * S::LDD + (ff0 + j) * 16 + (lane & 15)] = accw[i][j][r];
  __syncthreads();
  const size_t ro = (size_t)(blockIdx.x % p.replicas) * N * K;
#pragma unroll 8
  for (int e = tid; e < N * K; e += NT) red_add(p.dw, ro + e, sD[(e / K) * S::LDD + e % K], CFL_FX_G);
}

}  // namespace

bool pw_bwd_supported(const PwBwdParams& p) {
  // the 128^2 level's two pointwise layers. The 64^2 level's (K = 128) were built and measured slower than pw.hip's
  // dgrad + the mixed launch's share of their wgrads (profiles/r6_pwb: 31.6 + 22.8 vs ~41 us per step) - their
  // tiles are per-block latency bound at the <= 4 tiles per block the 65,536-pixel layers give 256 CUs
  const bool kn = p.K == 64 && (p.N == 32 || p.N == 64);
  return kn && p.M > 0 && p.M % TP == 0 && p.replicas >= 1 && p.bwd.reps >= 1 && p.bwd.reps <= BNB_MAX_REPS;
}

template <int K, int N>
static int launch(const PwBwdParams& p, hipStream_t st) {
  const int tiles = p.M / TP;
  // default grids measured per shape (profiles/r6_pwb): more blocks add replica-row atomics, fewer leave CUs idle
  int grid = cfl_tune(TUNE_PWB_BLOCKS) > 0 ? cfl_tune(TUNE_PWB_BLOCKS) : (N == 32 ? 384 : 256);
  if (grid > tiles) grid = tiles;
  hipLaunchKernelGGL((pw_bwd_kernel<K, N>), dim3(grid), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int pw_bwd(const PwBwdParams& p, hipStream_t st) {
  if (!pw_bwd_supported(p)) return 1;
  return p.N == 32 ? launch<64, 32>(p, st) : launch<64, 64>(p, st);
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_pw_bwd(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_pw_bwd(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
