// Streaming 1x1 convolution on gfx950 MFMA: the SeparableConv2D pointwise convs (forward, with the next BatchNorm's
// batch statistics) and the 1x1 data gradients of the pointwise and residual convs
// (/root/reference/client_fit_model.py:107-116, 118-121, 133-136).
//
// These GEMMs have K = Cin = 32-256 and M = B*H*W = 16k-262k pixels: 1-8 K-steps per output tile, i.e. a streaming
// pass over the input. conv_igemm's tile-per-block form (one 64x64 tile, LDS-staged operands, block barriers,
// per-block statistics atomics) measured 2.2-3.7 TB/s against 6.8 TB/s for a copy of the same bytes, and its
// statistics epilogue alone cost 9 us of 22.5 at 128^2 (tools/pw_probe.py: 4,096 blocks x 128 atomics).
//
// Here the MFMA operands are swapped - D = W * X^T - so that
//   * the B operand (16 pixels x 32 channels per fragment: lane = (pixel, 8 channels)) is a plain 16-byte global
//     load of the NHWC input straight into the MFMA registers (no LDS staging of the activations, no barrier);
//   * the accumulator holds 4 consecutive output channels of one pixel per lane: 8-byte bf16 stores straight from
//     the registers, no LDS transpose;
//   * the weights (A operand) of the block's output-channel slice stay resident in LDS for the whole launch
//     (swizzled 16-byte quarters: conflict-free fragment reads).
// Each wave is its own pipeline: a persistent loop over WR-pixel tiles whose next tile's loads are issued right after
// the current tile's MFMAs, so they are in flight during its epilogue. Statistics (from the rounded bf16 outputs, as
// in conv_igemm) stay in registers across the tiles: one atomic per (channel, statistic) per block at the end.
//
// Because the input goes straight from global memory into the MFMA registers, producer passes of a data gradient
// fold into this load (the kernel also stores the formed input for the weight gradient that reads it later):
//   BWD - the BN-backward apply of (g, y) (common.h BnBwdIn; the encoder pointwise dgrads), and
//   S2  - the 2x2-block sum of a full-resolution gradient (the decoder residual conv's upsample gradient).
#include "common.h"
#include "launch.h"
#include "side_bodies.h"

namespace {

constexpr int NT = 256;

// bf16 offset of 16-byte quarter q of weight row n in a [rows][32] k-block: quarter q stored at q ^ ((n >> 1) & 3)
// (conv_igemm.hip's swizzle: a fragment read of 16 consecutive rows at one quarter covers all 64 banks)
CFL_DEVICE int wswz(int n, int q) { return n * 32 + ((q ^ ((n >> 1) & 3)) << 3); }

// pixels per wave tile (B operand: WR*K/128 VGPRs; the 2x2-sum input holds four times that while loading, so its
// tiles are halved below K = 128)
template <int K, bool S2 = false>
constexpr int pw_rows() { return K >= 128 ? 4096 / K : (S2 ? 32 : 64); }

// BWD: the input is the gradient g w.r.t. a BatchNorm output and the operand is its BN-backward apply (common.h
// BnBwdIn, the bn_bwd_apply arithmetic): g and the BN input y are loaded into the B-fragment registers and combined
// right before the MFMAs; the blocks of output slice 0 also store dx (each pixel once) for the weight gradient, and
// block 0 writes dgamma / dbeta. Replaces a bn_bwd_apply pass (one write + read of dx and a launch fewer).
// S2: the input is the 2x2-block sum of p.sum2x2 (the decoder residual conv's upsample gradient): the four full-
// resolution pixels of each B-fragment pixel are loaded and summed ((o00 + o01) + (o10 + o11), rounded once: node_bwd's
// GM_SUM2X2), and the slice-0 blocks store the sums into x for the weight gradient.
// SIDE: the launch also carries an independent streaming pass (launch.h SideJob) whose blocks are interleaved with the
// conv's in groups of 8, so a conv block keeps its dispatch-order XCD (block b -> XCD b % 8, which the slice mapping
// below relies on) and both kinds are resident on every CU from the start: conv groups at even, side groups at odd
// group positions while both last, then the remaining conv blocks, then the remaining side blocks. The conv code reads
// the kernel argument p directly (a body function taking it by reference made the compiler copy it into registers at
// entry: 182 -> 256 VGPRs and spills in the BN-backward form).
template <int NB, int K, int D, bool BWD, bool S2 = false, int SIDE = SIDE_NONE>
__global__ __launch_bounds__(NT, 2) void pw_kernel(const ConvParams p, int nslices, int conv_blocks) {
  CFL_TS_GUARD;
  int bid = blockIdx.x;
  const int nblocks = conv_blocks;
  if constexpr (SIDE != SIDE_NONE) {
    const int side_blocks = gridDim.x - conv_blocks;
    const int pairs = imin(conv_blocks >> 3, side_blocks >> 3);
    const int b = blockIdx.x, grp = b >> 3;
    bool conv;
    int idx;
    if (grp < 2 * pairs) {
      conv = (grp & 1) == 0;
      idx = (grp >> 1) * 8 + (b & 7);
    } else {                                           // the rest: conv blocks first, then side blocks
      const int rb = b - 16 * pairs, conv_rest = conv_blocks - 8 * pairs;
      conv = rb < conv_rest;
      idx = pairs * 8 + (conv ? rb : rb - conv_rest);
    }
    if (!conv) {
      if constexpr (SIDE == SIDE_BBA) side::bba_body(p.side.bba, idx, side_blocks);
      else side::node_pool_body<1>(p.side.pool, idx, side_blocks);
      return;
    }
    bid = idx;
  }
  constexpr int WR = pw_rows<K, S2>();
  constexpr int MF = WR / 16, NF = NB / 16, KS = K / 32;
  __shared__ __attribute__((aligned(16))) bf16_t sW[KS * NB * 32];
  __shared__ __attribute__((aligned(16))) float sBias[NB];
  __shared__ float sred[2][NT / 64][NB];
  __shared__ __attribute__((aligned(16))) float sco[BWD ? 5 * K + NT : 1];   // BN-backward coefficients (bnb_prologue)

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, q = lane >> 4;
  // block -> (output-channel slice, block within the slice); the slices of one pixel range sit on one XCD
  // (dispatch order b, b + 8, ... share an XCD and its L2, which then serves the second slice's input reads)
  const int j = bid >> 3;
  const int slice = j % nslices, bs = (j / nslices) * 8 + (bid & 7);
  const int bps = nblocks / nslices;
  const int n0 = slice * NB;
  const int tiles = (p.M + WR - 1) / WR;
  const int wstride = bps * (NT / 64);
  int t = bs * (NT / 64) + wid;

  // B operand: lane (r16, q) holds pixel m0 + i*16 + r16, channels s*32 + q*8 .. +7. Rows past M are clamped to the
  // last pixel (their results are neither stored nor counted).
  s8v a[D][MF][KS];
  uint4 ya[BWD ? D : 1][MF][KS];                         // BWD: the BN input y of the same elements
  uint4 qa[S2 ? D : 1][MF][KS][3];                       // S2: the other three pixels of each 2x2 block
  auto load = [&](int d, int tt) {
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      int m = tt * WR + i * 16 + r16;
      m = m < p.M ? m : p.M - 1;
      const size_t off = (size_t)m * K + q * 8;
      if constexpr (S2) {
        const int hw = p.Hin * p.Win, b = m / hw, r = m - b * hw, h = r / p.Win, w = r - h * p.Win;
        const size_t W2 = (size_t)p.Win * 2;
        const size_t o00 = (((size_t)b * 2 * p.Hin + 2 * h) * W2 + 2 * w) * K + q * 8;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          a[d][i][s] = *reinterpret_cast<const s8v*>(p.sum2x2 + o00 + s * 32);
          qa[d][i][s][0] = *reinterpret_cast<const uint4*>(p.sum2x2 + o00 + K + s * 32);
          qa[d][i][s][1] = *reinterpret_cast<const uint4*>(p.sum2x2 + o00 + W2 * K + s * 32);
          qa[d][i][s][2] = *reinterpret_cast<const uint4*>(p.sum2x2 + o00 + (W2 + 1) * K + s * 32);
        }
      } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          a[d][i][s] = *reinterpret_cast<const s8v*>(p.x + off + s * 32);
          if constexpr (BWD) ya[d][i][s] = *reinterpret_cast<const uint4*>(p.bwd.y + off + s * 32);
        }
      }
    }
  };
  // D tiles in flight per wave: the first D tiles' loads are issued while the weights are staged
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (t + d * wstride < tiles) load(d, t + d * wstride);

  // the weight slice, bias and (BWD) the BN-backward replica rows are issued together with the first tiles: the
  // prologue waits one memory round trip (a strided weight-copy loop waited one per iteration: ~6 us per block)
  Stage16<NT, NB * K / 8> wst;
  wst.load([&](int c) { const int n = c / (K / 8), kc = c - n * (K / 8); return p.wt + (size_t)(n0 + n) * K + kc * 8; });
  const float bias_v = p.bias ? p.bias[n0 + imin(tid, NB - 1)] : 0.f;
  if constexpr (BWD) bnb_prologue<NT>(p.bwd, K, sco, sco + 5 * K, bid == 0);   // ends with a barrier
  wst.store([&](int c) { const int n = c / (K / 8), kc = c - n * (K / 8); return sW + (kc >> 2) * NB * 32 + wswz(n, kc & 3); });
  if (tid < NB) sBias[tid] = bias_v;
  __syncthreads();

  const bool stats = p.stats != nullptr;
  float s1[NF][4], s2[NF][4];
#pragma unroll
  for (int nf = 0; nf < NF; ++nf)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[nf][r] = s2[nf][r] = 0.f;

  cfl_ts_phase(0);
  for (; t < tiles; t += D * wstride) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int tt = t + d * wstride;
      if (tt >= tiles) break;
      // opaque zero: keeps the (loop-invariant) weight fragment / BN-coefficient reads inside the loop - hoisted,
      // they would stay live in registers across the whole loop and spill
      int wo = 0;
      asm volatile("" : "+v"(wo));
      const bf16_t* sWt = sW + wo;
      if constexpr (S2) {
        const bool side = slice == 0;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int m = tt * WR + i * 16 + r16;
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            float u0[8], u1[8], u2[8], u3[8], o[8];
            unpack8(*reinterpret_cast<const uint4*>(&a[d][i][s]), u0);
            unpack8(qa[d][i][s][0], u1);
            unpack8(qa[d][i][s][1], u2);
            unpack8(qa[d][i][s][2], u3);
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0.f + ((u0[j] + u1[j]) + (u2[j] + u3[j]));
            const uint4 v = pack8(o);
            a[d][i][s] = *reinterpret_cast<const s8v*>(&v);
            if (side && m < p.M) *reinterpret_cast<uint4*>(const_cast<bf16_t*>(p.x) + (size_t)m * K + s * 32 + q * 8) = v;
          }
        }
      }
      if constexpr (BWD) {
        // dx = BN-backward apply of (g, y); slice-0 blocks store it (rows past M are clamped copies: not stored)
        const bool side = slice == 0 && p.bwd.dx != nullptr;
        const float* co = sco + wo;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int m = tt * WR + i * 16 + r16;
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const uint4 dx = bnb_apply8(*reinterpret_cast<const uint4*>(&a[d][i][s]), ya[d][i][s], co, K,
                                        s * 32 + q * 8);
            a[d][i][s] = *reinterpret_cast<const s8v*>(&dx);
            if (side && m < p.M) *reinterpret_cast<uint4*>(p.bwd.dx + (size_t)m * K + s * 32 + q * 8) = dx;
          }
        }
      }
      f4v acc[NF][MF];
#pragma unroll
      for (int nf = 0; nf < NF; ++nf)
#pragma unroll
        for (int i = 0; i < MF; ++i) acc[nf][i] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int nf = 0; nf < NF; ++nf) {
          const s8v w = *reinterpret_cast<const s8v*>(sWt + s * NB * 32 + wswz(nf * 16 + r16, q));
#pragma unroll
          for (int i = 0; i < MF; ++i)
            acc[nf][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, a[d][i][s], acc[nf][i], 0, 0, 0);
        }
      const int m0 = tt * WR;
      if (tt + D * wstride < tiles) load(d, tt + D * wstride);   // refill this buffer: D tiles stay in flight

      // D = W * X^T: lane (r16, q) holds output channels n0 + nf*16 + q*4 + r (r = 0..3) of pixel m0 + i*16 + r16.
      // Fragments nf = 2h, 2h+1 are paired: lanes q, q^1 (lane +- 16) swap one 8-byte half each so every lane owns
      // 8 consecutive channels and each store instruction writes 64 contiguous bytes per pixel (8-byte stores of
      // 32-byte pieces measured at half the write rate: tools/pw_probe.py)
      const bool odd = q & 1;
#pragma unroll
      for (int h = 0; h < NF / 2; ++h) {
        const float4 b0 = *reinterpret_cast<const float4*>(&sBias[(2 * h) * 16 + q * 4]);
        const float4 b1 = *reinterpret_cast<const float4*>(&sBias[(2 * h + 1) * 16 + q * 4]);
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int m = m0 + i * 16 + r16;
          const f4v c0 = acc[2 * h][i], c1 = acc[2 * h + 1][i];
          const uint2 u0 = make_uint2(pack2bf(c0[0] + b0.x, c0[1] + b0.y), pack2bf(c0[2] + b0.z, c0[3] + b0.w));
          const uint2 u1 = make_uint2(pack2bf(c1[0] + b1.x, c1[1] + b1.y), pack2bf(c1[2] + b1.z, c1[3] + b1.w));
          const uint2 give = odd ? u0 : u1;
          const uint2 got = make_uint2(xor16_get(give.x), xor16_get(give.y));
          const uint4 v = odd ? make_uint4(got.x, got.y, u1.x, u1.y) : make_uint4(u0.x, u0.y, got.x, got.y);
          if (m < p.M) {
            *reinterpret_cast<uint4*>(p.y + (size_t)m * p.N + n0 + (2 * h + odd) * 16 + (q >> 1) * 8) = v;
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
    }
  }

  cfl_ts_phase(1);
  if (!stats) return;
  // lanes of one q group hold the same 4 channels per fragment column: reduce over r16, then over the 4 waves
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
  const size_t ro = (size_t)(bid % STAT_REPLICAS) * 2 * p.N;
  for (int e = tid; e < 2 * NB; e += NT) {
    const int st = e / NB, cc = e - st * NB;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) v += sred[st][w][cc];
    red_add(p.stats, ro + st * p.N + n0 + cc, v, red_scale(true, st));
  }
}

template <int NB, int K, int D>
void launch_d(const ConvParams& p, hipStream_t st) {
  const bool bwd = p.bwd.y != nullptr;
  const int WR = p.sum2x2 ? pw_rows<K, true>() : pw_rows<K>();
  const int nslices = p.N / NB;
  const int tiles = (p.M + WR - 1) / WR;
  // persistent grid: each wave takes a multiple of D tiles (ideally exactly D: its whole share in flight at once),
  // at most one round of resident blocks (2 per CU) per launch
  int cap = cfl_tune(TUNE_PW_BLOCKS);
  if (cap <= 0) cap = 512;
  int per_slice = cap / nslices / 8 * 8;
  if (per_slice < 8) per_slice = 8;
  int tpw = (tiles + per_slice * 4 - 1) / (per_slice * 4);           // tiles per wave
  tpw = (tpw + D - 1) / D * D;
  const int waves = (tiles + tpw - 1) / tpw;
  const int bps = ((waves + 3) / 4 + 7) / 8 * 8;
  const int cb = bps * nslices;
  if constexpr (D == 1 && NB <= 64) {     // (the 128-wide slices serve the plain and BN-backward forms only)
    if (p.side.kind == SIDE_BBA) {                 // the decoder residual dgrads + the BN_B backward apply
      const dim3 g(cb + bn_bwd_apply_grid(p.side.bba));
      if (p.sum2x2) hipLaunchKernelGGL((pw_kernel<NB, K, 1, false, true, SIDE_BBA>), g, dim3(NT), 0, st, p, nslices, cb);
      else hipLaunchKernelGGL((pw_kernel<NB, K, 1, false, false, SIDE_BBA>), g, dim3(NT), 0, st, p, nslices, cb);
      return;
    }
    if (p.side.kind == SIDE_POOL) {                // the encoder residual dgrads + the max-pool node gradient
      const dim3 g(cb + node_pool_grid(p.side.pool));
      hipLaunchKernelGGL((pw_kernel<NB, K, 1, false, false, SIDE_POOL>), g, dim3(NT), 0, st, p, nslices, cb);
      return;
    }
    if (p.sum2x2) {
      hipLaunchKernelGGL((pw_kernel<NB, K, 1, false, true>), dim3(cb), dim3(NT), 0, st, p, nslices, cb);
      return;
    }
  }
  if constexpr (D == 1) {
    if (bwd) {
      hipLaunchKernelGGL((pw_kernel<NB, K, 1, true>), dim3(cb), dim3(NT), 0, st, p, nslices, cb);
      return;
    }
  }
  hipLaunchKernelGGL((pw_kernel<NB, K, D, false>), dim3(cb), dim3(NT), 0, st, p, nslices, cb);
}

template <int NB, int K>
void launch(const ConvParams& p, hipStream_t st) {
  int d = cfl_tune(TUNE_PW_DEPTH);
  if (d <= 0 || p.bwd.y || p.sum2x2 || p.side.kind) d = 1;   // whole-step A/B: depth 1 / 2 (4 at K = 32) 1.459 / 1.478 ms per iteration; the
                                  // BN-backward form holds y as well and runs at depth 1 only (deeper rings spill)
  if constexpr (K == 32) {                                // deeper rings spill at K >= 64
    if (d >= 4) return launch_d<NB, K, 4>(p, st);
  }
  if (d >= 2) launch_d<NB, K, 2>(p, st);
  else launch_d<NB, K, 1>(p, st);
}

}  // namespace

bool pw_conv_supported(const ConvParams& p) {
  return cfl_tune(TUNE_PW) != 1 && cfl_tune(TUNE_IGEMM_CFG) == 0 && p.algo == 0 && p.ks == 1 && p.stride == 1 &&
         p.pad_t == 0 && p.pad_l == 0 && !p.up_in && p.Ho == p.Hin && p.Wo == p.Win && p.K == p.Cin &&
         (p.Cin == 32 || p.Cin == 64 || p.Cin == 128 || p.Cin == 256) && (p.N == 32 || p.N % 64 == 0) &&
         p.xf.ab == nullptr && !p.xf.relu && p.node.y == nullptr && p.join.mode == JOIN_NONE &&
         (p.bwd.y == nullptr || (p.bwd.dx != nullptr && p.bwd.reps <= BNB_MAX_REPS)) &&
         (p.sum2x2 == nullptr || (p.bwd.y == nullptr && p.bias == nullptr && p.stats == nullptr)) && p.pj.v == nullptr &&
         p.xfin.stats == nullptr && p.M > 0 &&
         (p.side.kind == SIDE_NONE || (p.bwd.y == nullptr && cfl_tune(TUNE_SIDE) != 1 &&
                                       (p.side.kind == SIDE_BBA ? bn_bwd_apply_ok(p.side.bba)
                                                                : node_pool_eligible(p.side.pool))));
}

int pw_conv(const ConvParams& p, hipStream_t st) {
  if (!pw_conv_supported(p)) return 1;
  const bool n32 = p.N == 32;
  // 128-channel output slices for the wide layers at large M (the 512^2 planned batch): each N slice re-reads (and in
  // the BN-backward form re-transforms) the whole input, so half the slices halve that traffic; whole step 5,581 ->
  // 5,753 img/s at 512^2 / b1,096. At 256^2 / b16 (M <= 65k for these layers) they measured slower (13,046 / 13,050 vs
  // 12,907 / 12,937: fewer blocks). TUNE_PW_NB: 64 = never, 128 = wherever the shape allows.
  const int nbt = cfl_tune(TUNE_PW_NB);
  if (nbt != 64 && p.N % 128 == 0 && p.Cin >= 128 && !p.sum2x2 && !p.side.kind &&
      (nbt == 128 || p.M >= (1 << 20))) {
    if (p.Cin == 128) launch<128, 128>(p, st);
    else launch<128, 256>(p, st);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  switch (p.Cin) {
    case 32: n32 ? launch<32, 32>(p, st) : launch<64, 32>(p, st); break;
    case 64: n32 ? launch<32, 64>(p, st) : launch<64, 64>(p, st); break;
    case 128: n32 ? launch<32, 128>(p, st) : launch<64, 128>(p, st); break;
    default: n32 ? launch<32, 256>(p, st) : launch<64, 256>(p, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_pw(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_pw(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
