// Split-K-in-block 3x3 / stride-1 / "same" convolution for the low-resolution decoder levels (16^2 and 32^2 maps at
// 256^2 input: M = 4k-16k pixels, Cin = 128-256 -> K = 1152-2304, N = 128-256), forward and data-gradient
// (/root/reference/client_fit_model.py:129,133).
//
// Why another 3x3 kernel. At these levels the whole layer is only M x N = 1-2M outputs: 256 CUs get one 64x64 or
// 128x64 output tile each, and every tile needs the FULL K = 9 * Cin reduction. The per-tile kernels (conv3x3.hip,
// conv3x3_deep.hip) split such a tile over their 4 waves by OUTPUT (2x2 waves of 32x16 / 64x32 pixels x channels on
// the 16x16x32 MFMA): every wave re-reads the shared A / B operands from LDS (1.5 ds_read_b128 per MFMA on the 8x8
// tiles, profiles/README.md: LDS-bound) and with one block per CU a single wave per SIMD waits out every barrier.
// Here the 4 waves split the block tile's REDUCTION instead: each wave accumulates the whole BM x BN tile on
// v_mfma_f32_32x32x16_bf16 (register blocking FM x FN 32x32 fragments: each A read feeds FN MFMAs, each B read FM)
// over a quarter of every chunk's 18 (tap, 16-channel k-step) units, and the four partial tiles are summed through
// LDS once at the end. LDS fragment traffic per MFMA drops 2-3x and the per-chunk work of a wave is 4-5 units of
// FM*FN back-to-back MFMAs.
//
// Operand pipeline (one 256-thread block per CU, 1 wave per SIMD):
//   * weights (9 taps x BN rows x 32 channels per chunk, the bulk of the bytes) stream global -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, no VGPR staging) into a 3-stage ring, two chunks ahead;
//   * the (TH+2) x (TW+2) x 32 input halo goes through registers one chunk ahead, so the producer's BN-apply + ReLU
//     and the nearest-2x upsample of the decoder input are applied on the way into LDS (padding stays exactly 0);
//   * one raw s_barrier per chunk with counted `s_waitcnt vmcnt` (a __syncthreads would drain the DMAs in flight).
// LDS images: 64-byte rows (32 bf16 channels) with the 16-byte quarter q of row r at slot q ^ ((r >> 2) & 3): a
// 32-row MFMA fragment read (ds_read_b128 lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ...) then touches 16
// distinct rows mod 16 = all 64 banks once. Halo lines are padded to HWL rows (24 for 8-wide tiles, 32 for 16-wide)
// so the 2-D pixel fragments keep that property for every tap shift.
// Epilogue (bias, bf16, LDS-staged 16-byte stores, BN statistics / BN-node gradient / decoder node join) as
// conv3x3.hip.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr int BK = 32;                    // channels per chunk
constexpr int WSTAGES = 3;                // weight ring (two chunks in flight)
constexpr int HSTAGES = 2;                // halo ring (one chunk ahead, via registers)
constexpr int SK_MAX_CIN = 256;           // XFIN coefficient staging

__device__ __attribute__((aligned(64))) uint4 g_sk_zero[4];     // 64 zero bytes: source of padding pieces

CFL_DEVICE int sk_off(int r, int q) { return r * BK + ((q ^ ((r >> 2) & 3)) << 3); }

CFL_DEVICE void sk_dma16(const void* src, bf16_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0, 0);
}

template <int N>
CFL_DEVICE void sk_wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// keep the issue order of the memory operations on either side (compiler and machine scheduler): the counted
// vmcnt waits assume the halo loads of a step are issued before its weight DMAs
CFL_DEVICE void sk_order() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS store the compiler cannot see (hipcc would order a visible LDS store after ALL outstanding LDS-DMA loads,
// draining the weight chunks in flight); it only touches the halo stage no DMA writes.
CFL_DEVICE void sk_store16(bf16_t* p, uint4 v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)p;
  const u4v d = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(d) : "memory");
}

template <int TH, int TW, int BN>
struct SkCfg {
  static constexpr int BM = TH * TW;
  static constexpr int HH = TH + 2, HWR = TW + 2, HWL = TW == 8 ? 24 : 32;
  static constexpr int HROWS = HH * HWL;                  // LDS rows per halo stage
  static constexpr int WROWS = 9 * BN;                    // LDS rows per weight stage
  static constexpr int W_INS = WROWS / 16;                // 1-KB DMA instructions per chunk
  static constexpr int W_PER = (W_INS + 3) / 4, W_REM = W_INS % 4;
  static constexpr int HPIECES = HH * HWR * 4, H_PER_T = (HPIECES + NT - 1) / NT;
  static constexpr int FM = BM / 32, FN = BN / 32;
  static constexpr int WST = WROWS * BK, HST = HROWS * BK;              // bf16 elements per stage
  static constexpr int RING_BYTES = 2 * (WSTAGES * WST + HSTAGES * HST);
  static constexpr int RPITCH = BM + 4;                   // fp32 reduction image [4][BN][RPITCH]
  static constexpr int LDC = BN + 8;
  static constexpr int RED_BYTES = 4 * BN * RPITCH * 4, C_BYTES = BM * LDC * 2;
  static constexpr int SMEM = RING_BYTES > RED_BYTES + C_BYTES ? RING_BYTES : RED_BYTES + C_BYTES;
  static_assert(W_INS * 16 == WROWS && BM % 32 == 0 && BN % 32 == 0 && TW <= 16, "tiling");
  static_assert(HWL >= HWR && HWL % 8 == 0, "halo pitch");
};

template <int TH, int TW, int BN, int NCH, bool PJ, bool XFIN>
__global__ __launch_bounds__(NT, 1) void conv3x3_sk_kernel(ConvParams p) {
  CFL_TS_GUARD;
  using S = SkCfg<TH, TW, BN>;
  constexpr int BM = S::BM, HWL = S::HWL, HWR = S::HWR, FM = S::FM, FN = S::FN;
  constexpr int W_PER = S::W_PER, W_REM = S::W_REM, H_PER_T = S::H_PER_T, HPIECES = S::HPIECES;
  constexpr int LDC = S::LDC;

  // ONE shared object (a second one can make hipcc drain the DMAs before every ds_read)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[S::SMEM + 2 * 4 * BN * 4 + 2 * SK_MAX_CIN * 4];
  bf16_t* wring = reinterpret_cast<bf16_t*>(smem);                    // [WSTAGES][9*BN rows][32]
  bf16_t* hring = wring + WSTAGES * S::WST;                           // [HSTAGES][HROWS][32]
  float (*sred)[4][BN] = reinterpret_cast<float (*)[4][BN]>(smem + S::SMEM);
  float* sxab = reinterpret_cast<float*>(smem + S::SMEM + 2 * 4 * BN * 4);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_w = p.Wo / TW, tiles_hw = tiles_w * (p.Ho / TH);
  const int nb = p.N / BN;
  const int lin = xcd_block_linear();                 // the column blocks of one pixel tile share an XCD
  const int bn_idx = lin % nb, tile = lin / nb;
  const int b = tile / tiles_hw, tr = tile - b * tiles_hw;
  const int ty0 = (tr / tiles_w) * TH, tx0 = (tr % tiles_w) * TW;
  const int nBlock = bn_idx * BN;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;
  const bool xform = has_ab || relu;

  // producer BN coefficients of every input channel in LDS (a transform reads them per chunk; a global load there
  // would be counted behind the weight DMAs in flight and drain them). XFIN: consumer-side BN finalize (computed
  // from the producer's replica sums; the first block writes the layer's ab rows).
  if constexpr (!XFIN) {
    if (has_ab && tid < p.Cin) {
      sxab[tid] = p.xf.ab[tid];
      sxab[SK_MAX_CIN + tid] = p.xf.ab[p.xf.C + tid];
    }
    __syncthreads();
  } else {
    if (tid < p.Cin) {
      float a, bb, mean, rstd;
      bn_coef_from_stats(p.xfin, p.Cin, tid, a, bb, mean, rstd);
      sxab[tid] = a;
      sxab[SK_MAX_CIN + tid] = bb;
      if (lin == 0) {
        float* ab = const_cast<float*>(p.xf.ab);
        ab[tid] = a;
        ab[p.Cin + tid] = bb;
        ab[2 * p.Cin + tid] = mean;
        ab[3 * p.Cin + tid] = rstd;
      }
    }
    __syncthreads();
  }

  // ---- weight DMA sources: instruction i = wid + 4 j covers LDS rows 16 i .. 16 i + 15 (row = tap * BN + n) ----
  const bf16_t* wsrc[W_PER];
#pragma unroll
  for (int j = 0; j < W_PER; ++j) {
    const int i = wid + 4 * j;
    const int row = 16 * (i < S::W_INS ? i : 0) + (lane >> 2), slot = lane & 3, q = slot ^ ((row >> 2) & 3);
    const int tap = row / BN, n = row - tap * BN;
    wsrc[j] = p.wt + (size_t)(nBlock + n) * p.K + (size_t)tap * p.Cin + q * 8;
  }
  const bool wfull = W_REM == 0 || wid < W_REM;      // wave-uniform: this wave issues W_PER DMAs per chunk
  auto issue_w = [&](int ch) {
    bf16_t* st = wring + (ch % WSTAGES) * S::WST;
#pragma unroll
    for (int j = 0; j < W_PER; ++j)
      if (j < W_PER - 1 || wfull) sk_dma16(wsrc[j] + ch * BK, st + (wid + 4 * j) * 512);
  };

  // ---- halo: piece e = tid + i NT -> halo pixel e / 4 (row-major over HH x HWR), channel quarter e % 4 ----
  const bf16_t* hsrc[H_PER_T];
  int hrow[H_PER_T];
  uint32_t hvalid = 0;
#pragma unroll
  for (int i = 0; i < H_PER_T; ++i) {
    const int e = tid + i * NT;
    const int hp = e >> 2, q = e & 3;
    const int hy = hp / HWR, hx = hp - hy * HWR;
    const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
    const bool ok = e < HPIECES && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl;
    hvalid |= (ok ? 1u : 0u) << i;
    hsrc[i] = ok ? p.x + (((size_t)b * p.Hin + (iy >> p.up_in)) * p.Win + (ix >> p.up_in)) * p.Cin + q * 8
                 : reinterpret_cast<const bf16_t*>(g_sk_zero);
    hrow[i] = e < HPIECES ? hy * HWL + hx : HWR;              // past the halo: line 0's first pad row (never read)
  }
  // The halo loads are inline asm: hipcc's waitcnt pass does not count the LDS-DMAs issued after them, so for a
  // compiler-visible load it drains vmcnt to 0 before the first use - and with it the weight DMAs of the chunk two
  // steps ahead. Here the counted sk_wait_h below is the only wait, and it ties the registers (no use moves above it).
  u4v rh[H_PER_T];
  auto load_h = [&](int ch) {                         // unconditional loads: a fixed vmcnt count per wave
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const bf16_t* src = hsrc[i] + (((hvalid >> i) & 1u) ? ch * BK : 0);
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(rh[i]) : "v"(src) : "memory");
    }
  };
  auto tie_h = [&]() {                                // after a counted wait: the halo registers are valid now
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) asm volatile("" : "+v"(rh[i]));
  };
  auto store_h = [&](int ch) {                        // producer transform on the way into LDS; padding stays 0
    float ha[8], hb[8];
    const int c8 = ch * BK + (tid & 3) * 8;           // every piece of this thread has channel quarter tid & 3
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ha[j] = has_ab ? sxab[c8 + j] : 1.f;
      hb[j] = has_ab ? sxab[SK_MAX_CIN + c8 + j] : 0.f;
    }
    bf16_t* st = hring + (ch % HSTAGES) * S::HST;
    // branch-free (divergent branches here made hipcc fall back to draining every DMA in flight): pieces past the
    // halo go to an unused pad row, out-of-image pieces keep their zero
    // (packed BN-apply + ReLU, common.h xform8; the mask zeroes out-of-image pieces)
    const uint32_t relu_lo = relu ? 0u : 0x80008000u;
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const uint32_t m = ((hvalid >> i) & 1u) ? 0xffffffffu : 0u;
      sk_store16(st + sk_off(hrow[i], (tid + i * NT) & 3),
                 xform8(make_uint4(rh[i][0], rh[i][1], rh[i][2], rh[i][3]), ha, hb, relu_lo, m));
    }
  };

  // decoder node join: this thread's half-resolution pixel and its mask / addend / sums-source vectors, in flight
  // during the K loop (one half-resolution pixel per thread: BM / 4 <= NT / (BN / 8))
  constexpr int CG = BN / 8, ROWS_PER_PASS = NT / CG;
  static_assert(!PJ || BM / 4 <= ROWS_PER_PASS, "one half-resolution pixel per thread");
  uint4 pjv = make_uint4(0, 0, 0, 0), pja = pjv, pjy = pjv;
  size_t pjoff = 0;
  bool pjok = false;
  if constexpr (PJ) {
    constexpr int HTW = TW / 2;
    const int hr = tid / CG, hy = hr / HTW, hx = hr % HTW;
    const int oy = ty0 + 2 * hy, ox = tx0 + 2 * hx;
    pjok = hr < BM / 4;
    pjoff = (((size_t)b * (p.Ho >> 1) + (oy >> 1)) * (p.Wo >> 1) + (ox >> 1)) * p.N + nBlock + (tid % CG) * 8;
    if (pjok) {
      pjv = *reinterpret_cast<const uint4*>(p.pj.v + pjoff);
      if (p.pj.add) pja = *reinterpret_cast<const uint4*>(p.pj.add + pjoff);
      if (p.pj.sy) pjy = *reinterpret_cast<const uint4*>(p.pj.sy + pjoff);
    }
  }

  // ---- fragments: A row of pixel fragment mf (tap (0,0)), B row of channel fragment nf, k-half of the lane ----
  int fa[FM];
#pragma unroll
  for (int mf = 0; mf < FM; ++mf) {
    const int pp = mf * 32 + (lane & 31);
    fa[mf] = (pp / TW) * HWL + pp % TW;
  }
  const int kh = lane >> 5;
  f16v acc[FM][FN];
#pragma unroll
  for (int mf = 0; mf < FM; ++mf)
#pragma unroll
    for (int nf = 0; nf < FN; ++nf)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mf][nf][r] = 0.f;

  // ---- pipeline, fully unrolled over the NCH chunks (no loop-carried accumulator or load registers: a loop made
  //      hipcc copy the accumulators AGPR <-> VGPR and drain every DMA in flight at the loop head) ----
  // issue order per chunk step c: [halo loads of c + 1] [weight DMAs of c + 2]; waits count the younger ops only.
  const int wcnt = wfull ? W_PER : W_PER - 1;                 // this wave's DMAs per chunk (wave-uniform)
  (void)wcnt;
  load_h(0);
  sk_order();
  issue_w(0);
  if (NCH > 1) issue_w(1);
  sk_order();
  if (NCH > 1) { if (wfull) sk_wait_vm<2 * W_PER>(); else sk_wait_vm<2 * W_PER - 2>(); }
  else { if (wfull) sk_wait_vm<W_PER>(); else sk_wait_vm<W_PER - 1>(); }
  tie_h();
  store_h(0);
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    // weights of chunk ch landed: only the DMAs of chunk ch + 1 may still be in flight
    if (ch + 1 < NCH) { if (wfull) sk_wait_vm<W_PER>(); else sk_wait_vm<W_PER - 1>(); }
    else sk_wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");        // this thread's halo stores of chunk ch
    __builtin_amdgcn_s_barrier();                             // every wave's part landed; stages of ch - 1 free
    if (ch + 1 < NCH) load_h(ch + 1);                         // in flight during this chunk's MFMAs
    sk_order();                                               // (the waits count the halo loads as the older ops)
    if (ch + 2 < NCH) issue_w(ch + 2);
    sk_order();
    const bf16_t* sw = wring + (ch % WSTAGES) * S::WST;
    const bf16_t* sh = hring + (ch % HSTAGES) * S::HST;
    // this wave's units u = wid + 4 j of the chunk's 18 (tap, 16-channel k-step) units; waves 2 and 3 run a
    // 5th unit against a zero weight fragment (no branch: the chunk step takes the 5-unit waves' time anyway).
    // Fragments are double-buffered in registers: unit j + 1's LDS reads are issued before unit j's MFMAs, so each
    // read has FM * FN MFMAs (>= 128 cycles) of cover instead of waiting in front of its own MFMAs.
    auto frag = [&](int j, s8v (&af)[FM], s8v (&bfg)[FN]) {
      const int u0 = wid + 4 * j;
      const bool live = j < 4 || u0 < 18;
      const int u = live ? u0 : 17;
      const int tap = u >> 1, s = u & 1;
      const int ky = (tap * 11) >> 5, kx = tap - 3 * ky;     // tap / 3 for tap < 9
      const int q = 2 * s + kh;
#pragma unroll
      for (int mf = 0; mf < FM; ++mf) af[mf] = *reinterpret_cast<const s8v*>(sh + sk_off(fa[mf] + ky * HWL + kx, q));
#pragma unroll
      for (int nf = 0; nf < FN; ++nf) {
        const s8v w = *reinterpret_cast<const s8v*>(sw + sk_off(tap * BN + nf * 32 + (lane & 31), q));
        bfg[nf] = live ? w : s8v{0, 0, 0, 0, 0, 0, 0, 0};
      }
    };
    auto mma = [&](const s8v (&af)[FM], const s8v (&bfg)[FN]) {
#pragma unroll
      for (int mf = 0; mf < FM; ++mf)
#pragma unroll
        for (int nf = 0; nf < FN; ++nf)
          acc[mf][nf] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[mf], bfg[nf], acc[mf][nf], 0, 0, 0);
    };
    s8v a0[FM], b0[FN], a1[FM], b1[FN];
    frag(0, a0, b0);
    frag(1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    frag(2, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    frag(3, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    frag(4, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, b0);
    if (ch + 1 < NCH) {                                       // halo of chunk ch + 1 -> the other halo stage
      __builtin_amdgcn_sched_barrier(0);                      // (the wait stays behind this chunk's MFMAs)
      if (ch + 2 < NCH) { if (wfull) sk_wait_vm<W_PER>(); else sk_wait_vm<W_PER - 1>(); }
      else sk_wait_vm<0>();
      tie_h();
      store_h(ch + 1);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();                                            // fragment reads done: the ring is free

  // ---- sum the four waves' partial tiles: red[w][n][m] fp32 (C/D map: col = lane & 31, rows (r & 3) + 8 (r >> 2)
  //      + 4 (lane >> 5)), then bias + bf16 into the C staging tile ----
  float* red = reinterpret_cast<float*>(smem);
  bf16_t (*sC)[LDC] = reinterpret_cast<bf16_t (*)[LDC]>(smem + S::RED_BYTES);
#pragma unroll
  for (int mf = 0; mf < FM; ++mf)
#pragma unroll
    for (int nf = 0; nf < FN; ++nf) {
      float* dst = red + ((size_t)wid * BN + nf * 32 + (lane & 31)) * S::RPITCH + mf * 32 + 4 * kh;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(dst + 8 * g) =
            make_float4(acc[mf][nf][4 * g], acc[mf][nf][4 * g + 1], acc[mf][nf][4 * g + 2], acc[mf][nf][4 * g + 3]);
    }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < BM * BN / 4 / NT; ++k) {           // item = (4 consecutive pixels, 1 channel)
    const int idx = tid + k * NT, n = idx % BN, m4 = (idx / BN) * 4;
    const float bias = p.bias ? p.bias[nBlock + n] : 0.f;
    float4 v = *reinterpret_cast<const float4*>(red + (size_t)n * S::RPITCH + m4);
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 t = *reinterpret_cast<const float4*>(red + ((size_t)w * BN + n) * S::RPITCH + m4);
      v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
    }
    sC[m4][n] = f2bf(v.x + bias);
    sC[m4 + 1][n] = f2bf(v.y + bias);
    sC[m4 + 2][n] = f2bf(v.z + bias);
    sC[m4 + 3][n] = f2bf(v.w + bias);
  }
  __syncthreads();

  // ---- epilogue (conv3x3.hip): plain store + BN statistics, BN-node gradient, or the decoder node join ----
  const int cg = tid % CG;
  const bool node = p.node.y != nullptr;
  NodeCoef nk;
  if (node) node_coef_load(p.node.ab, p.N, nBlock + cg * 8, nk);
  float s[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[0][q] = s[1][q] = 0.f;
  if constexpr (PJ) {
    float pm[8], pr[8];
    load_f8_or(p.pj.sab + 2 * p.N + nBlock + cg * 8, p.pj.sy != nullptr, 0.f, pm);
    load_f8_or(p.pj.sab + 3 * p.N + nBlock + cg * 8, p.pj.sy != nullptr, 0.f, pr);
    constexpr int HTW = TW / 2;
    if (pjok) {
      const int hr = tid / CG, hy = hr / HTW, hx = hr % HTW;
      uint4 o4[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) o4[q] = *reinterpret_cast<const uint4*>(&sC[(2 * hy + (q >> 1)) * TW + 2 * hx + (q & 1)][cg * 8]);
      *reinterpret_cast<uint4*>(p.pj.out + pjoff) = pool_join8(o4, pjv, pja, pjy, p.pj.add != nullptr,
                                                               p.pj.sy != nullptr, pm, pr, s[0], s[1]);
    }
  } else {
#pragma unroll
    for (int r0 = 0; r0 < BM; r0 += ROWS_PER_PASS) {
      const int row = r0 + tid / CG;
      const int m = (b * p.Ho + ty0 + row / TW) * p.Wo + tx0 + row % TW;
      const size_t off = (size_t)m * p.N + nBlock + cg * 8;
      uint4 v = *reinterpret_cast<const uint4*>(&sC[row][cg * 8]);
      if (node) {
        v = node_epi(v, p.node.y + off, nk, p.node.relu, s[0], s[1]);
      } else {
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          s[0][q] += f[q];
          s[1][q] += f[q] * f[q];
        }
      }
      *reinterpret_cast<uint4*>(p.y + off) = v;
    }
  }
  if (p.stats || node || (PJ && p.pj.sums)) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int o = CG; o < 64; o <<= 1) {
        s[0][q] = xor_add(s[0][q], o);
        s[1][q] = xor_add(s[1][q], o);
      }
    if (lane < CG) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        sred[0][wid][cg * 8 + q] = s[0][q];
        sred[1][wid][cg * 8 + q] = s[1][q];
      }
    }
    __syncthreads();
    float* rep = PJ ? p.pj.sums : node ? p.node.sums : p.stats;
    const int nrep = PJ ? (p.pj.reps > 1 ? p.pj.reps : 1) : node ? (p.node.reps > 1 ? p.node.reps : 1) : STAT_REPLICAS;
    const size_t ro = (size_t)(tile % nrep) * 2 * p.N;
    for (int e = tid; e < 2 * BN; e += NT) {
      const int st = e / BN, cc = e - st * BN;
      red_add(rep, ro + st * p.N + nBlock + cc, sred[st][0][cc] + sred[st][1][cc] + sred[st][2][cc] + sred[st][3][cc],
              red_scale(!PJ && !node, st));
    }
  }
}

template <int TH, int TW, int BN, int NCH>
int launch_sk_n(const ConvParams& p, hipStream_t st) {
  const int blocks = (p.Ho / TH) * (p.Wo / TW) * p.B * (p.N / BN);
  if (p.xfin.stats)
    hipLaunchKernelGGL((conv3x3_sk_kernel<TH, TW, BN, NCH, false, true>), dim3(blocks), dim3(NT), 0, st, p);
  else if (p.pj.v)
    hipLaunchKernelGGL((conv3x3_sk_kernel<TH, TW, BN, NCH, true, false>), dim3(blocks), dim3(NT), 0, st, p);
  else
    hipLaunchKernelGGL((conv3x3_sk_kernel<TH, TW, BN, NCH, false, false>), dim3(blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

template <int TH, int TW, int BN>
int launch_sk(const ConvParams& p, hipStream_t st) {
  switch (p.Cin / BK) {
    case 2: return launch_sk_n<TH, TW, BN, 2>(p, st);
    case 4: return launch_sk_n<TH, TW, BN, 4>(p, st);
    case 8: return launch_sk_n<TH, TW, BN, 8>(p, st);
  }
  return 1;
}

// tile configs: 1 = 8x8 px x 64 ch, 2 = 8x16 x 64, 4 = 8x16 x 32 (a 16x16 x 32 config measured slowest everywhere)
bool sk_cfg_fits(const ConvParams& p, int cfg) {
  switch (cfg) {
    case 1: return p.Ho % 8 == 0 && p.Wo % 8 == 0 && p.N % 64 == 0;
    case 2: return p.Ho % 8 == 0 && p.Wo % 16 == 0 && p.N % 64 == 0;
    case 4: return p.Ho % 8 == 0 && p.Wo % 16 == 0 && p.N % 32 == 0;
  }
  return false;
}

int sk_blocks(const ConvParams& p, int cfg) {
  const int tw = cfg == 1 ? 8 : 16, bn = cfg <= 2 ? 64 : 32;
  return (p.Ho / 8) * (p.Wo / tw) * p.B * (p.N / bn);
}

// default tile: the largest whole tile that still gives every CU a block (fewer weight re-reads per output)
int sk_pick(const ConvParams& p) {
  const int forced = cfl_tune(TUNE_CONV3_SK_CFG);
  if (forced > 0) return sk_cfg_fits(p, forced) ? forced : 0;
  for (int cfg : {2, 4, 1})
    if (sk_cfg_fits(p, cfg) && sk_blocks(p, cfg) >= 240) return cfg;
  return sk_cfg_fits(p, 1) ? 1 : 0;
}

}  // namespace

// Shapes: Cin = 64 / 128 / 256 (2, 4 or 8 chunks, compiled), maps tiled exactly by the config.
// TUNE_CONV3_SK: 0 = default, 1 = never, 2 = whenever the shape allows it, 3 = the low-resolution levels only.
bool conv3x3_sk_eligible(const ConvParams& p) {
  const int v = cfl_tune(TUNE_CONV3_SK);
  if (v == 1) return false;
  // another 3x3 kernel forced (tests / A/B sweeps) takes precedence over the default choice
  if (v == 0 && (cfl_tune(TUNE_CONV3_DEEP) == 2 || cfl_tune(TUNE_CONV3_SMALL) == 2 || cfl_tune(TUNE_CONV3_BIG) == 2 ||
                 cfl_tune(TUNE_CONV3_WS) == 2))
    return false;
  if (p.ks != 3 || p.stride != 1 || p.pad_t != 1 || p.pad_l != 1 || p.Cin % BK || p.K != 9 * p.Cin) return false;
  const int nch = p.Cin / BK;
  if (nch != 2 && nch != 4 && nch != 8) return false;        // compiled chunk counts
  if (p.Cin > SK_MAX_CIN) return false;                       // coefficient staging
  if (p.bwd.y || sk_pick(p) == 0) return false;
  if (p.xfin.stats && p.pj.v) return false;
  if (p.pj.v && (p.Ho % 2 || p.Wo % 2)) return false;
  // default: the 8-chunk (Cin = 256) convs of the <= 32^2 levels without the decoder node join. In-step per-position
  // trace A/B (tools/gpu_trace_ab.sh, 256^2 / b16): those five calls 1.5-1.9 / 0.3-0.4 us faster each; the Cin = 128
  // calls -0.1 .. +2.4 us and the node-join form +9.7 us (its join loads wait in front of the K loop), so not those.
  // Only at small M (<= 128k output pixels): at the 512^2 planned batch (1,096 images, M = 1.1M at 32^2) the four
  // such calls ran 2,627 / 2,742 us vs 1,732 / 1,898 us for the whole-chunk 8x16 kernel (profiles/r4_512) - with
  // that many tiles the in-block split of K only costs.
  // 3 = every low-resolution candidate (maps <= 32^2, Cin >= 128), 4 = 16^2 maps and 32^2 maps with N <= 128 (A/B).
  const bool low = p.Cin >= 128 && p.Ho * p.Wo <= 32 * 32;
  if (v == 0) return p.Cin == 256 && p.Ho * p.Wo <= 32 * 32 && (int64_t)p.B * p.Ho * p.Wo <= (1 << 17) && !p.pj.v;
  return v == 2 || (v == 3 && low) || (v == 4 && low && (p.Ho * p.Wo <= 16 * 16 || p.N <= 128));
}

int conv3x3_sk(const ConvParams& p, hipStream_t st) {
  if (!conv3x3_sk_eligible(p)) return 1;
  switch (sk_pick(p)) {
    case 1: return launch_sk<8, 8, 64>(p, st);
    case 2: return launch_sk<8, 16, 64>(p, st);
    case 4: return launch_sk<8, 16, 32>(p, st);
  }
  return 1;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_conv3x3_sk(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_conv3x3_sk(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
