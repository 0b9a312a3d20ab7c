// Deep-K 3x3 / stride-1 / "same" convolution for the low-resolution decoder levels (16^2 and 32^2 maps at 256^2 input:
// Cin = 128-256 -> K = 1152-2304, M = 4k-16k pixels), forward and data-gradient (/root/reference/client_fit_model.py
// :129,133). These layers are neither MFMA- nor HBM-bound: the per-tile halo kernel (conv3x3.hip) walks its 4-8
// input-channel chunks with ONE chunk in flight, so every chunk pays a full L2 / HBM latency (measured 10-16 % of
// the MFMA peak, 15-25 % of the roofline: profiles/r2_step1/roofline.txt, pmc_summary.txt).
// Here every chunk's operands - the 9 taps' 32 x 32 weight tiles and the (TH+2) x (TW+2) x 32 input halo - are
// copied global -> LDS by LDS-DMA loads (global_load_lds_dwordx4: no VGPR staging) into a 3-stage ring, so two
// chunks are in flight while the third is consumed. The DMA writes LDS lane-linearly; the XOR-swizzled images of
// conv3x3.hip (conflict-free fragment reads for any tap shift) are produced by permuting each lane's SOURCE address.
// Out-of-image halo pixels and pad rows read a 64-byte zero line. A producer BN-apply + ReLU (forward inputs) is
// applied in place in LDS after the chunk has landed (padding stays zero), one extra barrier per chunk.
// Waits: raw s_barrier + counted `s_waitcnt vmcnt` (a __syncthreads would drain every in-flight DMA:
// cdna_hip_programming.md §5 "Pipelining across barriers"); no other global load is issued inside the loop.
// Epilogue (bias, bf16, LDS-staged 16-byte stores, BN statistics / BN-node gradient) as conv3x3.hip.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr int BK = 32;                    // channels per chunk
constexpr int BN_ = 32;                   // output channels per block
constexpr int STAGES = 3;

__device__ __attribute__((aligned(64))) uint4 g_zero_line[4];   // 64 zero bytes: source of padding rows

CFL_DEVICE int swz_off(int r, int q) { return r * BK + ((q ^ ((r >> 1) & 2)) << 3); }

CFL_DEVICE void dma16(const void* src, bf16_t* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                   (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0, 0);
}

template <int N>
CFL_DEVICE void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// LDS store the compiler cannot see: hipcc orders every visible LDS store after ALL outstanding LDS-DMA loads
// (s_waitcnt vmcnt(0)), which would drain the two chunks in flight at every in-place halo transform. This store
// only touches the stage being consumed, never a stage a DMA is filling; the caller waits lgkmcnt before the barrier.
CFL_DEVICE void lds_store16(bf16_t* p, uint4 v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)p;
  const u4v d = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(d) : "memory");
}

constexpr int MAX_CIN = 512;              // producer BN coefficients staged in LDS

template <int TH, int TW, int WM, int WN>
__global__ __launch_bounds__(NT, 2) void conv3x3_deep_kernel(ConvParams p) {
  CFL_TS_GUARD;
  constexpr int BM = TH * TW;
  constexpr int HW = TW + 2, HP = (TH + 2) * HW;
  constexpr int TM = BM / WM, TN = BN_ / WN, FM = TM / 16, FN = TN / 16;
  constexpr int W_INS = 9 * BN_ / 16;                       // 1-KB DMA instructions per stage: weights (16 rows each)
  constexpr int H_INS = (HP + 15) / 16;                     // ... and halo
  constexpr int INS = W_INS + H_INS;
  constexpr int PW_MAX = (INS + 3) / 4, PW_REM = INS % 4;   // waves < PW_REM (or all, if 0) issue PW_MAX, others one less
  constexpr int STAGE = INS * 512;                          // bf16 elements per stage (1 KB per instruction)
  constexpr int LDC = BN_ + 8;
  static_assert(WM * WN == 4 && TM % 16 == 0 && TN % 16 == 0, "wave tiling");
  static_assert(BM * LDC <= STAGES * STAGE, "C staging tile must fit in the ring");

  // ONE shared object (a second one can make hipcc drain the DMAs before every ds_read: cdna_hip_programming.md §5)
  constexpr int RING_BYTES = STAGES * STAGE * 2, SRED_BYTES = 2 * 4 * BN_ * 4, SAB_BYTES = 2 * MAX_CIN * 4;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[RING_BYTES + SRED_BYTES + SAB_BYTES];
  bf16_t* ring = reinterpret_cast<bf16_t*>(smem);
  float (*sred)[4][BN_] = reinterpret_cast<float (*)[4][BN_]>(smem + RING_BYTES);
  float* sab = reinterpret_cast<float*>(smem + RING_BYTES + SRED_BYTES);   // [2][Cin]: a, b of the producer BN

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_w = p.Wo / TW, tiles_hw = tiles_w * (p.Ho / TH);
  const int lin = xcd_block_linear();                       // the column blocks of one pixel tile share an XCD
  const int nb = p.N / BN_;
  const int bn_idx = lin % nb, tile = lin / nb;
  const int b = tile / tiles_hw, tr = tile - b * tiles_hw;
  const int ty0 = (tr / tiles_w) * TH, tx0 = (tr % tiles_w) * TW;
  const int nBlock = bn_idx * BN_;
  const int chunks = p.Cin / BK;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;
  const bool xform = has_ab || relu;

  if (has_ab) {                                             // before any DMA: these are ordinary loads
    for (int c = tid; c < p.Cin; c += NT) {
      sab[c] = p.xf.ab[c];
      sab[MAX_CIN + c] = p.xf.ab[p.xf.C + c];
    }
  }
  __syncthreads();
  // ---- this lane's DMA sources, as (base pointer, per-chunk stride) pairs; instruction i = wid + 4 * j ----
  const bf16_t* src[PW_MAX];
  int cstep[PW_MAX];                                        // elements to advance per chunk (0: zero line)
#pragma unroll
  for (int j = 0; j < PW_MAX; ++j) {
    const int i = wid + 4 * j;
    if (i >= INS) {                                         // (this wave issues one instruction fewer)
      src[j] = reinterpret_cast<const bf16_t*>(g_zero_line);
      cstep[j] = 0;
    } else if (i < W_INS) {                                 // weights: row = tap*32 + n
      const int row = 16 * i + (lane >> 2), slot = lane & 3, q = slot ^ ((row >> 1) & 2);
      const int tap = row / BN_, n = row - tap * BN_;
      src[j] = p.wt + (size_t)(nBlock + n) * p.K + (size_t)tap * p.Cin + q * 8;
      cstep[j] = BK;
    } else {                                                // halo: row = halo pixel
      const int row = 16 * (i - W_INS) + (lane >> 2), slot = lane & 3, q = slot ^ ((row >> 1) & 2);
      const int hy = row / HW, hx = row - hy * HW;
      const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
      if (row < HP && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl) {
        src[j] = p.x + (((size_t)b * p.Hin + (iy >> p.up_in)) * p.Win + (ix >> p.up_in)) * p.Cin + q * 8;
        cstep[j] = BK;
      } else {
        src[j] = reinterpret_cast<const bf16_t*>(g_zero_line);
        cstep[j] = 0;
      }
    }
  }
  const bool full = PW_REM == 0 || wid < PW_REM;             // wave-uniform: this wave issues PW_MAX per chunk
  auto issue = [&](int ch) {                                // chunk ch -> ring stage ch % STAGES
    bf16_t* st = ring + (ch % STAGES) * STAGE;
#pragma unroll
    for (int j = 0; j < PW_MAX; ++j)
      if (j < PW_MAX - 1 || full) dma16(src[j] + ch * cstep[j], st + (wid + 4 * j) * 512);
  };

  // producer transform coefficients of the halo pieces this thread rewrites (chunk-dependent channel base)
  constexpr int HALO_PIECES = HP * 4, HPT = (HALO_PIECES + NT - 1) / NT;
  bool hvalid[HPT];
#pragma unroll
  for (int k = 0; k < HPT; ++k) {
    const int e = tid + k * NT, row = e >> 2;
    const int hy = row / HW, hx = row - hy * HW;
    const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
    hvalid[k] = e < HALO_PIECES && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl;
  }
  auto transform_halo = [&](int ch) {                       // in place: a*x + b, ReLU on in-image pixels
    bf16_t* sh = ring + (ch % STAGES) * STAGE + W_INS * 512;
#pragma unroll
    for (int k = 0; k < HPT; ++k) {
      if (!hvalid[k]) continue;
      const int e = tid + k * NT, row = e >> 2, slot = e & 3, q = slot ^ ((row >> 1) & 2);
      const int cq = ch * BK + q * 8;                       // slot `slot` of a row holds channel quarter q
      bf16_t* ptr = sh + row * BK + slot * 8;
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(ptr), f);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        if (has_ab) f[jj] = fmaf(sab[cq + jj], f[jj], sab[MAX_CIN + cq + jj]);
        if (relu) f[jj] = fmaxf(f[jj], 0.f);
      }
      lds_store16(ptr, pack8(f));
    }
  };

  int fhp[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pp = wm * TM + i * 16 + (lane & 15);
    fhp[i] = (pp / TW) * HW + pp % TW;
  }
  const int fq = lane >> 4;
  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  // prologue: STAGES - 1 chunks in flight
  issue(0);
  if (chunks > 1) issue(1);
  for (int ch = 0; ch < chunks; ++ch) {
    // chunk ch has landed once at most the DMAs of chunk ch + 1 (issued earlier) are outstanding
    if (ch + 1 < chunks) {
      if (full) wait_vm<PW_MAX>();
      else wait_vm<PW_MAX - 1>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();                           // every wave's part landed; stage (ch-1) % 3 is free
    if (ch + 2 < chunks) issue(ch + 2);
    if (xform) {
      transform_halo(ch);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    const bf16_t* sw = ring + (ch % STAGES) * STAGE;
    const bf16_t* sh = sw + W_INS * 512;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int ky = tap / 3, kx = tap - ky * 3;
      s8v af[FM], bfg[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const s8v*>(sh + swz_off(fhp[i] + ky * HW + kx, fq));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfg[j] = *reinterpret_cast<const s8v*>(sw + swz_off(tap * BN_ + wn * TN + j * 16 + (lane & 15), fq));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();                             // all fragment reads done: the ring becomes C staging

  bf16_t (*sC)[LDC] = reinterpret_cast<bf16_t (*)[LDC]>(ring);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int cl = wn * TN + j * 16 + (lane & 15);
    const float bias = p.bias ? p.bias[nBlock + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) sC[wm * TM + i * 16 + (lane >> 4) * 4 + r][cl] = f2bf(acc[i][j][r] + bias);
  }
  __syncthreads();
  constexpr int CG = BN_ / 8, ROWS_PER_PASS = NT / CG;
  const int cg = tid % CG;
  const bool node = p.node.y != nullptr;
  NodeCoef nk;
  if (node) node_coef_load(p.node.ab, p.N, nBlock + cg * 8, nk);
  float s[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[0][q] = s[1][q] = 0.f;
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
  if (p.stats || node) {
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
    float* rep = node ? p.node.sums : p.stats;
    const size_t ro = (size_t)(tile % (node ? (p.node.reps > 1 ? p.node.reps : 1) : STAT_REPLICAS)) * 2 * p.N;
    for (int e = tid; e < 2 * BN_; e += NT) {
      const int st = e / BN_, cc = e - st * BN_;
      red_add(rep, ro + st * p.N + nBlock + cc, sred[st][0][cc] + sred[st][1][cc] + sred[st][2][cc] + sred[st][3][cc],
              red_scale(!node, st));
    }
  }
}

}  // namespace

// Used where it measured faster (tools/kbench.py at 256^2 / B16, profiles/README.md): the 16^2-level data
// gradients (Cin 256, no producer transform): 16.8 / 14.1 -> 13.4 / 11.1 us. With a producer transform (the in-place
// LDS pass + barrier per chunk) or on the 32^2 / 64^2 levels (8x8 tiles vs the per-tile kernel's 8x16) it was
// 1.3-2.1x SLOWER, so those stay on conv3x3.hip. TUNE_CONV3_DEEP: 1 = never, 2 = whenever the shape allows (tests).
bool conv3x3_deep_eligible(const ConvParams& p) {
  const int v = cfl_tune(TUNE_CONV3_DEEP);
  if (v == 1) return false;
  if (p.ks != 3 || p.stride != 1 || p.pad_t != 1 || p.pad_l != 1 || p.Cin % BK || p.N % BN_) return false;
  if (p.Ho % 8 || p.Wo % 8 || p.K != 9 * p.Cin) return false;
  return v == 2 || (p.Cin >= 256 && p.Ho * p.Wo <= 256 && p.xf.ab == nullptr && !p.xf.relu && !p.up_in);
}

int conv3x3_deep(const ConvParams& p, hipStream_t st) {
  if (!conv3x3_deep_eligible(p) || p.Cin > MAX_CIN) return 1;
  const int blocks = (p.Ho / 8) * (p.Wo / 8) * p.B * (p.N / BN_);     // 8x8-pixel x 32-channel tiles, 2 blocks / CU
  hipLaunchKernelGGL((conv3x3_deep_kernel<8, 8, 2, 2>), dim3(blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_conv3x3_deep(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_conv3x3_deep(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
