// Convolution weight gradient on gfx950 MFMA:  dW[k][n] = sum_m im2col(T(x))[m][k] * dy[m][n].
//
// The reduction runs over pixels (M = B*Ho*Wo, up to millions), which in NHWC is the OUTER dimension of both
// operands. Both tiles are therefore staged in their natural [m][k] / [m][n] row layout (16-byte coalesced
// global loads, the producer's BN-apply + ReLU folded into the x load with coefficients held in registers - a
// block's k range is fixed, so each thread's channels never change) and the MFMA operands - which need 8
// consecutive m per lane - are read with the CDNA4 transposing LDS read ds_read_b64_tr_b16
// (__builtin_amdgcn_ds_read_tr16_b64): no register or LDS transpose pass.
//
// Output tile BKO(k) x BNO(n) (128x128 for the big K*N layers, down to 32x32), 4 waves 2x2, reduction step 32
// pixels, register-staged double buffer. The M range is split over gridDim.z so the grid holds ~512 long-running
// blocks; partial tiles are combined with fp32 atomics into the layer's slot of the flat gradient buffer (or into
// WGRAD_REPLICAS replica rows summed by grad_finish), writing Keras layouts (HWIO for Conv2D / pointwise; (kh,kw,out,in) with the spatial flip for Conv2DTranspose).
#include <cstdio>

#include "common.h"
#include "launch.h"
#include "wgrad3_body.h"

namespace {

constexpr int NT = 256;

typedef short s4v_lds __attribute__((ext_vector_type(4)));

CFL_DEVICE s4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4v_lds __attribute__((address_space(3)))*)(p));
}

// RM: pixels per pipeline stage (32 = one MFMA k-step; 128 = four k-steps per barrier and 4x the bytes in flight
// per stage for the small K x N tiles, which are latency-bound at 32)
template <int BKO, int BNO, int RM>
constexpr int wgrad_lds_bytes() { return 2 * RM * (BKO + 16) * 2 + 2 * RM * (BNO + 16) * 2; }

// DIRECT: a 1x1 / stride-1 / unpadded / not-upsampled conv (x pixel m = output pixel m): a step's x and dy rows are
// contiguous, read with raw buffer loads from per-step scalar resources whose range ends at the block's last pixel
// (past it both read 0 - a dy row of 0 contributes nothing whatever its x row holds), so a chunk costs no address
// math, no validity bits and no masking; the x transform runs on packed fp32 FMAs (common.h xform2). The
// general form decodes each chunk row's (b, oh, ow), builds 64-bit addresses and carries per-lane row counters:
// ~30 VALU ops per chunk against 8 MFMAs per wave per step in the <64, 32, 128> config.
constexpr bool wgrad_direct(const WgradParams& p) {
  return p.ks == 1 && p.stride == 1 && p.pad_t == 0 && p.pad_l == 0 && p.up_in == 0 && p.K == p.Cin;
}

template <int BKO, int BNO, int RM, bool DIRECT = false>
CFL_DEVICE void wgrad_body(const WgradParams& p, int chunk, int bx, int by, int bz, unsigned char* smem) {
  constexpr int TK = BKO / 2, TN = BNO / 2;
  constexpr int FK = TK / 16, FN = TN / 16;
  // LDS rows of 96 / 160 / 288 bytes (32 x odd): the 32 lanes of each ds_read_b64_tr_b16 read 8 CONSECUTIVE pixel
  // rows x 32 bytes (k-slot order below), which then cover all 64 banks. The previous 80-144-byte rows with rows
  // {8g+q, 8g+q+4} per lane group left 2-way conflicts: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 33-40 %
  // (profiles/r2_step1/pmc_summary.txt) - the same fix conv3x3_wgrad.hip got in round 1.
  constexpr int LDX = BKO + 16, LDG = BNO + 16;
  constexpr int XC = RM * BKO / 8, GC = RM * BNO / 8;   // 16-byte chunks per tile
  constexpr int XPT = (XC + NT - 1) / NT, GPT = (GC + NT - 1) / NT;
  bf16_t (*sX)[RM][LDX] = reinterpret_cast<bf16_t (*)[RM][LDX]>(smem);
  bf16_t (*sG)[RM][LDG] = reinterpret_cast<bf16_t (*)[RM][LDG]>(smem + 2 * RM * LDX * 2);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wk = wid >> 1, wn = wid & 1;
  const int kBlock = bx * BKO, nBlock = by * BNO;
  const int m_begin = bz * chunk;
  const int m_end = imin(p.M, m_begin + chunk);
  if (m_begin >= m_end) return;
  const int HWo = p.Ho * p.Wo;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;

  // x chunks: fixed channel group (k range of this block), rows xm + i * (NT / (BKO/8))
  constexpr int XW = BKO / 8;
  const int xk = kBlock + (tid % XW) * 8;
  const int tap = xk / p.Cin, xc = xk - tap * p.Cin;
  const int ky = tap / p.ks, kx = tap - ky * p.ks;
  const bool has_ab = p.xf.ab != nullptr;
  float ca[8], cb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ca[j] = has_ab ? p.xf.ab[xc + j] : 1.f;
    cb[j] = has_ab ? p.xf.ab[p.xf.C + xc + j] : 0.f;
  }
  constexpr int GW = BNO / 8;
  const int gn = nBlock + (tid % GW) * 8;

  // pixel decode (b, oh, ow) of each x chunk row, advanced incrementally by RM per step (no division in the loop)
  int db[XPT], doh[XPT], dow[XPT];
#pragma unroll
  for (int i = 0; i < (DIRECT ? 0 : XPT); ++i) {
    const int m = m_begin + (tid + i * NT) / XW;
    db[i] = m / HWo;
    const int r = m - db[i] * HWo;
    doh[i] = r / p.Wo;
    dow[i] = r - doh[i] * p.Wo;
  }
  // loaded RAW and branch-free (clamped addresses, validity bits); masked + transformed in store(), after the MFMAs
  // that the prefetch should overlap (see wgrad3_body.h)
  uint4 rx[XPT], rg[GPT];
  uint32_t xval = 0, gval = 0;
  const uint32_t relu_lo = p.xf.relu ? 0u : 0x80008000u;
  auto load = [&](int m0) {
    if constexpr (DIRECT) {
      // resources from the block's first channel of the step's first pixel (uniform) to the block's last pixel
      const int rows = m_end - m0;
      const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.x + (size_t)m0 * p.Cin + kBlock), 0, (rows * p.Cin - kBlock) * 2, 0x00020000);
      const __amdgpu_buffer_rsrc_t rs_g = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(p.dy + (size_t)m0 * p.N + nBlock), 0, (rows * p.N - nBlock) * 2, 0x00020000);
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int ch = tid + i * NT;
        const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs_x, (ch / XW) * p.Cin * 2 + (ch % XW) * 16, 0, 0);
        rx[i] = make_uint4(v.x, v.y, v.z, v.w);
      }
#pragma unroll
      for (int i = 0; i < GPT; ++i) {
        const int ch = tid + i * NT;
        const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs_g, (ch / GW) * p.N * 2 + (ch % GW) * 16, 0, 0);
        rg[i] = make_uint4(v.x, v.y, v.z, v.w);
      }
      return;
    }
    xval = 0;
    gval = 0;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int ch = tid + i * NT;
      const int m = m0 + ch / XW;
      const int b = db[i], oh = doh[i], ow = dow[i];
      const int ih = oh * p.stride - p.pad_t + ky, iw = ow * p.stride - p.pad_l + kx;
      const bool ok = ch < XC && m < m_end && ih >= 0 && ih < Hl && iw >= 0 && iw < Wl;
      // (rows past m_end decode past the last image: clamp the image too)
      const int bc = imin(b, p.B - 1), ihc = imin(imax(ih, 0), Hl - 1), iwc = imin(imax(iw, 0), Wl - 1);
      rx[i] = *reinterpret_cast<const uint4*>(
          p.x + (((size_t)bc * p.Hin + (ihc >> p.up_in)) * p.Win + (iwc >> p.up_in)) * p.Cin + xc);
      xval |= (uint32_t)ok << i;
      dow[i] += RM;                       // advance this chunk row to the next step's pixel
      while (dow[i] >= p.Wo) {
        dow[i] -= p.Wo;
        if (++doh[i] == p.Ho) {
          doh[i] = 0;
          ++db[i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int ch = tid + i * NT;
      const int m = m0 + ch / GW;
      const bool ok = ch < GC && m < m_end;
      rg[i] = *reinterpret_cast<const uint4*>(p.dy + (size_t)imin(m, p.M - 1) * p.N + gn);
      gval |= (uint32_t)ok << i;
    }
  };
  auto store = [&](int buf) {
    if constexpr (DIRECT) {
#pragma unroll
      for (int i = 0; i < XPT; ++i) {
        const int ch = tid + i * NT;
        if (ch < XC) {
          const uint4 v = rx[i];
          uint4 o;
          o.x = xform2(v.x, f32x2_t{ca[0], ca[1]}, f32x2_t{cb[0], cb[1]}, relu_lo);
          o.y = xform2(v.y, f32x2_t{ca[2], ca[3]}, f32x2_t{cb[2], cb[3]}, relu_lo);
          o.z = xform2(v.z, f32x2_t{ca[4], ca[5]}, f32x2_t{cb[4], cb[5]}, relu_lo);
          o.w = xform2(v.w, f32x2_t{ca[6], ca[7]}, f32x2_t{cb[6], cb[7]}, relu_lo);
          *reinterpret_cast<uint4*>(&sX[buf][ch / XW][(ch % XW) * 8]) = o;
        }
      }
#pragma unroll
      for (int i = 0; i < GPT; ++i) {
        const int ch = tid + i * NT;
        if (ch < GC) *reinterpret_cast<uint4*>(&sG[buf][ch / GW][(ch % GW) * 8]) = rg[i];
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int ch = tid + i * NT;
      if (ch < XC) {
        // packed transform (common.h xform8), padding / rows past the block exactly 0
        *reinterpret_cast<uint4*>(&sX[buf][ch / XW][(ch % XW) * 8]) =
            xform8(rx[i], ca, cb, relu_lo, ((xval >> i) & 1u) ? 0xffffffffu : 0u);
      }
    }
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int ch = tid + i * NT;
      if (ch < GC) *reinterpret_cast<uint4*>(&sG[buf][ch / GW][(ch % GW) * 8]) = ((gval >> i) & 1u) ? rg[i]
                                                                                                  : make_uint4(0, 0, 0, 0);
    }
  };

  f4v acc[FK][FN];
#pragma unroll
  for (int i = 0; i < FK; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  load(m_begin);
  store(0);
  __syncthreads();
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  int buf = 0;
  for (int m0 = m_begin; m0 < m_end; m0 += RM) {
    const bool more = m0 + RM < m_end;
    if (more) load(m0 + RM);
#pragma unroll
    for (int ks = 0; ks < RM / 32; ++ks) {
      // this lane's pixel rows: r0 (elements 0-3) and r0 + 16 (elements 4-7); the same pixel -> k-slot permutation
      // on both operands, so the reduction is unchanged
      const int r0 = 32 * ks + 4 * g + q;
      s8v af[FK], bfg[FN];
#pragma unroll
      for (int i = 0; i < FK; ++i) {
        const int kc = wk * TK + i * 16 + 4 * pq;
        const s4v lo = tr_read(&sX[buf][r0][kc]);
        const s4v hi = tr_read(&sX[buf][r0 + 16][kc]);
        af[i] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int nc = wn * TN + j * 16 + 4 * pq;
        const s4v lo = tr_read(&sG[buf][r0][nc]);
        const s4v hi = tr_read(&sG[buf][r0 + 16][nc]);
        bfg[j] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < FK; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // epilogue: D[k][n], col n = lane&15, row k = (lane>>4)*4 + r; slab mode spreads the split blocks' atomics
  // over replica rows (every block adding into ONE row serialises at the memory-side atomic units)
  const size_t ro = p.slabs > 0 ? (size_t)(bz % p.slabs) * p.K * p.N : 0;
#pragma unroll
  for (int i = 0; i < FK; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nBlock + wn * TN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = kBlock + wk * TK + i * 16 + (lane >> 4) * 4 + r;
        size_t dst;
        if (p.dst_mode == 1) {
          const int t = k / p.Cin, c = k - t * p.Cin;
          dst = ((size_t)(p.ks * p.ks - 1 - t) * p.N + n) * p.Cin + c;
        } else {
          dst = (size_t)k * p.N + n;
        }
        red_add(p.dw, ro + dst, acc[i][j][r], CFL_FX_G);
      }
    }
}

template <int BKO, int BNO, int RM>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_kernel(WgradParams p, int chunk) {
  CFL_TS_GUARD;
  __shared__ __attribute__((aligned(16))) unsigned char smem[wgrad_lds_bytes<BKO, BNO, RM>()];
  wgrad_body<BKO, BNO, RM>(p, chunk, blockIdx.x, blockIdx.y, blockIdx.z, smem);
}

// pixels per block (multiple of rm) and M splits of a generic weight gradient with a bko x bno output tile
void wgrad_shape(const WgradParams& p, int bko, int bno, int rm, int& chunk, int& zs) {
  const int tiles = (p.K / bko) * (p.N / bno);
  chunk = p.m_chunk;
  if (chunk <= 0) {
    // 320 blocks per layer: the deferred wgrads of a step are launched grouped (launch_group), so a layer's grid
    // need not fill the chip alone - fewer, longer blocks than 512 halve the replica-row atomics (whole-step A/B:
    // 1.691 -> 1.676 ms/iteration vs 512, profiles/README.md); re-swept after the round-2 folds: 256 / 320 / 384 /
    // 448 -> 1.4255-1.4340 / 1.4176-1.4187 / 1.4197-1.4201 / 1.4324-1.4345 ms
    const int target = cfl_tune(TUNE_WGRAD1_BLOCKS) > 0 ? cfl_tune(TUNE_WGRAD1_BLOCKS) : 320;
    const int minpix = cfl_tune(TUNE_WGRAD1_MINPIX) > 0 ? cfl_tune(TUNE_WGRAD1_MINPIX) : 512;
    int splits = (target + tiles - 1) / tiles;
    const int max_splits = (p.M + minpix - 1) / minpix;   // keep >= minpix pixels per block (512: 4 RM=128 stages)
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    chunk = (p.M + splits - 1) / splits;
  }
  chunk = (chunk + rm - 1) / rm * rm;
  zs = (p.M + chunk - 1) / chunk;
}

template <int BKO, int BNO, int RM = 32>
void launch(const WgradParams& p, hipStream_t st) {
  int chunk, zs;
  wgrad_shape(p, BKO, BNO, RM, chunk, zs);
  dim3 grid(p.K / BKO, p.N / BNO, zs);
  hipLaunchKernelGGL((conv_wgrad_kernel<BKO, BNO, RM>), grid, dim3(NT), 0, st, p, chunk);
}

// Grouped launch of several independent generic (1x1 / strided) weight gradients of ONE tile config: the deferred
// pointwise and residual-conv wgrads of a step are latency-bound grids of 64-512 blocks each (the low-resolution
// layers hold few pixels per block), so issued together their blocks co-run (the 3x3 halo ones are grouped the same
// way in conv3x3_wgrad.hip).
constexpr int WG1_MAX = 16;
struct WgradItem {
  WgradParams p;
  int chunk, gx, gy, block0;
};
struct WgradGroup {
  WgradItem it[WG1_MAX];
  int n;
};

template <int BKO, int BNO, int RM>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_group_kernel(const WgradGroup g) {
  CFL_TS_GUARD;
  __shared__ __attribute__((aligned(16))) unsigned char smem[wgrad_lds_bytes<BKO, BNO, RM>()];
  int k = 0;
  while (k + 1 < g.n && g.it[k + 1].block0 <= (int)blockIdx.x) ++k;
  const WgradItem& I = g.it[k];
  const int local = blockIdx.x - I.block0;
  const int bx = local % I.gx, r = local / I.gx;
  wgrad_body<BKO, BNO, RM>(I.p, I.chunk, bx, r % I.gy, r / I.gy, smem);
}

// tile config of a generic weight gradient (see conv_wgrad) and its (BKO, BNO, RM)
int wgrad_config(const WgradParams& p, int& bko, int& bno, int& rm) {
  const bool k128 = p.K % 128 == 0, n128 = p.N % 128 == 0;
  if (k128 && n128 && (int64_t)p.K * p.N >= 128 * 128 * 16) { bko = 128; bno = 128; rm = 32; return 0; }
  // K, N % 128 == 0 at large M (the wide pointwise / residual layers at 512^2): 128x128 output tiles with 64-pixel
  // stages - each operand is re-read N/128 resp. K/128 times instead of N/64, K/64 and a wave issues 16 MFMAs per
  // 32-pixel k-step instead of 4. tools/kbench.py at 512^2 / batch 256: 64x64 / 128x128 (32-px stages) / 128x128
  // (64-px stages) = 890.7 / 454.8 / 382.4 us (64^2, 256->256), 902.8 / 492.0 / 388.2 us (128^2, 128->128),
  // 224.9 / 120.0 / 115.1 us (32^2, 256->256). TUNE_WGRAD1_BIG: 1 = 64x64 tiles, 2 = 32-pixel stages.
  // Round 6: at every M (was M >= 64k): the low-resolution 256-channel layers at 256^2 / batch 16 (32^2 256 -> 256,
  // 128 -> 256, 16^2 256 -> 256 / 128) re-read x and dy K/64 resp. N/64 times on 64x64 tiles and were the mixed
  // launch's least efficient items (~3x the block time per MB of a streaming item, tools/mix_timeline.py); 128x128
  // tiles: their slot time 8.2k -> 3.9k block-us, the mixed launch 136.8 -> 127.9 us in the step
  // (profiles/r6_wgrad/trace_ab_big3.txt)
  const int big = cfl_tune(TUNE_WGRAD1_BIG);
  if (big != 1 && k128 && n128) {
    bko = 128; bno = 128;
    rm = big == 2 ? 32 : 64;
    return big == 2 ? 0 : 6;
  }
  rm = 128;
  if (p.K % 64 == 0 && p.N % 64 == 0) {
    bko = 64; bno = 64;
    // 64-pixel stages: 40 instead of 80 KB of LDS, 4 blocks per CU instead of 2 (whole step 1.524 -> 1.507 ms)
    if (cfl_tune(TUNE_WGRAD1_RM) == 128) return 1;
    rm = 64;
    return 5;
  }
  if (p.K % 64 == 0) { bko = 64; bno = 32; return 2; }
  if (p.N % 64 == 0) { bko = 32; bno = 64; return 3; }
  bko = 32; bno = 32;
  return 4;
}

template <int BKO, int BNO, int RM>
int launch_group(const WgradParams* ps, int n, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += WG1_MAX) {
    WgradGroup g{};
    int blocks = 0;
    for (int i = i0; i < n && i < i0 + WG1_MAX; ++i) {
      WgradItem& it = g.it[g.n++];
      it.p = ps[i];
      int zs;
      wgrad_shape(ps[i], BKO, BNO, RM, it.chunk, zs);
      it.gx = ps[i].K / BKO;
      it.gy = ps[i].N / BNO;
      it.block0 = blocks;
      blocks += it.gx * it.gy * zs;
    }
    hipLaunchKernelGGL((conv_wgrad_group_kernel<BKO, BNO, RM>), dim3(blocks), dim3(NT), 0, st, g);
    if (hipGetLastError() != hipSuccess) return 3;
  }
  return 0;
}

// Mixed launch: every deferred weight gradient of a step - the 3x3 halo ones (wgrad3_body.h) and the generic 1x1 /
// strided ones of every tile config - in ONE grid. Alone (or grouped per config, five launches) each is a
// latency-bound grid that leaves the chip part-idle in its tail; in one grid the blocks of all of them co-run and
// the four launch boundaries between the groups are gone. One LDS buffer sized for the largest body (the 64-wide
// halo config, 75.5 KB: 2 blocks per CU, as the halo groups had); the kernel's VGPR count is the largest body's.
// kind: 0-9 halo config (conv3x3_wgrad_config; 6-9 the 64-channel blocks), 10 + c
// generic config c (wgrad_config; 20 + c: its DIRECT form, wgrad_body; c = 1, the 80 KB
// 128-pixel-stage variant, is launched on its own)
constexpr int MIX_MAX = 24;
struct MixItem {
  WgradParams p;
  int kind;
  int a, b;                 // halo: pixel tiles, pixel splits; generic: pixels per block, unused
  int gx, gy, block0;
};
struct MixGroup {
  MixItem it[MIX_MAX];
  int n;
  int xcd;                  // XCD-grouped block order (TUNE_WGRAD_MIX_XCD != 1)
};
constexpr int cmax(int a, int b) { return a > b ? a : b; }
constexpr int MIX_LDS = cmax(cmax(cmax(cmax(wg3::wgrad3_lds_bytes<64>(), wg3::wgrad3_lds_bytes<64, 64, true>()),
                                       wgrad_lds_bytes<128, 128, 32>()),
                                  wgrad_lds_bytes<128, 128, 64>()),
                             cmax(cmax(wgrad_lds_bytes<64, 32, 128>(), wgrad_lds_bytes<32, 64, 128>()),
                                  cmax(wgrad_lds_bytes<32, 32, 128>(), wgrad_lds_bytes<64, 64, 64>())));
static_assert(MIX_LDS <= 80 * 1024, "two mixed blocks per CU");

__global__ __launch_bounds__(NT, 2) void wgrad_mix_kernel(const MixGroup g) {
  CFL_TS_GUARD;
  __shared__ __attribute__((aligned(16))) unsigned char smem[MIX_LDS];
  // XCD grouping: within every 64 dispatch slots, each XCD runs 8 consecutive logical blocks - the (up to 8) input-
  // channel blocks of one pixel split, which read the same dy tile, share an XCD's L2 and run at the same time (round-
  // robin dispatch spread them over 8 L2s: FETCH_SIZE of the mixed launch ~850 MB per step)
  const int base = blockIdx.x & ~63, span = imin(64, (int)gridDim.x - base);
  const int vb = base + (g.xcd ? xcd_swizzle(blockIdx.x & 63, span) : (blockIdx.x & 63));
  int k = 0;
  while (k + 1 < g.n && g.it[k + 1].block0 <= vb) ++k;
  // the item is copied out of the argument block first (a reference into it, indexed by a runtime k, made the
  // compiler spill the whole 3 KB block to scratch)
  const WgradParams P = g.it[k].p;
  const int kind = g.it[k].kind, a = g.it[k].a, b = g.it[k].b, gx = g.it[k].gx, gy = g.it[k].gy;
  const int local = vb - g.it[k].block0;
  const int bx = local % gx, r = local / gx, by = r % gy, bz = r / gy;
  switch (kind) {
    case 0: wg3::wgrad3_body<64, true>(P, a, b, bx, by, bz, smem); break;
    case 1: wg3::wgrad3_body<64, false>(P, a, b, bx, by, bz, smem); break;
    case 2: wg3::wgrad3_body<32, true>(P, a, b, bx, by, bz, smem); break;
    case 3: wg3::wgrad3_body<32, false>(P, a, b, bx, by, bz, smem); break;
    case 6: wg3::wgrad3_body<64, true, 64, true>(P, a, b, bx, by, bz, smem); break;
    case 7: wg3::wgrad3_body<64, false, 64, true>(P, a, b, bx, by, bz, smem); break;
    case 8: wg3::wgrad3_body<32, true, 64, true>(P, a, b, bx, by, bz, smem); break;
    case 9: wg3::wgrad3_body<32, false, 64, true>(P, a, b, bx, by, bz, smem); break;
    case 20: wgrad_body<128, 128, 32, true>(P, a, bx, by, bz, smem); break;
    case 26: wgrad_body<128, 128, 64, true>(P, a, bx, by, bz, smem); break;
    case 22: wgrad_body<64, 32, 128, true>(P, a, bx, by, bz, smem); break;
    case 23: wgrad_body<32, 64, 128, true>(P, a, bx, by, bz, smem); break;
    case 24: wgrad_body<32, 32, 128, true>(P, a, bx, by, bz, smem); break;
    case 25: wgrad_body<64, 64, 64, true>(P, a, bx, by, bz, smem); break;
    case 10: wgrad_body<128, 128, 32>(P, a, bx, by, bz, smem); break;
    case 16: wgrad_body<128, 128, 64>(P, a, bx, by, bz, smem); break;
    case 12: wgrad_body<64, 32, 128>(P, a, bx, by, bz, smem); break;
    case 13: wgrad_body<32, 64, 128>(P, a, bx, by, bz, smem); break;
    case 14: wgrad_body<32, 32, 128>(P, a, bx, by, bz, smem); break;
    default: wgrad_body<64, 64, 64>(P, a, bx, by, bz, smem); break;   // 15
  }
}

}  // namespace

bool conv3x3_wgrad_supported(const WgradParams& p);
int conv3x3_wgrad(const WgradParams& p, hipStream_t st);
int conv3x3_wgrad_splits(const WgradParams& p);

int conv_wgrad_slabs(const WgradParams& p) {
  if (p.algo != 1 && conv3x3_wgrad_supported(p)) return conv3x3_wgrad_splits(p);
  return cfl_tune(TUNE_WGRAD_REPS) > 0 ? cfl_tune(TUNE_WGRAD_REPS) : WGRAD_REPLICAS;
}

bool conv_wgrad_plain_slabs(const WgradParams& p) { return p.algo != 1 && conv3x3_wgrad_supported(p); }

int conv3x3_wgrad_config(const WgradParams& p);
int conv3x3_wgrad_cbt(const WgradParams& p);
int conv3x3_wgrad_grouped(const WgradParams* ps, int n, hipStream_t st);
void conv3x3_wgrad_shape(const WgradParams& p, int& bno, int& tiles, int& splits);

static bool generic_ok(const WgradParams& p) {
  return p.Cin % 8 == 0 && p.K == p.ks * p.ks * p.Cin && p.K % 32 == 0 && p.N % 32 == 0;
}

// the mixed launches of conv_wgrad_batch: halo items first (the longest blocks start first), MIX_MAX per launch
static int launch_mix(const WgradParams* ps, int n, hipStream_t st) {
  MixGroup g{};
  int blocks = 0;
  auto flush = [&]() -> int {
    if (g.n == 0) return 0;
    g.xcd = cfl_tune(TUNE_WGRAD_MIX_XCD) != 1;
    hipLaunchKernelGGL(wgrad_mix_kernel, dim3(blocks), dim3(NT), 0, st, g);
    g = MixGroup{};
    blocks = 0;
    return hipGetLastError() == hipSuccess ? 0 : 3;
  };
  const int only = cfl_tune(TUNE_WGRAD_MIX_ONLY), skip = cfl_tune(TUNE_WGRAD_MIX_SKIP);
  static bool listed = false;
  const bool list = cfl_tune(TUNE_WGRAD_MIX_LIST) == 1 && !listed;
  // item order (TUNE_WGRAD_MIX_ORDER): 2 (default) = halo and generic items alternating (the MFMA-heavy long halo
  // blocks and the HBM-heavy generic ones co-resident from the start: 155 vs 160 us per launch, two trace A/Bs), 3 =
  // every halo item first (the longest blocks start first), 1 = the generic items first (202 us)
  int order[64], no = 0, hl[64], gl[64], nh = 0, ngn = 0;
  for (int i = 0; i < n && i < 64; ++i) {
    if (ps[i].algo != 1 && conv3x3_wgrad_supported(ps[i])) hl[nh++] = i;
    else gl[ngn++] = i;
  }
  const int mode = cfl_tune(TUNE_WGRAD_MIX_ORDER) > 0 ? cfl_tune(TUNE_WGRAD_MIX_ORDER) : 2;
  if (mode == 2) {
    for (int a = 0, b = 0; a < nh || b < ngn;) {
      if (a < nh) order[no++] = hl[a++];
      if (b < ngn) order[no++] = gl[b++];
    }
  } else {
    const int* first = mode == 1 ? gl : hl;
    const int* second = mode == 1 ? hl : gl;
    const int n1 = mode == 1 ? ngn : nh, n2 = mode == 1 ? nh : ngn;
    for (int a = 0; a < n1; ++a) order[no++] = first[a];
    for (int a = 0; a < n2; ++a) order[no++] = second[a];
  }
  int idx = -1;
  for (int oi = 0; oi < no; ++oi) {
    {
      const int i = order[oi];
      const WgradParams& p = ps[i];
      const bool halo = p.algo != 1 && conv3x3_wgrad_supported(p);
      ++idx;
      if ((only > 0 && idx != only - 1) || (idx < 31 && ((skip >> idx) & 1))) continue;   // timing experiments
      if (g.n == MIX_MAX) {
        const int rc = flush();
        if (rc) return rc;
      }
      MixItem& it = g.it[g.n++];
      it.p = p;
      int zs;
      if (halo) {
        int bno;
        conv3x3_wgrad_shape(p, bno, it.a, it.b);
        if (p.slabs > 0 && p.slabs != it.b) return 2;
        it.kind = conv3x3_wgrad_config(p);
        it.gx = p.Cin / conv3x3_wgrad_cbt(p);
        it.gy = p.N / bno;
        zs = it.b;
      } else {
        int bko, bno, rm;
        const int cfg = wgrad_config(p, bko, bno, rm);
        wgrad_shape(p, bko, bno, rm, it.a, zs);
        // the direct body's per-step buffer ranges (a block's remaining rows x channels) must fit 31 bits
        const bool direct = wgrad_direct(p) && cfl_tune(TUNE_WGRAD_DIRECT) != 1 &&
                            (int64_t)it.a * (p.Cin > p.N ? p.Cin : p.N) * 2 < (1ll << 31);
        it.kind = (direct ? 20 : 10) + cfg;
        it.b = 0;
        it.gx = p.K / bko;
        it.gy = p.N / bno;
      }
      it.block0 = blocks;
      blocks += it.gx * it.gy * zs;
      if (list)
        fprintf(stderr, "[wgrad_mix] item %2d kind %2d B%d %dx%d Cin %d up %d -> %dx%d N %d ks %d s %d: %d blocks\n", idx,
                it.kind, p.B, p.Hin, p.Win, p.Cin, p.up_in, p.Ho, p.Wo, p.N, p.ks, p.stride, it.gx * it.gy * zs);
    }
  }
  if (list) listed = true;
  return flush();
}

static bool mix_ok(const WgradParams& p) {
  if (p.algo != 1 && conv3x3_wgrad_supported(p)) return true;
  int bko, bno, rm;
  return generic_ok(p) && wgrad_config(p, bko, bno, rm) != 1;
}


int conv_wgrad_batch(const WgradParams* ps, int n, hipStream_t st) {
  static thread_local WgradParams by_cfg[10][16], gen_cfg[7][32];  // halo configs 0-9 (conv3x3_wgrad_config)
  int cnt[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, gcnt[7] = {0, 0, 0, 0, 0, 0, 0};
  const bool group = cfl_tune(TUNE_WGRAD_GROUP) != 1;
  const bool group1 = group && cfl_tune(TUNE_WGRAD_GROUP) != 2;
  if (group1 && cfl_tune(TUNE_WGRAD_MIX) != 1) {            // default: one mixed launch (plus any odd ones out)
    static thread_local WgradParams mix[64];
    int nm = 0;
    for (int i = 0; i < n; ++i) {
      if (ps[i].slabs > 0 && ps[i].slabs != conv_wgrad_slabs(ps[i])) return 2;
      if (mix_ok(ps[i]) && nm < 64) {
        mix[nm++] = ps[i];
      } else {
        const int rc = conv_wgrad(ps[i], st);
        if (rc) return rc;
      }
    }
    return launch_mix(mix, nm, st);
  }
  for (int i = 0; i < n; ++i) {
    const WgradParams& p = ps[i];
    if (p.slabs > 0 && p.slabs != conv_wgrad_slabs(p)) return 2;
    if (p.algo != 1 && conv3x3_wgrad_supported(p) && group) {
      const int c = conv3x3_wgrad_config(p);
      if (c < 0 || c >= 10 || cnt[c] == 16) return 5;
      by_cfg[c][cnt[c]++] = p;
    } else if (!(p.algo != 1 && conv3x3_wgrad_supported(p)) && group1 && generic_ok(p)) {
      int bko, bno, rm;
      const int c = wgrad_config(p, bko, bno, rm);
      if (gcnt[c] == 32) return 5;
      gen_cfg[c][gcnt[c]++] = p;
    } else {
      const int rc = conv_wgrad(p, st);
      if (rc) return rc;
    }
  }
  for (int c = 0; c < 7; ++c) {
    if (!gcnt[c]) continue;
    int rc;
    switch (c) {
      case 0: rc = launch_group<128, 128, 32>(gen_cfg[c], gcnt[c], st); break;
      case 6: rc = launch_group<128, 128, 64>(gen_cfg[c], gcnt[c], st); break;
      case 1: rc = launch_group<64, 64, 128>(gen_cfg[c], gcnt[c], st); break;
      case 5: rc = launch_group<64, 64, 64>(gen_cfg[c], gcnt[c], st); break;
      case 2: rc = launch_group<64, 32, 128>(gen_cfg[c], gcnt[c], st); break;
      case 3: rc = launch_group<32, 64, 128>(gen_cfg[c], gcnt[c], st); break;
      default: rc = launch_group<32, 32, 128>(gen_cfg[c], gcnt[c], st); break;
    }
    if (rc) return rc;
  }
  for (int c = 0; c < 10; ++c)
    if (cnt[c]) {
      const int rc = conv3x3_wgrad_grouped(by_cfg[c], cnt[c], st);
      if (rc) return rc;
    }
  return 0;
}

int conv_wgrad(const WgradParams& p, hipStream_t st) {
  if (p.slabs > 0 && p.slabs != conv_wgrad_slabs(p)) return 2;
  if (p.algo != 1 && conv3x3_wgrad_supported(p)) return conv3x3_wgrad(p, st);
  if (!generic_ok(p)) return 1;
  int bko, bno, rm;
  switch (wgrad_config(p, bko, bno, rm)) {
    case 0: launch<128, 128>(p, st); break;
    case 6: launch<128, 128, 64>(p, st); break;
    case 1: launch<64, 64, 128>(p, st); break;
    case 5: launch<64, 64, 64>(p, st); break;
    case 2: launch<64, 32, 128>(p, st); break;
    case 3: launch<32, 64, 128>(p, st); break;
    default: launch<32, 32, 128>(p, st); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_conv_wgrad(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_conv_wgrad(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
