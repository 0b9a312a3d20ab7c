// 3x3 / stride 1 / "same" convolution with a spatial M-tile and an LDS halo (gfx950 MFMA 16x16x32 bf16).
//
// Serves every Conv2DTranspose of the decoder - forward (/root/reference/client_fit_model.py:129,133) and
// data-gradient - i.e. 66 % of the network's FLOPs. The generic implicit GEMM (conv_igemm.hip) re-loads and
// re-transforms each input element once per tap (9x). Here a block owns a TH x TW pixel tile of one image and
// BN output channels; for every 32-channel input chunk it loads the (TH+2) x (TW+2) halo tile ONCE into LDS -
// applying the producer's BN-apply + ReLU and the nearest-2x upsample fold (decoder inputs are stored at half
// resolution) on the way in - and all 9 taps read their MFMA A fragments as shifted views of that tile:
//   A fragment of tap (ky,kx), pixel p = (py,px): halo[py+ky][px+kx][8*(lane>>4) .. +7]   (one ds_read_b128)
// The packed weights [N][K] (K = tap*Cin + c) stream through a register-staged double buffer per (chunk, tap)
// K-step; the next chunk's halo is prefetched into registers during the current chunk's taps and written to the
// second halo buffer before the chunk boundary, so each K-step costs one barrier.
// LDS images are dense (64 B per halo pixel / weight row) with an XOR swizzle of the four 16-byte channel quarters,
// quarter q of row r stored at slot q ^ swz(r), swz(r) = (r >> 1) & 2: every ds_read_b128 lane group (16 lanes =
// 16 consecutive rows, mixed quarters) then covers all 64 banks for ANY starting row - the tap shifts move the
// start - and every ds_write_b128 group of 8 lanes (2 rows x 4 quarters) covers 32 banks. (A 40-bf16 padded
// stride left 3-way conflicts on the shifted taps: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 45 %.)
// Epilogue (bias, bf16, LDS-staged 16-byte stores, BN statistics) and split-K over input chunks (fp32 workspace
// + splitk epilogue) are shared with conv_igemm.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr int BK = 32;          // channels per chunk (one K-step = one tap of one chunk)
constexpr int LDH = BK;         // halo pixel stride (bf16), swizzled
constexpr int LDB = BK;

// bf16 offset of 16-byte quarter q of LDS row r in a swizzled dense image
__device__ __forceinline__ int swz_off(int r, int q) { return r * BK + ((q ^ ((r >> 1) & 2)) << 3); }

// WB ("whole-chunk B"): the block stages all 9 taps' weight tiles of a chunk at once ([tap][n][LDB], single LDS
// buffer, next chunk register-prefetched during the current chunk's 9 x FMxFN MFMAs): two barriers per CHUNK
// instead of one per tap, and no per-tap global-load latency on the critical path. Used for BN <= 64.
// PJ: the decoder node join epilogue (launch.h PoolJoinEpi) - its own instantiation, so the registers of its
// prefetched operands never cost the plain convs occupancy.
// XFIN: consumer-side BN finalize of the input transform (p.xfin): every block turns the producer's replica sums
// into the Cin channels' (a, b) in LDS (its loads in flight with the first chunk's); the first block writes the ab
// rows for the layer's later consumers.
template <int TH, int TW, int BN_, int WM, int WN, bool WB, bool PJ = false, bool XFIN = false>
__global__ __launch_bounds__(NT, 2) void conv3x3_kernel(ConvParams p, int chunks_per_split, float* __restrict__ ws) {
  CFL_TS_GUARD;
  constexpr int BM = TH * TW;
  constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;          // halo pixels
  // LDS pitch of a halo line: TW + 2, except 16 for the 8-wide tiles - there a 16-row A fragment spans two pixel rows,
  // and with 10-row lines every ds_read_b128 lane group hit 2-way bank conflicts under the row swizzle (measured
  // SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 28 %, profiles/r3_final); 16-row lines make every group conflict-free
  constexpr int HWL = TW == 8 ? 16 : HW, HPL = HH * HWL;
  constexpr int TM = BM / WM, TN = BN_ / WN, FM = TM / 16, FN = TN / 16;
  constexpr int HALO_CHUNKS = HP * (BK / 8);                      // 16-byte pieces per halo tile
  constexpr int H_PER_T = (HALO_CHUNKS + NT - 1) / NT;
  constexpr int B_CHUNKS = BN_ * BK / 8, B_PER_T = (B_CHUNKS + NT - 1) / NT;
  constexpr int BW_CHUNKS = 9 * B_CHUNKS, BW_PER_T = WB ? (BW_CHUNKS + NT - 1) / NT : 1;
  constexpr int SH = (WB ? 1 : 2) * HPL * LDH, SB = (WB ? 9 : 2) * BN_ * LDB;
  constexpr int LDC = BN_ + 8;
  static_assert(BM * LDC <= SH + SB, "C staging tile must fit");
  static_assert(WM * WN == 4 && TM % 16 == 0 && TN % 16 == 0, "wave tiling");

  __shared__ __attribute__((aligned(16))) bf16_t smem[SH + SB];
  __shared__ float sred[2][4][BN_];
  __shared__ float sxab[XFIN ? 2 * 256 : 1];            // consumer-side finalize: (a, b) of every input channel
  bf16_t* sH = smem;              // [2][HP][LDH]
  bf16_t* sB = smem + SH;         // [2][BN_][LDB]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_w = (p.Wo + TW - 1) / TW, tiles_h = (p.Ho + TH - 1) / TH;
  // logical block (XCD-aware): the N-blocks and K-splits of one pixel tile, and neighbouring tiles, share an XCD
  const int lin = xcd_block_linear();
  const int bn_idx = lin % gridDim.y, rest = lin / gridDim.y;
  const int bz = rest % gridDim.z;
  int t = rest / gridDim.z;
  const int tile_id = t;
  const int b = t / (tiles_w * tiles_h);
  t -= b * tiles_w * tiles_h;
  const int ty0 = (t / tiles_w) * TH, tx0 = (t % tiles_w) * TW;
  const int nBlock = bn_idx * BN_;
  const int chunks = p.Cin / BK;
  const int ch0 = bz * chunks_per_split;
  const int ch1 = imin(chunks, ch0 + chunks_per_split);
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;

  // ---- halo loading: piece e -> halo pixel e/4, channel quarter e%4 ----
  // The halo is loaded RAW (rh) and the producer's BN-apply + ReLU applied only right before it is written to LDS,
  // after the current chunk's MFMAs: a transform right after the load made every chunk wait for its own prefetch
  // first (tools/conv3_probe.py at 256^2 / B16: the transformed convs ran 1.1-5.4 us slower than untransformed ones).
  uint4 rh[H_PER_T];
  uint32_t hvalid = 0;                                  // bit i = piece i inside the image
  float ha[8], hb[8];                                   // producer coefficients of the loaded chunk (quarter tid & 3)
  auto load_coefs = [&](int chunk) {
    // a thread's pieces all have channel quarter tid & 3 (NT % 4 == 0): one coefficient load per chunk
    const int c8 = chunk * BK + (tid & 3) * 8;
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
  // The block's halo pieces sit at the same pixels for every chunk: their byte offsets in the tile image (padding:
  // the out-of-range offset, read as 0) are computed once, and a chunk's loads are buffer loads with the chunk as
  // the scalar offset - no per-chunk address math and no per-lane branch around a load.
  static_assert(div_small_ok<HW, H_PER_T * NT / 4>(), "halo pixel division");
  const __amdgpu_buffer_rsrc_t rs_x =
      buf_rsrc(p.x + (size_t)b * p.Hin * p.Win * p.Cin, (uint32_t)p.Hin * p.Win * p.Cin * 2u);
  uint32_t hoff[H_PER_T], hv_tile = 0;
#pragma unroll
  for (int i = 0; i < H_PER_T; ++i) {
    const int e = tid + i * NT;
    const int hp = e >> 2;
    const int hy = div_small<HW>(hp), hx = hp - hy * HW;
    const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;      // logical input coords (pad 1)
    const bool ok = e < HALO_CHUNKS && (unsigned)iy < (unsigned)Hl && (unsigned)ix < (unsigned)Wl;
    hoff[i] = ok ? __umul24((unsigned)iy >> p.up_in, (unsigned)p.Win * p.Cin * 2u) +
                       __umul24((unsigned)ix >> p.up_in, (unsigned)p.Cin * 2u) + (tid & 3) * 16u
                 : CFL_OOB;
    hv_tile |= (ok ? 1u : 0u) << i;
  }
  auto load_halo = [&](int chunk) {
    if (!XFIN) load_coefs(chunk);                       // (XFIN: after the prologue, below)
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) rh[i] = buf_load16(rs_x, hoff[i], chunk * BK * 2);
    hvalid = hv_tile;
  };
  // producer BN-apply + ReLU of the raw halo in rh (packed, common.h xform8); padding stays exactly 0
  const uint32_t relu_lo = relu ? 0u : 0x80008000u;
  auto xform_halo = [&]() {
    if (!(has_ab || relu)) return;
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) rh[i] = xform8(rh[i], ha, hb, relu_lo, ((hvalid >> i) & 1u) ? 0xffffffffu : 0u);
  };
  auto store_halo = [&](int buf) {
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < HALO_CHUNKS) {
        const int hp = e >> 2, hy = hp / HW, hx = hp - hy * HW;
        *reinterpret_cast<uint4*>(sH + buf * HPL * LDH + swz_off(hy * HWL + hx, e & 3)) = rh[i];
      }
    }
  };
  // ---- weight tile of K-step (chunk, tap): wt[n][tap*Cin + chunk*32 .. +32) ----
  // (buffer loads over the weight matrix; a piece's row / quarter is fixed, the tap and chunk are scalar offsets)
  const __amdgpu_buffer_rsrc_t rs_w = buf_rsrc(p.wt, (uint32_t)p.N * p.K * 2u);
  uint4 rb[B_PER_T];
  auto load_b = [&](int chunk, int tap) {
    const uint32_t kofs = (uint32_t)(tap * p.Cin + chunk * BK) * 2u;
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int e = tid + i * NT;
      rb[i] = buf_load16(rs_w, (B_CHUNKS % NT == 0 || e < B_CHUNKS)
                                   ? (uint32_t)((nBlock + (e >> 2)) * p.K + (e & 3) * 8) * 2u : CFL_OOB, kofs);
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < B_CHUNKS) *reinterpret_cast<uint4*>(sB + buf * BN_ * LDB + swz_off(e >> 2, e & 3)) = rb[i];
    }
  };

  // ---- whole-chunk weight tiles (WB): piece e -> tap e / B_CHUNKS, row n, 16-byte quarter q ----
  uint4 rbw[BW_PER_T];
  // NT % B_CHUNKS == 0 (B_CHUNKS = 128 / 256): piece i's tap is i * (NT / B_CHUNKS) + tid / B_CHUNKS and its weight
  // row / quarter tid % B_CHUNKS - one per-thread offset, the tap and chunk in the scalar offset
  static_assert(!WB || NT % B_CHUNKS == 0, "whole-chunk weight pieces");
  const int bw_w = tid % B_CHUNKS;
  const uint32_t bw_off = (uint32_t)((nBlock + (bw_w >> 2)) * p.K + (tid / B_CHUNKS) * p.Cin + (bw_w & 3) * 8) * 2u;
  auto load_bw = [&](int chunk) {
#pragma unroll
    for (int i = 0; i < BW_PER_T; ++i) {
      const int e = tid + i * NT;
      rbw[i] = buf_load16(rs_w, (BW_CHUNKS % NT == 0 || e < BW_CHUNKS) ? bw_off : CFL_OOB,
                          (uint32_t)(i * (NT / B_CHUNKS) * p.Cin + chunk * BK) * 2u);
    }
  };
  auto store_bw = [&]() {
#pragma unroll
    for (int i = 0; i < BW_PER_T; ++i) {
      const int e = tid + i * NT;
      if (BW_CHUNKS % NT == 0 || e < BW_CHUNKS) {
        const int tap = e / B_CHUNKS, w = e - tap * B_CHUNKS;
        *reinterpret_cast<uint4*>(sB + swz_off(tap * BN_ + (w >> 2), w & 3)) = rbw[i];
      }
    }
  };

  // per-lane fragment: halo row of tap (0,0) for each A fragment, B row, channel quarter
  int fhp[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pp = wm * TM + i * 16 + (lane & 15);
    fhp[i] = (pp / TW) * HWL + pp % TW;
  }
  const int fq = lane >> 4;
  const int brow = wn * TN + (lane & 15);

  // decoder node join (PoolJoinEpi): this thread's half-resolution pixel (one per thread: HB <= rows per pass)
  // and its mask / addend / sums-source vectors, loaded now so they are in flight during the K loop
  constexpr bool pj = PJ;
  static_assert(!PJ || BM / 4 <= NT / (BN_ / 8), "one half-resolution pixel per thread");
  uint4 pjv = make_uint4(0, 0, 0, 0), pja = pjv, pjy = pjv;
  size_t pjoff = 0;
  bool pjok = false;
  if constexpr (PJ) {
    constexpr int CGp = BN_ / 8, HTW = TW / 2, HB = BM / 4;
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

  f4v acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  if constexpr (WB) {
    if (ch0 < ch1) {
      load_halo(ch0);
      load_bw(ch0);
    }
    if constexpr (XFIN) {         // the first chunk's loads are in flight during the coefficient computation
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
      load_coefs(ch0);
    }
    if (ch0 < ch1) {
      xform_halo();
      store_halo(0);
      store_bw();
    }
    __syncthreads();
    for (int ch = ch0; ch < ch1; ++ch) {
      const bool next_chunk = ch + 1 < ch1;
      if (next_chunk) {                                      // in flight during this chunk's 9 taps
        load_halo(ch + 1);
        load_bw(ch + 1);
        if constexpr (XFIN) load_coefs(ch + 1);
      }
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
        s8v af[FM], bfg[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *reinterpret_cast<const s8v*>(sH + swz_off(fhp[i] + ky * HWL + kx, fq));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfg[j] = *reinterpret_cast<const s8v*>(sB + swz_off(tap * BN_ + brow + j * 16, fq));
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
      if (next_chunk) {
        xform_halo();
        store_halo(0);
        store_bw();
        __syncthreads();
      }
    }
  } else {
  if (ch0 < ch1) {
    load_halo(ch0);
    xform_halo();
    store_halo(0);
    load_b(ch0, 0);
    store_b(0);
  }
  __syncthreads();
  int bbuf = 0;
  for (int ch = ch0; ch < ch1; ++ch) {
    const int hbuf = (ch - ch0) & 1;
    const bool next_chunk = ch + 1 < ch1;
    if (next_chunk) load_halo(ch + 1);                       // in flight during this chunk's 9 taps
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const bool more = tap < 8 || next_chunk;
      if (more) {
        if (tap < 8) load_b(ch, tap + 1);
        else load_b(ch + 1, 0);
      }
      const int ky = tap / 3, kx = tap - ky * 3;
      s8v af[FM], bfg[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const s8v*>(sH + hbuf * HPL * LDH + swz_off(fhp[i] + ky * HWL + kx, fq));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfg[j] = *reinterpret_cast<const s8v*>(sB + bbuf * BN_ * LDB + swz_off(brow + j * 16, fq));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
      if (more) store_b(bbuf ^ 1);
      if (tap == 8 && next_chunk) {
        xform_halo();
        store_halo(hbuf ^ 1);
      }
      __syncthreads();
      bbuf ^= 1;
    }
  }
  }

  // pixel index of accumulator row r of fragment i -> (m valid?, global m)
  auto out_m = [&](int row, int& m) -> bool {
    const int py = row / TW, px = row % TW;
    const int oy = ty0 + py, ox = tx0 + px;
    m = (b * p.Ho + oy) * p.Wo + ox;
    return oy < p.Ho && ox < p.Wo;
  };

  if (ws != nullptr) {                    // split-K partials
    float* dst = ws + (size_t)bz * p.M * p.N;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = nBlock + wn * TN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          int m;
          if (out_m(wm * TM + i * 16 + (lane >> 4) * 4 + r, m)) dst[(size_t)m * p.N + n] = acc[i][j][r];
        }
      }
    return;
  }

  bf16_t (*sC)[LDC] = reinterpret_cast<bf16_t (*)[LDC]>(smem);
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
  const bool node = p.node.y != nullptr;           // fused BN-node gradient epilogue (dgrad of a BN node's input)
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
    int m;
    if (out_m(row, m)) {
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
  }
  if (p.stats || node || (pj && p.pj.sums)) {
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
    // replica row of this block (element offset: the deterministic mode's int64 rows use the same indices)
    float* rep = pj ? p.pj.sums : node ? p.node.sums : p.stats;
    const int nrep = pj ? (p.pj.reps > 1 ? p.pj.reps : 1) : node ? (p.node.reps > 1 ? p.node.reps : 1) : STAT_REPLICAS;
    const size_t ro = (size_t)(tile_id % nrep) * 2 * p.N;
    for (int e = tid; e < 2 * BN_; e += NT) {
      const int st = e / BN_, cc = e - st * BN_;
      red_add(rep, ro + st * p.N + nBlock + cc, sred[st][0][cc] + sred[st][1][cc] + sred[st][2][cc] + sred[st][3][cc],
              red_scale(!pj && !node, st));
    }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Weight-stationary persistent variant for the high-resolution decoder convs (Cin <= 64: the 128^2 / 64^2 maps at
// 256^2 input, M = 65k-262k pixels, N = 32-128, K = 288-576). The per-tile kernel above re-loads the block's whole
// weight tile (9 taps x BN x 32 per chunk) for every 128-pixel tile - more L2->LDS bytes than the activations - and
// pays one global-load latency per tile with nothing to overlap it. Here a block keeps ALL K of its 32 output
// channels in LDS for its lifetime (CH x 18.4 KB) and walks a strided list of pixel tiles; the next tile's raw halo
// (every chunk) is in flight in registers while the current tile's 9 x CH taps run, and is BN-applied / ReLU'd
// only when it is written to LDS (after the MFMAs), so the loads are never waited for early. BN statistics /
// BN-node sums accumulate in registers across the block's tiles: one set of channel atomics per block.
// LDS: weights CH*9*32 rows + halo CH*HP rows (64 B each, swizzled as above) + a bf16 C staging tile.
template <int TH, int TW, int CH, bool PJ = false, bool XFIN = false>
__global__ __launch_bounds__(NT, CH == 1 && !PJ ? 3 : 2) void conv3x3_ws_kernel(ConvParams p, int n_items) {
  CFL_TS_GUARD;
  constexpr int BN_ = 32, WM = 4;
  constexpr int BM = TH * TW;
  constexpr int HW = TW + 2, HP = (TH + 2) * HW;
  constexpr int TM = BM / WM, FM = TM / 16, FN = BN_ / 16;
  constexpr int HALO_CHUNKS = HP * (BK / 8);
  constexpr int H_PER_T = (HALO_CHUNKS + NT - 1) / NT;
  constexpr int SW = CH * 9 * BN_ * LDB, SH = CH * HP * LDH;
  constexpr int LDC = BN_ + 8;
  constexpr int CG = BN_ / 8, ROWS_PER_PASS = NT / CG;
  static_assert(TM % 16 == 0 && H_PER_T <= 32, "tiling");

  __shared__ __attribute__((aligned(16))) bf16_t smem[SW + SH + BM * LDC];
  __shared__ float sred[2][4][BN_];
  bf16_t* sB = smem;                 // [CH][9][BN_][32]
  bf16_t* sH = smem + SW;            // [CH][HP][32]
  bf16_t (*sC)[LDC] = reinterpret_cast<bf16_t (*)[LDC]>(smem + SW + SH);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int nb = p.N / BN_;
  const int nBlock = (blockIdx.x % nb) * BN_;       // gridDim.x % nb == 0: one column block per block
  const int tiles_w = p.Wo / TW, tiles_hw = tiles_w * (p.Ho / TH);
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;

  // ---- all weights of this column block: piece e -> (row = (ch*9 + tap)*BN_ + n, quarter q). Every piece's load
  //      is issued (index clamped) before the first LDS store: the strided copy loop waited one full memory round
  //      trip per iteration (5 / 9 of them per block, most of a block's time at 2-3 tiles per block).
  constexpr int WP = CH * 9 * BN_ * 4, WPT = (WP + NT - 1) / NT;
  u4v wr[WPT];
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    const int e = imin(tid + i * NT, WP - 1);
    const int row = e >> 2, q = e & 3;
    const int n = row % BN_, ct = row / BN_, ch = ct / 9, tap = ct - ch * 9;
    wr[i] = *reinterpret_cast<const u4v*>(p.wt + (size_t)(nBlock + n) * p.K + (size_t)tap * p.Cin + ch * BK + q * 8);
  }
#pragma unroll
  for (int i = 0; i < WPT; ++i) {
    const int e = tid + i * NT;
    if (e < WP) *reinterpret_cast<u4v*>(sB + swz_off(e >> 2, e & 3)) = wr[i];
  }
  // producer BN coefficients of this thread's channel quarter, per chunk (constant over the block's tiles); XFIN:
  // computed here from the producer's replica sums (consumer-side finalize, first block writes the ab rows)
  float a8[CH][8], b8[CH][8];
  if constexpr (XFIN) {
    __shared__ float sxab[2 * CH * BK];
    if (tid < CH * BK) {
      float a, bb, mean, rstd;
      bn_coef_from_stats(p.xfin, p.Cin, tid, a, bb, mean, rstd);
      sxab[tid] = a;
      sxab[CH * BK + tid] = bb;
      if (blockIdx.x == 0) {
        float* ab = const_cast<float*>(p.xf.ab);
        ab[tid] = a;
        ab[p.Cin + tid] = bb;
        ab[2 * p.Cin + tid] = mean;
        ab[3 * p.Cin + tid] = rstd;
      }
    }
    __syncthreads();
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        a8[ch][j] = sxab[ch * BK + (tid & 3) * 8 + j];
        b8[ch][j] = sxab[CH * BK + ch * BK + (tid & 3) * 8 + j];
      }
  } else {
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
      load_f8_or(p.xf.ab + ch * BK + (tid & 3) * 8, has_ab, 1.f, a8[ch]);
      load_f8_or(p.xf.ab + p.xf.C + ch * BK + (tid & 3) * 8, has_ab, 0.f, b8[ch]);
    }
  }

  auto tile_of = [&](int item, int& b, int& ty0, int& tx0) {
    int t = item / nb;
    b = t / tiles_hw;
    t -= b * tiles_hw;
    ty0 = (t / tiles_w) * TH;
    tx0 = (t % tiles_w) * TW;
  };
  // raw halo of a tile into registers (no use of the values here: the loads stay in flight). Buffer loads from the
  // tile image's resource: a piece costs a few full-rate ops (24-bit products into a 32-bit offset; padding = the
  // out-of-range offset, read as 0 - no per-lane branch around the load) and the chunk is the scalar offset.
  uint4 rh[CH][H_PER_T];
  uint32_t rvalid = 0;                                  // bit i: piece i lies inside the image
  const uint32_t x_row = (uint32_t)p.Win * p.Cin * 2u, x_px = (uint32_t)p.Cin * 2u;
  const uint32_t x_img = (uint32_t)p.Hin * p.Win * p.Cin * 2u;
  static_assert(div_small_ok<HW, H_PER_T * NT / 4>(), "halo pixel division");
  auto load_halo = [&](int item) {
    int b, ty0, tx0;
    tile_of(item, b, ty0, tx0);
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(p.x + (size_t)b * p.Hin * p.Win * p.Cin, x_img);
    rvalid = 0;
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      const int hp = e >> 2;
      const int hy = div_small<HW>(hp), hx = hp - hy * HW;
      const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
      const bool ok = e < HALO_CHUNKS && (unsigned)iy < (unsigned)Hl && (unsigned)ix < (unsigned)Wl;
      rvalid |= (ok ? 1u : 0u) << i;
      const uint32_t off = ok ? __umul24((unsigned)iy >> p.up_in, x_row) + __umul24((unsigned)ix >> p.up_in, x_px) +
                                    (tid & 3) * 16u
                              : CFL_OOB;
#pragma unroll
      for (int ch = 0; ch < CH; ++ch) rh[ch][i] = buf_load16(rs, off, ch * BK * 2);
    }
  };
  // producer BN-apply + ReLU on the way into LDS (packed, common.h xform8); padding stays exactly 0
  const uint32_t relu_lo = relu ? 0u : 0x80008000u;
  auto store_halo = [&]() {
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e >= HALO_CHUNKS) continue;
      const uint32_t m = ((rvalid >> i) & 1u) ? 0xffffffffu : 0u;
#pragma unroll
      for (int ch = 0; ch < CH; ++ch)
        *reinterpret_cast<uint4*>(sH + ch * HP * LDH + swz_off(e >> 2, e & 3)) =
            xform8(rh[ch][i], a8[ch], b8[ch], relu_lo, m);
    }
  };

  int fhp[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int pp = wid * TM + i * 16 + (lane & 15);
    fhp[i] = (pp / TW) * HW + pp % TW;
  }
  const int fq = lane >> 4;
  const int cg = tid % CG;
  const bool node = p.node.y != nullptr;
  constexpr bool pj = PJ;
  NodeCoef nk;
  if (node) node_coef_load(p.node.ab, p.N, nBlock + cg * 8, nk);
  float pm[8], pr[8];
  load_f8_or(p.pj.sab + 2 * p.N + nBlock + cg * 8, pj && p.pj.sy != nullptr, 0.f, pm);
  load_f8_or(p.pj.sab + 3 * p.N + nBlock + cg * 8, pj && p.pj.sy != nullptr, 0.f, pr);
  float biasf[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) biasf[j] = p.bias ? p.bias[nBlock + j * 16 + (lane & 15)] : 0.f;
  float s[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) s[0][q] = s[1][q] = 0.f;

  int item = blockIdx.x;
  if (item < n_items) load_halo(item);
  if (item < n_items) store_halo();
  __syncthreads();
  cfl_ts_phase(0);
  for (; item < n_items; item += gridDim.x) {
    const int next = item + gridDim.x;
    if (next < n_items) load_halo(next);               // in flight during this tile's MFMAs
    // decoder node join: this tile's half-resolution vectors (one pixel per thread), in flight during the MFMAs
    uint4 pjv = make_uint4(0, 0, 0, 0), pja = pjv, pjy = pjv;
    size_t pjoff = 0;
    const int pjr = tid / CG;
    if (PJ && pjr < BM / 4) {
      int pb, pty0, ptx0;
      tile_of(item, pb, pty0, ptx0);
      const int hy = pjr / (TW / 2), hx = pjr % (TW / 2);
      pjoff = (((size_t)pb * (p.Ho >> 1) + (pty0 >> 1) + hy) * (p.Wo >> 1) + (ptx0 >> 1) + hx) * p.N + nBlock + cg * 8;
      pjv = *reinterpret_cast<const uint4*>(p.pj.v + pjoff);
      if (p.pj.add) pja = *reinterpret_cast<const uint4*>(p.pj.add + pjoff);
      if (p.pj.sy) pjy = *reinterpret_cast<const uint4*>(p.pj.sy + pjoff);
    }
    f4v acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < CH; ++ch)
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int ky = tap / 3, kx = tap - ky * 3;
        s8v af[FM], bfg[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *reinterpret_cast<const s8v*>(sH + ch * HP * LDH + swz_off(fhp[i] + ky * HW + kx, fq));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfg[j] = *reinterpret_cast<const s8v*>(sB + swz_off((ch * 9 + tap) * BN_ + j * 16 + (lane & 15), fq));
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfg[j], acc[i][j], 0, 0, 0);
      }
    // accumulators + bias -> bf16 staging tile (one rounding, as the per-tile kernel)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int cl = j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sC[wid * TM + i * 16 + (lane >> 4) * 4 + r][cl] = f2bf(acc[i][j][r] + biasf[j]);
    }
    __syncthreads();                                    // halo reads done, C tile complete
    if (next < n_items) store_halo();
    int b, ty0, tx0;
    tile_of(item, b, ty0, tx0);
    if constexpr (PJ) {                                 // decoder node join at half resolution (PoolJoinEpi)
      constexpr int HTW = TW / 2, HB = BM / 4;
      static_assert(HB <= ROWS_PER_PASS, "one half-resolution pass");
      if (pjr < HB) {
        const int hy = pjr / HTW, hx = pjr % HTW;
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
    __syncthreads();                                    // next halo visible, C tile consumed
  }
  cfl_ts_phase(1);
  if (p.stats || node || (pj && p.pj.sums)) {
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
    const int rb = blockIdx.x / nb;                     // replica row (blocks of one column block spread)
    float* rep = pj ? p.pj.sums : node ? p.node.sums : p.stats;
    const int nrep = pj ? (p.pj.reps > 1 ? p.pj.reps : 1) : node ? (p.node.reps > 1 ? p.node.reps : 1) : STAT_REPLICAS;
    const size_t ro = (size_t)(rb % nrep) * 2 * p.N;
    for (int e = tid; e < 2 * BN_; e += NT) {
      const int st = e / BN_, cc = e - st * BN_;
      red_add(rep, ro + st * p.N + nBlock + cc, sred[st][0][cc] + sred[st][1][cc] + sred[st][2][cc] + sred[st][3][cc],
              red_scale(!pj && !node, st));
    }
  }
}

// every 3x3 / stride-1 conv with Cin in {32, 64} on maps tiled exactly by 8x16 (or 16x8) pixel tiles
// (TUNE_CONV3_WS: 1 = never, 2 = whenever the shape allows it, regardless of the tile count - tests)
static bool ws_eligible(const ConvParams& p) {
  const int v = cfl_tune(TUNE_CONV3_WS);
  if (v == 1) return false;
  if (!(p.Cin == 32 || p.Cin == 64) || p.N % 32) return false;
  const int tw = p.Wo >= 16 ? 16 : 8, th = 128 / tw;
  if (p.Ho % th || p.Wo % tw) return false;
  const int items = (p.Ho / th) * (p.Wo / tw) * p.B * (p.N / 32);
  // measured (tools/kbench.py, 256^2 / B16): the 128^2 level (2048-4096 items, >= 3 tiles per block) gains 15-22 %,
  // the 64^2 level (1024 items, 2 tiles per block) loses 15 % - the per-tile kernel stays there
  return v == 2 || items >= 2048;
}

template <int TH, int TW, int CH>
void launch_ws(const ConvParams& p, hipStream_t st) {
  const int nb = p.N / 32;
  const int items = (p.Ho / TH) * (p.Wo / TW) * p.B * nb;
  int grid = cfl_tune(TUNE_CONV3_WS_GRID) > 0 ? cfl_tune(TUNE_CONV3_WS_GRID) : (CH == 1 ? 768 : 512);
  grid = grid / nb * nb;
  if (grid < nb) grid = nb;
  if (grid > items) grid = items;
  if (p.xfin.stats) hipLaunchKernelGGL((conv3x3_ws_kernel<TH, TW, CH, false, true>), dim3(grid), dim3(NT), 0, st, p, items);
  else if (p.pj.v) hipLaunchKernelGGL((conv3x3_ws_kernel<TH, TW, CH, true>), dim3(grid), dim3(NT), 0, st, p, items);
  else hipLaunchKernelGGL((conv3x3_ws_kernel<TH, TW, CH>), dim3(grid), dim3(NT), 0, st, p, items);
}

template <int TH, int TW, int BN_, int WM, int WN, bool WB = false>
int launch(const ConvParams& p, int splits, hipStream_t st) {
  const int chunks = p.Cin / BK;
  const int per = (chunks + splits - 1) / splits;
  splits = (chunks + per - 1) / per;
  const int tiles = ((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * p.B;
  dim3 grid(tiles, p.N / BN_, splits);
  if constexpr (WB) {
    if (p.xfin.stats) {
      hipLaunchKernelGGL((conv3x3_kernel<TH, TW, BN_, WM, WN, true, false, true>), grid, dim3(NT), 0, st, p,
                         per, splits > 1 ? p.ws : nullptr);
      return splits;
    }
    if constexpr (TH * TW / 4 <= NT / (BN_ / 8)) {     // (the node join needs one half-res pixel per thread)
      if (p.pj.v) {
        hipLaunchKernelGGL((conv3x3_kernel<TH, TW, BN_, WM, WN, true, true>), grid, dim3(NT), 0, st, p, per, nullptr);
        return 1;
      }
    }
  }
  hipLaunchKernelGGL((conv3x3_kernel<TH, TW, BN_, WM, WN, WB>), grid, dim3(NT), 0, st, p, per,
                     splits > 1 ? p.ws : nullptr);
  return splits;
}

}  // namespace

// output-channel tile of the whole-chunk path: 64 (fewer halo re-loads) unless tuned to 32 (more blocks, 122 vs 208
// VGPRs -> 4 vs 2 waves per SIMD). Counters behind the tile choices (profiles/r2_pmc/pmc_summary.txt and
// pmc_latency.txt, 256^2 / B16 bench step): the 8x16 x 64 tile runs at 14 % of the MFMA peak and 0.8 TB/s with
// 1.3 % LDS bank conflicts (the swizzle), an 89 % L2 hit rate and ~320-cycle L1->L2 latency - neither MFMA, HBM nor
// LDS bound but latency-bound per block, which is why the halo is prefetched a chunk ahead, the producer transform
// deferred to the LDS store and the 128^2 level moved to the weight-stationary persistent kernel (weights loaded
// once per block instead of per tile: 8.7 % MFMA, 2.5 TB/s). tools/conv3_probe.py times the variants per shape.
static int wb_bn(const ConvParams& p) {
  const int v = cfl_tune(TUNE_CONV3_BN);
  if (v == 32 || p.N % 64 != 0) return 32;
  return 64;
}

static bool use_wb(const ConvParams& p) {
  const int v = cfl_tune(TUNE_CONV3_WB);
  return v == 0 ? true : v == 1;           // 0 = default (whole-chunk B, BN <= 64), 2 = per-tap B (BN up to 128)
}

// Low-M layers (the 16x16 maps at 256^2: 4096 pixels, K up to 2304): rather than split K over a fp32 workspace and
// a second epilogue launch, cut the output into 8x8-pixel x 32-channel tiles - enough blocks without a K split.
static bool small_tiles(const ConvParams& p) {
  const int v = cfl_tune(TUNE_CONV3_SMALL);
  if (v == 1 || !use_wb(p) || p.N % 32 || p.Ho < 8 || p.Wo < 8) return false;
  if (v == 2) return true;
  const int tw = p.Wo >= 16 ? 16 : 8, th = 128 / tw, bn = p.N >= 64 ? 64 : p.N;
  const int blocks = ((p.Ho + th - 1) / th) * ((p.Wo + tw - 1) / tw) * p.B * (p.N / bn);
  const int small = ((p.Ho + 7) / 8) * ((p.Wo + 7) / 8) * p.B * (p.N / 32);
  return blocks < 192 && p.Cin / BK >= 2 && small >= 384;
}

// Large-M layers (the 32^2-128^2 decoder levels at the 512^2 planned batch: 1.1-18M pixels, Cin 64-256): 16x16-
// pixel tiles. The whole-chunk weight tile (9 taps x 64 x 32, 36 KB) is re-read from L2 for every pixel tile, and at
// this M the 8x16 tiles ran at ~28 % of the MFMA peak on that L2 stream; 256 pixels per tile halve the weight bytes
// per MFMA. TUNE_CONV3_BIG: 1 = off, 2 = whenever the shape allows.
static bool big_tiles(const ConvParams& p) {
  const int v = cfl_tune(TUNE_CONV3_BIG);
  if (v == 1 || p.pj.v || !use_wb(p) || wb_bn(p) != 64 || p.Ho % 16 || p.Wo % 16) return false;
  // (>= 1M pixels: the 32^2 level at the 512^2 planned batch, 1.1M, gained 250-430 us per call over the 8x16 tiles
  // with the 4 x 1 wave grid - profiles/r5_conv/trace_ab_big_tiles_1M_512.txt; the 256^2 bench's largest is 262k)
  return v == 2 || (int64_t)p.B * p.Ho * p.Wo >= (1 << 20);
}

bool conv3x3_deep_eligible(const ConvParams& p);
bool conv3x3_sk_eligible(const ConvParams& p);
int conv3x3_sk(const ConvParams& p, hipStream_t st);
int conv3x3_splits(const ConvParams& p) {
  return conv3x3_sk_eligible(p) || small_tiles(p) || ws_eligible(p) || conv3x3_deep_eligible(p) || big_tiles(p)
             ? 1 : conv3x3_split_k(p);
}

// K splits of the 8x16 / 16x8-pixel tiles (the fp8 kernel has no small-tile variant and always uses this)
int conv3x3_split_k(const ConvParams& p) {
  const int tw = p.Wo >= 16 ? 16 : 8;
  const int th = 128 / tw;
  const int bn = use_wb(p) ? wb_bn(p) : (p.N >= 128 ? 128 : p.N);
  const int blocks = ((p.Ho + th - 1) / th) * ((p.Wo + tw - 1) / tw) * p.B * (p.N / bn);
  const int chunks = p.Cin / BK;
  const int below = cfl_tune(TUNE_CONV3_SPLIT_BLOCKS) > 0 ? cfl_tune(TUNE_CONV3_SPLIT_BLOCKS) : 192;
  const int target = cfl_tune(TUNE_CONV3_SPLIT_TARGET) > 0 ? cfl_tune(TUNE_CONV3_SPLIT_TARGET) : 384;
  if (blocks >= below || chunks < 2) return 1;
  int s = (target + blocks - 1) / blocks;
  if (s > chunks) s = chunks;
  const int per = (chunks + s - 1) / s;
  return (chunks + per - 1) / per;
}

bool conv3x3_supported(const ConvParams& p) {
  // the halo loaders read one image through a buffer resource with 32-bit offsets from 24-bit row / pixel products
  const bool fits = (int64_t)p.Hin * p.Win * p.Cin * 2 < (1ll << 31) && (int64_t)p.Win * p.Cin * 2 < (1 << 24);
  return p.ks == 3 && p.stride == 1 && p.pad_t == 1 && p.pad_l == 1 && p.Cin % BK == 0 && p.N % 32 == 0 &&
         p.Wo >= 8 && p.Ho >= 8 && (p.N % 128 == 0 || p.N == 64 || p.N == 32) && fits;
}

bool conv3x3_deep_eligible(const ConvParams& p);
int conv3x3_deep(const ConvParams& p, hipStream_t st);

int conv3x3(const ConvParams& p, hipStream_t st) {
  if (p.wt8) {
    // block-scaled fp8 operands (fp8.hip). TUNE_CONV3_F8: 0 = default - fp8 for the decoder node-join data gradients
    // (the convT1 dgrads with the pj epilogue) unless the bf16 weight-stationary kernel takes the call; the other
    // calls measured faster on the bf16 kernels once those moved to 16x16 tiles on a 4 x 1 wave grid (per position
    // at 512^2: bf16 -77 .. -276 us, the node-join form +217 us - profiles/r5_conv/trace_ab_fp8_routing_512.txt),
    // 1 = never. Round 6 closed the whole-network fp8 modes (profiles/r6_fp8: every routed kernel 23-150 % slower,
    // VALU / MFMA 56-168 against 3-9 in bf16 - the per-32 amax / scale / convert of every staged halo chunk); 2 stays
    // only as a TEST hook (kernel coverage of the non-join shapes, tests/test_gpu_kernels.py), never a product mode.
    const int v = cfl_tune(TUNE_CONV3_F8);
    if (v == 2 || (v == 0 && p.pj.v && !ws_eligible(p))) return conv3x3_f8(p, st);
    ConvParams q = p;
    q.wt8 = nullptr;
    q.ws8 = nullptr;
    return conv3x3(q, st);
  }
  if (!conv3x3_supported(p)) return 1;
  if (p.bwd.y) return 6;                    // the BN-backward operand is applied by a separate pass (conv_igemm)
  // low-resolution deep-K layers: K split over the block's waves, 32x32 MFMA register tiles (conv3x3_sk.hip)
  if (conv3x3_sk_eligible(p)) return conv3x3_sk(p, st);
  if (p.xfin.stats && (p.pj.v || p.xf.C > 256 || !(ws_eligible(p) || use_wb(p)))) {
    // a kernel without the consumer-side finalize: finalize first, then the plain call
    const int rc = bn_finalize(p.xfin.stats, p.xfin.gamma, p.xfin.beta, nullptr, nullptr, const_cast<float*>(p.xf.ab),
                               p.Cin, p.xfin.count, p.xfin.eps, 1, st);
    if (rc) return rc;
    ConvParams q = p;
    q.xfin = BnStatsIn{};
    return conv3x3(q, st);
  }
  // LDS-DMA ring, no split-K
  if (conv3x3_deep_eligible(p) && !ws_eligible(p) && !p.pj.v)
    return conv3x3_deep(p, st);
  if (ws_eligible(p)) {                     // weight-stationary persistent tiles (no split-K)
    const bool w16 = p.Wo >= 16;
    if (p.Cin == 32) {
      if (w16) launch_ws<8, 16, 1>(p, st);
      else launch_ws<16, 8, 1>(p, st);
    } else {
      if (w16) launch_ws<8, 16, 2>(p, st);
      else launch_ws<16, 8, 2>(p, st);
    }
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  if (p.pj.v && !use_wb(p)) return 8;        // the node join needs one half-resolution pixel per thread (BN <= 64)
  int splits = conv3x3_splits(p);
  if (splits > 1 && (p.ws == nullptr || p.ws_elems < (int64_t)splits * p.M * p.N || p.pj.v)) splits = 1;
  const bool w16 = p.Wo >= 16;
  if (small_tiles(p)) {
    splits = launch<8, 8, 32, 2, 2, true>(p, 1, st);
  } else if (big_tiles(p)) {
    // 4 x 1 waves of 64 pixels x 64 channels: 8 fragment reads per 16 MFMAs instead of 10 (128 x 32 per wave) - these
    // large-M calls are LDS-read bound (measured: profiles/README.md round 5)
    if (cfl_tune(TUNE_CONV3_BIG_WAVES) == 1) splits = launch<16, 16, 64, 2, 2, true>(p, 1, st);
    else splits = launch<16, 16, 64, 4, 1, true>(p, 1, st);
  } else if (use_wb(p) && wb_bn(p) == 64) {
    if (w16) splits = launch<8, 16, 64, 2, 2, true>(p, splits, st);
    else splits = launch<16, 8, 64, 2, 2, true>(p, splits, st);
  } else if (use_wb(p)) {
    if (w16) splits = launch<8, 16, 32, 4, 1, true>(p, splits, st);
    else splits = launch<16, 8, 32, 4, 1, true>(p, splits, st);
  } else if (p.N % 128 == 0) {
    if (w16) splits = launch<8, 16, 128, 2, 2>(p, splits, st);
    else splits = launch<16, 8, 128, 2, 2>(p, splits, st);
  } else if (p.N == 64) {
    if (w16) splits = launch<8, 16, 64, 2, 2>(p, splits, st);
    else splits = launch<16, 8, 64, 2, 2>(p, splits, st);
  } else {
    if (w16) splits = launch<8, 16, 32, 4, 1>(p, splits, st);
    else splits = launch<16, 8, 32, 4, 1>(p, splits, st);
  }
  if (hipGetLastError() != hipSuccess) return 3;
  return splits > 1 ? -splits : 0;   // negative: caller must run the split-K epilogue
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_conv3x3(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_conv3x3(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
