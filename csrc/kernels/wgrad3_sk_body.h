// Split-K-in-block weight gradient of the 3x3 / stride-1 / "same" convolutions (the decoder's Conv2DTranspose
// layers, /root/reference/client_fit_model.py:129,133) for the low-resolution levels:
//   dW[tap][c][n] = sum_pixels T(x)[p + (ky-1, kx-1)][c] * dy[p][n]
//
// Why a second halo body (wgrad3_body.h is the other). There, a block owns a 32-channel x 64-output-channel tile and
// its 4 waves split the tile's (c, n) fragment COMBOS; every wave walks every pixel of the block's share, so a block
// is as long as its pixel share: at the 16^2 - 64^2 levels 32 blocks of 32 serial 128-pixel tiles each, ~68 us per
// block alone (profiles/r4_probe/mix_probe_head.txt), which the mixed weight-gradient launch must wait out in its
// tail. Here the 4 waves split the REDUCTION instead: each 128-pixel tile's four 32-pixel MFMA k-steps go one to
// each wave, and every wave accumulates the whole block tile - 32 input channels x 32 output channels x 9 taps
// (2 x 2 16x16 fragments per tap, 144 fp32 accumulators) - over its quarter of every tile. Per k-step a wave reads
// its dy fragments once for all 9 taps and each halo fragment once for both output fragments: 40 transposing LDS
// reads per 36 MFMAs (the combo split: 2.2 per MFMA). The four partial tiles are summed through LDS once, at the end.
// With the block tile a quarter of the combo split's (32 x 32 instead of 32 x 64 per 4 waves x ... ) and pixel splits
// chosen for ~16 tiles per block, a 16^2 / 32^2 / 64^2 layer becomes 128-256 short blocks instead of 32 long ones.
//
// Staging is the combo body's: per 128-pixel tile the (8+2) x (16+2) x 32 input halo (producer BN-apply + ReLU and
// the nearest-2x upsample folded into the load, padding exactly 0) and the 128 x 32 dy tile, loaded RAW one tile
// ahead into registers (clamped in-image addresses, validity bits) and masked + transformed on the LDS store after
// the current tile's MFMAs; 96-byte LDS rows keep the transposing reads (8 consecutive pixel rows x 32 bytes per
// 32-lane group) conflict-free for every tap shift.
#pragma once
#include "common.h"
#include "launch.h"

namespace {
namespace wg3s {

constexpr int NT = 256;
constexpr int CB = 32;                    // input channels per block (A rows)
constexpr int NB = 32;                    // output channels per block (B columns)
constexpr int TH = 8, TW = 16, TP = TH * TW;
constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;
constexpr int LDH = CB + 16, LDD = NB + 16;                    // 96-byte rows
constexpr int HALO_CH = HP * (CB / 8), H_PER_T = (HALO_CH + NT - 1) / NT;
constexpr int D_CH = TP * (NB / 8), D_PER_T = (D_CH + NT - 1) / NT;
constexpr int LDS_BYTES = 2 * HP * LDH * 2 + 2 * TP * LDD * 2;
constexpr int RED_ITEMS = 3 * 2 * 2 * 4;                       // accumulators per lane per 3-tap reduction round
static_assert(4 * RED_ITEMS * 64 * 4 <= LDS_BYTES, "reduction rounds fit the staging buffers");
static_assert(D_CH % NT == 0, "dy staging: whole chunks per thread");

typedef short s4v_lds __attribute__((ext_vector_type(4)));

CFL_DEVICE s4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4v_lds __attribute__((address_space(3)))*)(p));
}

// TR: accumulate D[n][c] (16 contiguous c per output row: the Conv2DTranspose (kh,kw,out,in) layout), else D[c][n]
template <bool TR>
CFL_DEVICE void wgrad3sk_body(const WgradParams& p, int tiles_total, int splits, int bx, int by, int bz,
                              unsigned char* smem) {
  bf16_t (*sH)[HP][LDH] = reinterpret_cast<bf16_t (*)[HP][LDH]>(smem);
  bf16_t (*sD)[TP][LDD] = reinterpret_cast<bf16_t (*)[TP][LDD]>(smem + 2 * HP * LDH * 2);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cbase = bx * CB, nBlock = by * NB;
  const int tiles_w = (p.Wo + TW - 1) / TW, tiles_h = (p.Ho + TH - 1) / TH;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;
  float a8[8], b8[8];                      // this thread's 8 halo channels are fixed: quarter tid & 3
  load_f8_or(p.xf.ab + cbase + (tid & 3) * 8, has_ab, 1.f, a8);
  load_f8_or(p.xf.ab + p.xf.C + cbase + (tid & 3) * 8, has_ab, 0.f, b8);

  uint4 rh[H_PER_T], rd[D_PER_T];
  uint32_t hval = 0, dval = 0;
  auto load = [&](int t) {
    const int b = t / (tiles_w * tiles_h);
    const int r = t - b * tiles_w * tiles_h;
    const int ty0 = (r / tiles_w) * TH, tx0 = (r % tiles_w) * TW;
    hval = 0;
    dval = 0;
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      const int ec = e < HALO_CH ? e : HALO_CH - 1;
      const int hp = ec >> 2, q = ec & 3;
      const int hy = hp / HW, hx = hp - hy * HW;
      const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
      const bool ok = e < HALO_CH && iy >= 0 && iy < Hl && ix >= 0 && ix < Wl;
      const int iyc = imin(imax(iy, 0), Hl - 1), ixc = imin(imax(ix, 0), Wl - 1);
      rh[i] = *reinterpret_cast<const uint4*>(
          p.x + (((size_t)b * p.Hin + (iyc >> p.up_in)) * p.Win + (ixc >> p.up_in)) * p.Cin + cbase + q * 8);
      hval |= (uint32_t)ok << i;
    }
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      const int e = tid + i * NT;
      const int pp = e >> 2, q = e & 3;
      const int oy = ty0 + pp / TW, ox = tx0 + pp % TW;
      const bool ok = oy < p.Ho && ox < p.Wo;
      rd[i] = *reinterpret_cast<const uint4*>(
          p.dy + (((size_t)b * p.Ho + imin(oy, p.Ho - 1)) * p.Wo + imin(ox, p.Wo - 1)) * p.N + nBlock + q * 8);
      dval |= (uint32_t)ok << i;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < HALO_CH) {
        uint4 v = rh[i];
        if (!((hval >> i) & 1u)) {
          v = make_uint4(0, 0, 0, 0);                 // padding stays exactly 0 (TF SAME pads the transformed input)
        } else if (has_ab || relu) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (has_ab) f[j] = fmaf(a8[j], f[j], b8[j]);
            if (relu) f[j] = fmaxf(f[j], 0.f);
          }
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(&sH[buf][e >> 2][(e & 3) * 8]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      const int e = tid + i * NT;
      *reinterpret_cast<uint4*>(&sD[buf][e >> 2][(e & 3) * 8]) = ((dval >> i) & 1u) ? rd[i] : make_uint4(0, 0, 0, 0);
    }
  };

  f4v acc[9][2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int cf = 0; cf < 2; ++cf)
#pragma unroll
      for (int nf = 0; nf < 2; ++nf) acc[t][cf][nf] = f4v{0.f, 0.f, 0.f, 0.f};

  // this wave's k-step of every tile: pixels 32 wid .. 32 wid + 31; lane rows p0 (elements 0-3) and p0 + 16 (4-7)
  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
  const int p0 = 32 * wid + 4 * g + q, p1 = p0 + 16;
  const int h0 = (p0 / TW) * HW + (p0 % TW), h1 = (p1 / TW) * HW + (p1 % TW);

  int t = bz;
  if (t < tiles_total) {
    load(t);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (; t < tiles_total; t += splits) {
    const bool more = t + splits < tiles_total;
    if (more) load(t + splits);
    s8v bop[2];
#pragma unroll
    for (int nf = 0; nf < 2; ++nf) {
      const s4v lo = tr_read(&sD[buf][p0][16 * nf + 4 * pq]);
      const s4v hi = tr_read(&sD[buf][p1][16 * nf + 4 * pq]);
      bop[nf] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int sh = (tap / 3) * HW + (tap % 3);
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) {
        const s4v lo = tr_read(&sH[buf][h0 + sh][16 * cf + 4 * pq]);
        const s4v hi = tr_read(&sH[buf][h1 + sh][16 * cf + 4 * pq]);
        const s8v aop = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int nf = 0; nf < 2; ++nf) {
          if (TR) acc[tap][cf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bop[nf], aop, acc[tap][cf][nf], 0, 0, 0);
          else acc[tap][cf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aop, bop[nf], acc[tap][cf][nf], 0, 0, 0);
        }
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // ---- the four waves' partial tiles -> one, through LDS, 3 taps per round (the loop ended on a barrier: the
  //      staging buffers are free). red[w][item][lane], item = ((tt * 2 + cf) * 2 + nf) * 4 + r. Output element of
  //      (tap, cf, nf, r, lane): D col = lane & 15, row = (lane >> 4) * 4 + r.
  //      Slab mode: this split's own row of the slab, plain stores (one writer per element); otherwise fp32
  //      atomics (int64 fixed point in the deterministic mode) into the destination.
  float* red = reinterpret_cast<float*>(smem);
  const bool slab = p.slabs > 0;
  float* dwb = slab ? p.dw + (size_t)bz * 9 * p.Cin * p.N : p.dw;
#pragma unroll
  for (int R = 0; R < 3; ++R) {
#pragma unroll
    for (int tt = 0; tt < 3; ++tt)
#pragma unroll
      for (int cf = 0; cf < 2; ++cf)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            red[(wid * RED_ITEMS + ((tt * 2 + cf) * 2 + nf) * 4 + r) * 64 + lane] = acc[3 * R + tt][cf][nf][r];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RED_ITEMS * 64 / NT; ++k) {
      const int e = tid + k * NT, it = e >> 6, ln = e & 63;
      const float v = red[(0 * RED_ITEMS + it) * 64 + ln] + red[(1 * RED_ITEMS + it) * 64 + ln] +
                      red[(2 * RED_ITEMS + it) * 64 + ln] + red[(3 * RED_ITEMS + it) * 64 + ln];
      const int r = it & 3, nf = (it >> 2) & 1, cf = (it >> 3) & 1, tap = 3 * R + (it >> 4);
      const int rr = (ln >> 4) * 4 + r, cc = ln & 15;
      size_t dst;
      if (TR) {
        const int n = nBlock + 16 * nf + rr, c = cbase + 16 * cf + cc;
        dst = ((size_t)(8 - tap) * p.N + n) * p.Cin + c;
      } else {
        const int n = nBlock + 16 * nf + cc, c = cbase + 16 * cf + rr;
        dst = ((size_t)tap * p.Cin + c) * p.N + n;
      }
      if (slab) dwb[dst] = v;
      else red_add(p.dw, dst, v, CFL_FX_G);
    }
    __syncthreads();
  }
}

}  // namespace wg3s
}  // namespace
