// The halo weight-gradient body of conv3x3_wgrad.hip (its design notes are there), in a header so the mixed
// weight-gradient launch of conv_wgrad.hip (wgrad_mix_kernel) can run it next to the generic bodies.
#pragma once
#include "common.h"
#include "launch.h"

namespace {
namespace wg3 {

constexpr int NT = 256;
constexpr int CB = 32;            // input channels per block (the A-operand rows)
constexpr int TH = 8, TW = 16, TP = TH * TW;
constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;
constexpr int LDH = CB + 16;     // 96-byte halo rows (see the layout note in conv3x3_wgrad.hip)

typedef short s4v_lds __attribute__((ext_vector_type(4)));

CFL_DEVICE s4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4v_lds __attribute__((address_space(3)))*)(p));
}

// LDS bytes of one block of the BNO config: two halo images + two dy tiles (the caller owns the allocation, so a
// grouped launch of several wgrad kinds can share one buffer: conv_wgrad.hip wgrad_mix_kernel)
template <int BNO>
constexpr int wgrad3_lds_bytes() { return 2 * HP * LDH * 2 + 2 * TP * (BNO + 16) * 2; }

// TR: accumulate D[n][c] instead of D[c][n] so that the 16 contiguous accumulator columns land on contiguous
// addresses of the destination layout (c for the Conv2DTranspose (kh,kw,out,in) layout, n for HWIO): each atomic
// wave-instruction then adds 4 x 64 B segments instead of 64 scattered dwords.
template <int BNO, bool TR>
CFL_DEVICE void wgrad3_body(const WgradParams& p, int tiles_total, int splits, int bx, int by, int bz,
                            unsigned char* smem) {
  constexpr int NF = BNO / 16;              // n fragments
  constexpr int COMBOS = 2 * NF;            // (c fragment, n fragment) pairs per tap
  constexpr int CPW = COMBOS / 4;           // combos per wave
  constexpr int LDD = BNO + 16;    // 96 / 160-byte dy rows
  constexpr int HALO_CH = HP * (CB / 8), H_PER_T = (HALO_CH + NT - 1) / NT;
  constexpr int D_CH = TP * (BNO / 8), D_PER_T = (D_CH + NT - 1) / NT;
  static_assert(COMBOS % 4 == 0, "combos must split over 4 waves");
  bf16_t (*sH)[HP][LDH] = reinterpret_cast<bf16_t (*)[HP][LDH]>(smem);
  bf16_t (*sD)[TP][LDD] = reinterpret_cast<bf16_t (*)[TP][LDD]>(smem + 2 * HP * LDH * 2);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cbase = bx * CB, nBlock = by * BNO;
  const int tiles_w = (p.Wo + TW - 1) / TW, tiles_h = (p.Ho + TH - 1) / TH;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  float a8[8], b8[8];
  load_f8_or(p.xf.ab + cbase + (tid & 3) * 8, has_ab, 1.f, a8);
  load_f8_or(p.xf.ab + p.xf.C + cbase + (tid & 3) * 8, has_ab, 0.f, b8);

  // The next tile's halo / dy chunks are loaded RAW, branch-free (clamped in-image addresses, a validity bit per
  // chunk) and only masked + transformed (producer BN-apply + ReLU) in store(), after the current tile's MFMAs:
  // transformed right after the load, the prefetch was consumed at issue and every tile waited its full load
  // latency (~2.4 us per 128-pixel tile against ~0.5 us of MFMAs).
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
      const int ec = e < D_CH ? e : D_CH - 1;
      const int pp = ec / (BNO / 8), q = ec % (BNO / 8);
      const int oy = ty0 + pp / TW, ox = tx0 + pp % TW;
      const bool ok = e < D_CH && oy < p.Ho && ox < p.Wo;
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
        } else if (has_ab || p.xf.relu) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            if (has_ab) f[j] = fmaf(a8[j], f[j], b8[j]);
            if (p.xf.relu) f[j] = fmaxf(f[j], 0.f);
          }
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(&sH[buf][e >> 2][(e & 3) * 8]) = v;
      }
    }
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < D_CH)
        *reinterpret_cast<uint4*>(&sD[buf][e / (BNO / 8)][(e % (BNO / 8)) * 8]) =
            ((dval >> i) & 1u) ? rd[i] : make_uint4(0, 0, 0, 0);
    }
  };

  // this wave's (c fragment, n fragment) combos
  int cf[CPW], nf[CPW];
#pragma unroll
  for (int u = 0; u < CPW; ++u) {
    const int combo = wid * CPW + u;
    cf[u] = combo / NF;
    nf[u] = combo % NF;
  }
  f4v acc[9][CPW];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < CPW; ++u) acc[t][u] = f4v{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane & 15) >> 2, pq = lane & 3;
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
#pragma unroll
    for (int j = 0; j < TP / 32; ++j) {            // pixel k-steps of 32
      const int p0 = 32 * j + 4 * g + q;            // this lane's pixel rows: p0 (elements 0-3) and p0 + 16
      const int p1 = p0 + 16;
      s8v bop[CPW];
#pragma unroll
      for (int u = 0; u < CPW; ++u) {
        const s4v lo = tr_read(&sD[buf][p0][16 * nf[u] + 4 * pq]);
        const s4v hi = tr_read(&sD[buf][p1][16 * nf[u] + 4 * pq]);
        bop[u] = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int h0 = (p0 / TW) * HW + (p0 % TW), h1 = (p1 / TW) * HW + (p1 % TW);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int sh = (tap / 3) * HW + (tap % 3);
#pragma unroll
        for (int u = 0; u < CPW; ++u) {
          const s4v lo = tr_read(&sH[buf][h0 + sh][16 * cf[u] + 4 * pq]);
          const s4v hi = tr_read(&sH[buf][h1 + sh][16 * cf[u] + 4 * pq]);
          const s8v aop = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          if (TR) acc[tap][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bop[u], aop, acc[tap][u], 0, 0, 0);
          else acc[tap][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aop, bop[u], acc[tap][u], 0, 0, 0);
        }
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // D col = lane&15, row = (lane>>4)*4 + r;  TR: D[n][c] -> (8-tap, n, c) layout, else D[c][n] -> (tap, c, n).
  // Slab mode: this split's own row of the slab, plain stores (each element has exactly one writer); otherwise
  // fp32 atomics into the destination.
  const bool slab = p.slabs > 0;
  float* dwb = slab ? p.dw + (size_t)bz * 9 * p.Cin * p.N : p.dw;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int u = 0; u < CPW; ++u) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        size_t dst;
        if (TR) {
          const int n = nBlock + 16 * nf[u] + rr, c = cbase + 16 * cf[u] + cc;
          dst = ((size_t)(8 - tap) * p.N + n) * p.Cin + c;
        } else {
          const int n = nBlock + 16 * nf[u] + cc, c = cbase + 16 * cf[u] + rr;
          dst = ((size_t)tap * p.Cin + c) * p.N + n;
        }
        if (slab) dwb[dst] = acc[tap][u][r];
        else red_add(p.dw, dst, acc[tap][u][r], CFL_FX_G);
      }
    }
}

}  // namespace wg3
}  // namespace
