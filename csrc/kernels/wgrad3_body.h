// The halo weight-gradient body of conv3x3_wgrad.hip (its design notes are there), in a header so the mixed
// weight-gradient launch of conv_wgrad.hip (wgrad_mix_kernel) can run it next to the generic bodies.
#pragma once
#include "common.h"
#include "launch.h"

namespace {
namespace wg3 {

constexpr int NT = 256;
constexpr int CB = 32;            // input channels per block (the A-operand rows) of the default configs
constexpr int TH = 8, TW = 16, TP = TH * TW;
constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;
static_assert(div_small_ok<HW, HP>(), "halo pixel division by multiply-shift (common.h div_small)");

typedef short s4v_lds __attribute__((ext_vector_type(4)));

CFL_DEVICE s4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4v_lds __attribute__((address_space(3)))*)(p));
}

// halo rows: CBT input channels + 16 bf16 of padding (96 / 160 bytes, see the layout note in conv3x3_wgrad.hip)
#ifndef WG3_HPAD
#define WG3_HPAD 16
#endif
#ifndef WG3_DPAD
#define WG3_DPAD 16
#endif
template <int CBT>
constexpr int ldh() { return CBT + WG3_HPAD; }

// LDS bytes of one block of the (BNO, CBT) config: two halo images + two dy tiles, SB (single buffer): one of each
// (the caller owns the allocation, so a grouped launch of several wgrad kinds can share one buffer: conv_wgrad.hip
// wgrad_mix_kernel)
template <int BNO, int CBT = CB, bool SB = false>
constexpr int wgrad3_lds_bytes() { return (SB ? 1 : 2) * (HP * ldh<CBT>() * 2 + TP * (BNO + WG3_DPAD) * 2); }

// TR: accumulate D[n][c] instead of D[c][n] so that the 16 contiguous accumulator columns land on contiguous
// addresses of the destination layout (c for the Conv2DTranspose (kh,kw,out,in) layout, n for HWIO): each atomic
// wave-instruction then adds 4 x 64 B segments instead of 64 scattered dwords.
// CBT: input channels per block (32, or 64 for the large launches: each dy tile then serves twice the channels, so
// a layer's dy is re-read Cin / 64 instead of Cin / 32 times, and each staged byte feeds twice the MFMAs).
// SB: one LDS buffer (the 64-channel configs: two would leave one block per CU); the next tile's registers are
// stored between two barriers instead of into the other buffer.
template <int BNO, bool TR, int CBT = CB, bool SB = false>
CFL_DEVICE void wgrad3_body(const WgradParams& p, int tiles_total, int splits, int bx, int by, int bz,
                            unsigned char* smem) {
  constexpr int NF = BNO / 16;              // n fragments
  constexpr int COMBOS = (CBT / 16) * NF;   // (c fragment, n fragment) pairs per tap
  constexpr int CPW = COMBOS / 4;           // combos per wave
  constexpr int LDH = ldh<CBT>();
  constexpr int LDD = BNO + WG3_DPAD;    // 96 / 160-byte dy rows
  constexpr int QP = CBT / 8;               // 16-byte pieces per halo pixel
  constexpr int HALO_CH = HP * QP, H_PER_T = (HALO_CH + NT - 1) / NT;
  constexpr int D_CH = TP * (BNO / 8), D_PER_T = (D_CH + NT - 1) / NT;
  constexpr int NBUF = SB ? 1 : 2;
  static_assert(COMBOS % 4 == 0, "combos must split over 4 waves");
  static_assert(CPW <= NF && NF % CPW == 0, "a wave's combos share one c fragment (one A read per tap)");
  static_assert(NT % QP == 0, "a thread's halo channel piece is the same in every staged chunk");
  bf16_t (*sH)[HP][LDH] = reinterpret_cast<bf16_t (*)[HP][LDH]>(smem);
  bf16_t (*sD)[TP][LDD] = reinterpret_cast<bf16_t (*)[TP][LDD]>(smem + NBUF * HP * LDH * 2);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cbase = bx * CBT, nBlock = by * BNO;
  const int tiles_w = (p.Wo + TW - 1) / TW, tiles_h = (p.Ho + TH - 1) / TH;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  // producer BN coefficients of this thread's 8 halo channels: held in registers, or (the 144-accumulator config)
  // re-read at each tile's store (L1 / L2 hits) to leave the registers to the accumulators
  constexpr bool AB_REG = CPW < 4;
  float a8[8], b8[8];
  if constexpr (AB_REG) {
    load_f8_or(p.xf.ab + cbase + (tid % QP) * 8, has_ab, 1.f, a8);
    load_f8_or(p.xf.ab + p.xf.C + cbase + (tid % QP) * 8, has_ab, 0.f, b8);
  }

  // The next tile's halo / dy chunks are loaded RAW, branch-free (clamped in-image addresses, a validity bit per
  // chunk) and only masked + transformed (producer BN-apply + ReLU) in store(), after the current tile's MFMAs:
  // transformed right after the load, the prefetch was consumed at issue and every tile waited its full load
  // latency (~2.4 us per 128-pixel tile against ~0.5 us of MFMAs).
  uint4 rh[H_PER_T], rd[D_PER_T];
  uint32_t hval = 0;
  // Chunk addressing: a thread's 16-byte channel piece is the same in every chunk (NT % QP == 0, NT % (BNO/8) == 0)
  // and its chunk pixels step by a constant, so per tile a chunk costs a few full-rate ops: 24-bit products into a
  // 32-bit byte offset from the tile image's base pointer (uniform, 64-bit: one layer of the 512^2 planned batch
  // spans more than 4 GB, one image never does). The generic form (64-bit products and runtime divisions per chunk,
  // ~150 VALU ops of which ~50 quarter-rate) took ~1,350 of the ~4,900 cycles of a 128-pixel tile step (s_memtime
  // phase stamps of wave 0: issue 1.35k, MFMAs 1.57k, store 1.63k, barrier 0.13k).
  const int hq = tid % QP, hp0 = tid / QP;
  const int dq = tid % (BNO / 8), dp0 = tid / (BNO / 8);
  const unsigned x_row = (unsigned)p.Win * p.Cin * 2u, x_px = (unsigned)p.Cin * 2u;
  const unsigned d_row = (unsigned)p.Wo * p.N * 2u, d_px = (unsigned)p.N * 2u;
  const int x_img = p.Hin * p.Win * p.Cin * 2, d_img = p.Ho * p.Wo * p.N * 2;   // < 2^31 (conv3x3_wgrad_supported)
  constexpr uint32_t OOB = 0x80000000u;          // past every resource's range: the buffer load returns 0
  // tile cursor (image, tile row, tile column) of the tile index, advanced by `splits` per step with carries instead
  // of two runtime divisions per tile (~50 scalar instructions on the step's issue path)
  const int tpi = tiles_w * tiles_h;
  const int s_b = splits / tpi, s_r = splits - s_b * tpi, s_y = s_r / tiles_w, s_x = s_r - s_y * tiles_w;
  int cb = bz / tpi, cy = (bz - cb * tpi) / tiles_w, cx = bz - cb * tpi - cy * tiles_w;
  auto advance = [&]() {
    cx += s_x;
    cy += s_y;
    cb += s_b;
    if (cx >= tiles_w) { cx -= tiles_w; ++cy; }
    if (cy >= tiles_h) { cy -= tiles_h; ++cb; }
  };
  auto load = [&]() {
    const int b = cb, ty0 = cy * TH, tx0 = cx * TW;
    // raw buffer resources over the tile's image (base in scalar registers: no 64-bit address math per chunk)
    const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.x + (size_t)b * p.Hin * p.Win * p.Cin + cbase), 0, x_img, 0x00020000);
    const __amdgpu_buffer_rsrc_t rs_d = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.dy + (size_t)b * p.Ho * p.Wo * p.N + nBlock), 0, d_img, 0x00020000);
    hval = 0;
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int hp = hp0 + i * (NT / QP);
      const bool in = (i + 1) * NT <= HALO_CH || hp < HP;
      const int hpc = (i + 1) * NT <= HALO_CH ? hp : imin(hp, HP - 1);
      const int hy = div_small<HW>(hpc), hx = hpc - hy * HW;
      const int iy = ty0 - 1 + hy, ix = tx0 - 1 + hx;
      const bool ok = in && (unsigned)iy < (unsigned)Hl && (unsigned)ix < (unsigned)Wl;
      const unsigned iyc = (unsigned)imin(imax(iy, 0), Hl - 1) >> p.up_in;
      const unsigned ixc = (unsigned)imin(imax(ix, 0), Wl - 1) >> p.up_in;
      const u4v v = __builtin_amdgcn_raw_buffer_load_b128(rs_x, __umul24(iyc, x_row) + __umul24(ixc, x_px) + hq * 16,
                                                          0, 0);
      rh[i] = make_uint4(v.x, v.y, v.z, v.w);
      hval |= (uint32_t)ok << i;
    }
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      // dy outside the map (a partial tile) reads as 0 from the out-of-range offset
      const int pp = dp0 + i * (NT / (BNO / 8));
      const int oy = ty0 + pp / TW, ox = tx0 + pp % TW;
      const bool ok = ((i + 1) * NT <= D_CH || pp < TP) && oy < p.Ho && ox < p.Wo;
      const u4v v = __builtin_amdgcn_raw_buffer_load_b128(
          rs_d, ok ? __umul24((unsigned)oy, d_row) + __umul24((unsigned)ox, d_px) + dq * 16 : OOB, 0, 0);
      rd[i] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  const uint32_t relu_lo = p.xf.relu ? 0u : 0x80008000u;
  auto store = [&](int buf) {
    if constexpr (!AB_REG) {
      load_f8_or(p.xf.ab + cbase + hq * 8, has_ab, 1.f, a8);
      load_f8_or(p.xf.ab + p.xf.C + cbase + hq * 8, has_ab, 0.f, b8);
    }
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < HALO_CH) {
        // producer BN-apply + ReLU, then padding exactly 0 (TF SAME pads the transformed input)
        const uint32_t m = ((hval >> i) & 1u) ? 0xffffffffu : 0u;
        const uint4 v = rh[i];
        uint4 o;
        o.x = xform2(v.x, f32x2_t{a8[0], a8[1]}, f32x2_t{b8[0], b8[1]}, relu_lo) & m;
        o.y = xform2(v.y, f32x2_t{a8[2], a8[3]}, f32x2_t{b8[2], b8[3]}, relu_lo) & m;
        o.z = xform2(v.z, f32x2_t{a8[4], a8[5]}, f32x2_t{b8[4], b8[5]}, relu_lo) & m;
        o.w = xform2(v.w, f32x2_t{a8[6], a8[7]}, f32x2_t{b8[6], b8[7]}, relu_lo) & m;
        *reinterpret_cast<uint4*>(&sH[buf][e / QP][(e % QP) * 8]) = o;
      }
    }
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < D_CH) *reinterpret_cast<uint4*>(&sD[buf][e / (BNO / 8)][(e % (BNO / 8)) * 8]) = rd[i];
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
    load();
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (; t < tiles_total; t += splits) {
    const bool more = t + splits < tiles_total;
    advance();
    if (more) load();
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
        // the wave's combos share c fragment cf[0] (static_assert above): one A read per tap
        const s4v lo = tr_read(&sH[buf][h0 + sh][16 * cf[0] + 4 * pq]);
        const s4v hi = tr_read(&sH[buf][h1 + sh][16 * cf[0] + 4 * pq]);
        const s8v aop = s8v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int u = 0; u < CPW; ++u) {
          if (TR) acc[tap][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bop[u], aop, acc[tap][u], 0, 0, 0);
          else acc[tap][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aop, bop[u], acc[tap][u], 0, 0, 0);
        }
        // 144 accumulators (CBT = BNO = 64): no room to hoist every tap's operand reads
        if constexpr (CPW == 4) __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (SB) {
      __syncthreads();                               // every wave's reads of this tile done
      if (more) store(0);
    } else {
      if (more) store(buf ^ 1);
    }
    __syncthreads();
    buf ^= NBUF - 1;
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
