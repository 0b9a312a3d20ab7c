// Weight gradient of the 3x3 / stride-1 / "same" convolutions (every Conv2DTranspose of the decoder,
// /root/reference/client_fit_model.py:129,133) on gfx950 MFMA with an LDS halo:
//   dW[tap][c][n] = sum_pixels T(x)[p + (ky-1, kx-1)][c] * dy[p][n]
// A block owns one 32-channel input chunk, an N tile (32 or 64 output channels) and a strided set of TH x TW pixel
// tiles. Per pixel tile it stages the (TH+2) x (TW+2) input halo ONCE (BN-apply + ReLU + nearest-2x upsample folded
// into the load) and the dy tile once; the 9 taps are shifted views of the halo. Both MFMA operands need 8
// consecutive PIXELS per lane (the reduction index), which in NHWC are the rows of the staged tiles: they are read
// with the transposing ds_read_b64_tr_b16, each lane supplying its own pixel-row address (so the halo shift is
// just a different address). The next tile is prefetched into registers during the current tile's 9x4 MFMA
// k-steps (one barrier per tile pair). Partial sums over the block's tiles are either added with one fp32 atomic
// per output element per block into the Keras-layout gradient slot, or (slab mode, used by the engine) stored
// plainly into the block's pixel-split row of a slab that grad_finish sums: plain stores run at ~5x the
// memory-side atomic rate and have no same-address serialisation.
// Reduction order / LDS layout: the MFMA k-slots of a 32-pixel step are assigned so that the 32 lanes of each
// ds_read_b64_tr_b16 read 8 CONSECUTIVE pixel rows (lo: 4g+q, hi: 16+4g+q; the same permutation on both operands,
// so the sum is unchanged); with 96-byte halo rows and 96/160-byte dy rows those 8 rows x 32 bytes cover all 64
// banks for any row base (the halo tap shifts move the base). The previous {b..b+3, b+8..b+11} assignment with
// 80/144-byte rows left 2-4-way conflicts (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 46 %).
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr int CB = 32;            // input channels per block (the A-operand rows)
constexpr int TH = 8, TW = 16, TP = TH * TW;
constexpr int HH = TH + 2, HW = TW + 2, HP = HH * HW;
constexpr int LDH = CB + 16;     // 96-byte halo rows (see the layout note above)

typedef short s4v_lds __attribute__((ext_vector_type(4)));

CFL_DEVICE s4v tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4v_lds __attribute__((address_space(3)))*)(p));
}

// TR: accumulate D[n][c] instead of D[c][n] so that the 16 contiguous accumulator columns land on contiguous
// addresses of the destination layout (c for the Conv2DTranspose (kh,kw,out,in) layout, n for HWIO): each atomic
// wave-instruction then adds 4 x 64 B segments instead of 64 scattered dwords.
template <int BNO, bool TR>
CFL_DEVICE void wgrad3_body(const WgradParams& p, int tiles_total, int splits, int bx, int by, int bz) {
  constexpr int NF = BNO / 16;              // n fragments
  constexpr int COMBOS = 2 * NF;            // (c fragment, n fragment) pairs per tap
  constexpr int CPW = COMBOS / 4;           // combos per wave
  constexpr int LDD = BNO + 16;    // 96 / 160-byte dy rows
  constexpr int HALO_CH = HP * (CB / 8), H_PER_T = (HALO_CH + NT - 1) / NT;
  constexpr int D_CH = TP * (BNO / 8), D_PER_T = (D_CH + NT - 1) / NT;
  static_assert(COMBOS % 4 == 0, "combos must split over 4 waves");
  __shared__ __attribute__((aligned(16))) bf16_t sH[2][HP][LDH];
  __shared__ __attribute__((aligned(16))) bf16_t sD[2][TP][LDD];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cbase = bx * CB, nBlock = by * BNO;
  const int tiles_w = (p.Wo + TW - 1) / TW, tiles_h = (p.Ho + TH - 1) / TH;
  const int Hl = p.Hin << p.up_in, Wl = p.Win << p.up_in;
  const bool has_ab = p.xf.ab != nullptr;
  float a8[8], b8[8];
  load_f8_or(p.xf.ab + cbase + (tid & 3) * 8, has_ab, 1.f, a8);
  load_f8_or(p.xf.ab + p.xf.C + cbase + (tid & 3) * 8, has_ab, 0.f, b8);

  uint4 rh[H_PER_T], rd[D_PER_T];
  auto load = [&](int t) {
    const int b = t / (tiles_w * tiles_h);
    const int r = t - b * tiles_w * tiles_h;
    const int ty0 = (r / tiles_w) * TH, tx0 = (r % tiles_w) * TW;
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < HALO_CH) {
        const int hp = e >> 2, q = e & 3;
        const int hy = hp / HW, hx = hp - hy * HW;
        const int iy = ty0 + hy - 1, ix = tx0 + hx - 1;
        if (iy >= 0 && iy < Hl && ix >= 0 && ix < Wl) {
          v = *reinterpret_cast<const uint4*>(
              p.x + (((size_t)b * p.Hin + (iy >> p.up_in)) * p.Win + (ix >> p.up_in)) * p.Cin + cbase + q * 8);
          if (has_ab || p.xf.relu) {
            float f[8];
            unpack8(v, f);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              if (has_ab) f[j] = fmaf(a8[j], f[j], b8[j]);
              if (p.xf.relu) f[j] = fmaxf(f[j], 0.f);
            }
            v = pack8(f);
          }
        }
      }
      rh[i] = v;
    }
#pragma unroll
    for (int i = 0; i < D_PER_T; ++i) {
      const int e = tid + i * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < D_CH) {
        const int pp = e / (BNO / 8), q = e % (BNO / 8);
        const int oy = ty0 + pp / TW, ox = tx0 + pp % TW;
        if (oy < p.Ho && ox < p.Wo)
          v = *reinterpret_cast<const uint4*>(p.dy + (((size_t)b * p.Ho + oy) * p.Wo + ox) * p.N + nBlock + q * 8);
      }
      rd[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < H_PER_T; ++i) {
      const int e = tid + i * NT;
      if (e < HALO_CH) *reinterpret_cast<uint4*>(&sH[buf][e >> 2][(e & 3) * 8]) = rh[i];
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
        else atomicAdd(&dwb[dst], acc[tap][u][r]);
      }
    }
}

template <int BNO, bool TR>
__global__ __launch_bounds__(NT, 2) void conv3x3_wgrad_kernel(WgradParams p, int tiles_total, int splits) {
  wgrad3_body<BNO, TR>(p, tiles_total, splits, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Grouped launch: several independent weight gradients (different layers, same tile config) in ONE grid. Every
// layer's wgrad is off the backward critical path and, alone, a latency-bound grid of a few hundred blocks; the
// engine defers them to the end of backward and issues one launch per tile config, so their blocks co-run.
constexpr int WG_MAX = 8;
struct Wgrad3Item {
  WgradParams p;
  int tiles, splits, gx, gy, block0;
};
struct Wgrad3Group {
  Wgrad3Item it[WG_MAX];
  int n;
};

template <int BNO, bool TR>
__global__ __launch_bounds__(NT, 2) void conv3x3_wgrad_group_kernel(const Wgrad3Group g) {
  int k = 0;
  while (k + 1 < g.n && g.it[k + 1].block0 <= (int)blockIdx.x) ++k;
  const Wgrad3Item& I = g.it[k];
  const int local = blockIdx.x - I.block0;
  const int bx = local % I.gx, r = local / I.gx;
  wgrad3_body<BNO, TR>(I.p, I.tiles, I.splits, bx, r % I.gy, r / I.gy);
}

}  // namespace

bool conv3x3_wgrad_supported(const WgradParams& p) {
  return p.ks == 3 && p.stride == 1 && p.pad_t == 1 && p.pad_l == 1 && p.Cin % CB == 0 && p.N % 32 == 0 &&
         p.Ho >= 8 && p.Wo >= 8;
}

static void wgrad3_shape(const WgradParams& p, int& bno, int& tiles, int& splits) {
  bno = p.N % 64 == 0 ? 64 : 32;
  tiles = ((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * p.B;
  const int xy = (p.Cin / CB) * (p.N / bno);
  const int target = cfl_tune(TUNE_WGRAD3_BLOCKS) > 0 ? cfl_tune(TUNE_WGRAD3_BLOCKS) : 512;
  // >= 16 pixel tiles per block: the engine launches the decoder's halo wgrads grouped (conv3x3_wgrad_grouped), so
  // long blocks still fill the chip, and every pixel split is one plain-stored slab row that grad_finish must read
  // (whole-step A/B on one MI355X: 4 / 8 / 16 / 24 / 32 -> 1.733 / 1.706 / 1.691 / 1.729 / 1.782 ms/iteration)
  int min_tiles = cfl_tune(TUNE_WGRAD3_MINTILES) > 0 ? cfl_tune(TUNE_WGRAD3_MINTILES) : 16;
  // the 32-wide output tiles (the N = 32 layers at 128^2: 1-2 channel blocks, so few blocks per pixel split) take
  // shorter blocks: 4 tiles (whole step 1.4289-1.4326 -> 1.4230-1.4278 ms; 8 = 16 = unchanged, 32 slower)
  if (bno == 32) min_tiles = cfl_tune(TUNE_WGRAD3_MINTILES32) > 0 ? cfl_tune(TUNE_WGRAD3_MINTILES32) : 4;
  splits = (target + xy - 1) / xy;
  const int max_splits = (tiles + min_tiles - 1) / min_tiles;   // amortise each block's output write
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
}

int conv3x3_wgrad_splits(const WgradParams& p) {
  int bno, tiles, splits;
  wgrad3_shape(p, bno, tiles, splits);
  return splits;
}

// tile config of a (supported) 3x3 wgrad: 0 = <64,TR>, 1 = <64,HWIO>, 2 = <32,TR>, 3 = <32,HWIO>
int conv3x3_wgrad_config(const WgradParams& p) {
  int bno, tiles, splits;
  wgrad3_shape(p, bno, tiles, splits);
  return (bno == 64 ? 0 : 2) + (p.dst_mode == 1 ? 0 : 1);
}

// n problems of ONE tile config (conv3x3_wgrad_config) in grouped launches of up to WG_MAX
int conv3x3_wgrad_grouped(const WgradParams* ps, int n, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += WG_MAX) {
    Wgrad3Group g{};
    int blocks = 0, cfg = -1;
    for (int i = i0; i < n && i < i0 + WG_MAX; ++i) {
      const WgradParams& p = ps[i];
      if (!conv3x3_wgrad_supported(p)) return 1;
      int bno, tiles, splits;
      wgrad3_shape(p, bno, tiles, splits);
      if (p.slabs > 0 && p.slabs != splits) return 2;
      const int c = conv3x3_wgrad_config(p);
      if (cfg >= 0 && c != cfg) return 4;
      cfg = c;
      Wgrad3Item& it = g.it[g.n++];
      it.p = p;
      it.tiles = tiles;
      it.splits = splits;
      it.gx = p.Cin / CB;
      it.gy = p.N / bno;
      it.block0 = blocks;
      blocks += it.gx * it.gy * splits;
    }
    switch (cfg) {
      case 0: hipLaunchKernelGGL((conv3x3_wgrad_group_kernel<64, true>), dim3(blocks), dim3(NT), 0, st, g); break;
      case 1: hipLaunchKernelGGL((conv3x3_wgrad_group_kernel<64, false>), dim3(blocks), dim3(NT), 0, st, g); break;
      case 2: hipLaunchKernelGGL((conv3x3_wgrad_group_kernel<32, true>), dim3(blocks), dim3(NT), 0, st, g); break;
      default: hipLaunchKernelGGL((conv3x3_wgrad_group_kernel<32, false>), dim3(blocks), dim3(NT), 0, st, g); break;
    }
    if (hipGetLastError() != hipSuccess) return 3;
  }
  return 0;
}

int conv3x3_wgrad(const WgradParams& p, hipStream_t st) {
  if (!conv3x3_wgrad_supported(p)) return 1;
  int bno, tiles, splits;
  wgrad3_shape(p, bno, tiles, splits);
  if (p.slabs > 0 && p.slabs != splits) return 2;
  dim3 grid(p.Cin / CB, p.N / bno, splits);
  const bool tr = p.dst_mode == 1;
  if (bno == 64 && tr) hipLaunchKernelGGL((conv3x3_wgrad_kernel<64, true>), grid, dim3(NT), 0, st, p, tiles, splits);
  else if (bno == 64) hipLaunchKernelGGL((conv3x3_wgrad_kernel<64, false>), grid, dim3(NT), 0, st, p, tiles, splits);
  else if (tr) hipLaunchKernelGGL((conv3x3_wgrad_kernel<32, true>), grid, dim3(NT), 0, st, p, tiles, splits);
  else hipLaunchKernelGGL((conv3x3_wgrad_kernel<32, false>), grid, dim3(NT), 0, st, p, tiles, splits);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
