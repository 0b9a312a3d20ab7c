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

#include "wgrad3_body.h"

namespace {

using namespace wg3;

template <int BNO, bool TR, int CBT = CB, bool SB = false>
__global__ __launch_bounds__(NT, 2) void conv3x3_wgrad_kernel(WgradParams p, int tiles_total, int splits) {
  CFL_TS_GUARD;
  __shared__ __attribute__((aligned(16))) unsigned char smem[wgrad3_lds_bytes<BNO, CBT, SB>()];
  wgrad3_body<BNO, TR, CBT, SB>(p, tiles_total, splits, blockIdx.x, blockIdx.y, blockIdx.z, smem);
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
  CFL_TS_GUARD;
  __shared__ __attribute__((aligned(16))) unsigned char smem[wgrad3_lds_bytes<BNO>()];
  int k = 0;
  while (k + 1 < g.n && g.it[k + 1].block0 <= (int)blockIdx.x) ++k;
  const Wgrad3Item& I = g.it[k];
  const int local = blockIdx.x - I.block0;
  const int bx = local % I.gx, r = local / I.gx;
  wgrad3_body<BNO, TR>(I.p, I.tiles, I.splits, bx, r % I.gy, r / I.gy, smem);
}

}  // namespace

// input channels per block: 64 (wgrad3_body CBT = 64, one LDS buffer) for the large launches - a layer's dy is then
// re-read Cin / 64 times instead of Cin / 32 and each staged tile feeds twice the MFMAs - else 32
// (TUNE_WGRAD3_WIDE: 0 = auto, 1 = never, 2 = whenever Cin % 64 == 0)
int conv3x3_wgrad_cbt(const WgradParams& p) {
  const int v = cfl_tune(TUNE_WGRAD3_WIDE);
  if (v == 1 || p.Cin % 64) return CB;
  if (v == 2) return 64;
  const int64_t tiles = (int64_t)((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * p.B;
  return tiles * (p.Cin / CB) >= 65536 ? 64 : CB;
}

bool conv3x3_wgrad_supported(const WgradParams& p) {
  // the body reads one image through a buffer resource with 32-bit byte offsets built from 24-bit products, and
  // 0x80000000 as its out-of-range offset (wgrad3_body.h load)
  const bool fits = (int64_t)p.Hin * p.Win * p.Cin * 2 < (1ll << 31) && (int64_t)p.Win * p.Cin * 2 < (1 << 24) &&
                    (int64_t)p.Ho * p.Wo * p.N * 2 < (1ll << 31) && (int64_t)p.Wo * p.N * 2 < (1 << 24);
  return p.ks == 3 && p.stride == 1 && p.pad_t == 1 && p.pad_l == 1 && p.Cin % CB == 0 && p.N % 32 == 0 &&
         p.Ho >= 8 && p.Wo >= 8 && fits;
}

void conv3x3_wgrad_shape(const WgradParams& p, int& bno, int& tiles, int& splits) {
  tiles = ((p.Ho + TH - 1) / TH) * ((p.Wo + TW - 1) / TW) * p.B;
  bno = p.N % 64 == 0 ? 64 : 32;
  const int xy = (p.Cin / conv3x3_wgrad_cbt(p)) * (p.N / bno);
  const int target = cfl_tune(TUNE_WGRAD3_BLOCKS) > 0 ? cfl_tune(TUNE_WGRAD3_BLOCKS) : 512;
  // >= 16 pixel tiles per block: the engine launches the decoder's halo wgrads grouped (conv3x3_wgrad_grouped), so
  // long blocks still fill the chip, and every pixel split is one plain-stored slab row that grad_finish must read
  // (whole-step A/B on one MI355X: 4 / 8 / 16 / 24 / 32 -> 1.733 / 1.706 / 1.691 / 1.729 / 1.782 ms/iteration)
  // (mixed launch, round 3: 16 / 32 tiles -> 1.3718 / 1.3554 ms per iteration: fewer, longer blocks co-run with the
  // other weight gradients and leave a third of the slab rows for grad_finish)
  int min_tiles = cfl_tune(TUNE_WGRAD3_MINTILES) > 0 ? cfl_tune(TUNE_WGRAD3_MINTILES) : 32;
  // the 32-wide output tiles (the N = 32 layers at 128^2: 1-2 channel blocks, so few blocks per pixel split): alone
  // in their group launch they took shorter blocks (4 tiles); in the mixed launch (conv_wgrad.hip wgrad_mix_kernel),
  // co-running with the other layers, longer blocks - a quarter of the slab rows for grad_finish - measured faster:
  // 4 / 8 / 16 tiles -> 1.3797 / 1.3770 / 1.3698 ms per iteration (one MI355X, driver-style bench)
  if (bno == 32) min_tiles = cfl_tune(TUNE_WGRAD3_MINTILES32) > 0 ? cfl_tune(TUNE_WGRAD3_MINTILES32) : 16;
  splits = (target + xy - 1) / xy;
  const int max_splits = (tiles + min_tiles - 1) / min_tiles;   // amortise each block's output write
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
}

int conv3x3_wgrad_splits(const WgradParams& p) {
  int bno, tiles, splits;
  conv3x3_wgrad_shape(p, bno, tiles, splits);
  return splits;
}

// tile config of a (supported) 3x3 wgrad: 0 = <64,TR>, 1 = <64,HWIO>, 2 = <32,TR>, 3 = <32,HWIO>; 64-channel
// blocks: 6 = <64,TR>, 7 = <64,HWIO>, 8 = <32,TR>, 9 = <32,HWIO> (4, 5: retired split-K-in-block body, round 6)
int conv3x3_wgrad_config(const WgradParams& p) {
  int bno, tiles, splits;
  conv3x3_wgrad_shape(p, bno, tiles, splits);
  return (conv3x3_wgrad_cbt(p) == 64 ? 6 : 0) + (bno == 64 ? 0 : 2) + (p.dst_mode == 1 ? 0 : 1);
}

int conv3x3_wgrad(const WgradParams& p, hipStream_t st);

// n problems of ONE tile config (conv3x3_wgrad_config) in grouped launches of up to WG_MAX
int conv3x3_wgrad_grouped(const WgradParams* ps, int n, hipStream_t st) {
  for (int i0 = 0; i0 < n; i0 += WG_MAX) {
    Wgrad3Group g{};
    int blocks = 0, cfg = -1;
    for (int i = i0; i < n && i < i0 + WG_MAX; ++i) {
      const WgradParams& p = ps[i];
      if (!conv3x3_wgrad_supported(p)) return 1;
      int bno, tiles, splits;
      conv3x3_wgrad_shape(p, bno, tiles, splits);
      if (p.slabs > 0 && p.slabs != splits) return 2;
      const int c = conv3x3_wgrad_config(p);
      if (c >= 4) {                                   // 64-channel bodies: launched on their own
        const int rc = conv3x3_wgrad(p, st);
        if (rc) return rc;
        continue;
      }
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
    if (g.n == 0) continue;
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
  conv3x3_wgrad_shape(p, bno, tiles, splits);
  if (p.slabs > 0 && p.slabs != splits) return 2;
  dim3 grid(p.Cin / conv3x3_wgrad_cbt(p), p.N / bno, splits);
  const bool tr = p.dst_mode == 1;
  if (conv3x3_wgrad_cbt(p) == 64) {
    if (bno == 64 && tr)
      hipLaunchKernelGGL((conv3x3_wgrad_kernel<64, true, 64, true>), grid, dim3(NT), 0, st, p, tiles, splits);
    else if (bno == 64)
      hipLaunchKernelGGL((conv3x3_wgrad_kernel<64, false, 64, true>), grid, dim3(NT), 0, st, p, tiles, splits);
    else if (tr)
      hipLaunchKernelGGL((conv3x3_wgrad_kernel<32, true, 64, true>), grid, dim3(NT), 0, st, p, tiles, splits);
    else
      hipLaunchKernelGGL((conv3x3_wgrad_kernel<32, false, 64, true>), grid, dim3(NT), 0, st, p, tiles, splits);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  if (bno == 64 && tr) hipLaunchKernelGGL((conv3x3_wgrad_kernel<64, true>), grid, dim3(NT), 0, st, p, tiles, splits);
  else if (bno == 64) hipLaunchKernelGGL((conv3x3_wgrad_kernel<64, false>), grid, dim3(NT), 0, st, p, tiles, splits);
  else if (tr) hipLaunchKernelGGL((conv3x3_wgrad_kernel<32, true>), grid, dim3(NT), 0, st, p, tiles, splits);
  else hipLaunchKernelGGL((conv3x3_wgrad_kernel<32, false>), grid, dim3(NT), 0, st, p, tiles, splits);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_conv3x3_wgrad(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_conv3x3_wgrad(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
