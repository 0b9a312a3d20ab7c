// Depthwise 3x3 convolution (SeparableConv2D's first stage, depth_multiplier 1, "same" pad 1):
// /root/reference/client_fit_model.py:109,113. Memory-bound (9 MAC per element).
//
// Work item = 8 channels (one 16-byte vector) x a strip of SW consecutive pixels of one row. The strip's input
// window (3 rows x SW+2 columns) is loaded once, the producer's BN-apply + ReLU (coefficients held in registers)
// applied once per loaded element, and reused by the 3 horizontal taps of every output in the strip. Blocks walk
// whole rows (32-bit indices, shifts). Keras depthwise kernel layout (3,3,C,1) = [tap][C].
// wgrad keeps 72 fp32 partial sums per thread across its items, reduces over the wave's pixel lanes with shuffles
// and over the block's waves through LDS, then one atomic per (tap, channel) per block into one of `replicas`
// copies of the gradient row (grad_finish in optim.hip sums the copies).
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

struct Coef8 {
  float a[8], b[8];
};

CFL_DEVICE void load_coef(const InXform& xf, int c0, Coef8& k) {
  load_f8_or(xf.ab + c0, xf.ab != nullptr, 1.f, k.a);
  load_f8_or(xf.ab + xf.C + c0, xf.ab != nullptr, 0.f, k.b);
}

CFL_DEVICE void load_x8(const bf16_t* p, const Coef8& k, bool has_ab, int relu, float* f) {
  unpack8(*reinterpret_cast<const uint4*>(p), f);
  if (has_ab) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaf(k.a[j], f[j], k.b[j]);
  }
  if (relu) {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
  }
}

CFL_DEVICE void load_w9(const float* w, int C, int c0, float (&wt)[9][8], bool flip) {
#pragma unroll
  for (int t = 0; t < 9; ++t) load_f8(w + (flip ? 8 - t : t) * C + c0, wt[t]);
}

// out[h][w] = sum_{ky,kx} in[h+ky-1][w+kx-1] * wt[ky*3+kx]   (dgrad: the flipped kernel, same form)
template <int SW>
__global__ __launch_bounds__(NT) void dw_conv_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                     bf16_t* __restrict__ y, InXform xf, int B, int H, int W, int C,
                                                     int flip) {
  CFL_TS_GUARD;
  const int G = C >> 3, lg = ilog2(G);
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  const bool has_ab = xf.ab != nullptr;
  Coef8 k;
  load_coef(xf, c0, k);
  float wt[9][8];
  load_w9(w, C, c0, wt, flip != 0);
  const int rows = B * H, items = (W / SW) << lg;
  for (int row = xcd_swizzle(blockIdx.x, gridDim.x); row < rows; row += gridDim.x) {   // halo rows on one XCD
    const int b = row / H, h = row - b * H;
    for (int it = threadIdx.x; it < items; it += NT) {
      const int w0 = (it >> lg) * SW;
      float acc[SW][8];
#pragma unroll
      for (int i = 0; i < SW; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int ih = h + ky - 1;
        if (ih < 0 || ih >= H) continue;
        const bf16_t* src = x + (size_t)(b * H + ih) * W * C + c0;
#pragma unroll
        for (int cx = 0; cx < SW + 2; ++cx) {
          const int iw = w0 + cx - 1;
          if (iw < 0 || iw >= W) continue;
          float f[8];
          load_x8(src + (size_t)iw * C, k, has_ab, xf.relu, f);
#pragma unroll
          for (int kx = 0; kx < 3; ++kx) {
            const int o = cx - kx;
            if (o < 0 || o >= SW) continue;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[o][j] = fmaf(f[j], wt[ky * 3 + kx][j], acc[o][j]);
          }
        }
      }
      bf16_t* dst = y + ((size_t)row * W + w0) * C + c0;
#pragma unroll
      for (int i = 0; i < SW; ++i) *reinterpret_cast<uint4*>(dst + (size_t)i * C) = pack8(acc[i]);
    }
  }
}

template <int SW>
__global__ __launch_bounds__(NT) void dw_wgrad_kernel(DwParams p, int replicas) {
  CFL_TS_GUARD;
  __shared__ float red[4][9][256];
  const int G = p.C >> 3, lg = ilog2(G);
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool has_ab = p.xf.ab != nullptr;
  Coef8 k;
  load_coef(p.xf, c0, k);
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  // flat items (row, strip, channel group): every thread gets work whatever the row width
  const int strips = p.W / SW;
  const int total = (p.B * p.H * strips) << lg;
  for (int it = xcd_swizzle(blockIdx.x, gridDim.x) * NT + threadIdx.x; it < total; it += gridDim.x * NT) {
    const int pix = it >> lg;                       // row * strips + strip
    const int row = pix / strips;
    const int w0 = (pix - row * strips) * SW;
    const int b = row / p.H, h = row - b * p.H;
    float g[SW][8];
#pragma unroll
    for (int i = 0; i < SW; ++i) load8(p.dy + ((size_t)row * p.W + w0 + i) * p.C + c0, g[i]);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int ih = h + ky - 1;
      if (ih < 0 || ih >= p.H) continue;
      const bf16_t* src = p.x + (size_t)(b * p.H + ih) * p.W * p.C + c0;
#pragma unroll
      for (int cx = 0; cx < SW + 2; ++cx) {
        const int iw = w0 + cx - 1;
        if (iw < 0 || iw >= p.W) continue;
        float f[8];
        load_x8(src + (size_t)iw * p.C, k, has_ab, p.xf.relu, f);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int o = cx - kx;
          if (o < 0 || o >= SW) continue;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[ky * 3 + kx][j] = fmaf(f[j], g[o][j], acc[ky * 3 + kx][j]);
        }
      }
    }
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[t][j];
      for (int o = G; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      acc[t][j] = v;
    }
  if (lane < G) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][t][c0 + j] = acc[t][j];
  }
  __syncthreads();
  // one contiguous 9*C row of atomics per block, spread over `replicas` rows (reduced later by grad_finish):
  // every block adding into ONE row serialises at the memory-side atomic units
  const size_t ro = (size_t)(blockIdx.x % replicas) * 9 * p.C;
  for (int e = threadIdx.x; e < 9 * p.C; e += NT) {
    const int t = e / p.C, c = e - t * p.C;
    red_add(p.dw, ro + t * p.C + c, red[0][t][c] + red[1][t][c] + red[2][t][c] + red[3][t][c], CFL_FX_G);
  }
}

// ---- row-streaming variant (default) ----
// A block owns a 32-pixel column strip x 32 channels x a segment of rows and walks down it 4 output rows per step.
// Input rows live in an LDS ring of 10 rows: each input row is fetched once per segment (halo overhead
// (SEG+2)/SEG x 34/32 instead of 6/4 x 34/32 for independent tiles), and the next step's 4 new rows are in flight in
// registers while the current step computes. One barrier per step: the rows written after step s's compute and the
// rows step s reads are 10 consecutive rows, i.e. distinct ring slots.
// Thread = 4 channels x a strip of 4 pixels (8-byte vectors): 36 fp32 weights / tap sums per thread instead of 72
// keeps the kernel at 3 waves per SIMD without spilling.
namespace dws {
constexpr int CT = 32, CPT = 4, G = CT / CPT, P = NT / G, SL = 4, TW = 32, SR = P / (TW / SL);
constexpr int HWp = TW + 2, NRING = 2 * SR + 2;
static_assert(TW * G == NT, "staging map: one thread per (column, channel group) of a row");
// Ring rows are 34 unpadded 64-byte pixels (x0 - 1 .. x0 + 32), pixel px at position pxo(px) = px ^ ((px >> 2) & 3):
// a wave reads 8 pixels 4 apart (its threads' 4-pixel strips) x 8 channel groups, and a plain 64-B pixel stride puts
// those 8 pixels in the same 16 banks; the XOR rotates each group of 4 pixels over all 64 banks (2 passes, the minimum
// for 512 B), and a wave's staging writes (8 consecutive pixels) stay conflict-free. (The previous 80-byte padded
// pixels: 13.7 % bank-conflict cycles in dw_stream, 8.8 % in the fused backward, r5_final/pmc_summary.txt.)
CFL_DEVICE int pxo(int px) { return px ^ ((px >> 2) & 3); }
// SWZ = false: the 80-byte padded pixels (pixel px at px) - the fused backward's two-ring kernel keeps them: the
// swizzled offsets cost it 10 registers it does not have (256 VGPRs at 2 blocks per CU: spills)
template <bool SWZ>
constexpr int ldp() { return SWZ ? CT : CT + 8; }
template <bool SWZ>
CFL_DEVICE int pxs(int px) { return SWZ ? pxo(px) : px; }

CFL_DEVICE void unpack4(const uint2& v, float* f) {
  f[0] = __uint_as_float(v.x << 16);
  f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16);
  f[3] = __uint_as_float(v.y & 0xffff0000u);
}
CFL_DEVICE uint2 pack4(const float* f) {
  return make_uint2(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]));
}
CFL_DEVICE void load_f4(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
}
CFL_DEVICE void load_f4_or(const float* p, bool cond, float dflt, float* f) {
  float4 a = make_float4(dflt, dflt, dflt, dflt);
  if (cond) a = *reinterpret_cast<const float4*>(p);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
}

// Row-major staging map: thread t owns column t / G (0..31) of every staged row, and the first 2*G*NR threads also
// one element of the two right-halo columns 32, 33 (row t / (2G)); q = t % G in both cases. Addresses are then a
// per-thread constant plus a per-row stride, so staging NR rows costs NR + 1 loads and almost no address registers.
// src_b: image b's base + this thread's channel offset; offsets are 32-bit (every tensor < 2^31 elements).
// Every lane issues its loads (padding positions read a clamped in-image address; okm marks them and put() zeroes
// them when the rows are written to LDS, not here - a select right after a load made the compiler wait for it on
// the spot): per-lane branches around loads made the compiler's wait counting give up (vmcnt(0) at the first use of
// any load, draining the prefetch in flight); only block / wave-uniform conditions branch.
template <int NR>
CFL_DEVICE void fetch(const bf16_t* src_b, const DwParams& p, int x0, int row0, bool on, uint2 (&v)[NR + 1],
                      uint32_t& okm) {
  const int tid = threadIdx.x;
  okm = 0;
  v[NR] = make_uint2(0, 0);
  // (on == false - past the segment's last step - still loads, all marked invalid: straight-line code keeps the
  // wait counts exact)
  const int ix = x0 + tid / G - 1;
  const bool colok = on && (unsigned)ix < (unsigned)p.W;
  const int ixc = min(max(ix, 0), p.W - 1);
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int iy = row0 + r;
    const bool ok = colok && (unsigned)iy < (unsigned)p.H;
    const int iyc = min(max(iy, 0), p.H - 1);
    v[r] = *reinterpret_cast<const uint2*>(src_b + (iyc * p.W + ixc) * p.C);
    okm |= (uint32_t)ok << r;
  }
  if (__builtin_amdgcn_readfirstlane(tid) < 2 * G * NR) {    // the right-halo elements (whole waves branch)
    const int iye = row0 + tid / (2 * G), ixe = x0 + TW - 1 + (tid % (2 * G)) / G;
    const bool ok = on && tid < 2 * G * NR && (unsigned)iye < (unsigned)p.H && (unsigned)ixe < (unsigned)p.W;
    const int iyc = min(max(iye, 0), p.H - 1), ixc2 = min(ixe, p.W - 1);
    v[NR] = *reinterpret_cast<const uint2*>(src_b + (iyc * p.W + ixc2) * p.C);
    okm |= (uint32_t)ok << NR;
  }
}

CFL_DEVICE uint2 xform4(uint2 t, bool on, const float* a4, const float* b4, int relu) {
  if (!on) return t;                                         // padding stays zero (TF SAME pads the input)
  const uint32_t lo = relu ? 0u : 0x80008000u;               // packed BN-apply + ReLU (common.h xform2)
  return make_uint2(xform2(t.x, f32x2_t{a4[0], a4[1]}, f32x2_t{b4[0], b4[1]}, lo),
                    xform2(t.y, f32x2_t{a4[2], a4[3]}, f32x2_t{b4[2], b4[3]}, lo));
}

template <int NR, bool SWZ>
CFL_DEVICE void put(bf16_t* sH, const uint2 (&v)[NR + 1], uint32_t okm, int row0, bool xform, const float* a4,
                    const float* b4, int relu) {
  const int tid = threadIdx.x, q = tid % G;
  const int slot0 = (row0 + NRING) % NRING;                  // row0 >= -1
  constexpr int LDP = ldp<SWZ>();
  bf16_t* col = sH + pxs<SWZ>(tid / G) * LDP + q * CPT;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int slot = slot0 + r >= NRING ? slot0 + r - NRING : slot0 + r;
    const bool ok = (okm >> r) & 1u;
    *reinterpret_cast<uint2*>(col + slot * HWp * LDP) = xform4(ok ? v[r] : make_uint2(0, 0), xform && ok, a4, b4, relu);
  }
  if (tid < 2 * G * NR) {
    const int re = tid / (2 * G), hxe = TW + (tid % (2 * G)) / G;
    const int slot = slot0 + re >= NRING ? slot0 + re - NRING : slot0 + re;
    const bool ok = (okm >> NR) & 1u;
    *reinterpret_cast<uint2*>(sH + (slot * HWp + pxs<SWZ>(hxe)) * LDP + q * CPT) =
        xform4(ok ? v[NR] : make_uint2(0, 0), xform && ok, a4, b4, relu);
  }
}
}  // namespace dws

// bid / nblocks: this block's index in, and the size of, its launch (or its item of a grouped launch)
template <int MODE>
CFL_DEVICE void dw_stream_body(const DwParams& p, int replicas, int seg_rows, int bid, int nblocks) {
  using namespace dws;
  constexpr int LDP = ldp<true>();
  __shared__ __attribute__((aligned(16))) bf16_t sH[NRING * HWp * LDP];
  __shared__ __attribute__((aligned(16))) float sNode[MODE == 1 ? 4 * CT : 4];   // dgrad node coefficients

  const int tid = threadIdx.x, cg = tid % G, pt = tid / G;
  const int sr = pt / (TW / SL), sc = (pt % (TW / SL)) * SL;
  const int nslices = p.C / CT, tiles_w = (p.W + TW - 1) / TW, nseg = (p.H + seg_rows - 1) / seg_rows;
  int lin = xcd_swizzle(bid, nblocks);
  const int cs = lin % nslices;
  lin /= nslices;
  const int tw = lin % tiles_w;
  lin /= tiles_w;
  const int sg = lin % nseg;
  const int b = lin / nseg;
  const int x0 = tw * TW, cbase = cs * CT, c0 = cbase + cg * CPT;
  const int ybeg = sg * seg_rows, yend = min(p.H, ybeg + seg_rows);
  const int nsteps = (yend - ybeg + SR - 1) / SR;

  const bool tx = MODE != 1;
  const bool has_ab = tx && p.xf.ab != nullptr;
  const int relu = tx ? p.xf.relu : 0;
  const bf16_t* src_b = (MODE == 1 ? p.dy : p.x) + (size_t)b * p.H * p.W * p.C + c0;
  float a4[4], b4[4];
  // forward with a consumer-side BN finalize (p.xfin): threads 0..CT-1 turn this channel slice's replica sums into
  // (a, b) in LDS (the slice's first block also writes the ab rows for the layer's later consumers)
  __shared__ float sAB[MODE == 0 ? 2 * CT : 1];
  const bool xfin = MODE == 0 && p.xfin.stats != nullptr;
  if (xfin) {
    if (tid < CT) {
      float a, bb, mean, rstd;
      bn_coef_from_stats(p.xfin, p.C, cbase + tid, a, bb, mean, rstd);
      sAB[MODE == 0 ? tid : 0] = a;
      sAB[MODE == 0 ? CT + tid : 0] = bb;
      if (tw == 0 && sg == 0 && b == 0) {
        float* ab = const_cast<float*>(p.xf.ab);
        ab[cbase + tid] = a;
        ab[p.C + cbase + tid] = bb;
        ab[2 * p.C + cbase + tid] = mean;
        ab[3 * p.C + cbase + tid] = rstd;
      }
    }
    __syncthreads();
    load_f4(&sAB[cg * CPT], a4);
    load_f4(&sAB[MODE == 0 ? CT + cg * CPT : 0], b4);
  } else {
    load_f4_or(p.xf.ab + c0, has_ab, 1.f, a4);
    load_f4_or(p.xf.ab + p.xf.C + c0, has_ab, 0.f, b4);
  }
  // fwd / dgrad taps live in LDS (re-read per input row: 36 fewer live registers than holding all 9 taps)
  __shared__ __attribute__((aligned(16))) float sW[MODE == 2 ? 4 : 9 * CT];
  if (MODE != 2) {
    for (int e = tid; e < 9 * CT; e += NT) {
      const int t = e / CT, c = e - t * CT;
      sW[MODE == 2 ? 0 : e] = p.w[(MODE == 1 ? 8 - t : t) * p.C + cbase + c];
    }
  }
  {
    uint2 v[SR + 3];
    uint32_t okm;
    fetch<SR + 2>(src_b, p, x0, ybeg - 1, true, v, okm);
    put<SR + 2, true>(sH, v, okm, ybeg - 1, has_ab || relu, a4, b4, relu);
  }
  // wgrad: this thread's dy strip of the current step (prefetched one step ahead like the halo rows)
  constexpr int NG = MODE == 2 ? SL : 1;
  uint2 gq[NG];
  auto fetch_dy = [&](int a, uint2* dst) {
    const int oy = a + sr;
#pragma unroll
    for (int i = 0; i < NG; ++i) {
      const bool ok = oy < yend && x0 + sc + i < p.W;
      uint2 t = make_uint2(0, 0);
      if (ok) t = *reinterpret_cast<const uint2*>(p.dy + (((size_t)b * p.H + oy) * p.W + x0 + sc + i) * p.C + c0);
      dst[i] = t;
    }
  };
  if (MODE == 2) fetch_dy(ybeg, gq);
  if (MODE == 1 && p.node.y != nullptr && tid < 4 * CT)
    sNode[MODE == 1 ? tid : 0] = p.node.ab[(tid / CT) * p.C + cbase + tid % CT];
  __syncthreads();

  constexpr int NA = MODE == 2 ? 9 : SL;
  float acc[NA][4];
#pragma unroll
  for (int t = 0; t < NA; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = 0.f;
  const bool node = MODE == 1 && p.node.y != nullptr;       // fused BN-node gradient epilogue (dgrad)
  float s0[4], s1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) s0[j] = s1[j] = 0.f;

  // halo rows are prefetched two steps ahead (register sets ra / rb alternate): one step's rows in flight per block
  // are too few bytes to cover HBM latency at 3 blocks per CU
  // (wgrad keeps one step: its dy strips and 36 tap sums leave no registers for a second set)
  constexpr bool D2 = MODE != 2;
  uint2 ra[SR + 1], rb[SR + 1];
  uint32_t oka = 0, okb = 0;
  if (D2) fetch<SR>(src_b, p, x0, ybeg + SR + 1, nsteps > 1, ra, oka);
  auto step = [&](int s, uint2 (&cur)[SR + 1], uint32_t& curok, uint2 (&nxt)[SR + 1], uint32_t& nxtok) {
    const int a = ybeg + s * SR;
    const bool more = s + 1 < nsteps;
    if (D2) fetch<SR>(src_b, p, x0, a + 2 * SR + 1, s + 2 < nsteps, nxt, nxtok);
    else fetch<SR>(src_b, p, x0, a + SR + 1, more, cur, curok);
    uint2 gn[NG];
    if (MODE == 2) fetch_dy(more ? a + SR : yend, gn);
    const int oy = a + sr;
    if (MODE != 2) {
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
    }
    float g[NG][4];
#pragma unroll
    for (int i = 0; i < NG; ++i) unpack4(gq[i], g[i]);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int slot = (oy - 1 + ky + NRING) % NRING;
      const bf16_t* hrow = &sH[slot * HWp * LDP + cg * CPT];
      float wt[MODE == 2 ? 1 : 3][4];
      if (MODE != 2) {
#pragma unroll
        for (int kx = 0; kx < (MODE == 2 ? 1 : 3); ++kx) load_f4(&sW[(ky * 3 + kx) * CT + cg * CPT], wt[kx]);
      }
#pragma unroll
      for (int cx = 0; cx < SL + 2; ++cx) {
        float f[4];
        unpack4(*reinterpret_cast<const uint2*>(hrow + pxo(sc + cx) * LDP), f);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int o = cx - kx;
          if (o < 0 || o >= SL) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (MODE == 2) acc[ky * 3 + kx][j] = fmaf(f[j], g[MODE == 2 ? o : 0][j], acc[ky * 3 + kx][j]);
            else acc[MODE == 2 ? 0 : o][j] = fmaf(f[j], wt[MODE == 2 ? 0 : kx][j], acc[MODE == 2 ? 0 : o][j]);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);   // one input row's 6 LDS reads in flight at a time (register pressure)
    }
    if (MODE != 2 && oy < yend) {
      const size_t off0 = (((size_t)b * p.H + oy) * p.W + x0 + sc) * p.C + c0;
#pragma unroll
      for (int i = 0; i < SL; ++i)
        if (x0 + sc + i < p.W) {
          uint2 v = pack4(acc[MODE == 2 ? 0 : i]);
          if (node) {                                        // g = mask * o (o already bf16) + BN-backward sums
            float o[4], y[4], na[4], nb[4], nmean[4], nrstd[4];   // coefficients re-read from LDS (registers)
            const float* nc = &sNode[cg * CPT];
            load_f4(nc, na);
            load_f4(nc + CT, nb);
            load_f4(nc + 2 * CT, nmean);
            load_f4(nc + 3 * CT, nrstd);
            unpack4(v, o);
            unpack4(*reinterpret_cast<const uint2*>(p.node.y + off0 + (size_t)i * p.C), y);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float gg = (!p.node.relu || fmaf(na[j], y[j], nb[j]) > 0.f) ? o[j] : 0.f;
              o[j] = gg;
              s0[j] += gg;
              s1[j] += gg * (y[j] - nmean[j]) * nrstd[j];
            }
            v = pack4(o);
          }
          *reinterpret_cast<uint2*>(p.y + off0 + (size_t)i * p.C) = v;
        }
    }
    if (more) put<SR, true>(sH, cur, curok, a + SR + 1, has_ab || relu, a4, b4, relu);
    if (MODE == 2) {
#pragma unroll
      for (int i = 0; i < NG; ++i) gq[i] = gn[i];
    }
    __syncthreads();
  };
  for (int s = 0; s < nsteps; s += 2) {
    step(s, ra, oka, rb, okb);
    if (s + 1 < nsteps) step(s + 1, rb, okb, ra, oka);
  }

  const int lane = tid & 63, wid = tid >> 6;
  float* red = reinterpret_cast<float*>(sH);                 // ring no longer needed (loop ended on a barrier)
  constexpr int NS = MODE == 2 ? 9 : 2;                      // rows of per-channel partials
  float part[NS][4];
  if (MODE == 2) {
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) part[t][j] = acc[MODE == 2 ? t : 0][j];
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      part[0][j] = s0[j];
      part[MODE == 2 ? 0 : 1][j] = s1[j];
    }
  }
  if (MODE == 2 || node) {                                   // block reduction, one atomic per (row, channel)
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v = part[t][j];
        for (int o = G; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
        part[t][j] = v;
      }
    if (lane < G) {
#pragma unroll
      for (int t = 0; t < NS; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[(wid * NS + t) * CT + cg * CPT + j] = part[t][j];
    }
    __syncthreads();
    float* dst;
    size_t ro;
    if (MODE == 2) {
      dst = p.dw;
      ro = (size_t)(bid % replicas) * 9 * p.C;
    } else {
      const int reps = p.node.reps > 1 ? p.node.reps : 1;
      dst = p.node.sums;
      ro = (size_t)(bid % reps) * 2 * p.C;
    }
    for (int e = tid; e < NS * CT; e += NT) {
      const int t = e / CT, c = e % CT;
      red_add(dst, ro + t * p.C + cbase + c, red[(0 * NS + t) * CT + c] + red[(1 * NS + t) * CT + c] +
                                                 red[(2 * NS + t) * CT + c] + red[(3 * NS + t) * CT + c], CFL_FX_G);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(NT, 3) void dw_stream_kernel(DwParams p, int replicas, int seg_rows) {
  CFL_TS_GUARD;
  dw_stream_body<MODE>(p, replicas, seg_rows, blockIdx.x, gridDim.x);
}

// Grouped launch of the deferred depthwise weight gradients of a step (the engine's 6 SeparableConv depthwise
// layers): each alone is a latency-bound row-streaming grid, so they share one launch and their blocks co-run.
constexpr int DWG_MAX = 8;
struct DwItem {
  DwParams p;
  int replicas, seg_rows, block0, nblocks;   // block0: multiple of 8 (an item's blocks keep their XCD order)
};
struct DwGroup {
  DwItem it[DWG_MAX];
  int n;
};

__global__ __launch_bounds__(NT, 3) void dw_wgrad_group_kernel(const DwGroup g) {
  CFL_TS_GUARD;
  int k = 0;
  while (k + 1 < g.n && g.it[k + 1].block0 <= (int)blockIdx.x) ++k;
  const DwItem& I = g.it[k];
  const int local = blockIdx.x - I.block0;
  if (local >= I.nblocks) return;                       // alignment padding between items
  dw_stream_body<2>(I.p, I.replicas, I.seg_rows, local, I.nblocks);
}

// Fused depthwise backward of one layer: dgrad and wgrad in one row-streaming pass. Both need the incoming gradient
// dy of the same rows (dgrad as a 3x3 halo, wgrad at the centre) and the wgrad needs the layer input x as a halo, so
// a block keeps TWO rings (dy raw, x with the producer's BN-apply + ReLU) and takes the wgrad's dy strip from the
// centre row of the dy ring: dy and x are each read once per segment instead of dy twice + x twice (separate dgrad
// with a BN-node epilogue reading x again, and wgrad), and one launch per layer instead of two.
// The x ring holds the TRANSFORMED input (BN-apply + ReLU once per staged element; the wgrad reads each element 4.5
// times, so transforming where read cost ~200 VALU ops per thread-step). NODE (the input is the BN node itself): the
// node epilogue's raw y of this step's 4 output pixels is loaded at the top of the step, ahead of the ring prefetch,
// so the epilogue's wait for it leaves the next step's rows in flight (they are rows the ring fetched a step ago:
// L2 hits).
template <bool NODE>
__global__ __launch_bounds__(NT, 2) void dw_bwd_stream_kernel(DwParams p, int replicas, int seg_rows) {
  CFL_TS_GUARD;
  using namespace dws;
  constexpr int LDP = ldp<false>();
  __shared__ __attribute__((aligned(16))) bf16_t sG[NRING * HWp * LDP];   // dy rows
  __shared__ __attribute__((aligned(16))) bf16_t sX[NRING * HWp * LDP];   // transformed x rows
  __shared__ __attribute__((aligned(16))) float sW[9 * CT];               // flipped taps (dgrad)
  __shared__ __attribute__((aligned(16))) float sNode[4 * CT];

  const int tid = threadIdx.x, cg = tid % G, pt = tid / G;
  const int sr = pt / (TW / SL), sc = (pt % (TW / SL)) * SL;
  const int nslices = p.C / CT, tiles_w = (p.W + TW - 1) / TW, nseg = (p.H + seg_rows - 1) / seg_rows;
  int lin = xcd_swizzle(blockIdx.x, gridDim.x);
  const int cs = lin % nslices;
  lin /= nslices;
  const int tw = lin % tiles_w;
  lin /= tiles_w;
  const int sg = lin % nseg;
  const int b = lin / nseg;
  const int x0 = tw * TW, cbase = cs * CT, c0 = cbase + cg * CPT;
  const int ybeg = sg * seg_rows, yend = min(p.H, ybeg + seg_rows);
  const int nsteps = (yend - ybeg + SR - 1) / SR;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;
  const size_t img = (size_t)b * p.H * p.W * p.C + c0;
  const bf16_t* g_b = p.dy + img;
  const bf16_t* x_b = p.x + img;
  constexpr bool node = NODE;
  float a4[4], b4[4];
  {
    // the first rows, the flipped taps, the node coefficients and the producer coefficients all issued before the
    // first wait (the strided tap copy waited one memory round trip per iteration)
    uint2 v[SR + 3], u[SR + 3];
    uint32_t okv, oku;
    fetch<SR + 2>(g_b, p, x0, ybeg - 1, true, v, okv);
    fetch<SR + 2>(x_b, p, x0, ybeg - 1, true, u, oku);
    constexpr int WT = (9 * CT + NT - 1) / NT;
    float wv[WT];
#pragma unroll
    for (int i = 0; i < WT; ++i) {
      const int e = imin(tid + i * NT, 9 * CT - 1), t = e / CT, c = e - t * CT;
      wv[i] = p.w[(8 - t) * p.C + cbase + c];
    }
    const int ne = imin(tid, 4 * CT - 1);
    const float nv = node ? p.node.ab[(ne / CT) * p.C + cbase + ne % CT] : 0.f;
    load_f4_or(p.xf.ab + c0, has_ab, 1.f, a4);
    load_f4_or(p.xf.ab + p.xf.C + c0, has_ab, 0.f, b4);
#pragma unroll
    for (int i = 0; i < WT; ++i)
      if (tid + i * NT < 9 * CT) sW[tid + i * NT] = wv[i];
    if (node && tid < 4 * CT) sNode[tid] = nv;
    put<SR + 2, false>(sG, v, okv, ybeg - 1, false, a4, b4, 0);
    put<SR + 2, false>(sX, u, oku, ybeg - 1, has_ab || relu, a4, b4, relu);   // transformed x (padding stays zero)
  }
  __syncthreads();

  float accw[9][4], s0[4], s1[4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) accw[t][j] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s0[j] = s1[j] = 0.f;
  uint2 rg[SR + 1], rx[SR + 1];
  uint32_t okg = 0, okx = 0;
  const bf16_t* hsrc = p.add_half ? p.add_half : p.dy;
  cfl_ts_phase(0);
  for (int s = 0; s < nsteps; ++s) {
    const int a = ybeg + s * SR;
    const bool more = s + 1 < nsteps;
    const int oy = a + sr;
    // this step's residual half-resolution gradient (even pixels) is loaded BEFORE the ring prefetch: the epilogue's
    // wait for it then leaves the next step's rows in flight (the node's y is the raw x ring's centre row)
    const size_t eoff = (((size_t)b * p.H + oy) * p.W + x0 + sc) * p.C + c0;
    uint2 hr[SL / 2];
#pragma unroll
    for (int i = 0; i < SL / 2; ++i) {                      // x0 + sc is a multiple of 4: even pixels are i = 0, 2
      // loaded unconditionally (clamped; from dy - a larger tensor - when there is no residual): see fetch
      const int xx = x0 + sc + 2 * i;
      const int Hh = (p.H + 1) >> 1, Wh = (p.W + 1) >> 1;
      const int hy = min(oy, p.H - 1) >> 1, hx = min(xx, p.W - 1) >> 1;
      hr[i] = *reinterpret_cast<const uint2*>(hsrc + (((size_t)b * Hh + hy) * Wh + hx) * p.C + c0);
    }
    uint2 yr[NODE ? SL : 1];                                 // the node's raw y at this step's output pixels
    if constexpr (NODE) {
      const int yy = min(oy, p.H - 1);
#pragma unroll
      for (int i = 0; i < SL; ++i)
        yr[i] = *reinterpret_cast<const uint2*>(x_b + (yy * p.W + min(x0 + sc + i, p.W - 1)) * p.C);
    }
    fetch<SR>(g_b, p, x0, a + SR + 1, more, rg, okg);       // next step's rows, in flight during this step
    fetch<SR>(x_b, p, x0, a + SR + 1, more, rx, okx);
    const float live = oy < yend ? 1.f : 0.f;              // rows past the segment belong to the next block
    float acc[SL][4], g[SL][4];
#pragma unroll
    for (int i = 0; i < SL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = g[i][j] = 0.f;
    // dgrad: flipped taps over the dy halo; the centre row's columns 1..SL are this strip's own dy (wgrad operand)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int slot = (oy - 1 + ky + NRING) % NRING;
      const bf16_t* hrow = &sG[(slot * HWp + sc) * LDP + cg * CPT];
      float wt[3][4];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) load_f4(&sW[(ky * 3 + kx) * CT + cg * CPT], wt[kx]);
#pragma unroll
      for (int cx = 0; cx < SL + 2; ++cx) {
        float f[4];
        unpack4(*reinterpret_cast<const uint2*>(hrow + cx * LDP), f);
        if (ky == 1 && cx >= 1 && cx <= SL) {
#pragma unroll
          for (int j = 0; j < 4; ++j) g[cx - 1][j] = f[j] * live;
        }
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int o = cx - kx;
          if (o < 0 || o >= SL) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[o][j] = fmaf(f[j], wt[kx][j], acc[o][j]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // wgrad: dW[tap] += x[p + tap - 1] * dy[p] over the x halo
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int slot = (oy - 1 + ky + NRING) % NRING;
      const bf16_t* hrow = &sX[(slot * HWp + sc) * LDP + cg * CPT];
#pragma unroll
      for (int cx = 0; cx < SL + 2; ++cx) {
        float f[4];
        unpack4(*reinterpret_cast<const uint2*>(hrow + cx * LDP), f);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int o = cx - kx;
          if (o < 0 || o >= SL) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) accw[ky * 3 + kx][j] = fmaf(f[j], g[o][j], accw[ky * 3 + kx][j]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (oy < yend) {
      const size_t off0 = eoff;
#pragma unroll
      for (int i = 0; i < SL; ++i)
        if (x0 + sc + i < p.W) {
          uint2 v = pack4(acc[i]);
          if (p.add_half || p.mask_x) {                      // residual join (node_bwd semantics, one rounding)
            float o[4];
            unpack4(v, o);
            if (p.mask_x) {                                  // transformed x at this pixel: the x ring's centre row
              float xv[4];
              unpack4(*reinterpret_cast<const uint2*>(&sX[((oy % NRING) * HWp + sc + i + 1) * LDP + cg * CPT]), xv);
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] = xv[j] > 0.f ? o[j] : 0.f;
            }
            if (p.add_half && (i & 1) == 0 && (oy & 1) == 0) {   // (oy < yend, x < W hold here)
              float r[4];
              unpack4(hr[i / 2], r);
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] += r[j];
            }
            v = pack4(o);
          }
          if constexpr (NODE) {                              // g = mask * o (o already bf16) + BN-backward sums
            // (the node's BN is the input transform's: its scale / shift are a4 / b4, checked by dw_bwd)
            float o[4], y[4], nmean[4], nrstd[4];
            const float* nc = &sNode[cg * CPT];
            load_f4(nc + 2 * CT, nmean);
            load_f4(nc + 3 * CT, nrstd);
            unpack4(v, o);
            unpack4(yr[i], y);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float gg = (!relu || fmaf(a4[j], y[j], b4[j]) > 0.f) ? o[j] : 0.f;
              o[j] = gg;
              s0[j] += gg;
              s1[j] += gg * (y[j] - nmean[j]) * nrstd[j];
            }
            v = pack4(o);
          }
          *reinterpret_cast<uint2*>(p.y + off0 + (size_t)i * p.C) = v;
        }
    }
    if (more) {
      put<SR, false>(sG, rg, okg, a + SR + 1, false, a4, b4, 0);
      put<SR, false>(sX, rx, okx, a + SR + 1, has_ab || relu, a4, b4, relu);
    }
    __syncthreads();
  }
  cfl_ts_phase(1);

  // block reduction of the 9 tap sums (+ the 2 node sums), one atomic per (row, channel) into replica rows
  const int lane = tid & 63, wid = tid >> 6;
  constexpr int NS = 11;
  float* red = reinterpret_cast<float*>(sG);                 // ring no longer needed (loop ended on a barrier)
  float part[NS][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) part[t][j] = accw[t][j];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    part[9][j] = s0[j];
    part[10][j] = s1[j];
  }
#pragma unroll
  for (int t = 0; t < NS; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = part[t][j];
      for (int o = G; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      part[t][j] = v;
    }
  if (lane < G) {
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(wid * NS + t) * CT + cg * CPT + j] = part[t][j];
  }
  __syncthreads();
  const size_t dro = (size_t)(blockIdx.x % replicas) * 9 * p.C;
  const int nreps = p.node.reps > 1 ? p.node.reps : 1;
  const size_t nro = (size_t)(blockIdx.x % nreps) * 2 * p.C;
  for (int e = tid; e < (node ? NS : 9) * CT; e += NT) {
    const int t = e / CT, c = e % CT;
    const float v = red[(0 * NS + t) * CT + c] + red[(1 * NS + t) * CT + c] + red[(2 * NS + t) * CT + c] +
                    red[(3 * NS + t) * CT + c];
    if (t < 9) red_add(p.dw, dro + t * p.C + cbase + c, v, CFL_FX_G);
    else red_add(p.node.sums, nro + (t - 9) * p.C + cbase + c, v, CFL_FX_G);
  }
}

// ---- fused depthwise backward with an LDS-DMA dy ring (the long-segment launches: dw_bwd's size rule) ----
// The register-budget restructure of dw_bwd_stream_kernel (256 VGPRs + 56 KB LDS: 2 blocks, 8 waves per CU) to 3 blocks
// per CU:
//   * dy (staged raw, no transform) goes global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds, no VGPR staging) into a
//     14-row ring, issued 1.5 steps ahead (after the step's epilogue stores);
//   * x (BN-apply + ReLU on the way in) stays register-staged one step ahead in a 6-row ring: its rows are written
//     between two barriers at the end of the step (10 rows without the second barrier would not fit 3 blocks);
//   * every global read is a buffer load on a per-image resource with a 32-bit offset: padding pieces take an
//     out-of-range offset and read 0 (no clamped addresses, no 64-bit address registers);
//   * rings in the dws swizzled layout (unpadded 64-byte pixels, dws::pxo);
//   * the dgrad epilogue runs before the wgrad (its 16 accumulators are dead while the 36 tap sums work).
// 45 KB LDS, 147 / 166 VGPRs, no scratch: 3 blocks per CU. Measured (profiles/r5_dw/): at the 512^2 planned batch
// (segments of whole maps, many rounds of blocks) 14-15 % faster per call than the two-ring kernel (19.3 vs 22.4 ms
// per step over the 6 calls); at 256^2 / batch 16 (one round of 6-8-step segments) 1-2 us per call slower - there the
// step chain (epilogue operands loaded at the top of a step and waited for mid-step, two barriers) and the deeper
// prologue bound it, not the resident wave count. (A first 54 KB version - x ring 10 rows - ran 2 blocks per CU at
// 768 blocks, 25 % slower: the hardware did not fit 3 x 53.9 KB.)
// Register loads and LDS stores are inline asm (for a compiler-visible load hipcc drains every DMA in flight before
// the first use, conv3x3_sk.hip); the counted `s_waitcnt vmcnt` below are the only waits. Issue order in step s:
// [half-res residual / node y of s] [x rows of s + 1] | wait for the first group | epilogue stores, [dy DMAs of
// s + 2] | wait for all but the DMAs: at any wait the stores are OLDER than everything it leaves in flight.
namespace dwd {
using dws::CPT;
using dws::CT;
using dws::G;
using dws::SL;
using dws::SR;
using dws::TW;
constexpr int PXB = CT * 2;                      // bytes per pixel (32 bf16 channels)
constexpr int ROWB = (TW + 2) * PXB;             // 2176: one ring row
constexpr int NRG = 3 * SR + 2, NRX = SR + 2;
constexpr int OFF_X = NRG * ROWB, OFF_W = OFF_X + NRX * ROWB, OFF_N = OFF_W + 9 * CT * 4, SMEM = OFF_N + 4 * CT * 4;
constexpr uint32_t OOB = 0x80000000u;            // buffer offset past every resource's range: the load returns 0
static_assert(3 * SMEM <= 160 * 1024, "three blocks per CU");
static_assert(ROWB > 2048 && ROWB - 2048 == 8 * 16, "a row = 2 full DMA instructions + 8 lanes of a third");
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef int i4v __attribute__((ext_vector_type(4)));

using dws::pxo;

// raw buffer resource over [base, base + bytes) (gfx9 dword 3); wave-uniform
CFL_DEVICE i4v rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i4v r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}
template <int N>
CFL_DEVICE void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
CFL_DEVICE void order() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
CFL_DEVICE u2v ld8(const i4v& rs, uint32_t off) {
  u2v v;
  asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(v) : "v"(off), "s"(rs) : "memory");
  return v;
}
CFL_DEVICE void st8(unsigned char* p, uint2 v) {
  const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)p;
  const u2v d = {v.x, v.y};
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(d) : "memory");
}
CFL_DEVICE uint2 u2(u2v v) { return make_uint2(v.x, v.y); }
}  // namespace dwd

namespace dwd {
// 16 bytes of the buffer at `off` -> LDS at the wave-uniform `lds` + 16 * lane. Inline asm (M0 = the LDS address):
// with the DMA visible, hipcc orders every later LDS read that may alias it (the tap reads too) behind vmcnt(0).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"        // M0 is reserved; this kernel has no other M0 user (checked ISA)
CFL_DEVICE void dma16(const i4v& rs, uint32_t off, unsigned char* lds) {
  const uint32_t a = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(a), "v"(off), "s"(rs)
               : "memory", "m0");
}
#pragma clang diagnostic pop

// x rows row0 .. row0 + NR - 1 of the staging map of dws::fetch (thread t: column t / G, the first 2 G NR threads
// also a right-halo piece - every thread issues that load, so a wave issues NR + 1 loads whatever its index).
// xcol: this thread's column byte offset in the image (OOB if the column is padding); hcol: its right-halo piece's
template <int NR>
CFL_DEVICE void fetchx(const i4v& rs, const DwParams& p, uint32_t xcol, uint32_t hcol, int hrow, int row0, bool on,
                       u2v (&v)[NR + 1], uint32_t& okm) {
  okm = 0;
  const uint32_t rowb = (uint32_t)p.W * p.C * 2;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int iy = row0 + r;                                 // wave-uniform
    const bool ok = on && (unsigned)iy < (unsigned)p.H && xcol != OOB;
    v[r] = ld8(rs, ok ? (uint32_t)iy * rowb + xcol : OOB);
    okm |= (uint32_t)ok << r;
  }
  const int iy = row0 + hrow;
  const bool ok = on && hrow < NR && (unsigned)iy < (unsigned)p.H && hcol != OOB;
  v[NR] = ld8(rs, ok ? (uint32_t)iy * rowb + hcol : OOB);
  okm |= (uint32_t)ok << NR;
}

template <int NR>
CFL_DEVICE void putx(unsigned char* ring, const u2v (&v)[NR + 1], uint32_t okm, int row0, bool xform, const float* a4,
                     const float* b4, int relu) {
  const int tid = threadIdx.x, q = tid % G;
  const int slot0 = (row0 + NRX) % NRX;                      // row0 >= -1
  unsigned char* col = ring + pxo(tid / G) * PXB + q * CPT * 2;
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int slot = slot0 + r >= NRX ? slot0 + r - NRX : slot0 + r;
    const bool ok = (okm >> r) & 1u;
    st8(col + slot * ROWB, dws::xform4(ok ? u2(v[r]) : make_uint2(0, 0), xform && ok, a4, b4, relu));
  }
  if (__builtin_amdgcn_readfirstlane(tid) < 2 * G * NR) {   // the waves holding right-halo pieces
    const int re = tid / (2 * G), hxe = TW + (tid % (2 * G)) / G;
    if (re < NR) {
      const int slot = slot0 + re >= NRX ? slot0 + re - NRX : slot0 + re;
      const bool ok = (okm >> NR) & 1u;
      st8(ring + slot * ROWB + pxo(hxe) * PXB + q * CPT * 2,
          dws::xform4(ok ? u2(v[NR]) : make_uint2(0, 0), xform && ok, a4, b4, relu));
    }
  }
}
}  // namespace dwd

template <bool NODE>
__global__ __launch_bounds__(NT, 3) void dw_bwd_dma_kernel(DwParams p, int replicas, int seg_rows) {
  CFL_TS_GUARD;
  using namespace dws;
  using dwd::NRG;
  using dwd::NRX;
  using dwd::OOB;
  using dwd::PXB;
  using dwd::ROWB;
  using dwd::pxo;
  // ONE shared object (a second one can make hipcc drain the DMAs before every ds_read): [dy ring][x ring][taps][node]
  __shared__ __attribute__((aligned(1024))) unsigned char smem[dwd::SMEM];
  unsigned char* sX = smem + dwd::OFF_X;
  float* sW = reinterpret_cast<float*>(smem + dwd::OFF_W);
  float* sNode = reinterpret_cast<float*>(smem + dwd::OFF_N);

  const int tid = threadIdx.x, lane = tid & 63, cg = tid % G, pt = tid / G;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int sr = wid, sc = (pt % (TW / SL)) * SL;            // a wave = one output row of the step
  static_assert(NT / 64 == SR && TW / SL * G == 64, "wave w owns output row w of a step");
  const int nslices = p.C / CT, tiles_w = (p.W + TW - 1) / TW, nseg = (p.H + seg_rows - 1) / seg_rows;
  int lin = xcd_swizzle(blockIdx.x, gridDim.x);
  const int cs = lin % nslices;
  lin /= nslices;
  const int tw = lin % tiles_w;
  lin /= tiles_w;
  const int sg = lin % nseg;
  const int b = lin / nseg;
  const int x0 = tw * TW, cbase = cs * CT, c0 = cbase + cg * CPT;
  const int ybeg = sg * seg_rows, yend = min(p.H, ybeg + seg_rows);
  const int nsteps = (yend - ybeg + SR - 1) / SR;
  const bool has_ab = p.xf.ab != nullptr;
  const int relu = p.xf.relu;
  const size_t img = (size_t)b * p.H * p.W * p.C;
  const uint32_t img_bytes = (uint32_t)p.H * p.W * p.C * 2;
  const dwd::i4v rs_x = dwd::rsrc(p.x + img, img_bytes);
  const dwd::i4v rs_g = dwd::rsrc(p.dy + img, img_bytes);
  const int Hh = (p.H + 1) >> 1, Wh = (p.W + 1) >> 1;
  const bf16_t* hsrc = p.add_half ? p.add_half : p.dy;
  const dwd::i4v rs_h = dwd::rsrc(hsrc + (size_t)b * Hh * Wh * p.C, (uint32_t)Hh * Wh * p.C * 2);

  // plain loads first, waited for before the first DMA is issued
  float a4[4], b4[4];
  load_f4_or(p.xf.ab + c0, has_ab, 1.f, a4);
  load_f4_or(p.xf.ab + p.xf.C + c0, has_ab, 0.f, b4);
  for (int e = tid; e < 9 * CT; e += NT) {
    const int t = e / CT, c = e - t * CT;
    sW[e] = p.w[(8 - t) * p.C + cbase + c];
  }
  if (NODE && tid < 4 * CT) sNode[tid] = p.node.ab[(tid / CT) * p.C + cbase + tid % CT];
#pragma unroll
  for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(a4[j]), "+v"(b4[j]));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // dy DMA: lane l of instruction j of a row fills bytes 1024 j + 16 l of the row = pixel position 16 j + l / 4
  // (pixel pxo(position)), channel quarter l % 4; lanes 8.. of the third instruction are masked off
  uint32_t gcol[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int px = pxo(16 * j + (lane >> 2)), ix = x0 - 1 + px;
    const bool ok = (unsigned)ix < (unsigned)p.W && px < TW + 2;
    gcol[j] = ok ? (uint32_t)(ix * p.C + cbase + (lane & 3) * 8) * 2 : OOB;
  }
  const uint32_t rowb = (uint32_t)p.W * p.C * 2;
  // (issued unconditionally - a fixed count per step keeps the waits single constants: a row with on == false
  // reads zeros from an out-of-range offset into a ring slot no later step reads, no memory traffic)
  auto dma_row = [&](int r, bool on) {                       // wave-uniform image row r (>= -1)
    unsigned char* dst = smem + ((r + NRG) % NRG) * ROWB;
    const bool rok = on && (unsigned)r < (unsigned)p.H;
    const uint32_t ro = rok ? (uint32_t)r * rowb : 0u;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const uint32_t off = rok && gcol[j] != OOB ? ro + gcol[j] : OOB;
      if (j < 2) dwd::dma16(rs_g, off, dst + 1024 * j);
      else if (lane < 8) dwd::dma16(rs_g, off, dst + 2048);
    }
  };
  // x staging offsets (dws::fetch's map): column tid / G, right-halo piece (row tid / 2G, column 32 + (tid % 2G) / G)
  const int xix = x0 + tid / G - 1, hix = x0 + TW - 1 + (tid % (2 * G)) / G;
  const uint32_t xcol = (unsigned)xix < (unsigned)p.W ? (uint32_t)(xix * p.C + c0) * 2 : OOB;
  const uint32_t hcol = (unsigned)hix < (unsigned)p.W ? (uint32_t)(hix * p.C + c0) * 2 : OOB;
  const int hrow = tid / (2 * G);

  // prologue: dy rows of steps 0 (ybeg - 1 .. ybeg + SR) and 1, x rows of step 0
  {
    dma_row(ybeg - 1 + wid, true);
    dma_row(ybeg + SR - 1 + (wid & 1), true);                      // rows ybeg + 3, ybeg + 4 (twice: identical bytes)
    dwd::order();
    dwd::u2v u[SR + 3];
    uint32_t oku;
    dwd::fetchx<SR + 2>(rs_x, p, xcol, hcol, hrow, ybeg - 1, true, u, oku);
    dwd::order();
    dma_row(ybeg + SR + 1 + wid, nsteps > 1);
    dwd::order();
    dwd::wait_vm<3>();
#pragma unroll
    for (int i = 0; i < SR + 3; ++i) asm volatile("" : "+v"(u[i]));
    dwd::putx<SR + 2>(sX, u, oku, ybeg - 1, has_ab || relu, a4, b4, relu);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  float accw[9][4], s0[4], s1[4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) accw[t][j] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) s0[j] = s1[j] = 0.f;
  for (int s = 0; s < nsteps; ++s) {
    const int a = ybeg + s * SR;
    const bool more = s + 1 < nsteps, dma2 = s + 2 < nsteps;
    const int oy = a + sr;                                   // wave-uniform
    // [residual half-resolution gradient (even pixels) / node y of this step] (unconditional: fixed counts)
    dwd::u2v hr[SL / 2];
    {
      const uint32_t hrowo = (uint32_t)(min(oy, p.H - 1) >> 1) * Wh;
#pragma unroll
      for (int i = 0; i < SL / 2; ++i) {
        const int hx = min(x0 + sc + 2 * i, p.W - 1) >> 1;
        hr[i] = dwd::ld8(rs_h, ((hrowo + hx) * p.C + c0) * 2);
      }
    }
    dwd::u2v yr[NODE ? SL : 1];
    if constexpr (NODE) {
      const uint32_t yro = (uint32_t)min(oy, p.H - 1) * rowb;
#pragma unroll
      for (int i = 0; i < SL; ++i) yr[i] = dwd::ld8(rs_x, yro + (uint32_t)(min(x0 + sc + i, p.W - 1) * p.C + c0) * 2);
    }
    // [x rows of step s + 1] (the dy DMAs of step s + 2 follow the epilogue's stores)
    dwd::u2v rx[SR + 1];
    uint32_t okx;
    dwd::fetchx<SR>(rs_x, p, xcol, hcol, hrow, a + SR + 1, more, rx, okx);
    dwd::order();

    const float live = oy < yend ? 1.f : 0.f;               // rows past the segment belong to the next block
    float acc[SL][4], g[SL][4];
#pragma unroll
    for (int i = 0; i < SL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = g[i][j] = 0.f;
    // dgrad: flipped taps over the dy halo; the centre row's columns 1..SL are this strip's own dy (wgrad operand)
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const unsigned char* hrow_p = smem + ((oy - 1 + ky + NRG) % NRG) * ROWB + cg * CPT * 2;
      float wt[3][4];
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) load_f4(&sW[(ky * 3 + kx) * CT + cg * CPT], wt[kx]);
#pragma unroll
      for (int cx = 0; cx < SL + 2; ++cx) {
        float f[4];
        unpack4(*reinterpret_cast<const uint2*>(hrow_p + pxo(sc + cx) * PXB), f);
        if (ky == 1 && cx >= 1 && cx <= SL) {
#pragma unroll
          for (int j = 0; j < 4; ++j) g[cx - 1][j] = f[j] * live;
        }
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int o = cx - kx;
          if (o < 0 || o >= SL) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[o][j] = fmaf(f[j], wt[kx][j], acc[o][j]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // (materialise the dgrad sums and the dy strip here: otherwise hipcc sinks the FMAs into their uses behind the
    // wait and the epilogue branch, keeping all 18 row reads + 9 tap vectors live across them)
#pragma unroll
    for (int i = 0; i < SL; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(acc[i][j]), "+v"(g[i][j]));
    // the epilogue operands have landed (the x rows of step s + 1 stay in flight)
    dwd::wait_vm<SR + 1>();
#pragma unroll
    for (int i = 0; i < SL / 2; ++i) asm volatile("" : "+v"(hr[i]));
#pragma unroll
    for (int i = 0; i < (NODE ? SL : 1); ++i) asm volatile("" : "+v"(yr[i]));
    if (oy < yend) {
      const size_t off0 = (((size_t)b * p.H + oy) * p.W + x0 + sc) * p.C + c0;
#pragma unroll
      for (int i = 0; i < SL; ++i)
        if (x0 + sc + i < p.W) {
          uint2 v = pack4(acc[i]);
          if (p.add_half || p.mask_x) {                      // residual join (node_bwd semantics, one rounding)
            float o[4];
            unpack4(v, o);
            if (p.mask_x) {                                  // transformed x at this pixel: the x ring's centre row
              float xv[4];
              unpack4(*reinterpret_cast<const uint2*>(sX + (oy % NRX) * ROWB + pxo(sc + i + 1) * PXB + cg * CPT * 2),
                      xv);
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] = xv[j] > 0.f ? o[j] : 0.f;
            }
            if (p.add_half && (i & 1) == 0 && (oy & 1) == 0) {   // (oy < yend, x < W hold here)
              float r[4];
              unpack4(dwd::u2(hr[i / 2]), r);
#pragma unroll
              for (int j = 0; j < 4; ++j) o[j] += r[j];
            }
            v = pack4(o);
          }
          if constexpr (NODE) {                              // g = mask * o (o already bf16) + BN-backward sums
            float o[4], y[4], nmean[4], nrstd[4];
            const float* nc = &sNode[cg * CPT];
            load_f4(nc + 2 * CT, nmean);
            load_f4(nc + 3 * CT, nrstd);
            unpack4(v, o);
            unpack4(dwd::u2(yr[NODE ? i : 0]), y);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const float gg = (!relu || fmaf(a4[j], y[j], b4[j]) > 0.f) ? o[j] : 0.f;
              o[j] = gg;
              s0[j] += gg;
              s1[j] += gg * (y[j] - nmean[j]) * nrstd[j];
            }
            v = pack4(o);
          }
          *reinterpret_cast<uint2*>(p.y + off0 + (size_t)i * p.C) = v;
        }
    }
    // [dy rows of step s + 2] - after the stores, so the end-of-step wait counts only these DMAs as younger than
    // the x rows
    dwd::order();
    dma_row(a + 2 * SR + 1 + wid, dma2);
    dwd::order();
    // wgrad: dW[tap] += x[p + tap - 1] * dy[p] over the x halo
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const unsigned char* hrow_p = sX + ((oy - 1 + ky + NRX) % NRX) * ROWB + cg * CPT * 2;
#pragma unroll
      for (int cx = 0; cx < SL + 2; ++cx) {
        float f[4];
        unpack4(*reinterpret_cast<const uint2*>(hrow_p + pxo(sc + cx) * PXB), f);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int o = cx - kx;
          if (o < 0 || o >= SL) continue;
#pragma unroll
          for (int j = 0; j < 4; ++j) accw[ky * 3 + kx][j] = fmaf(f[j], g[o][j], accw[ky * 3 + kx][j]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // everything but this step's dy DMAs (rows of step s + 2) has landed - the x rows of step s + 1, the epilogue's
    // stores and the DMAs of step s + 1
    dwd::wait_vm<3>();
#pragma unroll
    for (int i = 0; i < SR + 1; ++i) asm volatile("" : "+v"(rx[i]));
    // x rows of step s + 1 -> the slots of rows a - 1 .. a + 2, once every wave is done with step s (a 6-row x ring:
    // 8.7 KB less LDS than staging them beside the rows in use; past the last step: zeros into slots no step reads)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    dwd::putx<SR>(sX, rx, okx, a + SR + 1, has_ab || relu, a4, b4, relu);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");      // this thread's x ring stores
    __builtin_amdgcn_s_barrier();
  }

  // block reduction of the 9 tap sums (+ the 2 node sums), one atomic per (row, channel) into replica rows
  dwd::wait_vm<0>();                                         // the last step's (zero) DMAs land in the dy ring
  __builtin_amdgcn_s_barrier();
  constexpr int NS = 11;
  float* red = reinterpret_cast<float*>(smem);               // dy ring no longer needed
  float part[NS][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) part[t][j] = accw[t][j];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    part[9][j] = s0[j];
    part[10][j] = s1[j];
  }
#pragma unroll
  for (int t = 0; t < NS; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = part[t][j];
      for (int o = G; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      part[t][j] = v;
    }
  if (lane < G) {
#pragma unroll
    for (int t = 0; t < NS; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[(wid * NS + t) * CT + cg * CPT + j] = part[t][j];
  }
  __syncthreads();
  const size_t dro = (size_t)(blockIdx.x % replicas) * 9 * p.C;
  const int nreps = p.node.reps > 1 ? p.node.reps : 1;
  const size_t nro = (size_t)(blockIdx.x % nreps) * 2 * p.C;
  for (int e = tid; e < (NODE ? NS : 9) * CT; e += NT) {
    const int t = e / CT, c = e % CT;
    const float v = red[(0 * NS + t) * CT + c] + red[(1 * NS + t) * CT + c] + red[(2 * NS + t) * CT + c] +
                    red[(3 * NS + t) * CT + c];
    if (t < 9) red_add(p.dw, dro + t * p.C + cbase + c, v, CFL_FX_G);
    else red_add(p.node.sums, nro + (t - 9) * p.C + cbase + c, v, CFL_FX_G);
  }
}

// (grid size, rows per segment) of the row-streaming kernels
// target: grid size to aim for (one round of resident blocks: 256 CUs x blocks per CU)
void stream_shape(const DwParams& p, int& blocks, int& seg_rows, int target = 0) {
  const int steps = (p.H + dws::SR - 1) / dws::SR;
  const int strips = p.B * ((p.W + 31) / 32) * (p.C / dws::CT);
  if (target <= 0)
    target = cfl_tune(TUNE_DW_STREAM_BLOCKS) > 0 ? cfl_tune(TUNE_DW_STREAM_BLOCKS) : 768;   // A/B-measured (256 / 384 / 512 / 768 / 1024 / 2048)
  int nseg = (target + strips - 1) / strips;
  nseg = nseg < 1 ? 1 : (nseg > steps ? steps : nseg);
  seg_rows = ((steps + nseg - 1) / nseg) * dws::SR;
  nseg = (p.H + seg_rows - 1) / seg_rows;
  blocks = strips * nseg;
}

template <int MODE>
int launch_stream(const DwParams& p, int replicas, hipStream_t st) {
  int blocks, seg_rows;
  stream_shape(p, blocks, seg_rows);
  hipLaunchKernelGGL((dw_stream_kernel<MODE>), dim3(blocks), dim3(NT), 0, st, p, replicas, seg_rows);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

bool pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }

int launch_dw(const bf16_t* x, const float* w, bf16_t* y, InXform xf, int B, int H, int W, int C, int flip,
              hipStream_t st) {
  if (C % 8 || C > 256 || !pow2(C / 8)) return 1;
  int blocks = B * H < 4096 ? B * H : 4096;
  if (W % 4 == 0) hipLaunchKernelGGL(dw_conv_kernel<4>, dim3(blocks), dim3(NT), 0, st, x, w, y, xf, B, H, W, C, flip);
  else hipLaunchKernelGGL(dw_conv_kernel<1>, dim3(blocks), dim3(NT), 0, st, x, w, y, xf, B, H, W, C, flip);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

// algo 0 (default): the row-streaming LDS-ring kernels for C % 32 == 0; 1 (or other C): the generic strip kernels
static bool streamed(const DwParams& p) { return p.C % 32 == 0 && p.algo != 1; }

int dw_fwd(const DwParams& p, hipStream_t st) {
  if (streamed(p)) return launch_stream<0>(p, 1, st);
  if (p.xfin.stats) {                        // the other paths read a final ab: finalize it first
    const int rc = bn_finalize(p.xfin.stats, p.xfin.gamma, p.xfin.beta, nullptr, nullptr, const_cast<float*>(p.xf.ab),
                               p.C, p.xfin.count, p.xfin.eps, 1, st);
    if (rc) return rc;
    DwParams q = p;
    q.xfin = BnStatsIn{};
    return dw_fwd(q, st);
  }
  return launch_dw(p.x, p.w, p.y, p.xf, p.B, p.H, p.W, p.C, 0, st);
}

int dw_dgrad(const DwParams& p, hipStream_t st) {
  if (streamed(p)) return launch_stream<1>(p, 1, st);
  if (p.node.y) return 2;                        // the fused BN-node epilogue exists on the streaming path only
  return launch_dw(p.dy, p.w, p.y, InXform{nullptr, p.C, 0}, p.B, p.H, p.W, p.C, 1, st);
}

int dw_bwd(const DwParams& p, hipStream_t st) {
  if (!streamed(p)) {                                       // other paths: the two passes (no residual join)
    if (p.add_half || p.mask_x) return 2;
    const int rc = dw_dgrad(p, st);
    return rc ? rc : dw_wgrad(p, st);
  }
  // the fused pass takes the BN node's y from its raw x ring: the node must be the layer input itself
  if (p.node.y != nullptr && (p.node.y != p.x || p.node.ab != p.xf.ab || p.node.relu != p.xf.relu)) return 1;
  // two rings (56 KB LDS): 2 blocks per CU, so one round of resident blocks is 512 (the single-pass kernels' 768
  // left a half-empty second round)
  int blocks, seg_rows;
  // LDS-DMA kernel (3 blocks per CU, one round is 768) for the launches that stream long segments: at the 512^2
  // planned batch 14-15 % faster per call than the two-ring kernel, at 256^2 / batch 16 (one round of 6-8-step
  // segments, prologue-bound) 1-2 us slower (profiles/r5_dw/). Auto: >= 2 rounds of strips at 3 blocks per CU.
  const int strips = p.B * ((p.W + dws::TW - 1) / dws::TW) * (p.C / dws::CT);
  const int dma_knob = cfl_tune(TUNE_DW_BWD_DMA);
  if (dma_knob == 1 || (dma_knob == 0 && strips >= 1536)) {
    stream_shape(p, blocks, seg_rows, cfl_tune(TUNE_DW_BWD_BLOCKS) > 0 ? cfl_tune(TUNE_DW_BWD_BLOCKS) : 768);
    if (p.node.y) hipLaunchKernelGGL(dw_bwd_dma_kernel<true>, dim3(blocks), dim3(NT), 0, st, p,
                                     p.replicas > 1 ? p.replicas : 1, seg_rows);
    else hipLaunchKernelGGL(dw_bwd_dma_kernel<false>, dim3(blocks), dim3(NT), 0, st, p,
                            p.replicas > 1 ? p.replicas : 1, seg_rows);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  stream_shape(p, blocks, seg_rows, cfl_tune(TUNE_DW_BWD_BLOCKS) > 0 ? cfl_tune(TUNE_DW_BWD_BLOCKS) : 512);
  if (p.node.y) hipLaunchKernelGGL(dw_bwd_stream_kernel<true>, dim3(blocks), dim3(NT), 0, st, p,
                                   p.replicas > 1 ? p.replicas : 1, seg_rows);
  else hipLaunchKernelGGL(dw_bwd_stream_kernel<false>, dim3(blocks), dim3(NT), 0, st, p,
                          p.replicas > 1 ? p.replicas : 1, seg_rows);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int dw_wgrad_batch(const DwParams* ps, int n, hipStream_t st) {
  DwGroup g{};
  int blocks = 0;
  auto flush = [&]() -> int {
    if (g.n == 0) return 0;
    hipLaunchKernelGGL(dw_wgrad_group_kernel, dim3(blocks), dim3(NT), 0, st, g);
    g = DwGroup{};
    blocks = 0;
    return hipGetLastError() == hipSuccess ? 0 : 3;
  };
  for (int i = 0; i < n; ++i) {
    const DwParams& p = ps[i];
    if (!streamed(p) || cfl_tune(TUNE_WGRAD_GROUP) == 1) {   // other paths: one launch each
      const int rc = dw_wgrad(p, st);
      if (rc) return rc;
      continue;
    }
    if (g.n == DWG_MAX) {
      const int rc = flush();
      if (rc) return rc;
    }
    DwItem& it = g.it[g.n++];
    it.p = p;
    it.replicas = p.replicas > 1 ? p.replicas : 1;
    stream_shape(p, it.nblocks, it.seg_rows);
    it.block0 = blocks;
    blocks = (blocks + it.nblocks + 7) / 8 * 8;
  }
  return flush();
}

int dw_wgrad(const DwParams& p, hipStream_t st) {
  if (streamed(p)) return launch_stream<2>(p, p.replicas > 1 ? p.replicas : 1, st);
  if (p.C % 8 || p.C > 256 || !pow2(p.C / 8)) return 1;
  const int sw = (p.W % 4 == 0) ? 4 : 1;
  const int64_t items = (int64_t)p.B * p.H * (p.W / sw) * (p.C / 8);
  int blocks = (int)((items + 2 * NT - 1) / (2 * NT));          // >= 2 items per thread
  const int cap = cfl_tune(TUNE_DW_WGRAD_BLOCKS) > 0 ? cfl_tune(TUNE_DW_WGRAD_BLOCKS) : 1024;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  const int reps = p.replicas > 1 ? p.replicas : 1;
  if (sw == 4) hipLaunchKernelGGL(dw_wgrad_kernel<4>, dim3(blocks), dim3(NT), 0, st, p, reps);
  else hipLaunchKernelGGL(dw_wgrad_kernel<1>, dim3(blocks), dim3(NT), 0, st, p, reps);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_dwconv(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_dwconv(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
