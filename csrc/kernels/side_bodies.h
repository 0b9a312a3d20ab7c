// Bodies of the streaming BN-backward passes (bn.hip), callable from any kernel with an explicit (block index, block
// count): bn.hip launches them alone, and pw.hip runs them as the "side job" of a streaming 1x1 data gradient that
// is independent of them - one launch for two latency-bound passes that read the same incoming gradient
// (launch.h SideJob).
#pragma once
#include "common.h"
#include "launch.h"

namespace {
namespace side {

constexpr int NT = 256;

// Gradient of a BN node routed back through MaxPooling2D(3, s2, same) (encoder: node_bwd<GM_MAXPOOL, GM_NONE>
// without masks), one 2x2 input-pixel block per item: the four pooled windows (i-1..i) x (j-1..j) that can hold
// these pixels' maxima are read ONCE for all four pixels (the per-pixel gather read each window's gradient and
// argmax up to 4x from L2). Window (i,j) holds pixel (dy,dx) at tap dy*3+dx, window (i-1,j) the top row at tap
// 6+dx, window (i,j-1) the left column at tap dy*3+2, window (i-1,j-1) pixel (0,0) at tap 8. Same BN-backward sums
// as node_bwd (sum g, sum g * xhat).
// IPT items per thread per trip: all their window / argmax / BN-input loads are issued before any of them is routed
// (one memory round trip per IPT items; the grid is capped, so the 128^2 level runs several trips per thread).
template <int IPT>
CFL_DEVICE void node_pool_body(const NodeBwdParams& p, int bid, int nblocks) {
  __shared__ float red[2][4][256];
  const int G = p.C >> 3, lg = ilog2(G);
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  const bool stats = p.sums != nullptr && p.ab != nullptr;
  float mean[8], rstd[8];
  load_f8_or(p.ab + 2 * p.C + c0, stats, 0.f, mean);
  load_f8_or(p.ab + 3 * p.C + c0, stats, 0.f, rstd);
  float s[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[0][j] = s[1][j] = 0.f;
  const int Hh = p.H >> 1, Wh = p.W >> 1;
  const int total = (p.B * Hh * Wh) << lg;
  const int HWh = Hh * Wh;
  const int stride = nblocks * NT;                       // a multiple of G: a thread's channel group never changes
  for (int it0 = bid * NT + threadIdx.x; it0 < total; it0 += IPT * stride) {
    uint4 uw[IPT][4], yv[IPT][4];
    uint2 am[IPT][4];
    size_t pix0[IPT];
#pragma unroll
    for (int v = 0; v < IPT; ++v) {
      const int itv = it0 + v * stride;
      const int blk = (itv < total ? itv : it0) >> lg;   // clamped: every load issues, only valid items store
      const int b = blk / HWh, r = blk - b * HWh, i = r / Wh, j = r - i * Wh;
      // windows q = (wi, wj): 0 = (i, j), 1 = (i, j-1), 2 = (i-1, j), 3 = (i-1, j-1); missing ones read window 0
      // with a tap no argmax holds
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool up = q >= 2, left = q & 1;
        const bool ok = (!up || i > 0) && (!left || j > 0);
        const int wi = ok ? i - up : i, wj = ok ? j - left : j;
        const size_t o = ((size_t)(b * Hh + wi) * Wh + wj) * p.C + c0;
        am[v][q] = *reinterpret_cast<const uint2*>(p.argmax + o);
        uw[v][q] = *reinterpret_cast<const uint4*>(p.src[0].p + o);
        if (!ok) am[v][q] = make_uint2(0xffffffffu, 0xffffffffu);
      }
      pix0[v] = (size_t)(b * p.H + 2 * i) * p.W + 2 * j;
#pragma unroll
      for (int d = 0; d < 4; ++d)
        yv[v][d] = stats ? *reinterpret_cast<const uint4*>(p.v + (pix0[v] + (d >> 1) * p.W + (d & 1)) * p.C + c0)
                         : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int v = 0; v < IPT; ++v) {
      if (it0 + v * stride >= total) break;
      float u[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) unpack8(uw[v][q], u[q]);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int dy = d >> 1, dx = d & 1;
        const size_t pix = pix0[v] + dy * p.W + dx;
        // taps of this pixel in windows 0..3 (64 = not contained)
        const uint32_t tw[4] = {(uint32_t)(dy * 3 + dx), dx == 0 ? (uint32_t)(dy * 3 + 2) : 64u,
                                dy == 0 ? (uint32_t)(6 + dx) : 64u, (dy == 0 && dx == 0) ? 8u : 64u};
        float g[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          float t = 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint32_t word = jj < 4 ? am[v][q].x : am[v][q].y;
            if (((word >> (8 * (jj & 3))) & 0xffu) == tw[q]) t += u[q][jj];
          }
          g[jj] = t;
        }
        const uint4 gv = pack8(g);
        *reinterpret_cast<uint4*>(p.out + pix * p.C + c0) = gv;
        if (stats) {
          float gr[8], y[8];
          unpack8(gv, gr);
          unpack8(yv[v][d], y);
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            s[0][jj] += gr[jj];
            s[1][jj] += gr[jj] * (y[jj] - mean[jj]) * rstd[jj];
          }
        }
      }
    }
  }
  if (!p.sums) return;
  const int reps = p.sum_reps > 1 ? p.sum_reps : 1;
  block_channel_atomics<2>(s, G, p.C, p.sums, (size_t)(bid % reps) * 2 * p.C, false, red);
}

constexpr int BBA_IPT = 4;

CFL_DEVICE void bba_body(const BnBwdApplyParams& p, int bid, int nblocks) {
  __shared__ __attribute__((aligned(16))) float co[5 * BNB_MAX_C];
  __shared__ float part[NT];
  const int G = p.C >> 3, lg = ilog2(G);
  const int total = p.M << lg;
  // grid stride is a multiple of G, so a thread's channel group never changes
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  const int S = nblocks * NT;
  // the first BBA_IPT items are loaded BEFORE the replica reduction below, so their latency overlaps it (the
  // low-resolution layers run one iteration per thread: prologue and loads were two serial memory round trips)
  uint4 g[BBA_IPT], y[BBA_IPT];
  auto load_items = [&](int t0) {
#pragma unroll
    for (int u = 0; u < BBA_IPT; ++u) {
      const int t = t0 + u * S;
      const size_t m = (size_t)(t < total ? t : (t0 < total ? t0 : 0)) >> lg;   // clamped: loads unconditional
      g[u] = *reinterpret_cast<const uint4*>(p.g + m * p.C + c0);
      y[u] = *reinterpret_cast<const uint4*>(p.y + m * p.C + c0);
    }
  };
  int t0 = bid * NT + threadIdx.x;
  load_items(t0);
  // the same prologue and element arithmetic as the conv operands that fold this pass (common.h BnBwdIn)
  const BnBwdIn q{p.y, p.ab, p.sums, p.sum_reps, 1.f / (float)p.M, p.dy, p.dgamma, p.dbeta};
  bnb_prologue<NT>(q, p.C, co, part, bid == 0);
  // this thread's channel group: constant over its items. 16-byte reads: 8-float rows at an 8-float stride read as
  // scalars were 8-way LDS bank conflicts per read (SQ_LDS_BANK_CONFLICT 43 %, profiles/r3_final/pmc_summary.txt)
  // The two 16-byte halves are read in swapped order by the channel groups with bit 3 set: a ds_read_b128 lane group
  // holds 16 channel groups, whose 32-byte rows put groups l and l + 8 on the same banks (8 l dwords mod 64) when
  // C >= 128 (PMC: 14.6 % conflict cycles)
  const int sw = (c0 >> 6) & 1;
  float a[8], mean[8], rstd[8], k1[8], k2[8];
  auto load_co = [&](const float* r, float* f) {
    const float4 h0 = *reinterpret_cast<const float4*>(r + 4 * sw);
    const float4 h1 = *reinterpret_cast<const float4*>(r + 4 - 4 * sw);
    const float4 lo = sw ? h1 : h0, hi = sw ? h0 : h1;
    f[0] = lo.x; f[1] = lo.y; f[2] = lo.z; f[3] = lo.w; f[4] = hi.x; f[5] = hi.y; f[6] = hi.z; f[7] = hi.w;
  };
  load_co(co + c0, a);
  load_co(co + p.C + c0, mean);
  load_co(co + 2 * p.C + c0, rstd);
  load_co(co + 3 * p.C + c0, k1);
  load_co(co + 4 * p.C + c0, k2);
  // BBA_IPT items per thread per iteration, all loads issued before any math (memory-level parallelism: the small
  // layers launch few blocks, so one item in flight per thread would leave HBM latency-bound)
  for (; t0 < total; t0 += BBA_IPT * S) {
#pragma unroll
    for (int u = 0; u < BBA_IPT; ++u) {
      const int t = t0 + u * S;
      float gf[8], yf[8], of[8];
      unpack8(g[u], gf);
      unpack8(y[u], yf);
#pragma unroll
      for (int j = 0; j < 8; ++j) of[j] = bnb_apply(gf[j], yf[j], a[j], mean[j], rstd[j], k1[j], k2[j]);
      const uint4 o = pack8(of);
      if (t < total) *reinterpret_cast<uint4*>(p.dy + (size_t)(t >> lg) * p.C + c0) = o;
    }
    if (t0 + BBA_IPT * S < total) load_items(t0 + BBA_IPT * S);
  }
}

}  // namespace side
}  // namespace
