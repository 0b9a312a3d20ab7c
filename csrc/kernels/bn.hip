// BatchNormalization (training mode, Keras defaults: axis -1, momentum 0.99, eps 1e-3; client_fit_model.py:101,
// 110, 114, 130, 134) as small pieces around the convolutions that carry the heavy traffic:
//   bn_finalize      batch (or moving) statistics -> per-channel (a, b, mean, rstd); consumers apply a*y+b on load
//   bn_moving_update moving_mean / moving_variance (unbiased batch variance, TF fused-BN convention)
//   node_bwd         gradient of a graph node: sum of up to two incoming gradients, each with its own placement
//                    (same / stride-2 scatter / 2x2 upsample-sum / max-pool routing) and ReLU mask, the node's own
//                    ReLU mask, and the BN-backward reductions sum(g), sum(g * xhat) per channel
//   bn_bwd_apply     dy = a * (g - sum(g)/M - xhat * sum(g*xhat)/M); writes dgamma / dbeta
// Elementwise kernels walk whole NHWC rows per block (32-bit indices, shifts; see common.h).
#include "common.h"
#include "launch.h"
#include "side_bodies.h"

namespace {

constexpr int NT = 256;

// Replica-row reduction shared by the finalize / moving-statistics kernels: FT threads, thread -> (channel c,
// replica phase j), FT / C threads per channel, so every one of the STAT_REPLICAS * 2 loads of a channel is issued
// in ONE round (the 1-block kernel is latency-bound: a per-thread serial walk over 32 replicas took ~5 us).
constexpr int FT = 1024;

// sums of channel threadIdx.x (valid for threadIdx.x < C after the call) into (s, s2)
__device__ __forceinline__ void replica_sums(const float* stats, int C, float (*part)[FT], float& s, float& s2) {
  if (cfl_det()) {                                   // int64 fixed-point rows (common.h): exact in any order
    s = s2 = 0.f;
    if (threadIdx.x < C) stat_sums_det(stats, C, threadIdx.x, s, s2);
    return;
  }
  const int per = FT / C, c = threadIdx.x % C, j = threadIdx.x / C;
  float a = 0.f, b = 0.f;
  // fully unrolled with a guard: a thread's (up to STAT_REPLICAS / 4 for C = 256) loads all issue before the adds
  // (an unroll-by-4 runtime loop was two dependent memory round trips for C >= 128)
  float va[STAT_REPLICAS / 4], vb[STAT_REPLICAS / 4];
#pragma unroll
  for (int k = 0; k < STAT_REPLICAS / 4; ++k) {
    const int r = j + k * per;
    va[k] = r < STAT_REPLICAS ? stats[r * 2 * C + c] : 0.f;
    vb[k] = r < STAT_REPLICAS ? stats[r * 2 * C + C + c] : 0.f;
  }
#pragma unroll
  for (int k = 0; k < STAT_REPLICAS / 4; ++k) {
    a += va[k];
    b += vb[k];
  }
  part[0][threadIdx.x] = a;
  part[1][threadIdx.x] = b;
  __syncthreads();
  s = s2 = 0.f;
  if (threadIdx.x < C)
    for (int k = 0; k < per; ++k) {
      s += part[0][k * C + threadIdx.x];
      s2 += part[1][k * C + threadIdx.x];
    }
}

__global__ __launch_bounds__(FT) void bn_finalize_kernel(const float* stats, const float* gamma, const float* beta,
                                                         const float* mmean, const float* mvar, float* ab, int C,
                                                         float count, float eps, int train) {
  CFL_TS_GUARD;
  // one thread per channel, all of its 2 * STAT_REPLICAS loads in one round (bn_coef_from_stats: the same
  // arithmetic as the consumer-side finalize)
  const int c = threadIdx.x;
  if (c >= C) return;
  float a, b, mean, rstd;
  if (train) {
    bn_coef_from_stats(BnStatsIn{stats, gamma, beta, count, eps}, C, c, a, b, mean, rstd);
  } else {
    mean = mmean[c];
    rstd = rsqrtf(mvar[c] + eps);
    a = gamma[c] * rstd;
    b = beta[c] - mean * a;
  }
  ab[c] = a;
  ab[C + c] = b;
  ab[2 * C + c] = mean;
  ab[3 * C + c] = rstd;
}

__global__ __launch_bounds__(256) void bn_eval_kernel(const BnEval* layers) {
  CFL_TS_GUARD;
  const BnEval L = layers[blockIdx.x];
  for (int c = threadIdx.x; c < L.C; c += blockDim.x) {
    const float rstd = rsqrtf(L.mvar[c] + L.eps);
    const float a = L.gamma[c] * rstd;
    L.ab[c] = a;
    L.ab[L.C + c] = L.beta[c] - L.mmean[c] * a;
    L.ab[2 * L.C + c] = L.mmean[c];
    L.ab[3 * L.C + c] = rstd;
  }
}

__global__ __launch_bounds__(FT) void bn_moving_kernel(const BnMoving* layers, float momentum) {
  CFL_TS_GUARD;
  __shared__ float part[2][FT];
  const BnMoving L = layers[blockIdx.x];
  float s, s2;
  replica_sums(L.stats, L.C, part, s, s2);
  const int c = threadIdx.x;
  if (c < L.C) {
    const float mean = s / L.count;
    const float var = fmaxf(s2 / L.count - mean * mean, 0.f);
    const float unbiased = var * (L.count / fmaxf(L.count - 1.f, 1.f));
    L.mmean[c] = L.mmean[c] * momentum + mean * (1.f - momentum);
    L.mvar[c] = L.mvar[c] * momentum + unbiased * (1.f - momentum);
  }
}

// Gather the incoming gradient of one item (pixel `w` of row (b, h), channels c0..c0+7): loads only, so the
// caller can issue two items' gathers before any store (memory-level parallelism for a latency-bound walk).
// M0 / M1: compile-time GradMode of the two sources (-1 = read from p at run time)
template <int M0, int M1>
CFL_DEVICE void node_gather(const NodeBwdParams& p, int b, int h, int w, int c0, const float* a, const float* bb,
                            float* y, float* v, float* g) {
  const int Hh = (p.H + 1) >> 1, Wh = (p.W + 1) >> 1;
  const size_t pix = ((size_t)b * p.H + h) * p.W + w;
  load8(p.v + pix * p.C + c0, y);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    v[j] = p.ab ? fmaf(a[j], y[j], bb[j]) : y[j];
    g[j] = 0.f;
  }
#pragma unroll
  for (int si = 0; si < 2; ++si) {
    GradSrc src = p.src[si];
    const int cm = si == 0 ? M0 : M1;
    if (cm >= 0) src.mode = cm;
    if (src.mode == GM_NONE) continue;
    float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (src.mode == GM_SAME) {
      load8(src.p + pix * p.C + c0, t);
    } else if (src.mode == GM_SCATTER2) {
      if (((h | w) & 1) == 0) load8(src.p + ((size_t)(b * Hh + (h >> 1)) * Wh + (w >> 1)) * p.C + c0, t);
    } else if (src.mode == GM_SUM2X2) {
      const int W2 = p.W * 2;
      float u[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        load8(src.p + ((size_t)(b * 2 * p.H + 2 * h + (q >> 1)) * W2 + 2 * w + (q & 1)) * p.C + c0, u[q]);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = (u[0][j] + u[1][j]) + (u[2][j] + u[3][j]);
    } else if (src.mode == GM_MAXPOOL) {
      // pooled outputs whose 3x3/s2 window contains (h, w): oh = h>>1 (ky = h&1) and, for even h >= 2,
      // oh = h/2 - 1 (ky = 2); same for w
      // branch-free: the second candidate of each axis may not exist (clamped to a valid address, its tap id set
      // to one no argmax holds), so all four gathers issue back to back instead of one latency each
      const bool h2 = (h & 1) == 0 && h >= 2, w2 = (w & 1) == 0 && w >= 2;
      const int ohs[2] = {h >> 1, h2 ? (h >> 1) - 1 : 0};
      const int ows[2] = {w >> 1, w2 ? (w >> 1) - 1 : 0};
      const int kys[2] = {(h & 1) * 3, h2 ? 6 : 64};
      const int kxs[2] = {w & 1, w2 ? 2 : 64};
      uint2 am[4];
      float u[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const size_t o = ((size_t)(b * Hh + ohs[q >> 1]) * Wh + ows[q & 1]) * p.C + c0;
        am[q] = *reinterpret_cast<const uint2*>(p.argmax + o);
        load8(src.p + o, u[q]);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t want = (uint32_t)(kys[q >> 1] + kxs[q & 1]);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t word = j < 4 ? am[q].x : am[q].y;
          if (((word >> (8 * (j & 3))) & 0xffu) == want) t[j] += u[q][j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] += src.mask ? (v[j] > 0.f ? t[j] : 0.f) : t[j];
  }
}

// IPT items (pixel, 8-channel group) per thread per iteration, all gathered before any store: the walk is
// latency-bound (a 512-block grid leaves 8-16 items per thread at the 128^2 level), so the loads of several items
// must be in flight together
template <int M0, int M1, int IPT>
__global__ __launch_bounds__(NT) void node_bwd_kernel(NodeBwdParams p) {
  CFL_TS_GUARD;
  __shared__ float red[2][4][256];
  const int G = p.C >> 3, lg = ilog2(G);
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  const bool has_ab = p.ab != nullptr;
  const float* sab = p.sab ? p.sab : p.ab;        // statistics of the BN whose sums this pass accumulates
  float a[8], bb[8], mean[8], rstd[8];
  load_f8_or(p.ab + c0, has_ab, 1.f, a);
  load_f8_or(p.ab + p.C + c0, has_ab, 0.f, bb);
  load_f8_or(sab + 2 * p.C + c0, sab != nullptr, 0.f, mean);
  load_f8_or(sab + 3 * p.C + c0, sab != nullptr, 0.f, rstd);
  float s[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[0][j] = s[1][j] = 0.f;
  auto finish = [&](size_t pix, const float* y, const float* v, float* g) {
    if (p.relu_node) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = v[j] > 0.f ? g[j] : 0.f;
    }
    const uint4 gv = pack8(g);
    *reinterpret_cast<uint4*>(p.out + pix * p.C + c0) = gv;
    if (p.sums) {
      float gr[8], ys[8];
      unpack8(gv, gr);
      if (p.sy) load8(p.sy + pix * p.C + c0, ys);       // BN input of the node this gradient also feeds
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[0][j] += gr[j];
        s[1][j] += gr[j] * ((p.sy ? ys[j] : y[j]) - mean[j]) * rstd[j];   // rstd = 0 for a plain node
      }
    }
  };
  // flat items (pixel, channel group), IPT per iteration; the grid stride is a multiple of G
  const int total = (p.B * p.H * p.W) << lg;
  const int HW = p.H * p.W;
  const int stride = gridDim.x * NT;
  for (int it = blockIdx.x * NT + threadIdx.x; it < total; it += IPT * stride) {
    float y[IPT][8], v[IPT][8], g[IPT][8];
    int pix[IPT];
#pragma unroll
    for (int u = 0; u < IPT; ++u) {
      const int itu = it + u * stride;
      pix[u] = (itu < total ? itu : it) >> lg;            // clamped: every gather issues, only valid items store
      const int bu = pix[u] / HW, ru = pix[u] - bu * HW, hu = ru / p.W;
      node_gather<M0, M1>(p, bu, hu, ru - hu * p.W, c0, a, bb, y[u], v[u], g[u]);
    }
#pragma unroll
    for (int u = 0; u < IPT; ++u)
      if (it + u * stride < total) finish((size_t)pix[u], y[u], v[u], g[u]);
  }
  if (!p.sums) return;
  // replica row of this block: every block adding into ONE row of sums serialises at the memory-side atomic units
  const int reps = p.sum_reps > 1 ? p.sum_reps : 1;
  if (sab) block_channel_atomics<2>(s, G, p.C, p.sums, (size_t)(blockIdx.x % reps) * 2 * p.C, false, red);
  else {
    float s1[1][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[0][j] = s[0][j];
    block_channel_atomics<1>(s1, G, p.C, p.sums, (size_t)(blockIdx.x % reps) * p.C, false, red);
  }
}

template <int IPT>
__global__ __launch_bounds__(NT) void node_pool_bwd_kernel(NodeBwdParams p) {
  CFL_TS_GUARD;
  side::node_pool_body<IPT>(p, blockIdx.x, gridDim.x);
}

__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BnBwdApplyParams p) {
  CFL_TS_GUARD;
  side::bba_body(p, blockIdx.x, gridDim.x);
}

bool pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }

}  // namespace

int bn_finalize(const float* stats, const float* gamma, const float* beta, const float* mmean, const float* mvar,
                float* ab, int C, float count, float eps, int train, hipStream_t st) {
  if (C < 1 || C > FT) return 1;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(1), dim3(C <= 256 ? 256 : FT), 0, st, stats, gamma, beta, mmean, mvar, ab, C, count,
                     eps, train);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int bn_moving_update(const BnMoving* d_layers, int n_layers, int max_c, float momentum, hipStream_t st) {
  (void)max_c;                                 // every layer's C divides FT (checked when the table is built)
  hipLaunchKernelGGL(bn_moving_kernel, dim3(n_layers), dim3(FT), 0, st, d_layers, momentum);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int bn_eval_coefs(const BnEval* d_layers, int n_layers, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_kernel, dim3(n_layers), dim3(256), 0, st, d_layers);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

template <int IPT>
int launch_node(const NodeBwdParams& p, int blocks, hipStream_t st) {
  const int m0 = p.src[0].mode, m1 = p.src[1].mode;
  if (m0 == GM_SAME && m1 == GM_NONE) hipLaunchKernelGGL((node_bwd_kernel<GM_SAME, GM_NONE, IPT>), dim3(blocks), dim3(NT), 0, st, p);
  else if (m0 == GM_SUM2X2 && m1 == GM_NONE) hipLaunchKernelGGL((node_bwd_kernel<GM_SUM2X2, GM_NONE, IPT>), dim3(blocks), dim3(NT), 0, st, p);
  else if (m0 == GM_MAXPOOL && m1 == GM_NONE) hipLaunchKernelGGL((node_bwd_kernel<GM_MAXPOOL, GM_NONE, IPT>), dim3(blocks), dim3(NT), 0, st, p);
  else if (m0 == GM_SAME && m1 == GM_SAME) hipLaunchKernelGGL((node_bwd_kernel<GM_SAME, GM_SAME, IPT>), dim3(blocks), dim3(NT), 0, st, p);
  else if (m0 == GM_SUM2X2 && m1 == GM_SAME) hipLaunchKernelGGL((node_bwd_kernel<GM_SUM2X2, GM_SAME, IPT>), dim3(blocks), dim3(NT), 0, st, p);
  else if (m0 == GM_SAME && m1 == GM_SCATTER2) hipLaunchKernelGGL((node_bwd_kernel<GM_SAME, GM_SCATTER2, IPT>), dim3(blocks), dim3(NT), 0, st, p);
  else hipLaunchKernelGGL((node_bwd_kernel<-1, -1, 2>), dim3(blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

static int node_bwd_cap() {
  return cfl_tune(TUNE_NODE_BWD_BLOCKS) > 0 ? cfl_tune(TUNE_NODE_BWD_BLOCKS) : 512;   // A/B-measured
}

// the 2x2-block max-pool routing kernel serves this node gradient (node_pool_body)
bool node_pool_eligible(const NodeBwdParams& p) {
  return p.C % 8 == 0 && p.C <= 256 && pow2(p.C / 8) && p.src[0].mode == GM_MAXPOOL && p.src[1].mode == GM_NONE &&
         !p.src[0].mask && !p.relu_node && !p.sy && p.ab && p.argmax && ((p.H | p.W) & 1) == 0 &&
         cfl_tune(TUNE_NODE_POOL2X2) != 1;
}

int node_pool_grid(const NodeBwdParams& p) {
  const int64_t items2 = (int64_t)p.B * (p.H / 2) * (p.W / 2) * (p.C / 8);
  int b2 = (int)((items2 + NT - 1) / NT);
  const int pcap = cfl_tune(TUNE_NODE_POOL_BLOCKS) > 0 ? cfl_tune(TUNE_NODE_POOL_BLOCKS) : node_bwd_cap();
  if (b2 > pcap) b2 = pcap;
  return b2 < 1 ? 1 : b2;
}

int node_bwd(const NodeBwdParams& p, hipStream_t st) {
  if (p.C % 8 || p.C > 256 || !pow2(p.C / 8)) return 1;
  const int64_t items = (int64_t)p.B * p.H * p.W * (p.C / 8);
  int blocks = (int)((items + 2 * NT - 1) / (2 * NT));
  const int cap = node_bwd_cap();
  if (blocks > cap) blocks = cap;     // bounded grid: one set of channel atomics per block
  if (blocks < 1) blocks = 1;
  if (node_pool_eligible(p)) {
    const int b2 = node_pool_grid(p);
    // one item per thread per trip: 2 (TUNE_NODE_POOL_IPT=2) needs 188 VGPRs (occupancy 3 -> 2) and measured slower
    // (whole step 1.4652-1.4664 vs 1.4580-1.4616 ms/iteration)
    if (cfl_tune(TUNE_NODE_POOL_IPT) == 2) hipLaunchKernelGGL(node_pool_bwd_kernel<2>, dim3(b2), dim3(NT), 0, st, p);
    else hipLaunchKernelGGL(node_pool_bwd_kernel<1>, dim3(b2), dim3(NT), 0, st, p);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  // specialised instances for the engine's source combinations (fewer live registers, no mode branches)
  // 2 items in flight per thread: 4 doubles the registers (occupancy 3 -> 2 waves/SIMD) and measured slower
  // (whole step 1.684 vs 1.695 ms/iteration)
  if (cfl_tune(TUNE_NODE_BWD_IPT) == 4) return launch_node<4>(p, blocks, st);
  return launch_node<2>(p, blocks, st);
}

bool bn_bwd_apply_ok(const BnBwdApplyParams& p) {
  return p.C % 8 == 0 && pow2(p.C / 8) && p.C <= BNB_MAX_C && p.sum_reps <= BNB_MAX_REPS;
}

int bn_bwd_apply_grid(const BnBwdApplyParams& p) {
  int blocks = (int)(((int64_t)p.M * (p.C / 8) + side::BBA_IPT * NT - 1) / (side::BBA_IPT * NT));
  // 1024 -> 256 in round 6 (interleaved bench A/B: 13,861 -> 13,909 img/s; fewer blocks, each with its BN-backward
  // prologue, and the side-job launches stay within one round of resident blocks - profiles/r6_misc)
  const int cap = cfl_tune(TUNE_BBA_BLOCKS) > 0 ? cfl_tune(TUNE_BBA_BLOCKS) : 256;
  if (blocks > cap) blocks = cap;
  return blocks < 1 ? 1 : blocks;
}

int bn_bwd_apply(const BnBwdApplyParams& p, hipStream_t st) {
  if (!bn_bwd_apply_ok(p)) return 1;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(bn_bwd_apply_grid(p)), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_bn(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_bn(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
