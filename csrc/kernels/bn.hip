// BatchNormalization (training mode, Keras defaults: axis -1, momentum 0.99, eps 1e-3; client_fit_model.py:101,
// 110, 114, 130, 134) as three small pieces around the convolutions that carry the heavy traffic:
//   bn_finalize      batch (or moving) statistics -> per-channel (a, b, mean, rstd); consumers apply a*y+b on load
//   bn_moving_update moving_mean / moving_variance (unbiased batch variance, TF fused-BN convention)
//   node_bwd         gradient of a graph node: sum of up to two incoming gradients, each with its own placement
//                    (same / stride-2 scatter / 2x2 upsample-sum / max-pool routing) and ReLU mask, the node's own
//                    ReLU mask, and the BN-backward reductions sum(g), sum(g * xhat) per channel
//   bn_bwd_apply     dy = a * (g - sum(g)/M - xhat * sum(g*xhat)/M); writes dgamma / dbeta
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

__global__ void bn_finalize_kernel(const float* stats, const float* gamma, const float* beta, const float* mmean,
                                   const float* mvar, float* ab, int C, float count, float eps, int train) {
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mean, var;
    if (train) {
      float s = 0.f, s2 = 0.f;
      for (int r = 0; r < STAT_REPLICAS; ++r) {
        s += stats[(size_t)r * 2 * C + c];
        s2 += stats[(size_t)r * 2 * C + C + c];
      }
      mean = s / count;
      var = fmaxf(s2 / count - mean * mean, 0.f);
    } else {
      mean = mmean[c];
      var = mvar[c];
    }
    const float rstd = rsqrtf(var + eps);
    const float a = gamma[c] * rstd;
    ab[c] = a;
    ab[C + c] = beta[c] - mean * a;
    ab[2 * C + c] = mean;
    ab[3 * C + c] = rstd;
  }
}

__global__ void bn_moving_kernel(const BnMoving* layers, float momentum) {
  const BnMoving L = layers[blockIdx.x];
  for (int c = threadIdx.x; c < L.C; c += blockDim.x) {
    float s = 0.f, s2 = 0.f;
    for (int r = 0; r < STAT_REPLICAS; ++r) {
      s += L.stats[(size_t)r * 2 * L.C + c];
      s2 += L.stats[(size_t)r * 2 * L.C + L.C + c];
    }
    const float mean = s / L.count;
    const float var = fmaxf(s2 / L.count - mean * mean, 0.f);
    const float unbiased = var * (L.count / fmaxf(L.count - 1.f, 1.f));
    L.mmean[c] = L.mmean[c] * momentum + mean * (1.f - momentum);
    L.mvar[c] = L.mvar[c] * momentum + unbiased * (1.f - momentum);
  }
}

CFL_DEVICE void load8(const bf16_t* p, float* f) { unpack8(*reinterpret_cast<const uint4*>(p), f); }

__global__ __launch_bounds__(NT) void node_bwd_kernel(NodeBwdParams p) {
  __shared__ float red[2][NT / 64][256];
  const int G = p.C >> 3, lanes = NT / G;
  const int cg = threadIdx.x % G, c0 = cg * 8;
  const int64_t npix = (int64_t)p.B * p.H * p.W;
  const int Hh = (p.H + 1) >> 1, Wh = (p.W + 1) >> 1;
  float a[8], bb[8], mean[8], rstd[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = p.ab ? p.ab[c0 + j] : 1.f;
    bb[j] = p.ab ? p.ab[p.C + c0 + j] : 0.f;
    mean[j] = p.ab ? p.ab[2 * p.C + c0 + j] : 0.f;
    rstd[j] = p.ab ? p.ab[3 * p.C + c0 + j] : 0.f;
  }
  float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t pix = (int64_t)blockIdx.x * lanes + threadIdx.x / G; pix < npix; pix += (int64_t)gridDim.x * lanes) {
    const int w = (int)(pix % p.W), h = (int)((pix / p.W) % p.H);
    const int64_t b = pix / ((int64_t)p.W * p.H);
    float y[8], v[8], g[8];
    load8(p.v + pix * p.C + c0, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = p.ab ? fmaf(a[j], y[j], bb[j]) : y[j];
      g[j] = 0.f;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const GradSrc src = p.src[s];
      if (src.mode == GM_NONE) continue;
      float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (src.mode == GM_SAME) {
        load8(src.p + pix * p.C + c0, t);
      } else if (src.mode == GM_SCATTER2) {
        if (((h | w) & 1) == 0) load8(src.p + ((b * Hh + (h >> 1)) * Wh + (w >> 1)) * p.C + c0, t);
      } else if (src.mode == GM_SUM2X2) {
        const int W2 = p.W * 2;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy)
#pragma unroll
          for (int dx = 0; dx < 2; ++dx) {
            float u[8];
            load8(src.p + ((b * (2 * p.H) + 2 * h + dy) * W2 + 2 * w + dx) * p.C + c0, u);
#pragma unroll
            for (int j = 0; j < 8; ++j) t[j] += u[j];
          }
      } else if (src.mode == GM_MAXPOOL) {
        // pooled outputs whose 3x3/s2 window contains (h, w): oh = h>>1 (ky = h&1) and, for even h >= 2,
        // oh = h/2 - 1 (ky = 2); same for w
        const int ohs[2] = {h >> 1, ((h & 1) == 0 && h >= 2) ? (h >> 1) - 1 : -1};
        const int kys[2] = {h & 1, 2};
        const int ows[2] = {w >> 1, ((w & 1) == 0 && w >= 2) ? (w >> 1) - 1 : -1};
        const int kxs[2] = {w & 1, 2};
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if (ohs[i] < 0 || ohs[i] >= Hh) continue;
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            if (ows[k] < 0 || ows[k] >= Wh) continue;
            const int64_t o = ((b * Hh + ohs[i]) * Wh + ows[k]) * p.C + c0;
            const uint2 am = *reinterpret_cast<const uint2*>(p.argmax + o);
            const int want = kys[i] * 3 + kxs[k];
            float u[8];
            load8(src.p + o, u);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t word = j < 4 ? am.x : am.y;
              if ((int)((word >> (8 * (j & 3))) & 0xffu) == want) t[j] += u[j];
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] += src.mask ? (v[j] > 0.f ? t[j] : 0.f) : t[j];
    }
    if (p.relu_node) {
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = v[j] > 0.f ? g[j] : 0.f;
    }
    const uint4 gv = pack8(g);
    *reinterpret_cast<uint4*>(p.out + pix * p.C + c0) = gv;
    if (p.sums) {
      float gr[8];
      unpack8(gv, gr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += gr[j];
        if (p.ab) s2[j] += gr[j] * (y[j] - mean[j]) * rstd[j];
      }
    }
  }
  if (!p.sums) return;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    for (int o = G; o < 64; o <<= 1) {
      s1[j] += __shfl_xor(s1[j], o, 64);
      s2[j] += __shfl_xor(s2[j], o, 64);
    }
  }
  if (lane < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][wid][c0 + j] = s1[j];
      red[1][wid][c0 + j] = s2[j];
    }
  }
  __syncthreads();
  const int nst = p.ab ? 2 : 1;
  for (int e = threadIdx.x; e < nst * p.C; e += NT) {
    const int st = e / p.C, c = e - st * p.C;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) v += red[st][w][c];
    atomicAdd(&p.sums[st * p.C + c], v);
  }
}

__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BnBwdApplyParams p) {
  const int G = p.C >> 3;
  const float invM = 1.f / (float)p.M;
  const int64_t total = (int64_t)p.M * G;
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < p.C; c += NT) {
      if (p.dbeta) p.dbeta[c] = p.sums[c];
      if (p.dgamma) p.dgamma[c] = p.sums[p.C + c];
    }
  }
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c0 = (int)(t % G) * 8;
    const int64_t m = t / G;
    float g[8], y[8], o[8];
    load8(p.g + m * p.C + c0, g);
    load8(p.y + m * p.C + c0, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      const float xhat = (y[j] - p.ab[2 * p.C + c]) * p.ab[3 * p.C + c];
      o[j] = p.ab[c] * (g[j] - p.sums[c] * invM - xhat * p.sums[p.C + c] * invM);
    }
    *reinterpret_cast<uint4*>(p.dy + m * p.C + c0) = pack8(o);
  }
}

int grid_cap(int64_t work, int cap) {
  int64_t g = (work + NT - 1) / NT;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

}  // namespace

int bn_finalize(const float* stats, const float* gamma, const float* beta, const float* mmean, const float* mvar,
                float* ab, int C, float count, float eps, int train, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(1), dim3(256), 0, st, stats, gamma, beta, mmean, mvar, ab, C, count,
                     eps, train);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int bn_moving_update(const BnMoving* d_layers, int n_layers, int max_c, float momentum, hipStream_t st) {
  (void)max_c;
  hipLaunchKernelGGL(bn_moving_kernel, dim3(n_layers), dim3(256), 0, st, d_layers, momentum);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int node_bwd(const NodeBwdParams& p, hipStream_t st) {
  if (p.C % 8 || p.C > 256 || (NT % (p.C / 8)) != 0) return 1;
  const int lanes = NT / (p.C / 8);
  const int64_t npix = (int64_t)p.B * p.H * p.W;
  int64_t blocks = (npix + lanes - 1) / lanes;
  if (blocks > 2048) blocks = 2048;   // bounded grid: one set of channel atomics per block
  hipLaunchKernelGGL(node_bwd_kernel, dim3((int)blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int bn_bwd_apply(const BnBwdApplyParams& p, hipStream_t st) {
  if (p.C % 8) return 1;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(grid_cap((int64_t)p.M * (p.C / 8), 4096)), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
