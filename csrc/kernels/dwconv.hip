// Depthwise 3x3 convolution (SeparableConv2D's first stage, depth_multiplier 1, "same" pad 1):
// /root/reference/client_fit_model.py:109,113. Memory-bound (9 MAC per element): each thread owns 8 channels of
// one pixel (16-byte loads/stores), the 9 taps come through L1/L2; the producer's BN-apply + ReLU is applied on
// load, so the normalised activation is never materialised. Keras depthwise kernel layout (3,3,C,1) = [tap][C].
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void dw_fwd_kernel(DwParams p) {
  const int G = p.C >> 3;
  const int64_t total = (int64_t)p.B * p.H * p.W * G;
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cg = (int)(t % G);
    const int64_t pix = t / G;
    const int w = (int)(pix % p.W), h = (int)((pix / p.W) % p.H);
    const int64_t b = pix / ((int64_t)p.W * p.H);
    const int c0 = cg * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int ih = h + ky - 1;
      if (ih < 0 || ih >= p.H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iw = w + kx - 1;
        if (iw < 0 || iw >= p.W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(p.x + ((b * p.H + ih) * p.W + iw) * p.C + c0), f);
        const float4 w0 = *reinterpret_cast<const float4*>(p.w + (ky * 3 + kx) * p.C + c0);
        const float4 w1 = *reinterpret_cast<const float4*>(p.w + (ky * 3 + kx) * p.C + c0 + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(xform1(f[j], p.xf, c0 + j), wv[j], acc[j]);
      }
    }
    *reinterpret_cast<uint4*>(p.y + pix * p.C + c0) = pack8(acc);
  }
}

// d(input of dw) = correlation of dy with the flipped kernel
__global__ __launch_bounds__(NT) void dw_dgrad_kernel(DwParams p) {
  const int G = p.C >> 3;
  const int64_t total = (int64_t)p.B * p.H * p.W * G;
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cg = (int)(t % G);
    const int64_t pix = t / G;
    const int w = (int)(pix % p.W), h = (int)((pix / p.W) % p.H);
    const int64_t b = pix / ((int64_t)p.W * p.H);
    const int c0 = cg * 8;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int oh = h - ky + 1;
      if (oh < 0 || oh >= p.H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int ow = w - kx + 1;
        if (ow < 0 || ow >= p.W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(p.dy + ((b * p.H + oh) * p.W + ow) * p.C + c0), f);
        const float4 w0 = *reinterpret_cast<const float4*>(p.w + (ky * 3 + kx) * p.C + c0);
        const float4 w1 = *reinterpret_cast<const float4*>(p.w + (ky * 3 + kx) * p.C + c0 + 4);
        const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(f[j], wv[j], acc[j]);
      }
    }
    *reinterpret_cast<uint4*>(p.y + pix * p.C + c0) = pack8(acc);
  }
}

// dW[tap][c] = sum_pixels T(x)[pixel + tap - 1] * dy[pixel]; per-thread 72 partial sums, block reduction per tap
// through LDS, one fp32 atomic per (tap, channel) per block.
__global__ __launch_bounds__(NT) void dw_wgrad_kernel(DwParams p, int64_t pix_per_block) {
  __shared__ float red[NT][9];
  const int G = p.C >> 3;                 // channel groups (<= 32)
  const int lanes = NT / G;               // pixel lanes per block
  const int cg = threadIdx.x % G, pl = threadIdx.x / G;
  const bool active = pl < lanes;
  const int c0 = cg * 8;
  const int64_t npix = (int64_t)p.B * p.H * p.W;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_block;
  const int64_t p1 = p0 + pix_per_block < npix ? p0 + pix_per_block : npix;
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  if (active) {
    for (int64_t pix = p0 + pl; pix < p1; pix += lanes) {
      const int w = (int)(pix % p.W), h = (int)((pix / p.W) % p.H);
      const int64_t b = pix / ((int64_t)p.W * p.H);
      float g[8];
      unpack8(*reinterpret_cast<const uint4*>(p.dy + pix * p.C + c0), g);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        const int ih = h + ky - 1;
        if (ih < 0 || ih >= p.H) continue;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int iw = w + kx - 1;
          if (iw < 0 || iw >= p.W) continue;
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(p.x + ((b * p.H + ih) * p.W + iw) * p.C + c0), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[ky * 3 + kx][j] = fmaf(xform1(f[j], p.xf, c0 + j), g[j], acc[ky * 3 + kx][j]);
        }
      }
    }
  }
  // reduce over pixel lanes: one channel (of 8) at a time to keep LDS small
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int t = 0; t < 9; ++t) red[threadIdx.x][t] = active ? acc[t][j] : 0.f;
    __syncthreads();
    // thread (cg, t) sums over lanes
    for (int e = threadIdx.x; e < G * 9; e += NT) {
      const int tcg = e % G, t = e / G;
      float s = 0.f;
      for (int l = 0; l < lanes; ++l) s += red[l * G + tcg][t];
      atomicAdd(&p.dw[t * p.C + tcg * 8 + j], s);
    }
    __syncthreads();
  }
}

int grid_for(int64_t work) {
  int64_t g = (work + NT - 1) / NT;
  return (int)(g < 4096 ? (g < 1 ? 1 : g) : 4096);
}

}  // namespace

int dw_fwd(const DwParams& p, hipStream_t st) {
  if (p.C % 8) return 1;
  hipLaunchKernelGGL(dw_fwd_kernel, dim3(grid_for((int64_t)p.B * p.H * p.W * (p.C / 8))), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int dw_dgrad(const DwParams& p, hipStream_t st) {
  if (p.C % 8) return 1;
  hipLaunchKernelGGL(dw_dgrad_kernel, dim3(grid_for((int64_t)p.B * p.H * p.W * (p.C / 8))), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int dw_wgrad(const DwParams& p, hipStream_t st) {
  if (p.C % 8 || p.C / 8 > NT / 4) return 1;
  const int64_t npix = (int64_t)p.B * p.H * p.W;
  int blocks = 1024;
  int64_t per = (npix + blocks - 1) / blocks;
  if (per < 64) per = 64;
  blocks = (int)((npix + per - 1) / per);
  hipLaunchKernelGGL(dw_wgrad_kernel, dim3(blocks), dim3(NT), 0, st, p, per);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
