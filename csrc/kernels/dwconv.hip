// Depthwise 3x3 convolution (SeparableConv2D's first stage, depth_multiplier 1, "same" pad 1):
// /root/reference/client_fit_model.py:109,113. Memory-bound (9 MAC per element).
//
// Work item = 8 channels (one 16-byte vector) x a strip of SW consecutive pixels of one row. The strip's input
// window (3 rows x SW+2 columns) is loaded once, the producer's BN-apply + ReLU (coefficients held in registers)
// applied once per loaded element, and reused by the 3 horizontal taps of every output in the strip - instead of
// re-loading and re-transforming each input 9 times. Keras depthwise kernel layout (3,3,C,1) = [tap][C].
// wgrad keeps 72 fp32 partial sums per thread across a grid-stride sweep, reduces over the wave's pixel lanes
// with shuffles and over the block's waves through LDS, then one atomic per (tap, channel) per block.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

struct Coef8 {
  float a[8], b[8];
};

CFL_DEVICE void load_coef(const InXform& xf, int c0, Coef8& k) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k.a[j] = 1.f;
    k.b[j] = 0.f;
  }
  if (xf.ab) {
    const float4 a0 = *reinterpret_cast<const float4*>(xf.ab + c0);
    const float4 a1 = *reinterpret_cast<const float4*>(xf.ab + c0 + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(xf.ab + xf.C + c0);
    const float4 b1 = *reinterpret_cast<const float4*>(xf.ab + xf.C + c0 + 4);
    k.a[0] = a0.x; k.a[1] = a0.y; k.a[2] = a0.z; k.a[3] = a0.w;
    k.a[4] = a1.x; k.a[5] = a1.y; k.a[6] = a1.z; k.a[7] = a1.w;
    k.b[0] = b0.x; k.b[1] = b0.y; k.b[2] = b0.z; k.b[3] = b0.w;
    k.b[4] = b1.x; k.b[5] = b1.y; k.b[6] = b1.z; k.b[7] = b1.w;
  }
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
  for (int t = 0; t < 9; ++t) {
    const int src = flip ? 8 - t : t;
    const float4 w0 = *reinterpret_cast<const float4*>(w + src * C + c0);
    const float4 w1 = *reinterpret_cast<const float4*>(w + src * C + c0 + 4);
    wt[t][0] = w0.x; wt[t][1] = w0.y; wt[t][2] = w0.z; wt[t][3] = w0.w;
    wt[t][4] = w1.x; wt[t][5] = w1.y; wt[t][6] = w1.z; wt[t][7] = w1.w;
  }
}

// out[h][w] = sum_{ky,kx} in[h+ky-1][w+kx-1] * wt[ky*3+kx]   (dgrad uses the flipped kernel: same form)
template <int SW>
__global__ __launch_bounds__(NT) void dw_conv_kernel(const bf16_t* __restrict__ x, const float* __restrict__ w,
                                                     bf16_t* __restrict__ y, InXform xf, int B, int H, int W, int C,
                                                     int flip) {
  const int G = C >> 3, strips = W / SW;
  const int64_t total = (int64_t)B * H * strips * G;
  const bool has_ab = xf.ab != nullptr;
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cg = (int)(t % G);
    int64_t r = t / G;
    const int s = (int)(r % strips);
    r /= strips;
    const int h = (int)(r % H);
    const int64_t b = r / H;
    const int c0 = cg * 8, w0 = s * SW;
    Coef8 k;
    load_coef(xf, c0, k);
    float wt[9][8];
    load_w9(w, C, c0, wt, flip != 0);
    float acc[SW][8];
#pragma unroll
    for (int i = 0; i < SW; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int ih = h + ky - 1;
      if (ih < 0 || ih >= H) continue;
      const bf16_t* row = x + ((b * H + ih) * W) * C + c0;
#pragma unroll
      for (int cx = 0; cx < SW + 2; ++cx) {
        const int iw = w0 + cx - 1;
        if (iw < 0 || iw >= W) continue;
        float f[8];
        load_x8(row + (int64_t)iw * C, k, has_ab, xf.relu, f);
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int o = cx - kx;      // output index in the strip using this input at tap kx
          if (o < 0 || o >= SW) continue;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[o][j] = fmaf(f[j], wt[ky * 3 + kx][j], acc[o][j]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < SW; ++i)
      *reinterpret_cast<uint4*>(y + ((b * H + h) * W + w0 + i) * C + c0) = pack8(acc[i]);
  }
}

template <int SW>
__global__ __launch_bounds__(NT) void dw_wgrad_kernel(DwParams p) {
  __shared__ float red[NT / 64][9][256];
  const int G = p.C >> 3, strips = p.W / SW;
  const int cg = threadIdx.x % G, c0 = cg * 8;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t total = (int64_t)p.B * p.H * strips;        // strip work items per channel group
  const int lanes = NT / G;
  const bool has_ab = p.xf.ab != nullptr;
  Coef8 k;
  load_coef(p.xf, c0, k);
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[t][j] = 0.f;
  for (int64_t it = (int64_t)blockIdx.x * lanes + threadIdx.x / G; it < total; it += (int64_t)gridDim.x * lanes) {
    const int s = (int)(it % strips);
    const int64_t r = it / strips;
    const int h = (int)(r % p.H);
    const int64_t b = r / p.H;
    const int w0 = s * SW;
    float g[SW][8];
#pragma unroll
    for (int i = 0; i < SW; ++i) unpack8(*reinterpret_cast<const uint4*>(p.dy + ((b * p.H + h) * p.W + w0 + i) * p.C + c0), g[i]);
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int ih = h + ky - 1;
      if (ih < 0 || ih >= p.H) continue;
      const bf16_t* row = p.x + ((b * p.H + ih) * p.W) * p.C + c0;
#pragma unroll
      for (int cx = 0; cx < SW + 2; ++cx) {
        const int iw = w0 + cx - 1;
        if (iw < 0 || iw >= p.W) continue;
        float f[8];
        load_x8(row + (int64_t)iw * p.C, k, has_ab, p.xf.relu, f);
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
  // reduce the wave's lanes that share this channel group (lane stride G), then the block's waves via LDS
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
  for (int e = threadIdx.x; e < 9 * p.C; e += NT) {
    const int t = e / p.C, c = e - t * p.C;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) v += red[w][t][c];
    atomicAdd(&p.dw[t * p.C + c], v);
  }
}

int grid_for(int64_t work, int cap) {
  int64_t g = (work + NT - 1) / NT;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

int launch_dw(const bf16_t* x, const float* w, bf16_t* y, InXform xf, int B, int H, int W, int C, int flip,
              hipStream_t st) {
  if (C % 8 || C > 256) return 1;
  if (W % 4 == 0) {
    const int64_t work = (int64_t)B * H * (W / 4) * (C / 8);
    hipLaunchKernelGGL(dw_conv_kernel<4>, dim3(grid_for(work, 8192)), dim3(NT), 0, st, x, w, y, xf, B, H, W, C, flip);
  } else {
    const int64_t work = (int64_t)B * H * W * (C / 8);
    hipLaunchKernelGGL(dw_conv_kernel<1>, dim3(grid_for(work, 8192)), dim3(NT), 0, st, x, w, y, xf, B, H, W, C, flip);
  }
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

}  // namespace

int dw_fwd(const DwParams& p, hipStream_t st) { return launch_dw(p.x, p.w, p.y, p.xf, p.B, p.H, p.W, p.C, 0, st); }

int dw_dgrad(const DwParams& p, hipStream_t st) {
  return launch_dw(p.dy, p.w, p.y, InXform{nullptr, p.C, 0}, p.B, p.H, p.W, p.C, 1, st);
}

int dw_wgrad(const DwParams& p, hipStream_t st) {
  if (p.C % 8 || p.C > 256 || (NT % (p.C / 8)) != 0) return 1;
  const int G = p.C / 8, lanes = NT / G;
  const int sw = (p.W % 4 == 0) ? 4 : 1;
  const int64_t items = (int64_t)p.B * p.H * (p.W / sw);
  // ~16 strip items per thread keeps the per-block reduction + atomics amortised
  int64_t blocks = (items + (int64_t)lanes * 16 - 1) / ((int64_t)lanes * 16);
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  if (sw == 4) hipLaunchKernelGGL(dw_wgrad_kernel<4>, dim3((int)blocks), dim3(NT), 0, st, p);
  else hipLaunchKernelGGL(dw_wgrad_kernel<1>, dim3((int)blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
