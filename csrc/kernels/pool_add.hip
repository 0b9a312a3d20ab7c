// Forward elementwise joins of the U-Net (the places where a BatchNorm output meets a residual):
//   pool_res_fwd: x = MaxPooling2D(3, s2, "same")(BN(y)) + residual          client_fit_model.py:114-122
//                 (TF same at stride 2: window rows 2*oh .. 2*oh+2 clipped at the bottom/right edge);
//                 the argmax (0..8 per channel) is kept for the backward routing
//   bn_add_fwd:   x_lo = BN(y) + q   or  BN(y) + up2(q)                      client_fit_model.py:134-141
//                 - the decoder's UpSampling2D of both branches commutes with the add and the 1x1 residual
//                 conv, so the add runs at the LOW resolution and the upsample is folded into consumers.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

int grid_cap(int64_t work, int cap) {
  int64_t g = (work + NT - 1) / NT;
  return (int)(g < cap ? (g < 1 ? 1 : g) : cap);
}

__global__ __launch_bounds__(NT) void pool_res_kernel(PoolResParams p) {
  const int G = p.C >> 3;
  const int64_t total = (int64_t)p.B * p.Ho * p.Wo * G;
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c0 = (int)(t % G) * 8;
    const int64_t op = t / G;
    const int ow = (int)(op % p.Wo), oh = (int)((op / p.Wo) % p.Ho);
    const int64_t b = op / ((int64_t)p.Wo * p.Ho);
    float a[8], bb[8], mx[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = p.ab[c0 + j];
      bb[j] = p.ab[p.C + c0 + j];
      mx[j] = -INFINITY;
      am[j] = 0;
    }
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int ih = 2 * oh + ky;
      if (ih >= p.H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iw = 2 * ow + kx;
        if (iw >= p.W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(p.y + ((b * p.H + ih) * p.W + iw) * p.C + c0), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = fmaf(a[j], f[j], bb[j]);
          if (v > mx[j]) {
            mx[j] = v;
            am[j] = ky * 3 + kx;
          }
        }
      }
    }
    float r[8];
    unpack8(*reinterpret_cast<const uint4*>(p.res + op * p.C + c0), r);
#pragma unroll
    for (int j = 0; j < 8; ++j) mx[j] += r[j];
    *reinterpret_cast<uint4*>(p.out + op * p.C + c0) = pack8(mx);
    uint2 packed;
    packed.x = (uint32_t)am[0] | ((uint32_t)am[1] << 8) | ((uint32_t)am[2] << 16) | ((uint32_t)am[3] << 24);
    packed.y = (uint32_t)am[4] | ((uint32_t)am[5] << 8) | ((uint32_t)am[6] << 16) | ((uint32_t)am[7] << 24);
    *reinterpret_cast<uint2*>(p.argmax + op * p.C + c0) = packed;
  }
}

__global__ __launch_bounds__(NT) void bn_add_kernel(BnAddParams p) {
  const int G = p.C >> 3;
  const int64_t total = (int64_t)p.B * p.H * p.W * G;
  const int Hq = p.q_up ? p.H >> 1 : p.H, Wq = p.q_up ? p.W >> 1 : p.W;
  for (int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int c0 = (int)(t % G) * 8;
    const int64_t pix = t / G;
    const int w = (int)(pix % p.W), h = (int)((pix / p.W) % p.H);
    const int64_t b = pix / ((int64_t)p.W * p.H);
    float y[8], q[8];
    unpack8(*reinterpret_cast<const uint4*>(p.y + pix * p.C + c0), y);
    const int64_t qi = p.q_up ? ((b * Hq + (h >> 1)) * Wq + (w >> 1)) : pix;
    unpack8(*reinterpret_cast<const uint4*>(p.q + qi * p.C + c0), q);
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = fmaf(p.ab[c0 + j], y[j], p.ab[p.C + c0 + j]) + q[j];
    *reinterpret_cast<uint4*>(p.out + pix * p.C + c0) = pack8(y);
  }
}

}  // namespace

int pool_res_fwd(const PoolResParams& p, hipStream_t st) {
  if (p.C % 8 || p.Ho != (p.H + 1) / 2 || p.Wo != (p.W + 1) / 2) return 1;
  hipLaunchKernelGGL(pool_res_kernel, dim3(grid_cap((int64_t)p.B * p.Ho * p.Wo * (p.C / 8), 4096)), dim3(NT), 0, st,
                     p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int bn_add_fwd(const BnAddParams& p, hipStream_t st) {
  if (p.C % 8 || (p.q_up && ((p.H | p.W) & 1))) return 1;
  hipLaunchKernelGGL(bn_add_kernel, dim3(grid_cap((int64_t)p.B * p.H * p.W * (p.C / 8), 4096)), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
