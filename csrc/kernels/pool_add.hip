// Forward elementwise joins of the U-Net (the places where a BatchNorm output meets a residual):
//   pool_res_fwd: x = MaxPooling2D(3, s2, "same")(BN(y)) + residual          client_fit_model.py:114-122
//                 (TF same at stride 2: window rows 2*oh .. 2*oh+2 clipped at the bottom/right edge);
//                 the argmax (0..8 per channel) is kept for the backward routing
//   bn_add_fwd:   x_lo = BN(y) + q   or  BN(y) + up2(q)                      client_fit_model.py:134-141
//                 - the decoder's UpSampling2D of both branches commutes with the add and the 1x1 residual
//                 conv, so the add runs at the LOW resolution and the upsample is folded into consumers.
// Row-per-block walks with 32-bit indices and shifts (common.h).
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

__global__ __launch_bounds__(NT) void pool_res_kernel(PoolResParams p) {
  CFL_TS_GUARD;
  const int G = p.C >> 3, lg = ilog2(G);
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  float a[8], bb[8];
  load_f8(p.ab + c0, a);
  load_f8(p.ab + p.C + c0, bb);
  const int rows = p.B * p.Ho, items = p.Wo << lg;
  for (int row = xcd_swizzle(blockIdx.x, gridDim.x); row < rows; row += gridDim.x) {
    const int b = row / p.Ho, oh = row - b * p.Ho;
    for (int it = threadIdx.x; it < items; it += NT) {
      const int ow = it >> lg;
      float mx[8];
      int am[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
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
          load8(p.y + ((size_t)(b * p.H + ih) * p.W + iw) * p.C + c0, f);
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
      const size_t o = ((size_t)row * p.Wo + ow) * p.C + c0;
      float r[8];
      load8(p.res + o, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) mx[j] += r[j];
      *reinterpret_cast<uint4*>(p.out + o) = pack8(mx);
      uint2 packed;
      packed.x = (uint32_t)am[0] | ((uint32_t)am[1] << 8) | ((uint32_t)am[2] << 16) | ((uint32_t)am[3] << 24);
      packed.y = (uint32_t)am[4] | ((uint32_t)am[5] << 8) | ((uint32_t)am[6] << 16) | ((uint32_t)am[7] << 24);
      *reinterpret_cast<uint2*>(p.argmax + o) = packed;
    }
  }
}

__global__ __launch_bounds__(NT) void bn_add_kernel(BnAddParams p) {
  CFL_TS_GUARD;
  const int G = p.C >> 3, lg = ilog2(G);
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  float a[8], bb[8];
  load_f8(p.ab + c0, a);
  load_f8(p.ab + p.C + c0, bb);
  const int Hq = p.q_up ? p.H >> 1 : p.H, Wq = p.q_up ? p.W >> 1 : p.W;
  const int rows = p.B * p.H, items = p.W << lg;
  for (int row = xcd_swizzle(blockIdx.x, gridDim.x); row < rows; row += gridDim.x) {
    const int b = row / p.H, h = row - b * p.H;
    const int qrow = p.q_up ? b * Hq + (h >> 1) : row;
    for (int it = threadIdx.x; it < items; it += NT) {
      const int w = it >> lg;
      const size_t o = ((size_t)row * p.W + w) * p.C + c0;
      float y[8], q[8];
      load8(p.y + o, y);
      load8(p.q + ((size_t)qrow * Wq + (p.q_up ? w >> 1 : w)) * p.C + c0, q);
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = fmaf(a[j], y[j], bb[j]) + q[j];
      *reinterpret_cast<uint4*>(p.out + o) = pack8(y);
    }
  }
}

bool pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }

int row_blocks(int rows) { return rows < 2048 ? rows : 2048; }

}  // namespace

int pool_res_fwd(const PoolResParams& p, hipStream_t st) {
  if (p.C % 8 || !pow2(p.C / 8) || p.Ho != (p.H + 1) / 2 || p.Wo != (p.W + 1) / 2) return 1;
  hipLaunchKernelGGL(pool_res_kernel, dim3(row_blocks(p.B * p.Ho)), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int bn_add_fwd(const BnAddParams& p, hipStream_t st) {
  if (p.C % 8 || !pow2(p.C / 8) || (p.q_up && ((p.H | p.W) & 1))) return 1;
  hipLaunchKernelGGL(bn_add_kernel, dim3(row_blocks(p.B * p.H)), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_pool_add(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_pool_add(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
