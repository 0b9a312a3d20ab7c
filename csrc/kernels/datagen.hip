// On-device synthetic crack data: renders the same images/masks as data/synthetic.py::render_numpy (integer-hash
// value-noise concrete texture, dark random-walk crack polylines, mask = pixels within the crack half-width)
// from the host-drawn segment table, so an 8000-image 256^2 dataset is generated in HBM in milliseconds and stays
// resident there (288 GB per GPU) - batch assembly is then just an index vector (entry.hip / head.hip).
#include "common.h"
#include "launch.h"

namespace {

CFL_DEVICE uint32_t hash3(uint32_t x, uint32_t y, uint32_t seed) {
  uint32_t h = x * 374761393u + y * 668265263u + seed * 2246822519u;
  h = (h ^ (h >> 13)) * 1274126177u;
  return h ^ (h >> 16);
}

__global__ void render_kernel(const float* segs, const float* params, uint8_t* images, uint8_t* masks, int img,
                              int max_seg) {
  const int n = blockIdx.y;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.z;
  if (x >= img) return;
  const float* par = params + n * 8;
  const float bg = par[0], noise_amp = par[1], dark = par[2], tint_r = par[3], tint_b = par[4];
  const uint32_t seed = (uint32_t)par[5];
  int cell = (int)par[6];
  if (cell < 1) cell = 1;
  const float fine = (float)(hash3(x, y, seed) & 255u) / 255.0f;
  const float coarse = (float)(hash3(x / cell, y / cell, seed + 7919u) & 255u) / 255.0f;
  float v = __fadd_rn(bg, __fmul_rn(noise_amp, __fsub_rn(__fadd_rn(__fmul_rn(0.35f, fine), __fmul_rn(0.65f, coarse)), 0.5f)));
  const float px = x + 0.5f, py = y + 0.5f;
  float dmin = 1e9f;
  const float* sg = segs + (size_t)n * max_seg * 6;
  for (int k = 0; k < max_seg; ++k) {
    const float x0 = sg[k * 6 + 0], y0 = sg[k * 6 + 1], x1 = sg[k * 6 + 2], y1 = sg[k * 6 + 3], hw = sg[k * 6 + 4];
    if (hw <= 0.f) continue;
    const float dx = __fsub_rn(x1, x0), dy = __fsub_rn(y1, y0);
    const float l2 = __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy));
    float t = __fdiv_rn(__fadd_rn(__fmul_rn(__fsub_rn(px, x0), dx), __fmul_rn(__fsub_rn(py, y0), dy)), fmaxf(l2, 1e-12f));
    t = fminf(fmaxf(t, 0.f), 1.f);
    const float ex = __fsub_rn(px, __fadd_rn(x0, __fmul_rn(t, dx)));
    const float ey = __fsub_rn(py, __fadd_rn(y0, __fmul_rn(t, dy)));
    const float d = __fdiv_rn(__fsqrt_rn(__fadd_rn(__fmul_rn(ex, ex), __fmul_rn(ey, ey))), hw);
    if (d < dmin) dmin = d;
  }
  const float shade = fminf(fmaxf(__fsub_rn(1.6f, dmin), 0.f), 1.f);
  v = __fsub_rn(v, __fmul_rn(shade, __fsub_rn(v, dark)));
  const size_t o = ((size_t)n * img + y) * img + x;
  const float r = fminf(fmaxf(__fadd_rn(v, tint_r), 0.f), 255.f);
  const float g = fminf(fmaxf(v, 0.f), 255.f);
  const float b = fminf(fmaxf(__fadd_rn(v, tint_b), 0.f), 255.f);
  images[o * 3 + 0] = (uint8_t)r;
  images[o * 3 + 1] = (uint8_t)g;
  images[o * 3 + 2] = (uint8_t)b;
  masks[o] = dmin < 1.0f ? 1 : 0;
}

}  // namespace

int render_cracks(const float* segs, const float* params, uint8_t* images, uint8_t* masks, int n, int img,
                  int max_seg, hipStream_t st) {
  dim3 grid((img + 127) / 128, n, img), blk(128);
  hipLaunchKernelGGL(render_kernel, grid, blk, 0, st, segs, params, images, masks, img, max_seg);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
