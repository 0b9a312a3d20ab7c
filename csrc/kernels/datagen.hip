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
  CFL_TS_GUARD;
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

// ---------------------------------------------------------------------------------------------------------------
// Folder data path (/root/reference/client_fit_model.py:34-40: cv2.imread -> cvtColor -> cv2.resize INTER_LINEAR ->
// (mask) > 0): the decoded images of a whole dataset, each at its own size, resized on the device in one launch into
// the HBM-resident uint8 dataset [n, dh, dw, c] (the /255 normalisation stays folded into the entry conv).
// Sampling grid and arithmetic are the host reference's (csrc/native/module.cpp resize_rows: half-pixel centres,
// clamped borders, float lerps, round-to-nearest-even) with contraction-free float ops: bit-exact when down-scaling,
// within 1 LSB on < 1 % of the values when up-scaling (tests/test_gpu_kernels.py).
namespace {
__global__ void resize_batch_kernel(const uint8_t* __restrict__ src, const int64_t* __restrict__ offs,
                                    const int* __restrict__ dims, uint8_t* __restrict__ dst, int dh, int dw, int c,
                                    int binarize) {
  CFL_TS_GUARD;
  const int img = blockIdx.y;
  const int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= dh * dw) return;
  const int y = pix / dw, x = pix - y * dw;
  const int sh = dims[2 * img], sw = dims[2 * img + 1];
  const uint8_t* s = src + offs[img];
  const float fy = (float)sh / dh, fx = (float)sw / dw;
  float sx = __fsub_rn(__fmul_rn(x + 0.5f, fx), 0.5f);
  int ix = (int)floorf(sx);
  float a = __fsub_rn(sx, (float)ix);
  if (ix < 0) { ix = 0; a = 0.f; }
  if (ix >= sw - 1) { ix = sw - 1; a = 0.f; }
  const int ix1 = min(ix + 1, sw - 1);
  float sy = __fsub_rn(__fmul_rn(y + 0.5f, fy), 0.5f);
  int iy = (int)floorf(sy);
  float b = __fsub_rn(sy, (float)iy);
  if (iy < 0) { iy = 0; b = 0.f; }
  if (iy >= sh - 1) { iy = sh - 1; b = 0.f; }
  const int iy1 = min(iy + 1, sh - 1);
  const uint8_t* ra = s + (size_t)iy * sw * c;
  const uint8_t* rb = s + (size_t)iy1 * sw * c;
  uint8_t* o = dst + ((size_t)img * dh * dw + pix) * c;
  const float a1 = __fsub_rn(1.f, a), b1 = __fsub_rn(1.f, b);
  for (int k = 0; k < c; ++k) {
    const float t = __fadd_rn(__fmul_rn((float)ra[ix * c + k], a1), __fmul_rn((float)ra[ix1 * c + k], a));
    const float u = __fadd_rn(__fmul_rn((float)rb[ix * c + k], a1), __fmul_rn((float)rb[ix1 * c + k], a));
    const float v = __fadd_rn(__fmul_rn(t, b1), __fmul_rn(u, b));
    const uint8_t q = (uint8_t)fminf(255.f, fmaxf(0.f, rintf(v)));
    o[k] = binarize ? (uint8_t)(q > 0) : q;
  }
}
}  // namespace

int resize_batch(const uint8_t* src, const int64_t* offs, const int* dims, uint8_t* dst, int n, int dh, int dw, int c,
                 int binarize, hipStream_t st) {
  if (n <= 0) return 0;
  if (c < 1 || c > 4 || dh < 1 || dw < 1) return 1;
  dim3 grid((dh * dw + 255) / 256, n);
  hipLaunchKernelGGL(resize_batch_kernel, grid, dim3(256), 0, st, src, offs, dims, dst, dh, dw, c, binarize);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_datagen(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_datagen(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
