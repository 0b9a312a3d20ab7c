// Entry block Conv2D(32, 3, strides=2, padding="same") on the 3-channel image (client_fit_model.py:100).
// K = 27 is too small for an MFMA tile, so this is a direct VALU kernel that reads the uint8 dataset rows of the
// batch through the index vector (batch assembly and the /255 normalisation of client_fit_model.py:43 are folded
// into the load - no batch tensor is ever materialised). TF "same" at stride 2 pads bottom/right only.
// Forward writes bf16 y + BN batch statistics (replica rows); wgrad accumulates dW (3,3,3,Cout) in fp32.
// Blocks walk whole output rows (32-bit indices, shifts); the row's input pixels are staged in LDS with word loads.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

// Stage input rows ih0 .. ih0+nr-1 of image `img` (uint8 HWC) into LDS as normalised floats; rows past the bottom
// edge (TF "same" stride-2 bottom pad) are zeros. Word-wide loads: S*3 bytes per row is a multiple of 4 (S % 4 == 0).
CFL_DEVICE void stage_rows(const uint8_t* img, int S, int ih0, int nr, float* srow) {
  const int words = S * 3 / 4;
  for (int e = threadIdx.x; e < nr * words; e += NT) {
    const int r = e / words, wd = e - r * words;
    const int ih = ih0 + r;
    uint32_t v = 0;
    if (ih < S) v = reinterpret_cast<const uint32_t*>(img + (size_t)ih * S * 3)[wd];
    float* d = srow + r * S * 3 + wd * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = (float)((v >> (8 * q)) & 0xffu) * (1.f / 255.f);
  }
}

__global__ __launch_bounds__(NT) void entry_fwd_kernel(EntryParams p) {
  extern __shared__ float srow[];            // [3][S*3] normalised input rows of this output row
  __shared__ float sw[27 * 64];
  __shared__ float red[2][4][256];
  const int G = p.Cout >> 3, lg = ilog2(G);
  for (int i = threadIdx.x; i < 27 * p.Cout; i += NT) sw[i] = p.w[i];
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  float bias[8];
  load_f8(p.bias + c0, bias);
  float s[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[0][j] = s[1][j] = 0.f;
  const int rows = p.B * p.Ho, items = p.Wo << lg, S3 = p.S * 3;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int b = row / p.Ho, oh = row - b * p.Ho;
    __syncthreads();                          // previous row's readers are done
    stage_rows(p.images + (size_t)p.idx[b] * p.S * S3, p.S, 2 * oh, 3, srow);
    __syncthreads();
    for (int it = threadIdx.x; it < items; it += NT) {
      const int ow = it >> lg;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = bias[j];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          const int iw = ow * 2 + kx;
          if (iw >= p.S) continue;
          const float* px = srow + ky * S3 + iw * 3;
#pragma unroll
          for (int ci = 0; ci < 3; ++ci) {
            const float xv = px[ci];
            const float* wr = sw + ((ky * 3 + kx) * 3 + ci) * p.Cout + c0;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv, wr[j], acc[j]);
          }
        }
      }
      const uint4 v = pack8(acc);
      *reinterpret_cast<uint4*>(p.y + ((size_t)row * p.Wo + ow) * p.Cout + c0) = v;
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[0][j] += f[j];
        s[1][j] += f[j] * f[j];
      }
    }
  }
  if (p.stats) block_channel_atomics<2>(s, G, p.Cout, p.stats + (size_t)(blockIdx.x % STAT_REPLICAS) * 2 * p.Cout, red);
}

// dW[ky][kx][ci][co] = sum_pix x[2oh+ky][2ow+kx][ci] * dy[pix][co]; blockIdx.y = ky, thread = (pixel, 8 outputs).
// The input row is staged in LDS once per output row; per-block sums go to one of `replicas` copies of dW.
__global__ __launch_bounds__(NT) void entry_wgrad_kernel(EntryParams p, int replicas) {
  extern __shared__ float srow[];            // [S*3] normalised input row 2*oh + ky
  __shared__ float red[4][9][64];
  const int G = p.Cout >> 3, lg = ilog2(G);
  const int c0 = (threadIdx.x & (G - 1)) * 8;
  const int ky = blockIdx.y;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float acc[9][8];
#pragma unroll
  for (int a = 0; a < 9; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;
  const int rows = p.B * p.Ho, items = p.Wo << lg, S3 = p.S * 3;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int b = row / p.Ho, oh = row - b * p.Ho;
    const int ih = oh * 2 + ky;
    if (ih >= p.S) continue;                  // uniform per block
    __syncthreads();
    stage_rows(p.images + (size_t)p.idx[b] * p.S * S3, p.S, ih, 1, srow);
    __syncthreads();
    for (int it = threadIdx.x; it < items; it += NT) {
      const int ow = it >> lg;
      float g[8];
      load8(p.dy + ((size_t)row * p.Wo + ow) * p.Cout + c0, g);
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iw = ow * 2 + kx;
        if (iw >= p.S) continue;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) {
          const float xv = srow[iw * 3 + ci];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[kx * 3 + ci][j] = fmaf(xv, g[j], acc[kx * 3 + ci][j]);
        }
      }
    }
  }
#pragma unroll
  for (int a = 0; a < 9; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[a][j];
      for (int o = G; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      acc[a][j] = v;
    }
  if (lane < G) {
#pragma unroll
    for (int a = 0; a < 9; ++a)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][a][c0 + j] = acc[a][j];
  }
  __syncthreads();
  float* dst = p.dw + (size_t)((blockIdx.x + blockIdx.y * gridDim.x) % replicas) * 27 * p.Cout;
  for (int e = threadIdx.x; e < 9 * p.Cout; e += NT) {
    const int a = e / p.Cout, c = e - a * p.Cout;
    atomicAdd(&dst[(ky * 9 + a) * p.Cout + c], red[0][a][c] + red[1][a][c] + red[2][a][c] + red[3][a][c]);
  }
}

bool pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }

}  // namespace

int entry_fwd(const EntryParams& p, hipStream_t st) {
  if (p.Cout % 8 || p.Cout > 64 || !pow2(p.Cout / 8)) return 1;
  const int rows = p.B * p.Ho;
  if (p.S % 4) return 1;
  const size_t lds = (size_t)3 * p.S * 3 * sizeof(float);
  if (lds > 48 * 1024) return 1;
  const int cap = cfl_tune(TUNE_ENTRY_FWD_BLOCKS) > 0 ? cfl_tune(TUNE_ENTRY_FWD_BLOCKS) : 1024;
  hipLaunchKernelGGL(entry_fwd_kernel, dim3(rows < cap ? rows : cap), dim3(NT), lds, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int entry_wgrad(const EntryParams& p, hipStream_t st) {
  if (p.Cout % 8 || p.Cout > 64 || !pow2(p.Cout / 8)) return 1;
  const int rows = p.B * p.Ho;
  if (p.S % 4) return 1;
  const int cap = cfl_tune(TUNE_ENTRY_WGRAD_BLOCKS) > 0 ? cfl_tune(TUNE_ENTRY_WGRAD_BLOCKS) : 256;   // measured
  const int reps = p.replicas > 1 ? p.replicas : 1;
  hipLaunchKernelGGL(entry_wgrad_kernel, dim3(rows < cap ? rows : cap, 3), dim3(NT), (size_t)p.S * 3 * sizeof(float),
                     st, p, reps);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
