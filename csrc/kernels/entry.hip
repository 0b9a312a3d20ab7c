// Entry block Conv2D(32, 3, strides=2, padding="same") on the 3-channel image (client_fit_model.py:100).
// K = 27 is too small for an MFMA tile, so this is a direct VALU kernel that reads the uint8 dataset rows of the
// batch through the index vector (batch assembly and the /255 normalisation of client_fit_model.py:43 are folded
// into the load - no batch tensor is ever materialised). TF "same" at stride 2 pads bottom/right only.
// Forward writes bf16 y + BN batch statistics (replica rows); wgrad accumulates dW (3,3,3,Cout) in fp32.
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

// thread = (output pixel, 8-channel group); grid-stride; stats reduced in registers then per block
__global__ __launch_bounds__(NT) void entry_fwd_kernel(EntryParams p) {
  __shared__ float sw[27 * 64];
  __shared__ float red[2][NT / 64][64];
  const int G = p.Cout / 8;
  for (int i = threadIdx.x; i < 27 * p.Cout; i += NT) sw[i] = p.w[i];
  __syncthreads();
  const int cg = threadIdx.x % G;
  const int c0 = cg * 8;
  const int64_t npix = (int64_t)p.B * p.Ho * p.Wo;
  const int lanes = NT / G;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float bias[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias[j] = p.bias[c0 + j];
  const float inv = 1.f / 255.f;
  for (int64_t pix = (int64_t)blockIdx.x * lanes + threadIdx.x / G; pix < npix; pix += (int64_t)gridDim.x * lanes) {
    const int ow = (int)(pix % p.Wo), oh = (int)((pix / p.Wo) % p.Ho);
    const int b = (int)(pix / ((int64_t)p.Wo * p.Ho));
    const uint8_t* img = p.images + (int64_t)p.idx[b] * p.S * p.S * 3;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = bias[j];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int ih = oh * 2 + ky;
      if (ih >= p.S) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iw = ow * 2 + kx;
        if (iw >= p.S) continue;
        const uint8_t* px = img + ((int64_t)ih * p.S + iw) * 3;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) {
          const float xv = px[ci] * inv;
          const float* wr = sw + ((ky * 3 + kx) * 3 + ci) * p.Cout + c0;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv, wr[j], acc[j]);
        }
      }
    }
    const uint4 v = pack8(acc);
    *reinterpret_cast<uint4*>(p.y + pix * p.Cout + c0) = v;
    float f[8];
    unpack8(v, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += f[j];
      s2[j] += f[j] * f[j];
    }
  }
  if (!p.stats) return;
  // reduce over the pixel lanes of this wave that share the channel group (lane stride G), then over waves
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    for (int o = G; o < 64; o <<= 1) {
      s[j] += __shfl_xor(s[j], o, 64);
      s2[j] += __shfl_xor(s2[j], o, 64);
    }
  }
  if (lane < G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][wid][c0 + j] = s[j];
      red[1][wid][c0 + j] = s2[j];
    }
  }
  __syncthreads();
  float* rep = p.stats + (size_t)(blockIdx.x % STAT_REPLICAS) * 2 * p.Cout;
  for (int e = threadIdx.x; e < 2 * p.Cout; e += NT) {
    const int st = e / p.Cout, c = e - st * p.Cout;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) v += red[st][w][c];
    atomicAdd(&rep[st * p.Cout + c], v);
  }
}

// dW[ky][kx][ci][co] = sum_pix x[2oh+ky][2ow+kx][ci] * dy[pix][co]
// thread = (pixel lane, channel group, ky): 9 taps(kx,ci) x 8 channels = 72 accumulators
__global__ __launch_bounds__(NT) void entry_wgrad_kernel(EntryParams p, int64_t pix_per_block) {
  __shared__ float red[NT][9];
  const int G = p.Cout / 8;
  const int per_pix = G * 3;
  const int lanes = NT / per_pix;
  const int t = threadIdx.x;
  const bool active = t < lanes * per_pix;
  const int pl = t / per_pix, r = t % per_pix;
  const int cg = r % G, ky = r / G;
  const int c0 = cg * 8;
  const int64_t npix = (int64_t)p.B * p.Ho * p.Wo;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_block;
  const int64_t p1 = p0 + pix_per_block < npix ? p0 + pix_per_block : npix;
  float acc[9][8];
#pragma unroll
  for (int a = 0; a < 9; ++a)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[a][j] = 0.f;
  const float inv = 1.f / 255.f;
  if (active) {
    for (int64_t pix = p0 + pl; pix < p1; pix += lanes) {
      const int ow = (int)(pix % p.Wo), oh = (int)((pix / p.Wo) % p.Ho);
      const int b = (int)(pix / ((int64_t)p.Wo * p.Ho));
      const int ih = oh * 2 + ky;
      if (ih >= p.S) continue;
      float g[8];
      unpack8(*reinterpret_cast<const uint4*>(p.dy + pix * p.Cout + c0), g);
      const uint8_t* row = p.images + (int64_t)p.idx[b] * p.S * p.S * 3 + (int64_t)ih * p.S * 3;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int iw = ow * 2 + kx;
        if (iw >= p.S) continue;
#pragma unroll
        for (int ci = 0; ci < 3; ++ci) {
          const float xv = row[iw * 3 + ci] * inv;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[kx * 3 + ci][j] = fmaf(xv, g[j], acc[kx * 3 + ci][j]);
        }
      }
    }
  }
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int a = 0; a < 9; ++a) red[t][a] = active ? acc[a][j] : 0.f;
    __syncthreads();
    for (int e = t; e < per_pix * 9; e += NT) {
      const int rr = e % per_pix, a = e / per_pix;
      const int ecg = rr % G, eky = rr / G;
      float sum = 0.f;
      for (int l = 0; l < lanes; ++l) sum += red[l * per_pix + rr][a];
      const int kx = a / 3, ci = a % 3;
      atomicAdd(&p.dw[((eky * 3 + kx) * 3 + ci) * p.Cout + ecg * 8 + j], sum);
    }
    __syncthreads();
  }
}

}  // namespace

int entry_fwd(const EntryParams& p, hipStream_t st) {
  if (p.Cout % 8 || p.Cout > 64) return 1;
  const int G = p.Cout / 8;
  const int64_t npix = (int64_t)p.B * p.Ho * p.Wo;
  int64_t blocks = (npix + (NT / G) - 1) / (NT / G);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(entry_fwd_kernel, dim3((int)blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int entry_wgrad(const EntryParams& p, hipStream_t st) {
  if (p.Cout % 8 || p.Cout / 8 * 3 > NT) return 1;
  const int64_t npix = (int64_t)p.B * p.Ho * p.Wo;
  int blocks = 512;
  int64_t per = (npix + blocks - 1) / blocks;
  if (per < 64) per = 64;
  blocks = (int)((npix + per - 1) / per);
  hipLaunchKernelGGL(entry_wgrad_kernel, dim3(blocks), dim3(NT), 0, st, p, per);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
