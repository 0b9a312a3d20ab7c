// Segmentation head + loss: Conv2D(1, 1x1, activation="sigmoid") then binary_crossentropy / accuracy
// (client_fit_model.py:145,157). TF2 Keras evaluates BCE on a Sigmoid output from the logits
// (sigmoid_cross_entropy_with_logits), mean over all B*S*S pixels; accuracy = binary_accuracy at 0.5.
//
// The decoder's last UpSampling2D commutes with the 1x1 head, so logits are computed once per LOW-resolution
// pixel (R x R) and each covers a 2x2 block of the S x S target mask (S = 2R), read straight from the uint8
// dataset through the batch index vector. Optional Dice term (north-star "Dice/BCE loss").
//   head_fwd: h = x . w + b; accumulates bce, correct pixels and the Dice sums (I, P, T)
//   head_bwd: dh = sum_children (sigmoid(h) - t) / (B*S*S) [+ Dice grad]; dx = dh * w; dw, db reductions
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr float DICE_SMOOTH = 1.0f;

// metrics layout (double): [0] bce sum, [1] correct, [2] pixels, [3] dice loss sum, [4] I, [5] P, [6] T (soft, this
// step), [7] TP (predicted AND true crack pixels), [8] PP (predicted crack pixels) - hard-threshold IoU / Dice

template <int CIN>
__global__ __launch_bounds__(NT) void head_fwd_kernel(HeadParams p) {
  __shared__ double red[7][NT / 64];
  const int npix = p.B * p.R * p.R;
  const int S = 2 * p.R;
  double bce = 0, cor = 0, I = 0, P = 0, T = 0, TP = 0, PP = 0;
  for (int pix = blockIdx.x * NT + threadIdx.x; pix < npix; pix += gridDim.x * NT) {
    const int j = pix % p.R, i = (pix / p.R) % p.R;
    const int b = pix / (p.R * p.R);
    float h = p.bias[0];
#pragma unroll
    for (int c0 = 0; c0 < CIN; c0 += 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(p.x + pix * CIN + c0), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) h = fmaf(f[k], p.w[c0 + k], h);
    }
    p.h[pix] = h;
    const float sp = fmaxf(h, 0.f) + log1pf(expf(-fabsf(h)));   // softplus(h) = BCE for t = 0
    const float sg = 1.f / (1.f + expf(-h));
    const uint8_t* mrow = p.masks + (int64_t)p.idx[b] * S * S;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const float t = mrow[(2 * i + dy) * S + 2 * j + dx] ? 1.f : 0.f;
        bce += sp - h * t;
        cor += ((h > 0.f) == (t > 0.5f)) ? 1.0 : 0.0;
        TP += (h > 0.f && t > 0.5f) ? 1.0 : 0.0;
        PP += h > 0.f ? 1.0 : 0.0;
        I += sg * t;
        P += sg;
        T += t;
      }
  }
  double v[7] = {bce, cor, I, P, T, TP, PP};
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    double x = v[k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
    if (lane == 0) red[k][wid] = x;
  }
  __syncthreads();
  if (threadIdx.x < 7) {
    double s = 0;
    for (int w = 0; w < NT / 64; ++w) s += red[threadIdx.x][w];
    const int slot = threadIdx.x < 2 ? threadIdx.x : threadIdx.x + 2;   // 0,1 -> 0,1 ; 2..6 -> 4..8
    atomicAdd(&p.metrics[slot], s);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&p.metrics[2], (double)npix * 4.0);
}

template <int CIN>
__global__ __launch_bounds__(NT) void head_bwd_kernel(HeadParams p) {
  __shared__ float red[CIN + 1][NT / 64];
  const int npix = p.B * p.R * p.R;
  const int S = 2 * p.R;
  const float inv_n = 1.f / (float)(npix * 4);
  float dI = 0.f, dP = 0.f, den = 1.f;
  if (p.dice) {
    const float I = (float)p.metrics[4], P = (float)p.metrics[5], T = (float)p.metrics[6];
    den = P + T + DICE_SMOOTH;
    dI = -2.f / den;                                   // d/dI of -(2I+s)/den
    dP = (2.f * I + DICE_SMOOTH) / (den * den);        // d/dP (and d/dT)
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&p.metrics[3], (double)(1.f - (2.f * I + DICE_SMOOTH) / den));
  }
  float gw[CIN];
#pragma unroll
  for (int c = 0; c < CIN; ++c) gw[c] = 0.f;
  float gb = 0.f;
  for (int pix = blockIdx.x * NT + threadIdx.x; pix < npix; pix += gridDim.x * NT) {
    const int j = pix % p.R, i = (pix / p.R) % p.R;
    const int b = pix / (p.R * p.R);
    const float h = p.h[pix];
    const float sg = 1.f / (1.f + expf(-h));
    const uint8_t* mrow = p.masks + (int64_t)p.idx[b] * S * S;
    float dh = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const float t = mrow[(2 * i + dy) * S + 2 * j + dx] ? 1.f : 0.f;
        dh += (sg - t) * inv_n;
        if (p.dice) dh += (dI * t + dP) * sg * (1.f - sg);
      }
    gb += dh;
#pragma unroll
    for (int c0 = 0; c0 < CIN; c0 += 8) {
      float f[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(p.x + pix * CIN + c0), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = dh * p.w[c0 + k];
        gw[c0 + k] = fmaf(dh, f[k], gw[c0 + k]);
      }
      *reinterpret_cast<uint4*>(p.dx + pix * CIN + c0) = pack8(o);
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c <= CIN; ++c) {
    float x = c < CIN ? gw[c] : gb;
    x = wave_sum(x);
    if (lane == 0) red[c][wid] = x;
  }
  __syncthreads();
  if (threadIdx.x <= CIN) {
    float s = 0.f;
    for (int w = 0; w < NT / 64; ++w) s += red[threadIdx.x][w];
    if (threadIdx.x < CIN) atomicAdd(&p.dw[threadIdx.x], s);
    else atomicAdd(p.db, s);
  }
}

}  // namespace

int head_fwd(const HeadParams& p, hipStream_t st) {
  if (p.Cin != 32) return 1;
  int64_t blocks = ((int64_t)p.B * p.R * p.R + NT - 1) / NT;
  if (blocks > 512) blocks = 512;
  hipLaunchKernelGGL(head_fwd_kernel<32>, dim3((int)blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int head_bwd(const HeadParams& p, hipStream_t st) {
  if (p.Cin != 32) return 1;
  int64_t blocks = ((int64_t)p.B * p.R * p.R + NT - 1) / NT;
  if (blocks > 512) blocks = 512;
  hipLaunchKernelGGL(head_bwd_kernel<32>, dim3((int)blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}
