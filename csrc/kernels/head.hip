// Segmentation head + loss: Conv2D(1, 1x1, activation="sigmoid") then binary_crossentropy / accuracy
// (client_fit_model.py:145,157). TF2 Keras evaluates BCE on a Sigmoid output from the logits
// (sigmoid_cross_entropy_with_logits), mean over all B*S*S pixels; accuracy = binary_accuracy at 0.5.
//
// The decoder's last UpSampling2D commutes with the 1x1 head, so logits are computed once per LOW-resolution
// pixel (R x R) and each covers a 2x2 block of the S x S target mask (S = 2R), read straight from the uint8
// dataset through the batch index vector. Optional Dice term (north-star "Dice/BCE loss").
//   head_fwd: h = x . w + b; accumulates bce, correct pixels and the Dice sums (I, P, T)
//   head_bwd: dh = sum_children (sigmoid(h) - t) / (B*S*S) [+ Dice grad]; dx = dh * w; dw, db reductions
// Four lanes per low-resolution pixel: lane q = tid & 3 owns channels 8q .. 8q+7 (one 16-byte load; the partial dot
// products meet through two lane shuffles) and target sub-pixel (q >> 1, q & 1) of the pixel's 2x2 block, so a
// wave's activation loads / stores are 1 KiB contiguous and the loss terms spread over every lane (one pixel per
// thread with a 64-byte row each left the head latency-bound).
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;
constexpr float DICE_SMOOTH = 1.0f;
// grid cap: every block ends with same-address atomics (7 doubles fwd, 33 floats bwd) that serialise at the memory
// side - 1024 blocks: 19.9 / 19.4 us, 512: 15.0 / 13.7 us, 256: 17.1 / 13.4 us (fwd / bwd, bench shape). A per-block
// slot + last-block reduction needs device-scope release/acquire fences (an L2 writeback / invalidate per block on
// the multi-XCD part) and measured 84 / 153 us.
constexpr int HEAD_BLOCKS = 512;
constexpr int HPT = 4;            // pixels per lane per trip (all loads of a trip in flight together)

// target bit of sub-pixel (q >> 1, q & 1) of low-resolution pixel pix, through the batch index vector
CFL_DEVICE float mask_at(const HeadParams& p, int pix, int S, int q) {
  const int j = pix % p.R, i = (pix / p.R) % p.R;
  const int b = pix / (p.R * p.R);
  return p.masks[(int64_t)p.idx[b] * S * S + (2 * i + (q >> 1)) * S + 2 * j + (q & 1)] ? 1.f : 0.f;
}

// metrics layout (double): [0] bce sum, [1] correct, [2] pixels, [3] dice loss sum, [4] I, [5] P, [6] T (soft, this
// step), [7] TP (predicted AND true crack pixels), [8] PP (predicted crack pixels) - hard-threshold IoU / Dice

template <int CIN>
__global__ __launch_bounds__(NT) void head_fwd_kernel(HeadParams p) {
  CFL_TS_GUARD;
  static_assert(CIN == 32, "4 lanes x 8 channels per pixel");
  __shared__ double red[7][NT / 64];
  const int npix = p.B * p.R * p.R;
  const int S = 2 * p.R;
  const int q = threadIdx.x & 3;
  float w[8];
  load_f8(p.w + 8 * q, w);
  const float bias = p.bias[0];
  double bce = 0, cor = 0, I = 0, P = 0, T = 0, TP = 0, PP = 0;
  // the grid stride is a multiple of 4: the 4 lanes of a pixel take every trip together (shuffles below); each
  // trip issues all HPT items' loads (activations, batch index -> mask byte) before any math
  const int stride = gridDim.x * NT;
  for (int t0 = blockIdx.x * NT + threadIdx.x; (t0 >> 2) < npix; t0 += HPT * stride) {
    float f[HPT][8], tt[HPT];
    int pix[HPT];
#pragma unroll
    for (int u = 0; u < HPT; ++u) {
      const int t = t0 + u * stride;
      pix[u] = (t >> 2) < npix ? t >> 2 : -1;
      const int pc = pix[u] < 0 ? 0 : pix[u];
      load8(p.x + (size_t)pc * CIN + 8 * q, f[u]);
      tt[u] = mask_at(p, pc, S, q);
    }
#pragma unroll
    for (int u = 0; u < HPT; ++u) {
      float h = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) h = fmaf(f[u][k], w[k], h);
      h = xor_add(h, 1);        // commutative pairings: all 4 lanes end with the same bits
      h = xor_add(h, 2);
      h += bias;
      if (pix[u] < 0) continue;
      if (q == 0) p.h[pix[u]] = h;
      const float sp = fmaxf(h, 0.f) + log1pf(expf(-fabsf(h)));   // softplus(h) = BCE for t = 0
      const float sg = 1.f / (1.f + expf(-h));
      bce += sp - h * tt[u];
      cor += ((h > 0.f) == (tt[u] > 0.5f)) ? 1.0 : 0.0;
      TP += (h > 0.f && tt[u] > 0.5f) ? 1.0 : 0.0;
      PP += h > 0.f ? 1.0 : 0.0;
      I += sg * tt[u];
      P += sg;
      T += tt[u];
    }
  }
  double v[7] = {bce, cor, I, P, T, TP, PP};
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    double x = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = xor_add(x, o);
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

// NODE: dx is also the gradient of the decoder's last BN node (x_lo = BN_B(c2) + q, no ReLU): its BN-backward sums
// sum(g), sum(g * xhat) are accumulated here from the stored bf16 dx (what a separate node_bwd pass would read back)
// FWD (training step without the Dice term, whose gradient needs the whole batch's sums first): the forward is done
// in the same pass - the logit is formed from the x row this kernel loads anyway (the same arithmetic as
// head_fwd_kernel, so the same bits), the loss / accuracy sums accumulate here, and x is read once per step instead
// of twice (one launch and a 16.8 MB read fewer at the bench shape)
template <int CIN, bool NODE, bool FWD>
__global__ __launch_bounds__(NT) void head_bwd_kernel(HeadParams p) {
  CFL_TS_GUARD;
  static_assert(CIN == 32, "4 lanes x 8 channels per pixel");
  __shared__ float red[CIN + 1][NT / 64];
  __shared__ float nred[NODE ? 2 * CIN : 1][NT / 64];
  __shared__ double mred[FWD ? 7 : 1][NT / 64];
  const int npix = p.B * p.R * p.R;
  const int S = 2 * p.R;
  const int q = threadIdx.x & 3;
  const float inv_n = 1.f / (float)(npix * 4);
  float dI = 0.f, dP = 0.f, den = 1.f;
  if (p.dice) {
    const float I = (float)p.metrics[4], P = (float)p.metrics[5], T = (float)p.metrics[6];
    den = P + T + DICE_SMOOTH;
    dI = -2.f / den;                                   // d/dI of -(2I+s)/den
    dP = (2.f * I + DICE_SMOOTH) / (den * den);        // d/dP (and d/dT)
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&p.metrics[3], (double)(1.f - (2.f * I + DICE_SMOOTH) / den));
  }
  float w[8], gw[8];
  load_f8(p.w + 8 * q, w);
#pragma unroll
  for (int k = 0; k < 8; ++k) gw[k] = 0.f;
  float gb = 0.f;
  const float bias = FWD ? p.bias[0] : 0.f;
  double bce = 0, cor = 0, mI = 0, mP = 0, mT = 0, TP = 0, PP = 0;
  float nmean[8], nrstd[8], ns0[8], ns1[8];
  load_f8_or(p.node.ab + 2 * CIN + 8 * q, NODE, 0.f, nmean);
  load_f8_or(p.node.ab + 3 * CIN + 8 * q, NODE, 0.f, nrstd);
#pragma unroll
  for (int k = 0; k < 8; ++k) ns0[k] = ns1[k] = 0.f;
  const int stride = gridDim.x * NT;
  cfl_ts_phase(0);
  for (int t0 = blockIdx.x * NT + threadIdx.x; (t0 >> 2) < npix; t0 += HPT * stride) {
    float f[HPT][8], hv[HPT], tt[HPT], yn[NODE ? HPT : 1][8];
    int pix[HPT];
#pragma unroll
    for (int u = 0; u < HPT; ++u) {     // all loads first (see head_fwd_kernel)
      const int t = t0 + u * stride;
      pix[u] = (t >> 2) < npix ? t >> 2 : -1;
      const int pc = pix[u] < 0 ? 0 : pix[u];
      if constexpr (!FWD) hv[u] = p.h[pc];
      load8(p.x + (size_t)pc * CIN + 8 * q, f[u]);
      if constexpr (NODE) load8(p.node.y + (size_t)pc * CIN + 8 * q, yn[u]);
      tt[u] = mask_at(p, pc, S, q);
    }
    if constexpr (FWD) {
#pragma unroll
      for (int u = 0; u < HPT; ++u) {
        float h = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) h = fmaf(f[u][k], w[k], h);
        h = xor_add(h, 1);
        h = xor_add(h, 2);
        h += bias;
        hv[u] = h;
        if (pix[u] < 0) continue;
        if (q == 0) p.h[pix[u]] = h;
        const float sp = fmaxf(h, 0.f) + log1pf(expf(-fabsf(h)));
        const float sg = 1.f / (1.f + expf(-h));
        bce += sp - h * tt[u];
        cor += ((h > 0.f) == (tt[u] > 0.5f)) ? 1.0 : 0.0;
        TP += (h > 0.f && tt[u] > 0.5f) ? 1.0 : 0.0;
        PP += h > 0.f ? 1.0 : 0.0;
        mI += sg * tt[u];
        mP += sg;
        mT += tt[u];
      }
    }
#pragma unroll
    for (int u = 0; u < HPT; ++u) {
      const float sg = 1.f / (1.f + expf(-hv[u]));
      float dh = (sg - tt[u]) * inv_n;
      if (p.dice) dh += (dI * tt[u] + dP) * sg * (1.f - sg);
      dh = xor_add(dh, 1);      // the pixel's gradient: sum over its 2x2 target block
      dh = xor_add(dh, 2);
      if (pix[u] < 0) continue;
      if (q == 0) gb += dh;
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = dh * w[k];
        gw[k] = fmaf(dh, f[u][k], gw[k]);
      }
      const uint4 ov = pack8(o);
      *reinterpret_cast<uint4*>(p.dx + (size_t)pix[u] * CIN + 8 * q) = ov;
      if constexpr (NODE) {
        float g[8];
        unpack8(ov, g);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          ns0[k] += g[k];
          ns1[k] += g[k] * (yn[u][k] - nmean[k]) * nrstd[k];
        }
      }
    }
  }
  cfl_ts_phase(1);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if constexpr (FWD) {
    double v[7] = {bce, cor, mI, mP, mT, TP, PP};
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      double x = v[k];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) x = xor_add(x, o);
      if (lane == 0) mred[k][wid] = x;
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int o = 4; o < 64; o <<= 1) gw[k] = xor_add(gw[k], o);   // lanes of one q hold the same channels
  gb = wave_sum(gb);
  if (lane < 4) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[8 * lane + k][wid] = gw[k];
  }
  if (lane == 0) red[CIN][wid] = gb;
  if constexpr (NODE) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) {
        ns0[k] = xor_add(ns0[k], o);
        ns1[k] = xor_add(ns1[k], o);
      }
    if (lane < 4) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        nred[8 * lane + k][wid] = ns0[k];
        nred[CIN + 8 * lane + k][wid] = ns1[k];
      }
    }
  }
  __syncthreads();
  if constexpr (NODE) {
    const int reps = p.node.reps > 1 ? p.node.reps : 1;
    const size_t ro = (size_t)(blockIdx.x % reps) * 2 * CIN;
    if (threadIdx.x < 2 * CIN) {
      float s = 0.f;
      for (int w2 = 0; w2 < NT / 64; ++w2) s += nred[threadIdx.x][w2];
      red_add(p.node.sums, ro + threadIdx.x, s, CFL_FX_G);
    }
  }
  if (threadIdx.x <= CIN) {
    float s = 0.f;
    for (int w2 = 0; w2 < NT / 64; ++w2) s += red[threadIdx.x][w2];
    if (cfl_det()) red_add(p.dwfx, threadIdx.x, s, CFL_FX_G);   // int64 [Cin + 1]; grad_finish GF_FIXED converts
    else if (threadIdx.x < CIN) atomicAdd(&p.dw[threadIdx.x], s);
    else atomicAdd(p.db, s);
  }
  if constexpr (FWD) {
    const int k = threadIdx.x - 64;                    // a wave that did not take part in the atomics above
    if (k >= 0 && k < 7) {
      double s = 0;
      for (int w2 = 0; w2 < NT / 64; ++w2) s += mred[k][w2];
      atomicAdd(&p.metrics[k < 2 ? k : k + 2], s);     // 0,1 -> 0,1 ; 2..6 -> 4..8 (head_fwd_kernel layout)
    }
    if (blockIdx.x == 0 && threadIdx.x == 128) atomicAdd(&p.metrics[2], (double)npix * 4.0);
  }
}

int head_blocks(const HeadParams& p) {
  const int64_t blocks = ((int64_t)p.B * p.R * p.R * 4 + HPT * NT - 1) / (HPT * NT);
  const int cap = cfl_tune(TUNE_HEAD_BLOCKS) > 0 ? cfl_tune(TUNE_HEAD_BLOCKS) : HEAD_BLOCKS;
  return (int)(blocks > cap ? cap : (blocks < 1 ? 1 : blocks));
}

}  // namespace

int head_fwd(const HeadParams& p, hipStream_t st) {
  if (p.Cin != 32) return 1;
  hipLaunchKernelGGL(head_fwd_kernel<32>, dim3(head_blocks(p)), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int head_bwd(const HeadParams& p, hipStream_t st) {
  if (p.Cin != 32) return 1;
  if (p.fused && p.dice) return 2;                    // the Dice gradient needs the forward's whole-batch sums first
  const dim3 g(head_blocks(p));
  if (p.node.y && p.fused) hipLaunchKernelGGL((head_bwd_kernel<32, true, true>), g, dim3(NT), 0, st, p);
  else if (p.node.y) hipLaunchKernelGGL((head_bwd_kernel<32, true, false>), g, dim3(NT), 0, st, p);
  else if (p.fused) hipLaunchKernelGGL((head_bwd_kernel<32, false, true>), g, dim3(NT), 0, st, p);
  else hipLaunchKernelGGL((head_bwd_kernel<32, false, false>), g, dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_head(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_head(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
