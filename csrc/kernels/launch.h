// Host-callable launchers of the gfx950 kernels (no torch dependency; raw device pointers + hipStream_t).
// Every launcher returns 0 on success, nonzero on an unsupported shape or a launch error.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

// BN batch statistics are accumulated into STAT_REPLICAS replica rows [rep][2][C] (sum, sum of squares) so the
// per-block atomics of thousands of workgroups do not all hit the same 2*C words; the BN's first consumer (or
// bn_finalize) sums the replicas. Whole-step A/B: 32 -> 8 replicas cost 4 us with bn_finalize launches (1.581 vs
// 1.585 ms) and make the consumer-side finalize cheap (every consumer block reads 2 * 8 values per channel); 4
// replicas measured 1.548 vs 1.521 ms for 8.
#define STAT_REPLICAS 8

// Consumer-side BatchNorm finalize: the first kernel that applies a BN layer computes the layer's coefficients
// itself from the producer's replica sums (no separate 1-block bn_finalize launch in between); the blocks that own a
// channel range also write that range's ab rows (a, b, mean, rstd) for the later consumers of the layer.
struct BnStatsIn {
  const float* stats;      // [STAT_REPLICAS][2][C] batch sums (nullptr = off: ab is already final)
  const float* gamma;
  const float* beta;
  float count;             // pixels per channel
  float eps;
};

// Coefficients of channel c from the replica sums - THE arithmetic of bn_finalize (replicas summed in order, all
// loads issued together), so a consumer-side finalize and a bn_finalize launch agree bit for bit.
// Deterministic mode (common.h): int64 fixed-point rows summed as integers (exact in any order) and converted once.
__device__ __forceinline__ bool stat_sums_det(const float* stats, int C, int c, float& s, float& s2) {
  if (!cfl_det()) return false;
  long long a = 0, b = 0;
#pragma unroll
  for (int r = 0; r < STAT_REPLICAS; ++r) {
    a += red_raw(stats, (size_t)r * 2 * C + c);
    b += red_raw(stats, (size_t)r * 2 * C + C + c);
  }
  s = red_fx(a, CFL_FX_S0);
  s2 = red_fx(b, CFL_FX_S1);
  return true;
}

__device__ __forceinline__ void bn_coef_from_stats(const BnStatsIn& f, int C, int c, float& a, float& b, float& mean,
                                                   float& rstd) {
  float s = 0.f, s2 = 0.f;
  if (!stat_sums_det(f.stats, C, c, s, s2)) {
    float v0[STAT_REPLICAS], v1[STAT_REPLICAS];
#pragma unroll
    for (int r = 0; r < STAT_REPLICAS; ++r) {
      v0[r] = f.stats[r * 2 * C + c];
      v1[r] = f.stats[r * 2 * C + C + c];
    }
#pragma unroll
    for (int r = 0; r < STAT_REPLICAS; ++r) {
      s += v0[r];
      s2 += v1[r];
    }
  }
  mean = s / f.count;
  const float var = fmaxf(s2 / f.count - mean * mean, 0.f);
  rstd = rsqrtf(var + f.eps);
  a = f.gamma[c] * rstd;
  b = f.beta[c] - mean * a;
}

// ---------------------------------------------------------------- implicit-GEMM conv (conv_igemm.hip)
// BN-node gradient epilogue (backward). The kernel's output o is the incoming gradient of a BatchNorm node whose
// forward input was `y` (ab rows: a, b, mean, rstd). Instead of o the kernel writes the node gradient
// g = (relu ? [a*y + b > 0] : 1) * o (bf16) and accumulates sum(g), sum(g * xhat), xhat = (y - mean) * rstd, into
// replica rows sums[reps][2][C] - i.e. node_bwd fused into the producer's epilogue (one pass fewer).
struct BnNodeEpi {
  const bf16_t* y;     // nullptr = off
  const float* ab;
  float* sums;
  int reps;
  int relu;
};

// Fused residual join in the epilogue of a forward 1x1 residual conv (its output r never goes to memory):
//   JOIN_POOL   out[m] = maxpool3x3s2_same(a*y + b)[m] + r[m], argmax recorded   (encoder, replaces pool_res_fwd)
//   JOIN_ADD    out[m] = a*y[m] + b + r[m]                                        (decoder level 0, bn_add_fwd)
//   JOIN_ADD_UP out[p] = a*y[p] + b + r[p/2] for the 4 pixels p of each conv pixel (decoder, bn_add_fwd q_up)
// y: the BN input at resolution H x W; ab: its BN coefficients (C = N rows).
enum { JOIN_NONE = 0, JOIN_POOL = 1, JOIN_ADD = 2, JOIN_ADD_UP = 3 };
struct ConvJoin {
  int mode;
  const bf16_t* y;
  const float* ab;
  bf16_t* out;
  uint8_t* argmax;         // JOIN_POOL only
  int H, W;
  BnStatsIn fin;           // consumer-side finalize of y's BN (ab computed here and its rows written), or off
};

// Decoder node join in a 3x3 data-gradient conv's epilogue (backward of x_lo_{k-1} -> UpSampling2D -> ReLU ->
// Conv2DTranspose, plus the residual conv's input gradient): the conv output o (full resolution, the gradient of
// the upsampled input) is never stored; instead, at half resolution,
//   out[h][w] = [v[h][w] > 0] * sum_{2x2} o[2h+dy][2w+dx] + add[h][w]
// and, if sums != nullptr, the BN-backward sums of the BN node out is also the gradient of (sum g, sum g * xhat,
// xhat from sy with the sab rows) - node_bwd(GM_SUM2X2 masked, GM_SAME, sy / sab) in the producer.
struct PoolJoinEpi {
  const bf16_t* v;     // nullptr = off: ReLU-mask source [B, Ho/2, Wo/2, N] (the conv's raw input)
  const bf16_t* add;   // addend [B, Ho/2, Wo/2, N] or nullptr
  bf16_t* out;         // [B, Ho/2, Wo/2, N]
  const bf16_t* sy;    // BN input for the sums' xhat (same layout) or nullptr (no sums)
  const float* sab;    // its BN rows (mean, rstd at rows 2, 3)
  float* sums;         // [reps][2][N]
  int reps;
};

struct GradSrc {
  const bf16_t* p;
  int mode;
  int mask;                // multiply this source by [v > 0]
};
struct NodeBwdParams {
  GradSrc src[2];
  const uint8_t* argmax;   // GM_MAXPOOL: [B, ceil(H/2), ceil(W/2), C] in 0..8
  const bf16_t* v;         // node value source: raw y (BN node: v = a*y+b) or plain x
  const float* ab;         // BN coefficients (4 rows) or nullptr for a plain node
  int relu_node;           // mask the total by [v > 0]
  bf16_t* out;             // gradient w.r.t. the BN output (BN node) or w.r.t. x (plain node)
  float* sums;             // [sum_reps][2][C]: sum g, sum g*xhat (BN node) / [sum_reps][C] sum g (plain) / nullptr
  const bf16_t* sy;        // optional: xhat for the sums from THIS tensor + sab (mean, rstd rows) instead of v / ab -
  const float* sab;        //   the gradient of a plain node that is also the (unmasked) gradient of a BN node
  int B, H, W, C;
  int sum_reps;            // replica rows of sums (block b adds into row b % sum_reps); <= 1: one row
};
struct BnBwdApplyParams {
  const bf16_t* g;         // gradient w.r.t. BN output (masked)
  const bf16_t* y;         // raw BN input
  const float* ab;         // 4 rows: a, b, mean, rstd
  const float* sums;       // [sum_reps][2][C] (node_bwd replica rows, summed here)
  bf16_t* dy;              // gradient w.r.t. y
  float* dgamma;           // flat-grad slots (written, not accumulated) or nullptr
  float* dbeta;
  int M, C;
  int sum_reps;
};
// A streaming BN-backward pass run as the "side job" of a streaming 1x1 data gradient (pw.hip) that reads the same
// incoming gradient and does not depend on it: its blocks are interleaved with the conv's in ONE launch (two
// latency-bound passes co-run instead of back to back). kind 0 = none; shapes pw.hip does not take run it first,
// alone (conv_igemm).
enum SideKind { SIDE_NONE = 0, SIDE_BBA = 1, SIDE_POOL = 2 };
struct SideJob {
  int kind;
  BnBwdApplyParams bba;    // SIDE_BBA: bn_bwd_apply
  NodeBwdParams pool;      // SIDE_POOL: node_bwd routed through the max-pool (node_pool_eligible)
};

struct ConvParams {
  const bf16_t* x;     // [B, Hin, Win, Cin] NHWC (physical; logical = upsample2 if up_in)
  const bf16_t* wt;    // [N][K] packed bf16 weights, K = ks*ks*Cin, k = (ky*ks + kx)*Cin + ci
  const float* bias;   // [N] or nullptr
  bf16_t* y;           // [B, Ho, Wo, N]
  float* stats;        // [STAT_REPLICAS][2][N] (sum, sum of squares), atomically accumulated, or nullptr
  InXform xf;          // transform applied to x on load
  int B, Hin, Win, Cin, up_in;
  int Ho, Wo, N, ks, stride, pad_t, pad_l;
  int M, K;
  float* ws;           // split-K fp32 workspace (nullptr: no split)
  int64_t ws_elems;
  int algo;            // 0 auto (3x3/s1 -> halo-tile conv3x3.hip, else generic), 1 generic only, 2 conv3x3 only
  BnNodeEpi node;      // optional BN-node gradient epilogue (dgrad producers); excludes stats / bias
  PoolJoinEpi pj;      // optional decoder node join (3x3 s1 dgrads, even tiles); excludes stats / bias / node / split
  BnStatsIn xfin;      // optional consumer-side finalize of xf's BN (xf.ab computed here from the sums, rows written)
  ConvJoin join;       // optional residual join (forward 1x1 residual convs); excludes stats / node / split-K
  BnBwdIn bwd;         // optional BN-backward apply folded into the operand load (x = the BN node gradient g;
                       // common.h). Data-gradient convs only: 1x1/s1 or 3x3/s1, no upsample, no xf; shapes a kernel
                       // does not fold fall back to bn_bwd_apply into bwd.dx + the plain conv (same results)
  SideJob side;        // optional independent streaming pass co-launched with a streaming 1x1 conv (pw.hip)
  const bf16_t* sum2x2;  // optional: x = the 2x2-block sums of this [B, 2*Hin, 2*Win, Cin] gradient (node_bwd
                         // GM_SUM2X2 order), formed on load by the streaming 1x1 kernel and stored into x (const cast)
                         // for the weight gradient; other kernels run node_bwd into x first (same results)
  const uint8_t* wt8;    // optional fp8 operands of a 3x3 conv (fp8.hip): e4m3 weights [N][K] (quant_w8 of wt) ...
  const uint8_t* ws8;    // ... and their e8m0 block scales [N][K / 32]; the activations are quantised on load
};
bool conv3x3_f8_supported(const ConvParams& p);
int conv3x3_f8(const ConvParams& p, hipStream_t st);
int quant_w8(const bf16_t* const* src, uint8_t* const* dst, uint8_t* const* sc, const int* nblk, int n, hipStream_t st);
int conv_igemm(const ConvParams& p, hipStream_t st);
// plain 1x1 / stride-1 convs (no input transform, epilogue = bias + optional BN statistics; input optionally formed
// on load: bwd = BN-backward apply, sum2x2 = 2x2-block sums): streaming MFMA kernel with swapped operands and resident
// weights (pw.hip); conv_igemm routes them there unless TUNE_PW = 1
bool pw_conv_supported(const ConvParams& p);
int pw_conv(const ConvParams& p, hipStream_t st);
int conv_igemm_splits(const ConvParams& p);   // K splits the launcher would use (workspace = splits*M*N floats)
int conv3x3_splits(const ConvParams& p);
int conv3x3_split_k(const ConvParams& p);     // K splits of the standard 8x16 / 16x8 tiles
int splitk_epilogue(const ConvParams& p, int splits, hipStream_t st);   // sum partials + bias/stats/node epilogue



// ---------------------------------------------------------------- weight gradient (conv_wgrad.hip)
struct WgradParams {
  const bf16_t* x;     // conv input (as in ConvParams)
  const bf16_t* dy;    // [M][N] gradient w.r.t. the conv output
  float* dw;           // fp32 destination (atomic accumulate)
  InXform xf;
  int B, Hin, Win, Cin, up_in;
  int Ho, Wo, N, ks, stride, pad_t, pad_l;
  int M, K;
  int dst_mode;        // 0: dw[k*N + n] (Keras HWIO / pointwise layout)   1: Conv2DTranspose (kh,kw,out,in) flip
  int m_chunk;         // pixels per block along M (multiple of 32), 0 = auto
  int algo;            // 0 auto (3x3/s1 -> halo wgrad conv3x3_wgrad.hip, else generic), 1 generic only
  int slabs;           // 0: accumulate into dw with atomics.  >0: dw is [slabs][K*N] (destination layout) and must
                       //    hold exactly conv_wgrad_slabs(p) rows; the rows are summed later by grad_finish
                       //    (halo kernel: one plain-stored row per pixel split; generic: atomic replica rows)
};
int conv_wgrad(const WgradParams& p, hipStream_t st);
// several independent weight gradients: the 3x3 halo ones grouped by tile config into shared launches
// (conv3x3_wgrad.hip conv3x3_wgrad_group_kernel), the rest launched one by one
int conv_wgrad_batch(const WgradParams* ps, int n, hipStream_t st);
int conv_wgrad_slabs(const WgradParams& p);
bool conv_wgrad_plain_slabs(const WgradParams& p);   // slab rows are plain-stored (else atomic replica rows)
#define WGRAD_REPLICAS 8     // 16 -> 8 in round 6: grad_finish -3 us, bench +0.3 % (profiles/r6_misc)

// ---------------------------------------------------------------- fused pointwise backward (pw_bwd.hip)
// dgrad + wgrad of a pointwise conv whose output feeds a BatchNorm, the BN backward folded in:
//   dy = bnb_apply(g, y);  dd = dy * W^T (stored);  dW = d^T dy (added into replica row blockIdx % replicas)
struct PwBwdParams {
  const bf16_t* g;         // [M][K] gradient w.r.t. the BN output (K = pw output channels)
  const bf16_t* y;         // [M][K] BN input (the pw output)  -- bwd.y mirrors it
  const bf16_t* d;         // [M][N] pw input (N = pw input channels)
  const bf16_t* w;         // [N][K] dgrad weights (pack PK_PW_DGRAD)
  bf16_t* dd;              // [M][N] dgrad output
  float* dw;               // [replicas][N * K] weight-gradient replica rows (Keras (1,1,N,K); int64 in det mode)
  BnBwdIn bwd;             // BN coefficients / node sums / dgamma, dbeta (dx unused)
  int M, K, N, replicas;
};
bool pw_bwd_supported(const PwBwdParams& p);
int pw_bwd(const PwBwdParams& p, hipStream_t st);

// ---------------------------------------------------------------- fused SeparableConv forward (sepconv.hip)
// y = pointwise(depthwise3x3(T(x))) + bias with the BN statistics of y; d = the depthwise output (side-stored for the
// pointwise weight gradient). T = xf (BN-apply + ReLU; xfin: computed here from the producer's replica sums).
struct SepParams {
  const bf16_t* x;     // [B,H,W,K]
  InXform xf;
  BnStatsIn xfin;
  const float* wdw;    // depthwise taps, Keras (3,3,K,1) = [tap][K]
  const bf16_t* wpw;   // pointwise weights packed [N][K] (pack_weights PK_PW)
  const float* bias;   // [N]
  bf16_t* d;           // [B,H,W,K]
  bf16_t* y;           // [B,H,W,N]
  float* stats;        // [STAT_REPLICAS][2][N] or nullptr
  int B, H, W, K, N;
};
bool sep_fwd_supported(const SepParams& p);
int sep_fwd(const SepParams& p, hipStream_t st);

// ---------------------------------------------------------------- depthwise 3x3 (dwconv.hip)
struct DwParams {
  const bf16_t* x;     // [B,H,W,C] (transform applied on load)
  const float* w;      // Keras depthwise kernel (3,3,C,1) fp32
  const bf16_t* dy;    // gradient of the dw output (dgrad / wgrad)
  bf16_t* y;           // fwd output / dgrad output
  float* dw;           // wgrad destination (fp32, atomic accumulate): [replicas][9][C]
  InXform xf;
  int B, H, W, C;
  int replicas;        // wgrad: >1 = spread block atomics over that many copies of the row (summed by grad_finish)
  int algo;            // 0 auto (C % 32 == 0 -> row-streaming LDS ring), 1 row-strip kernels, 2 LDS halo tiles
  BnNodeEpi node;      // dgrad only (halo-tile path): fused BN-node gradient epilogue
  // dw_bwd only: the dgrad output joins the residual branch's gradient before it is stored (the encoder's input
  // node, node_bwd(dz0 same [masked], dres stride-2 scatter) folded into the producer):
  const bf16_t* add_half;   // dres [B, ceil(H/2), ceil(W/2), C] added at even (h, w) (before the node epilogue)
  int mask_x;               // multiply the dgrad value (not add_half) by [x > 0] (x = the layer's transformed input)
  BnStatsIn xfin;           // dw_fwd: xf.ab computed here from these sums (and written to xf.ab, 4 rows)
};
int dw_fwd(const DwParams& p, hipStream_t st);
int dw_dgrad(const DwParams& p, hipStream_t st);
int dw_wgrad(const DwParams& p, hipStream_t st);
// dgrad (p.dy -> p.y, optional BN-node epilogue p.node) and wgrad (p.x with p.xf, p.dy -> p.dw replicas) of one
// layer in one fused pass (dwconv.hip dw_bwd_stream_kernel)
int dw_bwd(const DwParams& p, hipStream_t st);
// several independent depthwise weight gradients: the row-streaming ones in one grouped launch (dwconv.hip)
int dw_wgrad_batch(const DwParams* ps, int n, hipStream_t st);

// ---------------------------------------------------------------- entry conv 3x3 s2, Cin = 3 (entry.hip)
struct EntryParams {
  const uint8_t* images;   // dataset [Ndata, S, S, 3] uint8
  const int32_t* idx;      // [B] dataset indices of this batch
  const float* w;          // Keras kernel (3,3,3,Cout) fp32
  const float* bias;       // [Cout]
  bf16_t* y;               // [B, Ho, Wo, Cout]
  float* stats;            // [STAT_REPLICAS][2][Cout]
  const bf16_t* dy;        // wgrad: [B,Ho,Wo,Cout]
  float* dw;               // wgrad destination (3,3,3,Cout) fp32: [replicas][27*Cout]
  int B, S, Cout, Ho, Wo;
  int replicas;            // wgrad: >1 = spread block atomics over that many row copies (summed by grad_finish)
  BnBwdIn bwd;             // wgrad: dy is the gradient g w.r.t. the entry BN's output and the operand its BN-backward
                           // apply (common.h; y = the conv output, computed on load; dx stored only on the fallback)
};
int entry_fwd(const EntryParams& p, hipStream_t st);
int entry_wgrad(const EntryParams& p, hipStream_t st);

// ---------------------------------------------------------------- BatchNorm / elementwise (bn.hip, pool_add.hip)
// ab (4 rows of C): a = gamma*rstd, b = beta - mean*a, mean, rstd. train: batch stats from the replica rows;
// eval: moving statistics.
int bn_finalize(const float* stats, const float* gamma, const float* beta, const float* mmean, const float* mvar,
                float* ab, int C, float count, float eps, int train, hipStream_t st);

struct BnMoving {          // one BatchNorm layer for the moving-statistics update
  const float* stats;      // [STAT_REPLICAS][2][C] batch sums
  float* mmean;
  float* mvar;
  int C;
  float count;
};
int bn_moving_update(const BnMoving* d_layers, int n_layers, int max_c, float momentum, hipStream_t st);

struct BnEval {             // one BatchNorm layer's inference coefficients (moving statistics)
  const float* gamma;
  const float* beta;
  const float* mmean;
  const float* mvar;
  float* ab;               // [4][C]
  int C;
  float eps;
};
// every layer's ab from its moving statistics in ONE launch (blockIdx = layer): an inference forward needs them all
int bn_eval_coefs(const BnEval* d_layers, int n_layers, hipStream_t st);

enum GradMode { GM_NONE = 0, GM_SAME = 1, GM_SCATTER2 = 2, GM_SUM2X2 = 3, GM_MAXPOOL = 4 };
int node_bwd(const NodeBwdParams& p, hipStream_t st);

int bn_bwd_apply(const BnBwdApplyParams& p, hipStream_t st);
bool bn_bwd_apply_ok(const BnBwdApplyParams& p);
int bn_bwd_apply_grid(const BnBwdApplyParams& p);
bool node_pool_eligible(const NodeBwdParams& p);
int node_pool_grid(const NodeBwdParams& p);

struct PoolResParams {     // x = maxpool3x3s2_same(a*y + b) + res ; argmax recorded
  const bf16_t* y;
  const float* ab;
  const bf16_t* res;       // [B,Ho,Wo,C]
  bf16_t* out;
  uint8_t* argmax;
  int B, H, W, C, Ho, Wo;
};
int pool_res_fwd(const PoolResParams& p, hipStream_t st);

struct BnAddParams {       // out = (a*y + b) + (up ? q[h/2][w/2] : q[h][w])
  const bf16_t* y;
  const float* ab;
  const bf16_t* q;
  int q_up;
  bf16_t* out;
  int B, H, W, C;
};
int bn_add_fwd(const BnAddParams& p, hipStream_t st);

// ---------------------------------------------------------------- head + loss (head.hip)
struct HeadParams {
  const bf16_t* x;         // x7_lo [B, R, R, Cin] (the logits are up2(conv1x1(x)))
  const float* w;          // (1,1,Cin,1)
  const float* bias;       // (1,)
  const uint8_t* masks;    // dataset masks [Ndata, 2R, 2R]
  const int32_t* idx;      // [B]
  float* h;                // [B, R, R] logits at low resolution
  double* metrics;         // [8]: bce_sum, correct, sum(p*t), sum(p), sum(t), n_pix, batches, unused
  bf16_t* dx;              // [B,R,R,Cin]
  float* dw;               // grad slots for w (Cin) and bias (1) - accumulated
  float* db;
  float* dwfx;             // deterministic mode: int64 fixed-point accumulators [Cin + 1] of dw, db (converted into
                           // them by grad_finish, GF_FIXED); required when the mode is on
  int B, R, Cin;
  int dice;                // add the Dice loss
  int fused;               // head_bwd: also do the forward (logits, loss / accuracy sums) in the same pass (dice 0)
  BnNodeEpi node;          // head_bwd: dx is also the (unmasked) gradient of a BN node whose input is node.y (same
                           // layout as x): accumulate its BN-backward sums (the decoder's last BN_B; node.relu unused)
};
int head_fwd(const HeadParams& p, hipStream_t st);
int head_bwd(const HeadParams& p, hipStream_t st);

// ---------------------------------------------------------------- optimizer / packing (optim.hip)
struct AdamParams {
  float* p;
  const float* g;
  float* m;
  float* v;
  const uint8_t* trainable;
  int64_t n;
  float lr, b1, b2, eps;
  int* step;               // device step counter (incremented by adam_step_done)
};
int adam_update(const AdamParams& p, hipStream_t st);
int adam_step_done(int* step, hipStream_t st);

enum PackKind { PK_CONV = 0, PK_CONV_DGRAD1x1 = 1, PK_CONVT = 2, PK_CONVT_DGRAD = 3, PK_PW = 4, PK_PW_DGRAD = 5 };
struct PackView {
  int kind;
  int64_t src;             // offset in the flat fp32 buffer
  int64_t dst;             // offset in the bf16 pack buffer
  int ks, cin, cout;       // layer geometry (Keras meaning)
  int64_t dst_scale;       // (unused; kept for the table's layout)
};
// step != nullptr: also increments the Adam step counter (adam_step_done folded into this launch)
int pack_weights(const float* flat, bf16_t* packed, const PackView* d_views, int n_views, int max_elems,
                 hipStream_t st, int* step = nullptr, int* cursor = nullptr);   // cursor: BatchSelect's, += 1

// opt_step: the whole optimizer tail of a training step in ONE launch (adam_update + bn_moving_update + pack_weights
// + the step / cursor advance), one block per work item:
//   OI_FLAT    Adam over flat[src, src + n) (n <= 1024), trainable entries only (the params without GEMM views)
//   OI_TILE    Adam over a 64x64 tile of a GEMM weight seen as a row-major [rows][cols] matrix at flat + src, then
//              both bf16 views of the updated tile: the transpose (packed + dst_t)[c * rows + r] and the row-mapped
//              copy (packed + dst_b)[(r % q) * s1 + (r / q) * s2 + base2 + c] - every pack_weights view is one of
//              the two (1x1 conv / pointwise [cin][cout]: PK_CONV / PK_PW transpose, the dgrad views copies; ConvT
//              (3,3,out,in) as [9 cout][cin]: PK_CONVT_DGRAD the transpose, PK_CONVT the tap-flipped row map)
//   OI_MOVING  the BN moving statistics of one layer from its replica batch sums
// The last block to finish (ticket) advances the Adam step and the batch cursor: every block has read the step.
enum OptKind { OI_FLAT = 0, OI_TILE = 1, OI_MOVING = 2 };
struct OptItem {
  int kind;
  int n;                   // flat: elements; moving: channels
  int r0, c0, rows, cols;  // tile
  int q, s1, s2, base2;    // tile: row map of the copy view
  int64_t src;             // flat / tile: offset into the flat master buffer
  int64_t dst_t, dst_b;    // tile: offsets into the bf16 pack buffer
  const float* stats;      // moving: [STAT_REPLICAS][2][C] batch sums
  float* mmean;
  float* mvar;
  float count;
};
struct OptParams {
  float* p;
  const float* g;
  float* m;
  float* v;
  const uint8_t* trainable;
  bf16_t* packed;
  const OptItem* items;
  int n_items;
  float lr, b1, b2, eps, momentum;
  int* step;
  int* cursor;             // nullable
  int* ticket;             // one int, zero between launches
  const float* lr_t;       // nullable: the step's Adam rate, computed by its zero_spans launch (StepAdvance), which
                           // also advanced the step and cursor - then step / cursor / ticket are unused (no ticket)
};
int opt_step(const OptParams& p, hipStream_t st);

// ---------------------------------------------------------------- step bookkeeping (optim.hip)
// grad_finish: ONE launch at the end of backward for every gradient that was accumulated into replica rows
// (GF_REDUCE: dst[i] += sum_r src[r*n + i], then the replicas are re-zeroed for the next step; GF_SUM: the same
// for rows that are fully overwritten every step, so no re-zeroing) or that equals
// another gradient (GF_COPY: dst[i] = src[i], e.g. a residual conv's bias grad == its BN's beta grad).
// GF_SUM: like GF_REDUCE, rows not re-zeroed; GF_FIXED (deterministic mode): dst[i] = int64 fixed-point src[i]
// converted (CFL_FX_G), src re-zeroed, any n. In the deterministic mode GF_REDUCE rows are int64 fixed point too and
// every entry is one group per tile (rows summed in order, no atomics); the grid must be re-derived
// (grad_finish_work) after cfl_det_set.
enum GradFinishMode { GF_REDUCE = 0, GF_COPY = 1, GF_SUM = 2, GF_FIXED = 3 };
struct GradFinish {
  float* src;
  float* dst;
  int n, replicas, mode;   // n % 4 == 0, src / dst 16-byte aligned
  int work_begin;          // first work item (set by grad_finish_work)
};
int grad_finish_work(GradFinish* h_entries, int n_entries);   // fills work_begin, returns the grid size
int grad_finish(const GradFinish* d_entries, int n_entries, int total_work, hipStream_t st);
// zero_spans: ONE launch zeroing a list of 16-byte aligned spans (the per-step gradient / statistics buffers)
struct ZeroSpan {
  void* p;
  int64_t bytes;           // multiple of 16
};
// batch: optionally also selects the step's dataset indices on the device, idx[0..B) = table[(*cursor) % nb]
// (a batch table bound once per epoch; the cursor is advanced by this launch's StepAdvance, or else by opt_step /
// pack_weights at the end of the step), so the replayed step needs no host-issued index copy
struct BatchSelect {
  const int32_t* table;    // [nb][B] or nullptr
  int* cursor;
  int32_t* idx;
  int B, nb;
};
// step: optionally advances the training step at its START (the engine's fused step): lr_t = the Adam rate of step
// *step + 1 (the formula opt_step uses), then *step += 1 and, with a batch table, *cursor += 1 after the batch
// select - so opt_step reads lr_t and needs no end-of-launch ticket (which kept every one of its blocks alive for a
// device-scope atomic round trip: 4 us of the step, profiles/README.md)
struct StepAdvance {
  int* step;               // nullptr: nothing advanced
  float* lr_t;
  float lr, b1, b2;
};
int zero_spans(const ZeroSpan* d_spans, int n_spans, int64_t max_bytes, hipStream_t st,
               BatchSelect batch = BatchSelect{}, StepAdvance adv = StepAdvance{});

// launch-shape tuning knobs (0 = built-in heuristic), set from Python for micro-benchmark sweeps
enum TuneKey {
  TUNE_NODE_BWD_BLOCKS = 0, TUNE_DW_WGRAD_BLOCKS = 1, TUNE_ENTRY_WGRAD_BLOCKS = 2,
  TUNE_WGRAD3_BLOCKS = 3,      // halo wgrad: target grid size (default 512)
  TUNE_WGRAD3_MINTILES = 4,    // halo wgrad: min pixel tiles per block (default 32)
  TUNE_IGEMM_CFG = 5,          // generic implicit GEMM: force a tile config 1..7 (see conv_igemm.hip)
  TUNE_CONV3_WB = 6,           // conv3x3: 1 = whole-chunk weight staging (default), 2 = per-tap double buffer
  TUNE_ENTRY_FWD_BLOCKS = 7,   // entry conv forward grid cap (default 1,024; 2,048 at >= 64k row steps)
  TUNE_DW_STREAM_BLOCKS = 8,   // depthwise row-streaming kernels: target grid size (default 768)
  TUNE_CONV3_SMALL = 9,        // conv3x3 low-M layers: 0 = heuristic, 1 = split-K (+ epilogue launch), 2 = 8x8x32 tiles
  TUNE_CONV3_BN = 10,          // conv3x3 whole-chunk path: output-channel tile (0 = 64 when N % 64 == 0, else 32)
  TUNE_NODE_POOL2X2 = 11,      // max-pool node gradient: 0 = 2x2-block kernel, 1 = per-pixel gather
  TUNE_ENTRY_ALGO = 12,        // entry conv (Cout 32): 0 = MFMA kernels, 1 = VALU kernels
  TUNE_HEAD_BLOCKS = 13,       // head fwd / bwd grid cap (default 512)
  TUNE_CONV3_WS = 14,          // conv3x3 Cin <= 64: 0 = weight-stationary persistent kernel, 1 = per-tile kernel
  TUNE_CONV3_WS_GRID = 15,     // weight-stationary conv3x3: persistent grid size (default 512)
  TUNE_WGRAD_GROUP = 16,       // conv_wgrad_batch: 1 = launch every wgrad on its own, 2 = group the 3x3 ones only
  TUNE_CONV3_DEEP = 17,        // conv3x3 Cin >= 128: 0 = LDS-DMA 3-stage deep-K kernel, 1 = off, 2 = force (any Cin)
  TUNE_WGRAD1_BLOCKS = 18,     // generic (1x1) wgrad: target blocks per layer (default 320)
  TUNE_WGRAD1_MINPIX = 19,     // generic (1x1) wgrad: min pixels per block (default 512)
  TUNE_NODE_BWD_IPT = 20,      // node_bwd: items in flight per thread (2 or 4; default 2)
  TUNE_DW_BWD_BLOCKS = 21,     // fused depthwise backward: target grid size (default 512)
  TUNE_BBA_BLOCKS = 22,        // bn_bwd_apply grid cap (default 256)
  TUNE_NODE_POOL_BLOCKS = 23,  // max-pool node gradient grid cap (default: TUNE_NODE_BWD_BLOCKS / 512)
  TUNE_WGRAD1_RM = 24,         // generic wgrad 64x64 tiles: pixels per pipeline stage (0 = 64, 128)
  TUNE_PW = 25,                // plain 1x1 convs: 0 = streaming kernel (pw.hip), 1 = conv_igemm tiles
  TUNE_PW_BLOCKS = 26,         // streaming 1x1 kernel: resident-grid cap (default 512 = 2 blocks per CU)
  TUNE_PW_DEPTH = 27,          // streaming 1x1 kernel: tiles in flight per wave (1 default, 2, 4 at K = 32)
  TUNE_NODE_POOL_IPT = 28,     // max-pool node gradient: 2x2 items per thread per trip (1 default, 2)
  TUNE_WGRAD3_MINTILES32 = 29, // halo wgrad, 32-wide output tiles: min pixel tiles per block (default 16)
  TUNE_WGRAD_MIX = 30,         // conv_wgrad_batch: 0 = every deferred wgrad in ONE mixed launch, 1 = a launch per config
  TUNE_CONV3_SPLIT_BLOCKS = 31, // conv3x3 8x16 tiles: split K when the grid has fewer blocks than this (default 192)
  TUNE_CONV3_SPLIT_TARGET = 32, // ... into about this many blocks (default 384)
  TUNE_SEP = 33,               // SeparableConv forward: 0 = fused depthwise + pointwise (sepconv.hip), 1 = two passes
  TUNE_SEP_BLOCKS = 34,        // fused SeparableConv forward: target grid size (default 512)
  TUNE_WGRAD_MIX_XCD = 35,     // mixed wgrad launch: 0 = XCD-grouped block order, 1 = dispatch order
  TUNE_SIDE = 36,              // streaming 1x1 dgrads: 0 = co-launch their side job (SideJob), 1 = run it alone first
  TUNE_WGRAD1_BIG = 37,        // generic wgrad, K and N % 128 == 0 (any M since round 6): 0 = 128x128 tiles, 64-pixel stages;
                               // 1 = 64x64 tiles; 2 = 128x128 tiles, 32-pixel stages
  TUNE_CONV3_BIG = 38,         // conv3x3 whole-chunk path at M >= 1M pixels: 0 = 16x16-pixel tiles, 1 = off, 2 = force
  TUNE_PW_NB = 39,             // streaming 1x1 kernel, N % 128 == 0 and K >= 128: 0 = 128-channel output slices at
                               // M >= 1M pixels (else 64), 64 = always 64, 128 = always 128
  TUNE_CONV3_SK = 40,          // split-K-in-block 32x32 MFMA 3x3 kernel (conv3x3_sk.hip): 0 = default (Cin 256 at <= 32^2), 1 = off,
                               //   2 = force wherever the shape allows, 3 = the low-resolution levels (<= 32^2, Cin >= 128)
  TUNE_CONV3_SK_CFG = 41,      // ... tile config: 0 = heuristic, 1 = 8x8 px x 64 ch, 2 = 8x16 x 64, 3 = 16x16 x 32,
                               //   4 = 8x16 x 32
  TUNE_WGRAD_MIX_ONLY = 42,    // TIMING ONLY (wrong gradients): mixed wgrad launch keeps only item k - 1 (mix order)
  TUNE_WGRAD_MIX_SKIP = 43,    // TIMING ONLY: mixed wgrad launch drops the items of this bit mask (bit k = item k)
  TUNE_WGRAD_MIX_LIST = 44,    // 1: print the mixed launch's items (index, kind, shape, blocks) to stderr once
  TUNE_WGRAD_MIX_ORDER = 45,   // mixed wgrad launch item order: 0 = default (2), 1 = generic first, 2 = alternating,
                               //   3 = halo items first (round 6: longest-block-first orders measured +4 / +8.5 us)
  TUNE_OPT_SCALAR = 46,        // opt_step: 1 = per-column tile form for every tile (default: 16-byte form where aligned)
  // 47: retired (opt_step timing knob without its ticket; the training step no longer uses the ticket)
  // 48, 49: retired (split-K-in-block halo wgrad body: slower in the slot-bound mixed launch, deleted in round 6)
  TUNE_CONV3_F8 = 50,          // fp8 3x3 routing: 0 = default (fp8 for the node-join dgrads the weight-stationary bf16
                               //   kernel does not take), 1 = never; 2 = TEST hook only (every call carrying fp8
                               //   operands: kernel coverage; the whole-network modes were closed in round 6)
  TUNE_DW_BWD_DMA = 51,        // fused depthwise backward: 0 = default (LDS-DMA dy ring kernel, 3 blocks / CU, when
                               //   the launch has >= 1,536 strips, else the register-staged two-ring kernel), 1 = always
                               //   the DMA kernel, 2 = never
  TUNE_WGRAD3_WIDE = 52,       // halo wgrad 64-input-channel blocks (one LDS buffer): 0 = default (launches of >= 64k
                               //   32-channel tile-blocks: the 512^2 planned batch), 1 = never, 2 = whenever Cin % 64 == 0
  TUNE_CONV3_BIG_WAVES = 53,   // conv3x3 16x16-pixel tiles: wave grid 0 = default (4 x 1: 64 px x 64 ch per wave), 1 = 2 x 2
  TUNE_WGRAD_DIRECT = 54,      // generic wgrad, 1x1 / stride-1 convs in the mixed launch: 0 = direct-row body, 1 = general
  TUNE_PWB_BLOCKS = 55,        // fused pointwise backward (pw_bwd.hip): grid (default 384 at N = 32, 256 at N = 64)
  TUNE_PWB = 56,               // encoder pointwise backward: 0 = fused dgrad + wgrad (pw_bwd.hip), 1 = pw.hip dgrad +
                               //   deferred wgrad (round 5)
  TUNE_WGRAD_REPS = 57,         // generic weight-gradient replica rows (conv_wgrad_slabs; default WGRAD_REPLICAS)
  TUNE_N = 58
};
int cfl_tune(int key);
void cfl_set_tune(int key, int value);
// deterministic reduction mode (common.h): sets the constant flag of every kernel translation unit (before any graph
// capture: the flag is read by the kernels at run time, so captured graphs follow the value at their replay) and the
// host copy; 0 on success
int cfl_det_set(int v);
// one scaled fp8 MFMA on raw lane registers (fp8.hip): a, b [64][8] int32, sa, sb [64], d [64][4] (16x16x128) or
// [64][16] (32x32x64)
int mfma_scale_probe(const int* a, const int* b, const int* sa, const int* sb, float* d, int shape, hipStream_t st);
int cfl_fx_overflow();
int cfl_det_host();
int cfl_det_upload_bn(int v);
int cfl_det_upload_conv3x3(int v);
int cfl_det_upload_conv3x3_deep(int v);
int cfl_det_upload_conv3x3_sk(int v);
int cfl_det_upload_conv3x3_wgrad(int v);
int cfl_det_upload_conv_igemm(int v);
int cfl_det_upload_conv_wgrad(int v);
int cfl_det_upload_datagen(int v);
int cfl_det_upload_dwconv(int v);
int cfl_det_upload_entry(int v);
int cfl_det_upload_fp8(int v);
int cfl_det_upload_head(int v);
int cfl_det_upload_optim(int v);
int cfl_det_upload_pool_add(int v);
int cfl_det_upload_pw(int v);
int cfl_det_upload_pw_bwd(int v);
int cfl_det_upload_sepconv(int v);

// block timeline (common.h CflTsGuard): buf = [cap][2] u64 (dispatch, retire) s_memrealtime stamps per linear block id
// of every instrumented kernel launched while set; nullptr = off. 0 on success.
int cfl_ts_set(void* buf, int cap);
int cfl_ts_upload_bn(void* buf, int cap);
int cfl_ts_upload_conv3x3(void* buf, int cap);
int cfl_ts_upload_conv3x3_deep(void* buf, int cap);
int cfl_ts_upload_conv3x3_sk(void* buf, int cap);
int cfl_ts_upload_conv3x3_wgrad(void* buf, int cap);
int cfl_ts_upload_conv_igemm(void* buf, int cap);
int cfl_ts_upload_conv_wgrad(void* buf, int cap);
int cfl_ts_upload_datagen(void* buf, int cap);
int cfl_ts_upload_dwconv(void* buf, int cap);
int cfl_ts_upload_entry(void* buf, int cap);
int cfl_ts_upload_fp8(void* buf, int cap);
int cfl_ts_upload_head(void* buf, int cap);
int cfl_ts_upload_optim(void* buf, int cap);
int cfl_ts_upload_pool_add(void* buf, int cap);
int cfl_ts_upload_pw(void* buf, int cap);
int cfl_ts_upload_pw_bwd(void* buf, int cap);
int cfl_ts_upload_sepconv(void* buf, int cap);

// ---------------------------------------------------------------- misc (optim.hip / datagen.hip)
int fill_f32(float* p, float v, int64_t n, hipStream_t st);
int gather_rows_u8(const uint8_t* src, const int32_t* idx, uint8_t* dst, int rows, int64_t row_bytes,
                   hipStream_t st);
int render_cracks(const float* segs, const float* params, uint8_t* images, uint8_t* masks, int n, int img,
                  int max_seg, hipStream_t st);
// n decoded images (src bytes at offs[i], dims[i] = {h, w}, c channels) bilinearly resized into dst [n, dh, dw, c]
// (binarize: masks -> {0, 1}); datagen.hip
int resize_batch(const uint8_t* src, const int64_t* offs, const int* dims, uint8_t* dst, int n, int dh, int dw, int c,
                 int binarize, hipStream_t st);

