// Optimizer and weight packing.
//   adam_update:   Keras OptimizerV2 Adam (compile(optimizer="Adam"), client_fit_model.py:157; defaults lr 1e-3,
//                  beta_1 0.9, beta_2 0.999, epsilon 1e-7) over the single flat fp32 master buffer, trainable
//                  entries only (BN moving statistics are skipped):
//                    lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t);  m,v EMA;  w -= lr_t * m / (sqrt(v) + eps)
//                  t lives on the device so the whole step can be replayed as one hipGraph.
//   pack_weights:  fp32 master (Keras layouts) -> bf16 GEMM operands [N][K] for conv_igemm, forward and dgrad,
//                  including the Conv2DTranspose flip/transposition; one launch for all layers (descriptor table).
#include "common.h"
#include "launch.h"

namespace {

constexpr int NT = 256;

// THE Adam element update (adam_kernel and opt_step share it). The moment updates are explicit fmas: left as
// a*b + c*d, the compiler contracted them differently in the vectorised and the scalar kernel (m differed by an ulp
// on ~5% of the elements); every other operation here feeds a division or a square root, nothing to contract.
CFL_DEVICE void adam_elem(float& w, float g, float& m, float& v, float lr_t, float b1, float b2, float eps) {
  m = fmaf(b1, m, (1.f - b1) * g);
  v = fmaf(b2, v, (1.f - b2) * g * g);
  w -= lr_t * m / (sqrtf(v) + eps);
}
CFL_DEVICE float adam_lr(const int* step, float lr, float b1, float b2) {
  const int t = *step + 1;
  return lr * sqrtf(1.f - powf(b2, (float)t)) / (1.f - powf(b1, (float)t));
}

// opt_step's rate: computed by the step's zero_spans launch (StepAdvance), else from the step counter
CFL_DEVICE float step_lr(const OptParams& p) {
  return p.lr_t != nullptr ? *p.lr_t : adam_lr(p.step, p.lr, p.b1, p.b2);
}

__global__ __launch_bounds__(NT) void adam_kernel(AdamParams p) {
  CFL_TS_GUARD;
  const float lr_t = adam_lr(p.step, p.lr, p.b1, p.b2);
  const int64_t n4 = p.n / 4;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n4; i += (int64_t)gridDim.x * NT) {
    const uint32_t tm = *reinterpret_cast<const uint32_t*>(p.trainable + 4 * i);
    if (!tm) continue;
    float4 w = reinterpret_cast<float4*>(p.p)[i];
    const float4 g = reinterpret_cast<const float4*>(p.g)[i];
    float4 m = reinterpret_cast<float4*>(p.m)[i];
    float4 v = reinterpret_cast<float4*>(p.v)[i];
    float* wp = &w.x;
    const float* gp = &g.x;
    float* mp = &m.x;
    float* vp = &v.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!((tm >> (8 * j)) & 0xffu)) continue;
      adam_elem(wp[j], gp[j], mp[j], vp[j], lr_t, p.b1, p.b2, p.eps);
    }
    reinterpret_cast<float4*>(p.p)[i] = w;
    reinterpret_cast<float4*>(p.m)[i] = m;
    reinterpret_cast<float4*>(p.v)[i] = v;
  }
}

__global__ void step_done_kernel(int* step) {
  CFL_TS_GUARD;
  *step += 1;
}

__global__ __launch_bounds__(NT) void pack_kernel(const float* flat, bf16_t* packed, const PackView* views,
                                                  int* step, int* cursor) {
  CFL_TS_GUARD;
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    if (step != nullptr) *step += 1;                  // adam_step_done
    if (cursor != nullptr) *cursor += 1;              // next step's batch (BatchSelect)
  }
  const PackView v = views[blockIdx.y];
  const int taps = v.ks * v.ks;
  int N, K;
  switch (v.kind) {
    case PK_CONV: N = v.cout; K = taps * v.cin; break;
    case PK_CONV_DGRAD1x1: N = v.cin; K = v.cout; break;
    case PK_CONVT: N = v.cout; K = 9 * v.cin; break;
    case PK_CONVT_DGRAD: N = v.cin; K = 9 * v.cout; break;
    case PK_PW: N = v.cout; K = v.cin; break;
    default: N = v.cin; K = v.cout; break;   // PK_PW_DGRAD
  }
  const int total = N * K;                      // < 2^31 for every layer (32-bit index math, no 64-bit division)
  const float* src = flat + v.src;
  bf16_t* dst = packed + v.dst;
  if (v.kind == PK_CONV || v.kind == PK_CONVT_DGRAD || v.kind == PK_PW) {
    // these views are plain transposes of the Keras array: src is [K][N] (N contiguous), dst [N][K]. Staged
    // through a 64x64 LDS tile so both the fp32 reads and the bf16 writes are coalesced rows (a per-element
    // gather reads one float per cache line at stride N)
    __shared__ float tl[64][65];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int tk = (K + 63) >> 6, tn = (N + 63) >> 6;
    for (int t = blockIdx.x; t < tk * tn; t += gridDim.x) {   // block-uniform loop: the barriers are safe
      const int k0 = (t / tn) << 6, n0 = (t % tn) << 6;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int k = k0 + ty + 4 * j, n = n0 + tx;
        tl[ty + 4 * j][tx] = (k < K && n < N) ? src[k * N + n] : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int n = n0 + ty + 4 * j, k = k0 + tx;
        if (n < N && k < K) dst[n * K + k] = f2bf(tl[tx][ty + 4 * j]);
      }
      __syncthreads();
    }
    return;
  }
  for (int e = blockIdx.x * NT + threadIdx.x; e < total; e += gridDim.x * NT) {
    const int n = e / K, k = e - n * K;
    int s;
    switch (v.kind) {
      case PK_CONV: s = k * v.cout + n; break;                                   // HWIO [tap][ci][co]
      case PK_CONV_DGRAD1x1: s = n * v.cout + k; break;                          // [ci][co] as [N=ci][K=co]
      case PK_CONVT: {                                                          // (3,3,out,in), flipped
        const int tap = k / v.cin, c = k - tap * v.cin;
        s = ((8 - tap) * v.cout + n) * v.cin + c;
        break;
      }
      case PK_CONVT_DGRAD: {                                                    // k = tap*cout + o, n = c
        const int tap = k / v.cout, o = k - tap * v.cout;
        s = (tap * v.cout + o) * v.cin + n;
        break;
      }
      case PK_PW: s = k * v.cout + n; break;                                    // (1,1,C,F): [c][f]
      default: s = n * v.cout + k; break;                                       // pw dgrad: [N=c][K=f]
    }
    dst[e] = f2bf(src[s]);
  }
}

// opt_step (launch.h): one block per OptItem. A thread that uses the step (lr_t) has its read completed before the
// stores that depend on it, i.e. before the block's closing barrier and the ticket atomic after it, so the last block
// advances the step only after every read of it. The ticket is RELAXED: the ordering it needs is that of loads whose
// values were already consumed, and nothing the blocks stored is read by the last block (an agent-scope release made
// every block write back its XCD's L2 before retiring). With p.lr_t (the engine's training step) the step's
// zero_spans launch already computed the rate and advanced the step / cursor: no ticket.
//
// VEC: a tile whose row length, offsets and row maps are multiples of 4 elements (every GEMM weight of the model)
// is moved in 16-byte fp32 / 8-byte bf16 pieces - a quarter of the memory instructions of the per-column form.
// column swizzle of the 16-byte form's [64][65] transpose tile (ds_*_b32 banks: dword address mod 32, lanes 0-31 /
// 32-63 per LDS cycle): rows 32 apart and columns 32 apart share banks, so the writes (lanes 0-31: columns 4cq + k,
// cq = 0..15) and the transposed reads (rows 4rq + i, rq = 0..15) were 2-way conflicted (PMC: 50 % conflict
// cycles). Rotating a 32-column half by 2 when exactly one of (row >= 32, column >= 32) holds separates both (a
// bijection per row).
CFL_DEVICE int opt_swz(int R, int C) { return (C & 32) | ((C + (((R ^ C) >> 5) << 1)) & 31); }

template <bool VEC>
__global__ __launch_bounds__(NT) void opt_step_kernel(const OptParams p) {
  CFL_TS_GUARD;
  const OptItem it = p.items[blockIdx.x];
  const int tid = threadIdx.x;
  __shared__ float tl[64][65];
  if (it.kind == OI_MOVING) {                           // bn_moving_kernel's update, replica sums in order
    const int C = it.n;
    const float mom = p.momentum;
    for (int c = tid; c < C; c += NT) {
      float s = 0.f, s2 = 0.f;
      if (!stat_sums_det(it.stats, C, c, s, s2)) {
        float va[STAT_REPLICAS], vb[STAT_REPLICAS];
#pragma unroll
        for (int r = 0; r < STAT_REPLICAS; ++r) {
          va[r] = it.stats[r * 2 * C + c];
          vb[r] = it.stats[r * 2 * C + C + c];
        }
#pragma unroll
        for (int r = 0; r < STAT_REPLICAS; ++r) {
          s += va[r];
          s2 += vb[r];
        }
      }
      const float mean = s / it.count;
      const float var = fmaxf(s2 / it.count - mean * mean, 0.f);
      const float unbiased = var * (it.count / fmaxf(it.count - 1.f, 1.f));
      it.mmean[c] = it.mmean[c] * mom + mean * (1.f - mom);
      it.mvar[c] = it.mvar[c] * mom + unbiased * (1.f - mom);
    }
  } else if (it.kind == OI_FLAT) {
    const float lr_t = step_lr(p);
    float w[4], g[4], m[4], v[4];
    bool on[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + u * NT;
      const int64_t e = it.src + i;
      on[u] = i < it.n && p.trainable[e];
      w[u] = on[u] ? p.p[e] : 0.f;
      g[u] = on[u] ? p.g[e] : 0.f;
      m[u] = on[u] ? p.m[e] : 0.f;
      v[u] = on[u] ? p.v[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (!on[u]) continue;
      const int64_t e = it.src + tid + u * NT;
      adam_elem(w[u], g[u], m[u], v[u], lr_t, p.b1, p.b2, p.eps);
      p.p[e] = w[u];
      p.m[e] = m[u];
      p.v[e] = v[u];
    }
  } else if (VEC && ((it.cols | it.rows | (int)it.src | it.s1 | it.s2 | it.base2 | (int)it.dst_t | (int)it.dst_b) &
                     3) == 0) {
    // 64x64 tile, thread (cq, rt) owns columns c0 + 4cq .. + 3 of rows r0 + rt + 16j: float4 loads / stores of the
    // fp32 arrays, 4 bf16 (8 bytes) per store of both views (the transpose through LDS: thread (rq, cc) writes rows
    // r0 + 4rq .. + 3 of column cc). Both LDS passes hit 64 distinct banks per wave (row stride 65).
    const float lr_t = step_lr(p);
    const int cq = tid & 15, rt = tid >> 4, c = it.c0 + 4 * cq;
    const bool cok = c < it.cols;                       // cols % 4 == 0: the whole quad is in range
    float4 w[4], g[4], m[4], v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = it.r0 + rt + 16 * j;
      // out-of-tile lanes load the tile's first quad (a select of the address, not of a pointer to a zero
      // constant: that made the compiler stage the constant in scratch and use flat loads); their values are unused
      const int64_t e = (cok && r < it.rows) ? it.src + (int64_t)r * it.cols + c : it.src;
      w[j] = *reinterpret_cast<const float4*>(p.p + e);
      g[j] = *reinterpret_cast<const float4*>(p.g + e);
      m[j] = *reinterpret_cast<const float4*>(p.m + e);
      v[j] = *reinterpret_cast<const float4*>(p.v + e);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = it.r0 + rt + 16 * j;
      if (cok && r < it.rows) {
        adam_elem(w[j].x, g[j].x, m[j].x, v[j].x, lr_t, p.b1, p.b2, p.eps);
        adam_elem(w[j].y, g[j].y, m[j].y, v[j].y, lr_t, p.b1, p.b2, p.eps);
        adam_elem(w[j].z, g[j].z, m[j].z, v[j].z, lr_t, p.b1, p.b2, p.eps);
        adam_elem(w[j].w, g[j].w, m[j].w, v[j].w, lr_t, p.b1, p.b2, p.eps);
        const int64_t e = it.src + (int64_t)r * it.cols + c;
        *reinterpret_cast<float4*>(p.p + e) = w[j];
        *reinterpret_cast<float4*>(p.m + e) = m[j];
        *reinterpret_cast<float4*>(p.v + e) = v[j];
        const uint2 b = make_uint2(pack2bf(w[j].x, w[j].y), pack2bf(w[j].z, w[j].w));
        *reinterpret_cast<uint2*>(p.packed + it.dst_b + (int64_t)(r % it.q) * it.s1 + (int64_t)(r / it.q) * it.s2 +
                                  it.base2 + c) = b;
      }
      const int R = rt + 16 * j;
      float* row = &tl[R][0];
      row[opt_swz(R, 4 * cq)] = w[j].x;
      row[opt_swz(R, 4 * cq + 1)] = w[j].y;
      row[opt_swz(R, 4 * cq + 2)] = w[j].z;
      row[opt_swz(R, 4 * cq + 3)] = w[j].w;
    }
    __syncthreads();
    const int rq = tid & 15, r = it.r0 + 4 * rq;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ccl = (tid >> 4) + 16 * j, cc = it.c0 + ccl;
      if (cc < it.cols && r < it.rows) {                 // rows % 4 == 0: the whole quad is in range
        const int R = 4 * rq;
        const uint2 b = make_uint2(pack2bf(tl[R][opt_swz(R, ccl)], tl[R + 1][opt_swz(R + 1, ccl)]),
                                   pack2bf(tl[R + 2][opt_swz(R + 2, ccl)], tl[R + 3][opt_swz(R + 3, ccl)]));
        *reinterpret_cast<uint2*>(p.packed + it.dst_t + (int64_t)cc * it.rows + r) = b;
      }
    }
  } else {
    // 64x64 tile, thread (tx, ty) owns column c0 + tx of rows r0 + ty + 4j: coalesced 256-B rows of every fp32 array
    const float lr_t = step_lr(p);
    const int tx = tid & 63, ty = tid >> 6, c = it.c0 + tx;
    const int64_t base = it.src;
    float w[16], g[16], m[16], v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = it.r0 + ty + 4 * j;
      const bool ok = r < it.rows && c < it.cols;
      const int64_t e = base + (int64_t)r * it.cols + c;
      w[j] = ok ? p.p[e] : 0.f;
      g[j] = ok ? p.g[e] : 0.f;
      m[j] = ok ? p.m[e] : 0.f;
      v[j] = ok ? p.v[e] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = it.r0 + ty + 4 * j;
      if (r < it.rows && c < it.cols) {
        const int64_t e = base + (int64_t)r * it.cols + c;
        adam_elem(w[j], g[j], m[j], v[j], lr_t, p.b1, p.b2, p.eps);
        p.p[e] = w[j];
        p.m[e] = m[j];
        p.v[e] = v[j];
        p.packed[it.dst_b + (int64_t)(r % it.q) * it.s1 + (int64_t)(r / it.q) * it.s2 + it.base2 + c] = f2bf(w[j]);
      }
      tl[ty + 4 * j][tx] = w[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int cc = it.c0 + ty + 4 * j, rr = it.r0 + tx;
      if (cc < it.cols && rr < it.rows) p.packed[it.dst_t + (int64_t)cc * it.rows + rr] = f2bf(tl[tx][ty + 4 * j]);
    }
  }
  __syncthreads();
  if (tid == 0 && p.lr_t == nullptr) {
    const int t = __hip_atomic_fetch_add(p.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (int)gridDim.x - 1) {                      // every block has read the step: advance it
      *p.ticket = 0;
      *p.step += 1;
      if (p.cursor != nullptr) *p.cursor += 1;
    }
  }
}

__global__ void fill_kernel(float* p, float v, int64_t n) {
  CFL_TS_GUARD;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) p[i] = v;
}

__global__ void gather_rows_kernel(const uint8_t* src, const int32_t* idx, uint8_t* dst, int rows, int64_t row_bytes) {
  CFL_TS_GUARD;
  const int r = blockIdx.y;
  const uint8_t* s = src + (int64_t)idx[r] * row_bytes;
  uint8_t* d = dst + (int64_t)r * row_bytes;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < row_bytes; i += (int64_t)gridDim.x * NT) d[i] = s[i];
}

// One block per work item = (entry, 1024-float element tile, group of GF_ROWS rows). Thread t owns elements
// 256 * u + t (u = 0..3) of the tile, so every load / store / atomic wave-instruction covers 256 contiguous bytes - the
// full-rate shape of the memory-side float atomics (a float4 per lane split into four scalar atomics put each
// instruction's lanes 16 B apart: four times the atomic requests). The GF_ROWS x 4 loads are issued before any sum
// (memory-level parallelism over a long row list); the sum goes to the destination plainly when the entry has a
// single row group, else with one atomic per element per group.
constexpr int GF_ROWS = 16;

// DET (deterministic mode, common.h): a separate instantiation - its int64 row registers would otherwise cost the
// default kernel 72 -> 246 VGPRs (occupancy 7 -> 2)
template <bool DET>
__global__ __launch_bounds__(NT) void grad_finish_kernel(const GradFinish* __restrict__ e, int n_entries) {
  CFL_TS_GUARD;
  // entry of this block: entries are sorted by work_begin; count how many begin at or before blockIdx.x
  const int wb = threadIdx.x < n_entries ? e[threadIdx.x].work_begin : 0x7fffffff;
  const int k = __syncthreads_count(wb <= (int)blockIdx.x) - 1;
  const GradFinish g = e[k];
  const int rows = g.mode == GF_COPY || g.mode == GF_FIXED ? 1 : g.replicas;
  constexpr bool det = DET;
  const int ngroups = det ? 1 : (rows + GF_ROWS - 1) / GF_ROWS;
  const int local = blockIdx.x - g.work_begin;
  const int tile = local / ngroups, rg = local - tile * ngroups;
  const int i0 = tile * 4 * NT + threadIdx.x;
  if (g.mode == GF_COPY) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * NT < g.n) g.dst[i0 + u * NT] = g.src[i0 + u * NT];
    return;
  }
  if (DET && g.mode == GF_FIXED) {  // deterministic mode: int64 fixed-point accumulators -> dst, re-zeroed
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * NT;
      if (i < g.n) {
        g.dst[i] = red_fx(red_raw(g.src, i), CFL_FX_G);
        reinterpret_cast<long long*>(g.src)[i] = 0;
      }
    }
    return;
  }
  if constexpr (DET) {              // one group per tile, every row in order: no atomics into dst
    // thread t owns the 4 consecutive elements 4t .. 4t+3 of the tile (n % 4 == 0, 16-byte aligned rows): 16-byte
    // row pieces through global-address-space pointers, several rows per load round
    typedef f4v __attribute__((address_space(1))) gf4;
    typedef long long i2v __attribute__((ext_vector_type(2)));
    typedef i2v __attribute__((address_space(1))) gi2;
    const int i = tile * 4 * NT + 4 * threadIdx.x;
    if (i >= g.n) return;
    gf4* dst = (gf4*)(g.dst + i);
    if (g.mode == GF_REDUCE) {      // int64 fixed-point rows (exact in any order), re-zeroed
      constexpr int GF_DROWS = 8;   // rows per load round (two 16-byte int64 pairs per row)
      gi2* src = (gi2*)(reinterpret_cast<long long*>(g.src) + i);
      const size_t n2 = (size_t)g.n >> 1;
      i2v q0 = {0, 0}, q1 = {0, 0};
      for (int r0 = 0; r0 < rows; r0 += GF_DROWS) {
        i2v a[GF_DROWS], b[GF_DROWS];
#pragma unroll
        for (int r = 0; r < GF_DROWS; ++r) {
          if (r0 + r < rows) {
            a[r] = src[(size_t)(r0 + r) * n2];
            b[r] = src[(size_t)(r0 + r) * n2 + 1];
          } else {
            a[r] = i2v{0, 0};
            b[r] = i2v{0, 0};
          }
        }
#pragma unroll
        for (int r = 0; r < GF_DROWS; ++r) {
          q0 += a[r];
          q1 += b[r];
          if (r0 + r < rows) {
            src[(size_t)(r0 + r) * n2] = i2v{0, 0};
            src[(size_t)(r0 + r) * n2 + 1] = i2v{0, 0};
          }
        }
      }
      *dst = *dst + f4v{red_fx(q0.x, CFL_FX_G), red_fx(q0.y, CFL_FX_G), red_fx(q1.x, CFL_FX_G),
                        red_fx(q1.y, CFL_FX_G)};
    } else {                        // GF_SUM: plainly stored float rows, summed in row order
      gf4* src = (gf4*)(g.src + i);
      const size_t n4 = (size_t)g.n >> 2;
      f4v s = {0.f, 0.f, 0.f, 0.f};
      for (int r0 = 0; r0 < rows; r0 += GF_ROWS) {
        f4v v[GF_ROWS];
#pragma unroll
        for (int r = 0; r < GF_ROWS; ++r) {
          if (r0 + r < rows) v[r] = src[(size_t)(r0 + r) * n4];
          else v[r] = f4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int r = 0; r < GF_ROWS; ++r) s += v[r];
      }
      *dst = *dst + s;
    }
    return;
  }
  if (ngroups == 1) {
    // single row group (no atomics into dst): thread t owns the 4 consecutive elements 4t .. 4t+3 of the tile, so
    // every row is one 16-byte load per lane (n % 4 == 0 and 16-byte aligned rows, make_grad_finish_table). The
    // table's pointers are cast to the global address space: as generic pointers they compiled to flat loads.
    typedef f4v __attribute__((address_space(1))) gf4;
    const int i = tile * 4 * NT + 4 * threadIdx.x;
    if (i >= g.n) return;
    gf4* src = (gf4*)(g.src + i);
    gf4* dst = (gf4*)(g.dst + i);
    const int n4 = g.n >> 2;
    f4v v[GF_ROWS];
#pragma unroll
    for (int r = 0; r < GF_ROWS; ++r) {
      if (r < rows) v[r] = src[(size_t)r * n4];
      else v[r] = f4v{0.f, 0.f, 0.f, 0.f};
    }
    f4v s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < GF_ROWS; ++r) s += v[r];   // the same row order as the per-element form: identical sums
    if (g.mode == GF_REDUCE) {
#pragma unroll
      for (int r = 0; r < GF_ROWS; ++r)
        if (r < rows) src[(size_t)r * n4] = f4v{0.f, 0.f, 0.f, 0.f};
    }
    *dst = *dst + s;
    return;
  }
  const int r0 = rg * GF_ROWS;
  float v[GF_ROWS][4];
#pragma unroll
  for (int r = 0; r < GF_ROWS; ++r)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * NT;
      v[r][u] = (r0 + r < rows && i < g.n) ? g.src[(size_t)(r0 + r) * g.n + i] : 0.f;
    }
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int r = 0; r < GF_ROWS; ++r)
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] += v[r][u];
  if (g.mode == GF_REDUCE) {        // atomic replica rows: re-zero for the next step
#pragma unroll
    for (int r = 0; r < GF_ROWS; ++r)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (r0 + r < rows && i0 + u * NT < g.n) g.src[(size_t)(r0 + r) * g.n + i0 + u * NT] = 0.f;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + u * NT;
    if (i >= g.n) continue;
    if (ngroups == 1) g.dst[i] += s[u];
    else atomicAdd(&g.dst[i], s[u]);
  }
}

constexpr int ZS_CHUNK = 4 * NT;   // zero_spans: 16-byte stores per block per chunk

__global__ void zero_spans_kernel(const ZeroSpan* __restrict__ spans, BatchSelect bs, StepAdvance adv) {
  CFL_TS_GUARD;
  if (blockIdx.x == 0 && blockIdx.y == 0) {            // block-uniform: the barrier is safe
    if (bs.table != nullptr) {                         // any batch size (the 512^2 plan: ~1,100)
      const size_t row = (size_t)(*bs.cursor % bs.nb) * bs.B;
      for (int i = threadIdx.x; i < bs.B; i += NT) bs.idx[i] = bs.table[row + i];
    }
    if (adv.step != nullptr) {
      __syncthreads();                                 // every thread has read the cursor
      if (threadIdx.x == 0) {
        *adv.lr_t = adam_lr(adv.step, adv.lr, adv.b1, adv.b2);
        *adv.step += 1;
        if (bs.table != nullptr) *bs.cursor += 1;
      }
    }
  }
  // block x of span y zeroes the 16-KB chunks x, x + gridDim.x, ...: four 16-byte stores per thread per chunk, issued
  // back to back, through a global-address-space pointer (the table's generic pointer compiled to flat stores)
  typedef u4v __attribute__((address_space(1))) gu4;
  const ZeroSpan z = spans[blockIdx.y];
  gu4* p = (gu4*)z.p;
  const int64_t n = z.bytes >> 4;
  for (int64_t c = (int64_t)blockIdx.x * ZS_CHUNK; c < n; c += (int64_t)gridDim.x * ZS_CHUNK) {
#pragma unroll
    for (int u = 0; u < ZS_CHUNK / NT; ++u) {
      const int64_t i = c + u * NT + threadIdx.x;
      if (i < n) p[i] = u4v{0u, 0u, 0u, 0u};
    }
  }
}

int g_tune[TUNE_N] = {0};

}  // namespace

int cfl_tune(int key) { return key >= 0 && key < TUNE_N ? g_tune[key] : 0; }

static int g_det_host = 0;
int cfl_det_host() { return g_det_host; }
static int (*const g_det_up[])(int) = {cfl_det_upload_bn, cfl_det_upload_conv3x3, cfl_det_upload_conv3x3_deep,
                            cfl_det_upload_conv3x3_sk, cfl_det_upload_conv3x3_wgrad, cfl_det_upload_conv_igemm,
                            cfl_det_upload_conv_wgrad, cfl_det_upload_datagen, cfl_det_upload_dwconv,
                            cfl_det_upload_entry, cfl_det_upload_fp8, cfl_det_upload_head, cfl_det_upload_optim, cfl_det_upload_pool_add,
                            cfl_det_upload_pw, cfl_det_upload_pw_bwd, cfl_det_upload_sepconv};
// 1 if any TU's fixed-point overflow flag is raised (cleared by cfl_det_set), 0 if none, 3 on a copy error
int cfl_fx_overflow() {
  int any = 0;
  for (auto f : g_det_up) {
    const int r = f(-1);
    if (r == 3) return 3;
    any |= r;
  }
  return any;
}
int cfl_det_set(int v) {
  v = v ? 1 : 0;
  int (*const up[])(int) = {cfl_det_upload_bn, cfl_det_upload_conv3x3, cfl_det_upload_conv3x3_deep,
                            cfl_det_upload_conv3x3_sk, cfl_det_upload_conv3x3_wgrad, cfl_det_upload_conv_igemm,
                            cfl_det_upload_conv_wgrad, cfl_det_upload_datagen, cfl_det_upload_dwconv,
                            cfl_det_upload_entry, cfl_det_upload_fp8, cfl_det_upload_head, cfl_det_upload_optim, cfl_det_upload_pool_add,
                            cfl_det_upload_pw, cfl_det_upload_pw_bwd, cfl_det_upload_sepconv};
  for (auto f : up)
    if (f(v)) return 3;
  g_det_host = v;
  return 0;
}
int cfl_ts_set(void* buf, int cap) {
  int (*const up[])(void*, int) = {cfl_ts_upload_bn, cfl_ts_upload_conv3x3, cfl_ts_upload_conv3x3_deep, cfl_ts_upload_conv3x3_sk, cfl_ts_upload_conv3x3_wgrad, cfl_ts_upload_conv_igemm, cfl_ts_upload_conv_wgrad, cfl_ts_upload_datagen, cfl_ts_upload_dwconv, cfl_ts_upload_entry, cfl_ts_upload_fp8, cfl_ts_upload_head, cfl_ts_upload_optim, cfl_ts_upload_pool_add, cfl_ts_upload_pw, cfl_ts_upload_pw_bwd, cfl_ts_upload_sepconv};
  for (auto f : up)
    if (f(buf, cap)) return 3;
  return 0;
}
void cfl_set_tune(int key, int value) {
  if (key >= 0 && key < TUNE_N) g_tune[key] = value;
}

int grad_finish_work(GradFinish* h_entries, int n_entries) {
  int w = 0;
  for (int i = 0; i < n_entries; ++i) {
    GradFinish& g = h_entries[i];
    const int rows = g.mode == GF_COPY || g.mode == GF_FIXED ? 1 : g.replicas;
    g.work_begin = w;
    w += ((g.n + 4 * NT - 1) / (4 * NT)) * (cfl_det_host() ? 1 : (rows + GF_ROWS - 1) / GF_ROWS);
  }
  return w;
}

int grad_finish(const GradFinish* d_entries, int n_entries, int total_work, hipStream_t st) {
  if (n_entries <= 0 || total_work <= 0) return 0;
  if (n_entries > NT) return 1;
  if (cfl_det_host()) hipLaunchKernelGGL(grad_finish_kernel<true>, dim3(total_work), dim3(NT), 0, st, d_entries, n_entries);
  else hipLaunchKernelGGL(grad_finish_kernel<false>, dim3(total_work), dim3(NT), 0, st, d_entries, n_entries);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int zero_spans(const ZeroSpan* d_spans, int n_spans, int64_t max_bytes, hipStream_t st, BatchSelect batch,
               StepAdvance adv) {
  if (n_spans <= 0) return batch.table != nullptr || adv.step != nullptr ? 1 : 0;   // nothing to launch them with
  if (batch.table != nullptr && (batch.B < 1 || batch.nb < 1)) return 1;
  if (adv.step != nullptr && adv.lr_t == nullptr) return 1;
  int64_t bx = (max_bytes / 16 + ZS_CHUNK - 1) / ZS_CHUNK;   // one chunk per block for spans up to 16 MB
  if (bx > 1024) bx = 1024;
  if (bx < 1) bx = 1;
  hipLaunchKernelGGL(zero_spans_kernel, dim3((int)bx, n_spans), dim3(NT), 0, st, d_spans, batch, adv);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int adam_update(const AdamParams& p, hipStream_t st) {
  if (p.n % 4) return 1;
  int64_t blocks = (p.n / 4 + NT - 1) / NT;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(adam_kernel, dim3((int)blocks), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int adam_step_done(int* step, hipStream_t st) {
  hipLaunchKernelGGL(step_done_kernel, dim3(1), dim3(1), 0, st, step);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int pack_weights(const float* flat, bf16_t* packed, const PackView* d_views, int n_views, int max_elems,
                 hipStream_t st, int* step, int* cursor) {
  int bx = (max_elems + NT - 1) / NT;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(pack_kernel, dim3(bx, n_views), dim3(NT), 0, st, flat, packed, d_views, step, cursor);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int opt_step(const OptParams& p, hipStream_t st) {
  if (p.n_items <= 0 || (!p.lr_t && (!p.ticket || !p.step)) || (p.lr_t && (p.step || p.cursor))) return 1;
  if (cfl_tune(TUNE_OPT_SCALAR)) hipLaunchKernelGGL(opt_step_kernel<false>, dim3(p.n_items), dim3(NT), 0, st, p);
  else hipLaunchKernelGGL(opt_step_kernel<true>, dim3(p.n_items), dim3(NT), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int fill_f32(float* p, float v, int64_t n, hipStream_t st) {
  int64_t blocks = (n + NT - 1) / NT;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(fill_kernel, dim3((int)(blocks < 1 ? 1 : blocks)), dim3(NT), 0, st, p, v, n);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int gather_rows_u8(const uint8_t* src, const int32_t* idx, uint8_t* dst, int rows, int64_t row_bytes,
                   hipStream_t st) {
  int bx = (int)((row_bytes + NT - 1) / NT);
  if (bx > 64) bx = 64;
  hipLaunchKernelGGL(gather_rows_kernel, dim3(bx, rows), dim3(NT), 0, st, src, idx, dst, rows, row_bytes);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_optim(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_optim(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
