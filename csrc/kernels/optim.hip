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

__global__ __launch_bounds__(NT) void adam_kernel(AdamParams p) {
  const int t = *p.step + 1;
  const float lr_t = p.lr * sqrtf(1.f - powf(p.b2, (float)t)) / (1.f - powf(p.b1, (float)t));
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
      mp[j] = p.b1 * mp[j] + (1.f - p.b1) * gp[j];
      vp[j] = p.b2 * vp[j] + (1.f - p.b2) * gp[j] * gp[j];
      wp[j] -= lr_t * mp[j] / (sqrtf(vp[j]) + p.eps);
    }
    reinterpret_cast<float4*>(p.p)[i] = w;
    reinterpret_cast<float4*>(p.m)[i] = m;
    reinterpret_cast<float4*>(p.v)[i] = v;
  }
}

__global__ void step_done_kernel(int* step) { *step += 1; }

__global__ __launch_bounds__(NT) void pack_kernel(const float* flat, bf16_t* packed, const PackView* views,
                                                  int* step, int* cursor) {
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

__global__ void fill_kernel(float* p, float v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) p[i] = v;
}

__global__ void gather_rows_kernel(const uint8_t* src, const int32_t* idx, uint8_t* dst, int rows, int64_t row_bytes) {
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

__global__ __launch_bounds__(NT) void grad_finish_kernel(const GradFinish* __restrict__ e, int n_entries) {
  // entry of this block: entries are sorted by work_begin; count how many begin at or before blockIdx.x
  const int wb = threadIdx.x < n_entries ? e[threadIdx.x].work_begin : 0x7fffffff;
  const int k = __syncthreads_count(wb <= (int)blockIdx.x) - 1;
  const GradFinish g = e[k];
  const int rows = g.mode == GF_COPY ? 1 : g.replicas;
  const int ngroups = (rows + GF_ROWS - 1) / GF_ROWS;
  const int local = blockIdx.x - g.work_begin;
  const int tile = local / ngroups, rg = local - tile * ngroups;
  const int i0 = tile * 4 * NT + threadIdx.x;
  if (g.mode == GF_COPY) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * NT < g.n) g.dst[i0 + u * NT] = g.src[i0 + u * NT];
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

__global__ void zero_spans_kernel(const ZeroSpan* __restrict__ spans, BatchSelect bs) {
  if (bs.table != nullptr && blockIdx.x == 0 && blockIdx.y == 0) {   // any batch size (the 512^2 plan: ~1,100)
    const size_t row = (size_t)(*bs.cursor % bs.nb) * bs.B;
    for (int i = threadIdx.x; i < bs.B; i += NT) bs.idx[i] = bs.table[row + i];
  }
  const ZeroSpan z = spans[blockIdx.y];
  uint4* p = reinterpret_cast<uint4*>(z.p);
  const int64_t n = z.bytes >> 4;
  for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
    p[i] = make_uint4(0, 0, 0, 0);
}

int g_tune[TUNE_N] = {0};

}  // namespace

int cfl_tune(int key) { return key >= 0 && key < TUNE_N ? g_tune[key] : 0; }
void cfl_set_tune(int key, int value) {
  if (key >= 0 && key < TUNE_N) g_tune[key] = value;
}

int grad_finish_work(GradFinish* h_entries, int n_entries) {
  int w = 0;
  for (int i = 0; i < n_entries; ++i) {
    GradFinish& g = h_entries[i];
    const int rows = g.mode == GF_COPY ? 1 : g.replicas;
    g.work_begin = w;
    w += ((g.n / 4 + NT - 1) / NT) * ((rows + GF_ROWS - 1) / GF_ROWS);
  }
  return w;
}

int grad_finish(const GradFinish* d_entries, int n_entries, int total_work, hipStream_t st) {
  if (n_entries <= 0 || total_work <= 0) return 0;
  if (n_entries > NT) return 1;
  hipLaunchKernelGGL(grad_finish_kernel, dim3(total_work), dim3(NT), 0, st, d_entries, n_entries);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int zero_spans(const ZeroSpan* d_spans, int n_spans, int64_t max_bytes, hipStream_t st, BatchSelect batch) {
  if (n_spans <= 0) return 0;
  if (batch.table != nullptr && (batch.B < 1 || batch.nb < 1)) return 1;
  int64_t bx = (max_bytes / 16 + NT - 1) / NT;
  if (bx > 1024) bx = 1024;
  if (bx < 1) bx = 1;
  hipLaunchKernelGGL(zero_spans_kernel, dim3((int)bx, n_spans), dim3(NT), 0, st, d_spans, batch);
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
