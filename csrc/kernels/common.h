// Shared device helpers for the gfx950 (CDNA4) kernels: bf16 bit conversions, vector types, wave64 reductions.
//
// Conventions used by every kernel in csrc/kernels:
//   * activations are NHWC bf16 stored as uint16_t (RNE rounding, NaN preserved);
//   * accumulation, BN statistics, gradients of weights and the optimizer are fp32;
//   * wave = 64 lanes; block sizes are multiples of 64;
//   * no 64-bit integer division in any hot loop (it lowers to a ~100-instruction sequence on CDNA): NHWC
//     elementwise kernels walk whole rows (b*H + h) per block and split a row into (pixel, 8-channel group)
//     items with shifts - the channel-group count C/8 is a power of two for every layer of the network;
//   * launchers take a hipStream_t and never allocate / synchronise (graph-capture safe).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CFL_DEVICE __device__ __forceinline__

typedef uint16_t bf16_t;
typedef short s8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

CFL_DEVICE float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// fp32 -> bf16 round-to-nearest-even with gfx950's v_cvt_pk_bf16_f32 (one instruction per pair, NaN stays NaN)
// instead of the ~5-op integer rounding sequence: bf16 packing is a large share of the VALU work of every
// memory-bound epilogue / elementwise kernel.
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

CFL_DEVICE uint32_t pack2bf(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

CFL_DEVICE bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }

// 8 bf16 <-> 8 float through one 16-byte vector
CFL_DEVICE void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

CFL_DEVICE uint4 pack8(const float* f) {
  return make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
}

CFL_DEVICE void load8(const bf16_t* p, float* f) { unpack8(*reinterpret_cast<const uint4*>(p), f); }

typedef short s2v_ __attribute__((ext_vector_type(2)));

// two bf16 (one dword of a staged chunk) -> max(a * x + b, lo) in bf16, with one packed fp32 FMA, the hardware bf16
// pack and a packed signed 16-bit max: every negative bf16 is a negative int16, so max with 0 is the exact ReLU and
// max with 0x8000 (the int16 minimum) the identity. lo: 0 (ReLU) or 0x80008000u (none), a = 1 / b = 0 without a BN.
CFL_DEVICE uint32_t xform2(uint32_t w, f32x2_t a, f32x2_t b, uint32_t lo) {
  const f32x2_t x = {__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
  const f32x2_t y = __builtin_elementwise_fma(a, x, b);
  const s2v_ r = __builtin_elementwise_max(__builtin_bit_cast(s2v_, __builtin_convertvector(y, bf16x2_t)),
                                           __builtin_bit_cast(s2v_, lo));
  return __builtin_bit_cast(uint32_t, r);
}
// 8 channels (a 16-byte chunk) through xform2, then AND-masked (m = 0 zeroes padding exactly)
CFL_DEVICE uint4 xform8(const uint4& v, const float* a, const float* b, uint32_t lo, uint32_t m) {
  return make_uint4(xform2(v.x, f32x2_t{a[0], a[1]}, f32x2_t{b[0], b[1]}, lo) & m,
                    xform2(v.y, f32x2_t{a[2], a[3]}, f32x2_t{b[2], b[3]}, lo) & m,
                    xform2(v.z, f32x2_t{a[4], a[5]}, f32x2_t{b[4], b[5]}, lo) & m,
                    xform2(v.w, f32x2_t{a[6], a[7]}, f32x2_t{b[6], b[7]}, lo) & m);
}

// x / D for small non-negative x as one full-rate 24-bit multiply and a shift; div_small_ok<D, N>() checks it for
// every x < N at compile time (static_assert at each use)
template <int D>
constexpr uint32_t div_magic16() { return (65536u + D - 1) / D; }
template <int D, int N>
constexpr bool div_small_ok() {
  for (int x = 0; x < N; ++x)
    if ((int)((x * div_magic16<D>()) >> 16) != x / D) return false;
  return true;
}
template <int D>
CFL_DEVICE int div_small(int x) { return (int)(__umul24((unsigned)x, div_magic16<D>()) >> 16); }

// Raw buffer access: a wave-uniform resource (base, byte range) in scalar registers, 32-bit per-lane byte offsets and
// a scalar offset; an offset past the range (CFL_OOB) reads 0. The halo / row loaders use these instead of 64-bit
// per-lane address math.
constexpr uint32_t CFL_OOB = 0x80000000u;
CFL_DEVICE __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
CFL_DEVICE uint4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const u4v v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
  return make_uint4(v.x, v.y, v.z, v.w);
}

CFL_DEVICE void load_f8(const float* p, float* f) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// 8 floats from p when cond, else 8 copies of dflt. Written with float4 values (not a branch over array stores) so
// the two paths merge as register phis: a branch-dependent store into a private array makes the compiler keep the
// array in scratch memory.
CFL_DEVICE void load_f8_or(const float* p, bool cond, float dflt, float* f) {
  float4 a = make_float4(dflt, dflt, dflt, dflt), b = a;
  if (cond) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}

// XCD-aware block order. Workgroups are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8), and each
// XCD has its own L2: blocks that share input rows (halo tiles, neighbouring rows, the N-blocks of one M-tile)
// should sit on the same XCD. This maps the dispatch index to a logical index such that every XCD receives one
// contiguous range of logical indices (a bijection on [0, n)).
CFL_DEVICE int xcd_swizzle(int b, int n) {
  const int q = n >> 3, r = n & 7;
  const int x = b & 7, i = b >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// logical linear block index of a 3-D grid under xcd_swizzle
CFL_DEVICE int xcd_block_linear() {
  const int lin = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  return xcd_swizzle(lin, gridDim.x * gridDim.y * gridDim.z);
}

// v + (v of lane ^ o) for o in {1, 2, 4, 8, 16, 32} without the LDS crossbar: DPP lane moves within a 16-lane row
// (quad_perm, row_mirror, row_half_mirror; xor 4 / 8 as two of them) and gfx950's v_permlane16 / 32_swap across rows
// (swap(v, v) leaves v_i and v_(i^16) in the two results: their sum is v_i + v_(i^16) in every lane). The value in
// every lane is bit-identical to `v + __shfl_xor(v, o, 64)` (the partners are the same, fp add commutes); o must
// fold to a constant (unrolled loops). __shfl_xor was one ds_bpermute - an LDS round trip - per step: the BN
// statistics / wgrad reductions of the kernel epilogues ran hundreds of them per block.
template <int CTRL>
CFL_DEVICE float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
CFL_DEVICE float xor_add(float v, int o) {
  constexpr int QP_1032 = 0xB1, QP_2301 = 0x4E, QP_3210 = 0x1B, ROW_MIRROR = 0x140, ROW_HALF_MIRROR = 0x141;
  if (o == 1) return v + dppf<QP_1032>(v);
  if (o == 2) return v + dppf<QP_2301>(v);
  if (o == 4) return v + dppf<ROW_HALF_MIRROR>(dppf<QP_3210>(v));
  if (o == 8) return v + dppf<ROW_HALF_MIRROR>(dppf<ROW_MIRROR>(v));
  const unsigned u = __builtin_bit_cast(unsigned, v);
  if (o == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
  }
  const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

// the double form of xor_add: both 32-bit halves moved by the same lane permutation (bit-identical to
// v + __shfl_xor(v, o, 64) on a double)
template <int CTRL>
CFL_DEVICE double dppd(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)u, CTRL, 0xF, 0xF, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
CFL_DEVICE double xor_add(double v, int o) {
  constexpr int QP_1032 = 0xB1, QP_2301 = 0x4E, QP_3210 = 0x1B, ROW_MIRROR = 0x140, ROW_HALF_MIRROR = 0x141;
  if (o == 1) return v + dppd<QP_1032>(v);
  if (o == 2) return v + dppd<QP_2301>(v);
  if (o == 4) return v + dppd<ROW_HALF_MIRROR>(dppd<QP_3210>(v));
  if (o == 8) return v + dppd<ROW_HALF_MIRROR>(dppd<ROW_MIRROR>(v));
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const auto l = o == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                         : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h = o == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                         : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const double d0 = __builtin_bit_cast(double, ((unsigned long long)(unsigned)h[0] << 32) | (unsigned)l[0]);
  const double d1 = __builtin_bit_cast(double, ((unsigned long long)(unsigned)h[1] << 32) | (unsigned)l[1]);
  return d0 + d1;
}

// the value of lane ^ 16 (an exchange, not a sum): v_permlane16_swap leaves the partner in the first result on
// odd rows (lanes 16-31, 48-63) and in the second on even rows
CFL_DEVICE unsigned xor16_get(unsigned v) {
  const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return (threadIdx.x & 16) ? (unsigned)r[0] : (unsigned)r[1];
}

CFL_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = xor_add(v, o);
  return v;
}

CFL_DEVICE float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum of one value per thread (blockDim.x multiple of 64, <= 1024). Result valid in thread 0.
template <int NT>
CFL_DEVICE float block_sum(float v, float* red /* >= NT/64 floats of LDS */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < NT / 64; ++i) t += red[i];
  }
  __syncthreads();
  return t;
}

CFL_DEVICE int imin(int a, int b) { return a < b ? a : b; }
CFL_DEVICE int imax(int a, int b) { return a > b ? a : b; }

// ---------------------------------------------------------------- deterministic reduction mode
// Every cross-block reduction of a training step - BN batch statistics, BN-backward node sums, weight-gradient
// replica rows, the head's dW / db - is a float atomicAdd by default: the total depends on the order in which the
// blocks' atomics arrive, so two replays of one step differ in the last bits. In deterministic mode
// (CFL_DETERMINISTIC=1, models/engine.py) each of these atomics adds a 64-bit fixed-point integer instead,
// llrint(v * 2^s): integer addition is associative, so the totals and everything computed from them are bitwise
// reproducible. The reduction buffers then hold int64 elements at the SAME element indices (twice the bytes: the
// engine allocates them so), and their consumers sum replica rows as integers and convert once. Scales (|total|
// bound per element; resolution):
//   CFL_FX_S0 = 2^24  BN sums of the (bf16-rounded) layer outputs       (< 5.5e11; 6e-8)
//   CFL_FX_S1 = 2^16  BN sums of their squares                           (< 1.4e14; 1.5e-5)
//   CFL_FX_G  = 2^40  BN-backward node sums, weight gradients, head dW   (< 8.4e6;  9.1e-13)
// The flag is each translation unit's constant g_cfl_det (set through cfl_det_set() in every TU, launch.h, before
// any graph capture). The host copy (cfl_det_host) sizes grad_finish's work split.
namespace {
__constant__ int g_cfl_det;
__device__ unsigned int g_cfl_fx_ovf;   // set when a fixed-point add fell outside +-2^62 (clamped)
}
#define CFL_FX_S0 16777216.0
#define CFL_FX_S1 65536.0
#define CFL_FX_G 1099511627776.0
CFL_DEVICE bool cfl_det() { return g_cfl_det != 0; }
// element i of a reduction buffer += v: a float atomic, or (deterministic) an int64 fixed-point atomic at `scale`
// A fixed-point add beyond +-2^62 (a partial sum past the documented bounds, or a NaN / inf) would make the int64
// conversion undefined and the total silently wrong: it is clamped (NaN -> 0) and the TU's overflow flag raised
// (read by cfl_fx_overflow(); the engine checks it after deterministic-mode rounds).
CFL_DEVICE void red_add(float* buf, size_t i, float v, double scale) {
  if (cfl_det()) {
    constexpr double kFxMax = 4611686018427387904.0;     // 2^62
    double q = (double)v * scale;
    if (!(fabs(q) <= kFxMax)) {
      q = q > 0.0 ? kFxMax : (q < 0.0 ? -kFxMax : 0.0);
      atomicOr(&g_cfl_fx_ovf, 1u);
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(buf) + i, (unsigned long long)__double2ll_rn(q));
  } else {
    atomicAdd(buf + i, v);
  }
}
// raw int64 element i of a deterministic-mode reduction buffer
CFL_DEVICE long long red_raw(const float* buf, size_t i) { return reinterpret_cast<const long long*>(buf)[i]; }
CFL_DEVICE float red_fx(long long q, double scale) { return (float)((double)q / scale); }
// scale of the epilogue sums of a BN layer's statistics (st 0: sums, 1: sums of squares) or of node sums
CFL_DEVICE double red_scale(bool stats, int st) { return stats ? (st ? CFL_FX_S1 : CFL_FX_S0) : CFL_FX_G; }
// v >= 0: set this TU's mode flag and clear its overflow flag (0 ok, 3 error); v < 0: read the overflow flag
// (0 clear, 1 raised, 3 error)
static inline int cfl_det_upload(int v) {
  unsigned int f = 0;
  if (v < 0)
    return hipMemcpyFromSymbol(&f, HIP_SYMBOL(g_cfl_fx_ovf), sizeof(f)) == hipSuccess ? (f ? 1 : 0) : 3;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_cfl_fx_ovf), &f, sizeof(f)) != hipSuccess) return 3;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_cfl_det), &v, sizeof(int)) == hipSuccess ? 0 : 3;
}

// Block timeline instrumentation (tools/block_timeline.py): with a buffer installed (cfl_ts_set, launch.h), every
// instrumented kernel's blocks record [dispatch, retire] s_memrealtime stamps (100 MHz, chip-wide) at
// buf[2 * linear block id]; off (null buffer) it costs one constant load and a branch per block.
struct CflTs {
  unsigned long long* buf;
  int cap;                 // blocks
};
namespace {
__constant__ CflTs g_cfl_ts;
}
CFL_DEVICE unsigned long long cfl_ts_now() { return __builtin_amdgcn_s_memrealtime(); }
// RAII: the retire stamp is taken when thread 0 leaves the kernel by any path (no barrier: an early return of part of
// a block must not deadlock); wave 0's exit stands for the block's
struct CflTsGuard {
  unsigned long long t0;
  __device__ CflTsGuard() : t0(cfl_ts_now()) {}
  __device__ ~CflTsGuard() {
    if (g_cfl_ts.buf == nullptr || threadIdx.x != 0) return;
    const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (b < g_cfl_ts.cap) {
      g_cfl_ts.buf[2 * b] = t0;
      g_cfl_ts.buf[2 * b + 1] = cfl_ts_now();
    }
  }
};
#define CFL_TS_GUARD CflTsGuard cfl_ts_guard_
// phase stamp k (0 or 1) of this block, thread 0, at buf[2 * (cap / 2 + linear block id) + k]: the upper half of
// the buffer holds two in-kernel phase boundaries per block (tools/gpu phase probes; cap must cover twice the grid)
CFL_DEVICE void cfl_ts_phase(int k) {
  if (g_cfl_ts.buf == nullptr || threadIdx.x != 0) return;
  const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if (b < g_cfl_ts.cap / 2) g_cfl_ts.buf[2 * (g_cfl_ts.cap / 2 + b) + k] = cfl_ts_now();
}
static inline int cfl_ts_upload(void* buf, int cap) {
  const CflTs t{reinterpret_cast<unsigned long long*>(buf), cap};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_cfl_ts), &t, sizeof(t)) == hipSuccess ? 0 : 3;
}

// log2 of a power of two (host or device)
__host__ __device__ inline int ilog2(int x) {
  int l = 0;
  while ((1 << l) < x) ++l;
  return l;
}

// v[i] + the v[i] of every lane congruent to this one mod G (G a runtime power of two): strides 4..32 on the
// constant-stride DPP / permlane reductions (xor_add), anything else on the LDS shuffle
template <int N>
CFL_DEVICE void reduce_stride(float (&v)[N], int G) {
  auto red = [&](auto g_c) __attribute__((always_inline)) {
    constexpr int GC = decltype(g_c)::value;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
      for (int o = GC; o < 64; o <<= 1) v[i] = xor_add(v[i], o);
  };
  switch (G) {
    case 4: red(std::integral_constant<int, 4>{}); break;
    case 8: red(std::integral_constant<int, 8>{}); break;
    case 16: red(std::integral_constant<int, 16>{}); break;
    case 32: red(std::integral_constant<int, 32>{}); break;
    default:
#pragma unroll
      for (int i = 0; i < N; ++i)
        for (int o = G; o < 64; o <<= 1) v[i] += __shfl_xor(v[i], o, 64);
  }
}

// Per-channel sums of 8-channel vectors held by a 256-thread block where thread t owns channel group t % G:
// reduce the wave's lanes that share the group (stride G), then the 4 waves through LDS, then one atomic per
// channel into buf[off + 0..C) and (if NS == 2) buf[off + C..2C) (red_add: float, or int64 fixed point in the
// deterministic mode at the BN-statistics scales when `stats`, else the node-sum scale).
template <int NS>
CFL_DEVICE void block_channel_atomics(float (&s)[NS][8], int G, int C, float* buf, size_t off, bool stats,
                                      float (*red)[4][256]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, c0 = (threadIdx.x % G) * 8;
  // the lane stride is a runtime value: dispatched to a constant-stride DPP / permlane reduction per G (xor_add with
  // a runtime o measured slower than the LDS shuffle it replaces; other strides keep the shuffle)
  auto reduce = [&](auto g_c) __attribute__((always_inline)) {
    constexpr int GC = decltype(g_c)::value;
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int o = GC; o < 64; o <<= 1) s[k][j] = xor_add(s[k][j], o);
  };
  switch (G) {
    case 4: reduce(std::integral_constant<int, 4>{}); break;
    case 8: reduce(std::integral_constant<int, 8>{}); break;
    case 16: reduce(std::integral_constant<int, 16>{}); break;
    case 32: reduce(std::integral_constant<int, 32>{}); break;
    default:
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          for (int o = G; o < 64; o <<= 1) s[k][j] += __shfl_xor(s[k][j], o, 64);
  }
  if (lane < G) {
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[k][wid][c0 + j] = s[k][j];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < NS * C; e += 256) {
    const int k = e / C, c = e - k * C;
    const float v = red[k][0][c] + red[k][1][c] + red[k][2][c] + red[k][3][c];
    red_add(buf, off + (size_t)k * C + c, v, red_scale(stats, k));
  }
}

// BN per-channel coefficients produced by bn_finalize (csrc/kernels/bn.hip): 4 rows of C floats
//   ab[0*C + c] = scale a = gamma * rstd     ab[1*C + c] = shift b = beta - mean * a
//   ab[2*C + c] = mean                       ab[3*C + c] = rstd
// A "transform" applied on load to a raw conv output y is  relu?(a*y + b).
struct InXform {
  const float* ab;   // nullptr = identity
  int C;             // channel count of ab
  int relu;          // apply ReLU after the affine (or alone when ab == nullptr)
};

// Coefficients of a fused BN-node epilogue (launch.h BnNodeEpi) for 8 channels c0..c0+7 of C.
struct NodeCoef {
  float a[8], b[8], mean[8], rstd[8];
};

CFL_DEVICE void node_coef_load(const float* ab, int C, int c0, NodeCoef& k) {
  load_f8(ab + c0, k.a);
  load_f8(ab + C + c0, k.b);
  load_f8(ab + 2 * C + c0, k.mean);
  load_f8(ab + 3 * C + c0, k.rstd);
}

// g = mask * o for 8 bf16 values o (exact: o is already bf16, masked lanes become 0); accumulates the BN-backward
// sums from the stored g. yp points at the node input y for the same pixel / channels.
CFL_DEVICE uint4 node_epi(uint4 o_bits, const bf16_t* yp, const NodeCoef& k, int relu, float* s0, float* s1) {
  float o[8], y[8];
  unpack8(o_bits, o);
  load8(yp, y);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float g = (!relu || fmaf(k.a[j], y[j], k.b[j]) > 0.f) ? o[j] : 0.f;
    o[j] = g;
    s0[j] += g;
    s1[j] += g * (y[j] - k.mean[j]) * k.rstd[j];
  }
  return pack8(o);
}

// BatchNorm backward "apply" folded into the operand load of the data-gradient conv that consumes it (launch.h
// ConvParams::bwd). The conv input x is then the gradient g w.r.t. the BN output, and the operand is
//   dx = a * (g - s0 / M - xhat * s1 / M),  xhat = (y - mean) * rstd
// with s0 = sum(g), s1 = sum(g * xhat) the node sums (replica rows accumulated by the producer of g). dx is also
// stored (each input pixel once) for the weight gradient that reads it later, and one block writes dgamma = s1 /
// dbeta = s0. This replaces the separate bn_bwd_apply pass: one launch and one write + read of dx fewer.
struct BnBwdIn {
  const bf16_t* y;     // raw BN input (same layout as x); nullptr = off
  const float* ab;     // 4 rows: a, b, mean, rstd
  const float* sums;   // [reps][2][C]
  int reps;            // 1..16
  float invM;          // 1 / pixels per channel
  bf16_t* dx;          // side store of dx (nullptr = none)
  float* dgamma;       // flat-grad slots, written (not accumulated) by one block; nullptr = none
  float* dbeta;
};
#define BNB_MAX_C 256
#define BNB_MAX_REPS 16

// One element of the BN-backward apply (shared by bn_bwd_apply and the folded conv operands: same arithmetic,
// bit-identical results).
CFL_DEVICE float bnb_apply(float g, float y, float a, float mean, float rstd, float k1, float k2) {
  const float xhat = (y - mean) * rstd;
  return a * (g - k1 - xhat * k2);
}

// Block prologue of a BN-backward consumer (NTH threads; C <= BNB_MAX_C, C % 8 == 0): sums the replica rows of the
// node sums - every load of the block issued in one round - and stages the per-channel coefficients in LDS:
//   co[0..C) a, co[C..2C) mean, co[2C..3C) rstd, co[3C..4C) k1 = s0/M, co[4C..5C) k2 = s1/M
// `part`: NTH floats of LDS. write_grads: this block writes dgamma / dbeta. Ends with a barrier.
template <int NTH>
CFL_DEVICE void bnb_prologue(const BnBwdIn& q, int C, float* co, float* part, bool write_grads) {
  const int C2 = 2 * C, t = threadIdx.x;
  const int reps = q.reps > 1 ? q.reps : 1;
  float am = 0.f, mm = 0.f, rm = 0.f;
  const bool coef = t < C;
  if (coef) {                                   // BN coefficients: issued with the replica loads below
    am = q.ab[t];
    mm = q.ab[2 * C + t];
    rm = q.ab[3 * C + t];
  }
  float s_lo = 0.f, s_hi = 0.f;                 // sums of element t (and t + NTH when C2 > NTH)
  const bool det = cfl_det();                   // int64 fixed-point rows: summed as integers, converted once
  // every replica-row load is unconditional (row index clamped into range, rows past reps weighted 0) so all of
  // them issue back to back and the block waits ONE memory round trip: guarded per-row loads compiled to a branch
  // and a full wait per row (16 serial round trips at reps 16, measured as most of a block's fixed cost)
  const int rlast = reps - 1;
  if (C2 <= NTH) {
    const int per = NTH / C2, e = t % C2, j = t / C2;
    float v = 0.f;
    long long vi = 0;
    if (det) {
      long long x[BNB_MAX_REPS];
#pragma unroll
      for (int k = 0; k < BNB_MAX_REPS; ++k) x[k] = red_raw(q.sums, (size_t)imin(j + k * per, rlast) * C2 + e);
#pragma unroll
      for (int k = 0; k < BNB_MAX_REPS; ++k) vi += j + k * per < reps ? x[k] : 0ll;
    } else {
      float x[BNB_MAX_REPS];
#pragma unroll
      for (int k = 0; k < BNB_MAX_REPS; ++k) x[k] = q.sums[(size_t)imin(j + k * per, rlast) * C2 + e];
#pragma unroll
      for (int k = 0; k < BNB_MAX_REPS; ++k)
        if (j + k * per < reps) v += x[k];
    }
    part[t] = det ? red_fx(vi, CFL_FX_G) : v;
    __syncthreads();
    if (t < C2)
      for (int k = 0; k < per; ++k) s_lo += part[k * C2 + t];
  } else {                                      // C2 == 2 * NTH at most (C <= 256, NTH = 256)
    if (det) {
      long long xl[BNB_MAX_REPS], xh[BNB_MAX_REPS], lo = 0, hi = 0;
#pragma unroll
      for (int r = 0; r < BNB_MAX_REPS; ++r) {
        xl[r] = red_raw(q.sums, (size_t)imin(r, rlast) * C2 + t);
        xh[r] = red_raw(q.sums, (size_t)imin(r, rlast) * C2 + t + NTH);
      }
#pragma unroll
      for (int r = 0; r < BNB_MAX_REPS; ++r)
        if (r < reps) {
          lo += xl[r];
          hi += xh[r];
        }
      s_lo = red_fx(lo, CFL_FX_G);
      s_hi = red_fx(hi, CFL_FX_G);
    } else {
      float xl[BNB_MAX_REPS], xh[BNB_MAX_REPS];
#pragma unroll
      for (int r = 0; r < BNB_MAX_REPS; ++r) {
        xl[r] = q.sums[(size_t)imin(r, rlast) * C2 + t];
        xh[r] = q.sums[(size_t)imin(r, rlast) * C2 + t + NTH];
      }
#pragma unroll
      for (int r = 0; r < BNB_MAX_REPS; ++r)
        if (r < reps) {
          s_lo += xl[r];
          s_hi += xh[r];
        }
    }
  }
  // element e < C is s0[e], e >= C is s1[e - C]
  if (t < C2) {
    co[3 * C + t] = s_lo * q.invM;              // k1 for t < C, k2 (= co[4C + t - C]) for t >= C
    if (write_grads) {
      if (t < C) { if (q.dbeta) q.dbeta[t] = s_lo; }
      else if (q.dgamma) q.dgamma[t - C] = s_lo;
    }
  }
  if (C2 > NTH) {
    co[3 * C + t + NTH] = s_hi * q.invM;
    if (write_grads && q.dgamma) q.dgamma[t + NTH - C] = s_hi;
  }
  if (coef) {
    co[t] = am;
    co[C + t] = mm;
    co[2 * C + t] = rm;
  }
  __syncthreads();
}

// dx of 8 channels c0..c0+7 from 8 g and 8 y values (coefficients from bnb_prologue's LDS block)
// (co 16-byte aligned, C and c0 multiples of 8: the five coefficient rows are read as 16-byte vectors - 10 LDS reads
// per call instead of 40 scalar ones)
// Global -> LDS copy of NP 16-byte pieces (piece e: src(e) -> dst(e), pointers) by an NTH-thread block, the loads of
// up to G pieces per thread issued before their stores. A strided `for (e = tid; e < NP; e += NTH)` copy compiled
// to one full memory round trip per iteration - measured as most of the 3-6 us per-block prologues of the streaming
// kernels (tools/block_timeline.py phases, profiles/r6_misc).
template <int NTH, int NP, int G = 8, typename Src, typename Dst>
CFL_DEVICE void stage16(const Src& src, const Dst& dst) {
  constexpr int PT = (NP + NTH - 1) / NTH;
  const int tid = threadIdx.x;
#pragma unroll
  for (int i0 = 0; i0 < PT; i0 += G) {
    u4v r[G];
#pragma unroll
    for (int i = 0; i < G; ++i)
      if (i0 + i < PT) r[i] = *reinterpret_cast<const u4v*>(src(imin(tid + (i0 + i) * NTH, NP - 1)));
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int e = tid + (i0 + i) * NTH;
      if (i0 + i < PT && e < NP) *reinterpret_cast<u4v*>(dst(e)) = r[i];
    }
  }
}

// The same copy split in two: load() issues every piece (kept in registers), store() writes them - so the loads can
// be issued together with other prologue loads ahead of an unrelated wait
template <int NTH, int NP>
struct Stage16 {
  static constexpr int PT = (NP + NTH - 1) / NTH;
  u4v r[PT];
  template <typename Src>
  CFL_DEVICE void load(const Src& src) {
#pragma unroll
    for (int i = 0; i < PT; ++i) r[i] = *reinterpret_cast<const u4v*>(src(imin((int)threadIdx.x + i * NTH, NP - 1)));
  }
  template <typename Dst>
  CFL_DEVICE void store(const Dst& dst) const {
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int e = threadIdx.x + i * NTH;
      if (e < NP) *reinterpret_cast<u4v*>(dst(e)) = r[i];
    }
  }
};

// The five coefficient vectors of channels c0..c0+7 in registers, for callers that apply them to many pixels
// (pw_bwd.hip: a thread's channel group is fixed for the whole launch)
struct BnbCo8 {
  float a[8], mean[8], rstd[8], k1[8], k2[8];
};
CFL_DEVICE BnbCo8 bnb_co8(const float* co, int C, int c0) {
  BnbCo8 k;
  load_f8(co + c0, k.a);
  load_f8(co + C + c0, k.mean);
  load_f8(co + 2 * C + c0, k.rstd);
  load_f8(co + 3 * C + c0, k.k1);
  load_f8(co + 4 * C + c0, k.k2);
  return k;
}
CFL_DEVICE uint4 bnb_apply8(const uint4& gv, const uint4& yv, const BnbCo8& k) {
  float g[8], y[8], o[8];
  unpack8(gv, g);
  unpack8(yv, y);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bnb_apply(g[j], y[j], k.a[j], k.mean[j], k.rstd[j], k.k1[j], k.k2[j]);
  return pack8(o);
}
CFL_DEVICE uint4 bnb_apply8(const uint4& gv, const uint4& yv, const float* co, int C, int c0) {
  return bnb_apply8(gv, yv, bnb_co8(co, C, c0));
}

// One half-resolution pixel of a PoolJoinEpi (launch.h) from the four bf16 conv outputs of its 2x2 block and the
// (prefetched) mask source vv, addend av (has_add) and sums source syv (has_sy), in node_bwd's order
// (0 + masked((o00 + o01) + (o10 + o11)) + add, one rounding); accumulates the BN-backward sums from the rounded
// value (mean / rstd of the sab rows in mean8 / rstd8). Returns the stored bf16 vector.
CFL_DEVICE uint4 pool_join8(const uint4 (&o)[4], const uint4& vv, const uint4& av, const uint4& syv, bool has_add,
                            bool has_sy, const float* mean8, const float* rstd8, float* s0, float* s1) {
  float u[4][8], v[8], g[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) unpack8(o[q], u[q]);
  unpack8(vv, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    g[j] = 0.f;                                   // node_bwd's accumulation, bit for bit (signed zeros included)
    g[j] += v[j] > 0.f ? (u[0][j] + u[1][j]) + (u[2][j] + u[3][j]) : 0.f;
  }
  if (has_add) {
    float a[8];
    unpack8(av, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] += a[j];
  }
  const uint4 gv = pack8(g);
  if (has_sy) {
    float gr[8], y[8];
    unpack8(gv, gr);
    unpack8(syv, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s0[j] += gr[j];
      s1[j] += gr[j] * (y[j] - mean8[j]) * rstd8[j];
    }
  }
  return gv;
}

CFL_DEVICE float xform1(float v, const InXform& t, int c) {
  if (t.ab) v = fmaf(t.ab[c], v, t.ab[t.C + c]);
  if (t.relu) v = fmaxf(v, 0.f);
  return v;
}
