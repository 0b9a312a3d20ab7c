// Entry block Conv2D(32, 3, strides=2, padding="same") on the 3-channel image (client_fit_model.py:100).
// The kernels read the uint8 dataset rows of the batch through the index vector (batch assembly and the /255
// normalisation of client_fit_model.py:43 are folded into the load - no batch tensor is ever materialised).
// TF "same" at stride 2 pads bottom/right only. Cout == 32 runs on MFMA (K = 27 taps padded to 32, see the MFMA
// section below); the direct VALU kernels serve other widths.
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
  CFL_TS_GUARD;
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
  if (p.stats) {
    block_channel_atomics<2>(s, G, p.Cout, p.stats, (size_t)(blockIdx.x % STAT_REPLICAS) * 2 * p.Cout, true, red);
  }
}

// dW[ky][kx][ci][co] = sum_pix x[2oh+ky][2ow+kx][ci] * dy[pix][co]; blockIdx.y = ky, thread = (pixel, 8 outputs).
// The input row is staged in LDS once per output row; per-block sums go to one of `replicas` copies of dW.
__global__ __launch_bounds__(NT) void entry_wgrad_kernel(EntryParams p, int replicas) {
  CFL_TS_GUARD;
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
#pragma unroll
      for (int o = G; o < 64; o <<= 1) v = xor_add(v, o);
      acc[a][j] = v;
    }
  if (lane < G) {
#pragma unroll
    for (int a = 0; a < 9; ++a)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][a][c0 + j] = acc[a][j];
  }
  __syncthreads();
  const size_t ro = (size_t)((blockIdx.x + blockIdx.y * gridDim.x) % replicas) * 27 * p.Cout;
  for (int e = threadIdx.x; e < 9 * p.Cout; e += NT) {
    const int a = e / p.Cout, c = e - a * p.Cout;
    red_add(p.dw, ro + (ky * 9 + a) * p.Cout + c, red[0][a][c] + red[1][a][c] + red[2][a][c] + red[3][a][c],
            CFL_FX_G);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// MFMA forms for Cout == 32 (the network's entry width). A step covers ECH output pixels of one output row: the three
// input rows it reads (columns 2*ow0 .. 2*ow0 + 2*ECH) are staged as raw bytes in LDS with dword loads (zeros past the
// image's bottom / right edge = TF "same" padding), and every lane builds its MFMA operand straight from those
// bytes: the 27 taps (ky, kx, ci) of a pixel as the integers 0..255 - exact in bf16; the /255 goes onto the fp32
// accumulator - zero-padded to K = 32:
//   forward  y[pix][co]  = bias[co] + (1/255) * X[pix][0:32] . W[0:32][co]   (W rounded to bf16, held in registers)
//   wgrad    dW[tap][co] = (1/255) * sum_pix X[pix][tap] * dy[pix][co]      (the pixel reduction is the MFMA K axis;
//            the [pixel][channel] dy tile is read with the transposing ds_read_b64_tr_b16, as conv_wgrad.hip does)
// mfma_f32_16x16x32_bf16 lane maps: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col l&15], C[row 4(l>>4)+r][col l&15].
// The VALU kernels above stay for other widths (TUNE_ENTRY_ALGO=1 forces them): they are LDS-bandwidth bound, two
// 16-byte weight reads per 8 FMAs.
constexpr int ECH = 128;          // output pixels per step (4 waves x 32)
constexpr int ELD = 40;           // LDS row stride (bf16) of the [pixel][32] dy / y tiles (80-byte rows)
constexpr int ERB = 784;          // staged bytes per input row: (2 * ECH + 1) * 3 = 771, rounded up to 16
constexpr int EDW = ERB / 4;      // dwords per staged row

typedef short s4v_lds __attribute__((ext_vector_type(4)));
CFL_DEVICE s4v tr_read(const bf16_t* q) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((s4v_lds __attribute__((address_space(3)))*)(q));
}

// byte offset of tap T inside the staged [3][ERB] rows (relative to the pixel's column 2*px), or -1 for T >= 27
CFL_DEVICE int tap_off(int T) { return T < 27 ? (T / 9) * ERB + ((T / 3) % 3) * 3 + T % 3 : -1; }

// the three input rows of step (row = b*Ho + oh, first output column ow0): thread t holds dwords t, t + NT, t + 2NT
// of the [3][EDW] image (addresses clamped, loads unconditional)
CFL_DEVICE void rows_load(const EntryParams& p, int row, int ow0, uint32_t (&rv)[3]) {
  const int b = row / p.Ho, oh = row - b * p.Ho;
  const int rowbytes = p.S * 3;                       // multiple of 4 (S % 4 == 0)
  const uint8_t* img = p.images + (size_t)p.idx[b] * p.S * rowbytes;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int e = threadIdx.x + NT * k;
    const int r = e / EDW, byte = ow0 * 6 + (e - r * EDW) * 4;
    const int ih = 2 * oh + r;
    const bool ok = e < 3 * EDW && ih < p.S && byte < rowbytes;
    const uint32_t v = *reinterpret_cast<const uint32_t*>(img + (ok ? (size_t)ih * rowbytes + byte : 0));
    rv[k] = ok ? v : 0u;
  }
}

CFL_DEVICE void rows_store(uint8_t* sR, const uint32_t (&rv)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int e = threadIdx.x + NT * k;
    if (e < 3 * EDW) reinterpret_cast<uint32_t*>(sR)[e] = rv[k];
  }
}

// 8 staged bytes at sR + base + off[j] (off < 0: 0) as an MFMA operand of 8 bf16 integers
CFL_DEVICE s8v bytes_frag(const uint8_t* sR, const int (&off)[8], const int (&stride)[8], int base) {
  float f[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = off[j] < 0 ? 0.f : (float)sR[base + off[j] + stride[j]];
  return __builtin_bit_cast(s8v, u4v{pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]),
                                     pack2bf(f[6], f[7])});
}

__global__ __launch_bounds__(NT) void entry_fwd_mfma_kernel(EntryParams p, int nch, int steps) {
  CFL_TS_GUARD;
  __shared__ __attribute__((aligned(16))) uint8_t sR[2][3 * ERB];
  __shared__ __attribute__((aligned(16))) bf16_t sY[ECH][ELD];
  __shared__ float red[2][4][256];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  // B operand (fixed): lane holds output channel 16j + r16 at taps 8g .. 8g+7 (0 for the padding taps)
  s8v wv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int T = 8 * g + e;
      wv[j][e] = (short)f2bf(T < 27 ? p.w[T * 32 + 16 * j + r16] : 0.f);
    }
  // A operand: lane holds pixel 32*wid + 16i + r16 at taps 8g .. 8g+7
  int off[8], zero[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    off[e] = tap_off(8 * g + e);
    zero[e] = 0;
  }
  const float bias0 = p.bias[r16], bias1 = p.bias[16 + r16];
  float s[2][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[0][j] = s[1][j] = 0.f;
  uint32_t rv[3];
  int st = blockIdx.x;
  rows_load(p, st / nch, (st % nch) * ECH, rv);
  rows_store(sR[0], rv);
  __syncthreads();
  int buf = 0;
  for (; st < steps; st += gridDim.x) {
    const int nxt = st + gridDim.x;
    const bool more = nxt < steps;
    if (more) rows_load(p, nxt / nch, (nxt % nch) * ECH, rv);   // in flight during this step
    f4v acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const s8v a = bytes_frag(sR[buf], off, zero, 6 * (32 * wid + 16 * i + r16));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wv[j], f4v{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bf16_t* yr = &sY[32 * wid + 16 * i + 4 * g + r][r16];
        yr[0] = f2bf(fmaf(acc[i][0][r], 1.f / 255.f, bias0));
        yr[16] = f2bf(fmaf(acc[i][1][r], 1.f / 255.f, bias1));
      }
    __syncthreads();
    const int row = st / nch, ow0 = (st % nch) * ECH;
#pragma unroll
    for (int k = 0; k < 2; ++k) {       // 16-byte stores of 8 channels; channel group (tid & 3) fixed per thread
      const int e = tid + NT * k, px = e >> 2, cq = (e & 3) * 8;
      if (ow0 + px < p.Wo) {
        const uint4 v = *reinterpret_cast<const uint4*>(&sY[px][cq]);
        *reinterpret_cast<uint4*>(p.y + ((size_t)row * p.Wo + ow0 + px) * 32 + cq) = v;
        float f[8];
        unpack8(v, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[0][j] += f[j];
          s[1][j] += f[j] * f[j];
        }
      }
    }
    if (more) rows_store(sR[buf ^ 1], rv);
    __syncthreads();
    buf ^= 1;
  }
  if (p.stats) {
    block_channel_atomics<2>(s, 4, 32, p.stats, (size_t)(blockIdx.x % STAT_REPLICAS) * 64, true, red);
  }
}

// BWD: the entry BN's backward apply folded into the dy load (p.bwd; the bn_bwd_apply arithmetic, bit-identical):
// g and y are loaded together and dx = a * (g - s0/M - xhat * s1/M) is formed right before the LDS store, with this
// thread's 8 channels' coefficients held in registers; block 0 writes dgamma / dbeta. dx itself is never stored.
template <bool BWD>
__global__ __launch_bounds__(NT) void entry_wgrad_mfma_kernel(EntryParams p, int nch, int steps, int replicas) {
  CFL_TS_GUARD;
  __shared__ __attribute__((aligned(16))) uint8_t sR[2][3 * ERB];
  __shared__ __attribute__((aligned(16))) bf16_t sG[2][ECH][ELD];
  __shared__ float red[4][32 * 32];
  __shared__ __attribute__((aligned(16))) float sco[BWD ? 5 * 32 + NT : 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // this thread's dy channels (tid & 3) * 8 .. +7 (e & 3 below with e = tid + NT * k)
  float ca[8], cm[8], cr[8], k1[8], k2[8];
  if constexpr (BWD) {
    bnb_prologue<NT>(p.bwd, 32, sco, sco + 5 * 32, blockIdx.x == 0);
    const int c0 = (tid & 3) * 8;
    load_f8(sco + c0, ca);              // 16-byte LDS reads (scalar reads at an 8-float stride conflicted)
    load_f8(sco + 32 + c0, cm);
    load_f8(sco + 64 + c0, cr);
    load_f8(sco + 96 + c0, k1);
    load_f8(sco + 128 + c0, k2);
  }
  const int g = lane >> 4, r16 = lane & 15;
  // A operand (X^T): lane holds tap row 16i + r16 at pixels 32*wid + 8g + 0..7 (column stride 2 pixels = 6 bytes)
  int aoff[2][8], astr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    aoff[0][j] = tap_off(r16);
    aoff[1][j] = tap_off(16 + r16);
    astr[j] = 6 * j;
  }
  uint32_t rv[3];
  uint4 gv[2], yv[BWD ? 2 : 1];
  bool okv[2];
  auto load = [&](int s) {
    const int row = s / nch, ow0 = (s % nch) * ECH;
    rows_load(p, row, ow0, rv);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + NT * k, ow = ow0 + (e >> 2);
      const size_t off = ((size_t)row * p.Wo + ow) * 32 + (e & 3) * 8;
      okv[k] = ow < p.Wo;
      gv[k] = okv[k] ? *reinterpret_cast<const uint4*>(p.dy + off) : make_uint4(0, 0, 0, 0);
      if constexpr (BWD) yv[k] = okv[k] ? *reinterpret_cast<const uint4*>(p.bwd.y + off) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int b) {
    rows_store(sR[b], rv);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + NT * k;
      uint4 v = gv[k];
      if constexpr (BWD) {
        if (okv[k]) {                                  // pixels past the row stay zero
          float g[8], y[8], o[8];
          unpack8(v, g);
          unpack8(yv[k], y);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = bnb_apply(g[j], y[j], ca[j], cm[j], cr[j], k1[j], k2[j]);
          v = pack8(o);
        }
      }
      *reinterpret_cast<uint4*>(&sG[b][e >> 2][(e & 3) * 8]) = v;
    }
  };
  f4v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  int st = blockIdx.x;
  load(st);
  store(0);
  __syncthreads();
  // transposed dy reads: lane 4q + pq of each 16-lane group addresses row r0 (+4 for the upper half), columns
  // 16j + 4pq .. +3, and receives column 16j + (lane & 15) at pixels 32*wid + 8g + 0..7 (the MFMA K slice)
  const int q = r16 >> 2, pq = lane & 3;
  const int r0 = 32 * wid + 8 * g + q;
  const int pbase = 6 * (32 * wid + 8 * g);
  int buf = 0;
  for (; st < steps; st += gridDim.x) {
    const bool more = st + gridDim.x < steps;
    if (more) load(st + gridDim.x);
    s8v af[2], bg[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      af[i] = bytes_frag(sR[buf], aoff[i], astr, pbase);
      const s4v glo = tr_read(&sG[buf][r0][16 * i + 4 * pq]);
      const s4v ghi = tr_read(&sG[buf][r0 + 4][16 * i + 4 * pq]);
      bg[i] = s8v{glo[0], glo[1], glo[2], glo[3], ghi[0], ghi[1], ghi[2], ghi[3]};
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bg[j], acc[i][j], 0, 0, 0);
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // C: tap 16i + 4g + r, channel 16j + (lane & 15); the 4 waves' pixel slices summed through LDS
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wid][(16 * i + 4 * g + r) * 32 + 16 * j + r16] = acc[i][j][r];
  __syncthreads();
  const size_t ro = (size_t)(blockIdx.x % replicas) * 27 * 32;
  for (int e = tid; e < 27 * 32; e += NT)
    red_add(p.dw, ro + e, (red[0][e] + red[1][e] + red[2][e] + red[3][e]) * (1.f / 255.f), CFL_FX_G);
}

bool pow2(int x) { return x > 0 && (x & (x - 1)) == 0; }

bool use_mfma(const EntryParams& p) { return p.Cout == 32 && cfl_tune(TUNE_ENTRY_ALGO) != 1; }

}  // namespace

int entry_fwd(const EntryParams& p, hipStream_t st) {
  if (p.Cout % 8 || p.Cout > 64 || !pow2(p.Cout / 8)) return 1;
  const int rows = p.B * p.Ho;
  if (p.S % 4) return 1;
  // grid cap: 1,024 at 256^2 / batch 16 (2,048 row steps: two per block; per-position trace A/Bs 15.7 / 15.7 vs
  // 16.6 / 17.0 us for 512, 20.2 us for 2,048 - round 1 had picked 512 for fewer same-address statistics atomics);
  // the many-step problems (512^2 planned batch: 561k steps) need more resident blocks to hide each block's
  // one-step-ahead row prefetch: kbench 512^2 / b256 cap 512 / 1,024 / 2,048 = 583 / 432 / 424 us
  const int cap = cfl_tune(TUNE_ENTRY_FWD_BLOCKS) > 0 ? cfl_tune(TUNE_ENTRY_FWD_BLOCKS)
                                                     : rows * ((p.Wo + ECH - 1) / ECH) >= 65536 ? 2048 : 1024;
  if (use_mfma(p)) {
    const int nch = (p.Wo + ECH - 1) / ECH, steps = rows * nch;
    hipLaunchKernelGGL(entry_fwd_mfma_kernel, dim3(steps < cap ? steps : cap), dim3(NT), 0, st, p, nch, steps);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  const size_t lds = (size_t)3 * p.S * 3 * sizeof(float);
  if (lds > 48 * 1024) return 1;
  hipLaunchKernelGGL(entry_fwd_kernel, dim3(rows < cap ? rows : cap), dim3(NT), lds, st, p);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

int entry_wgrad(const EntryParams& p, hipStream_t st) {
  if (p.Cout % 8 || p.Cout > 64 || !pow2(p.Cout / 8)) return 1;
  const int rows = p.B * p.Ho;
  if (p.S % 4) return 1;
  const int reps = p.replicas > 1 ? p.replicas : 1;
  if (p.bwd.y && (!use_mfma(p) || p.bwd.reps > BNB_MAX_REPS)) {   // unfolded: bn_bwd_apply into bwd.dx, then dy = dx
    if (p.bwd.dx == nullptr) return 5;
    BnBwdApplyParams a{};
    a.g = p.dy;
    a.y = p.bwd.y;
    a.ab = p.bwd.ab;
    a.sums = p.bwd.sums;
    a.dy = p.bwd.dx;
    a.dgamma = p.bwd.dgamma;
    a.dbeta = p.bwd.dbeta;
    a.M = p.B * p.Ho * p.Wo;
    a.C = p.Cout;
    a.sum_reps = p.bwd.reps;
    const int rc = bn_bwd_apply(a, st);
    if (rc) return rc;
    EntryParams q = p;
    q.dy = p.bwd.dx;
    q.bwd = BnBwdIn{};
    return entry_wgrad(q, st);
  }
  if (use_mfma(p)) {
    const int nch = (p.Wo + ECH - 1) / ECH, steps = rows * nch;
    // (as entry_fwd: 512 at 256^2 / b16; kbench 512^2 / b256 cap 512 / 1,024 / 2,048 = 521 / 487 / 420 us)
    const int mcap = cfl_tune(TUNE_ENTRY_WGRAD_BLOCKS) > 0 ? cfl_tune(TUNE_ENTRY_WGRAD_BLOCKS)
                                                           : steps >= 65536 ? 2048 : 512;
    const dim3 grid(steps < mcap ? steps : mcap);
    if (p.bwd.y) hipLaunchKernelGGL(entry_wgrad_mfma_kernel<true>, grid, dim3(NT), 0, st, p, nch, steps, reps);
    else hipLaunchKernelGGL(entry_wgrad_mfma_kernel<false>, grid, dim3(NT), 0, st, p, nch, steps, reps);
    return hipGetLastError() == hipSuccess ? 0 : 3;
  }
  const int cap = cfl_tune(TUNE_ENTRY_WGRAD_BLOCKS) > 0 ? cfl_tune(TUNE_ENTRY_WGRAD_BLOCKS) : 256;   // measured
  hipLaunchKernelGGL(entry_wgrad_kernel, dim3(rows < cap ? rows : cap, 3), dim3(NT), (size_t)p.S * 3 * sizeof(float),
                     st, p, reps);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_entry(int v) { return cfl_det_upload(v); }
// block timeline buffer of this translation unit (common.h g_cfl_ts; set by cfl_ts_set)
int cfl_ts_upload_entry(void* buf, int cap) { return cfl_ts_upload(buf, cap); }
