// Block-scaled fp8 (OCP e4m3) MFMA on gfx950: v_mfma_scale_f32_16x16x128_f8f6f4 / _32x32x64_ with per-32-element
// e8m0 block scales (BASELINE config 5: the fp8 Conv2D MFMA path).
//
// mfma_scale_probe: one wave runs ONE scaled MFMA on caller-supplied lane registers (32 fp8 bytes of A and of B per
// lane, one int32 scale word each) and returns the raw accumulator registers - the operand lane maps are checked
// against a host GEMM with exact small-integer data (tests/test_gpu_kernels.py) before any kernel relies on them.
#include "common.h"
#include "launch.h"

namespace {

typedef int i8v __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(64) void mfma_scale_probe_kernel(const int* __restrict__ a, const int* __restrict__ b,
                                                              const int* __restrict__ sa, const int* __restrict__ sb,
                                                              float* __restrict__ d, int shape) {
  const int l = threadIdx.x;
  i8v av, bv;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    av[j] = a[l * 8 + j];
    bv[j] = b[l * 8 + j];
  }
  if (shape == 16) {
    f4v c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, sa[l], 0, sb[l]);
#pragma unroll
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
  } else {
    f16v c = {};
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c, 0, 0, 0, sa[l], 0, sb[l]);
#pragma unroll
    for (int r = 0; r < 16; ++r) d[l * 16 + r] = c[r];
  }
}

}  // namespace

int mfma_scale_probe(const int* a, const int* b, const int* sa, const int* sb, float* d, int shape, hipStream_t st) {
  if (shape != 16 && shape != 32) return 1;
  hipLaunchKernelGGL(mfma_scale_probe_kernel, dim3(1), dim3(64), 0, st, a, b, sa, sb, d, shape);
  return hipGetLastError() == hipSuccess ? 0 : 3;
}

// deterministic reduction mode flag of this translation unit (common.h g_cfl_det; set by cfl_det_set)
int cfl_det_upload_fp8(int v) { return cfl_det_upload(v); }
