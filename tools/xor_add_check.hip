// standalone check (tools/xor_add_check.hip): common.h xor_add(v, o) == v + __shfl_xor(v, o, 64) bit for bit in every
// lane for o = 1..32 (float and double) and xor16_get == __shfl_xor(v, 16). Build: hipcc -O3 -std=c++17
// --offload-arch=gfx950 -Icsrc -Icsrc/kernels tools/xor_add_check.hip -o /tmp/xor_add_check; run on the GPU.
#include "common.h"
#include <cstdio>
#include <vector>
__global__ void k(const float* in, int* bad) {
  const float v = in[blockIdx.x * 64 + threadIdx.x];
  int nb = 0;
  const int os[6] = {1, 2, 4, 8, 16, 32};
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float a = xor_add(v, os[i]), b = v + __shfl_xor(v, os[i], 64);
    nb += __builtin_bit_cast(unsigned, a) != __builtin_bit_cast(unsigned, b);
  }
  const double dv = (double)v * 1.000001 + 1e-7 * threadIdx.x;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const double a = xor_add(dv, os[i]), b = dv + __shfl_xor(dv, os[i], 64);
    nb += __builtin_bit_cast(unsigned long long, a) != __builtin_bit_cast(unsigned long long, b);
  }
  const unsigned u = __builtin_bit_cast(unsigned, v);
  nb += xor16_get(u) != (unsigned)__shfl_xor((int)u, 16, 64);
  if (nb) atomicAdd(bad, nb);
}
int main() {
  const int n = 64 * 64;
  std::vector<float> h(n);
  unsigned s = 12345;
  for (auto& x : h) { s = s * 1664525u + 1013904223u; x = (float)((int)(s >> 8) - (1 << 23)) * 1e-3f; }
  float* d; int* bad; int hb = 0;
  hipMalloc(&d, n * 4); hipMalloc(&bad, 4);
  hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  hipMemcpy(bad, &hb, 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(64), dim3(64), 0, 0, d, bad);
  hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost);
  printf("xor_add mismatches: %d\n", hb);
  return hb != 0;
}
