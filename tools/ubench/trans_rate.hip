// Micro-benchmark: issue throughput of v_fma_f32 vs v_exp_f32 vs v_rcp_f32 on gfx950.
// 8 independent chains per lane, full chip (8 waves/SIMD), cycles from s_memtime are
// not used: we report wave-instructions per ns per SIMD; compare ratios only.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIters = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float seed) {
  float a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = seed * (threadIdx.x + j + 1) * 1e-6f;
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (KIND == 0) a[j] = __builtin_fmaf(a[j], 0.999f, 1e-7f);
      if (KIND == 1) a[j] = __builtin_amdgcn_exp2f(a[j]) * -0.5f;    // exp + mul
      if (KIND == 2) a[j] = __builtin_amdgcn_rcpf(a[j]) + 1.0f;      // rcp + add
      if (KIND == 3) a[j] = __builtin_amdgcn_exp2f(a[j]);             // exp only
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j];
  if (s == 1234.5f) out[0] = s;
}

int main() {
  float* d;
  hipMalloc(&d, 4);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8;  // 8 blocks x 4 waves = 32 waves/CU
  const char* names[] = {"fma", "exp+mul", "rcp+add", "exp"};
  for (int kind = 0; kind < 4; ++kind) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
      if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
      if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
      if (kind == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
    }
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr = (double)blocks * 4 * kIters * 8;  // per loop-body instruction
    const double per_simd = wave_instr / (p.multiProcessorCount * 4);
    printf("%-8s %.3f ms  %.3f ns per wave-op per SIMD (%.2f cycles @2.4GHz)\n", names[kind], ms,
           ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4);
  }
  return 0;
}
