// Micro-benchmark: per-instruction issue cost on gfx950, full chip (8 waves/SIMD),
// 8 independent chains per lane.  Reports cycles per wave-instruction per SIMD at the
// measured clock-free rate (ns) and at 2.4 GHz.  Kinds:
//   fma      v_fma_f32                pk_fma   v_pk_fma_f32 (2 lanes' worth per instr)
//   exp      v_exp_f32                rcp      v_rcp_f32
//   add_abs  v_add_f32 |x|+c           bfi      v_bfi_b32 (copysign)
//   cmp_cnt  v_cmp + s_bcnt1 + s_add (ballot count; VALU->SALU dependency)
//   exp_fma  1 exp : 4 fma mix         cndadd   v_cndmask-free count: cnt += x<0
//   fract    v_fract_f32               cvt_flr  v_cvt_flr_i32_f32
//   med3     v_med3_f32                lshl_or  v_lshl_or_b32
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int kIters = 2048;

template <int KIND>
__global__ __launch_bounds__(256) void k(float* out, float seed) {
  float a[8];
  v2f b[8];
  int cnt = 0, ci[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = seed * (threadIdx.x + j + 1) * 1e-6f;
    b[j] = (v2f)(a[j]);
    ci[j] = 0;
  }
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (KIND == 0) a[j] = __builtin_fmaf(a[j], 0.999f, 1e-7f);
      if constexpr (KIND == 1) b[j] = b[j] * (v2f)(0.999f) + (v2f)(1e-7f);
      if constexpr (KIND == 2) a[j] = __builtin_amdgcn_exp2f(a[j]);
      if constexpr (KIND == 3) a[j] = __builtin_amdgcn_rcpf(a[j]);
      if constexpr (KIND == 4) a[j] = __builtin_fabsf(a[j]) + -0.5f;
      if constexpr (KIND == 5) a[j] = __builtin_copysignf(a[j], a[(j + 1) & 7]);
      if constexpr (KIND == 6) cnt += __builtin_popcountll(__builtin_amdgcn_ballot_w64(a[j] < (float)it));
      if constexpr (KIND == 7) {
        if (j % 4 == 0) a[j] = __builtin_amdgcn_exp2f(a[j]);
        else a[j] = __builtin_fmaf(a[j], 0.999f, 1e-7f);
      }
      if constexpr (KIND == 8) ci[j] += (a[j] < (float)it) ? 1 : 0;
      if constexpr (KIND == 9) a[j] = __builtin_amdgcn_fractf(a[j]);
      if constexpr (KIND == 10) {
        int kk;
        asm volatile("v_cvt_flr_i32_f32 %0, %1" : "=v"(kk) : "v"(a[j]));
        a[j] = __int_as_float(kk);
      }
      if constexpr (KIND == 11) a[j] = __builtin_amdgcn_fmed3f(a[j], -3.0f, seed);
      if constexpr (KIND == 12) {
        int kk;
        asm volatile("v_lshl_or_b32 %0, %1, 8, %2" : "=v"(kk) : "v"(ci[j]), "v"(cnt));
        ci[j] = kk;
      }
    }
  }
  float s = (float)cnt;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j] + b[j].x + b[j].y + (float)ci[j];
  if (s == 1234.5f) out[0] = s;
}

template <int KIND>
static float run(int blocks, float* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<KIND>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  return ms;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 4);
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8;  // 8 blocks x 4 waves = 32 waves/CU
  const char* names[] = {"fma", "pk_fma", "exp", "rcp", "add_abs", "bfi", "cmp_cnt", "exp1fma3",
                         "cndadd", "fract", "cvt_flr", "med3", "lshl_or"};
  constexpr int NK = 13;
  float ms[NK] = {run<0>(blocks, d), run<1>(blocks, d), run<2>(blocks, d), run<3>(blocks, d),
                  run<4>(blocks, d), run<5>(blocks, d), run<6>(blocks, d), run<7>(blocks, d),
                  run<8>(blocks, d), run<9>(blocks, d), run<10>(blocks, d), run<11>(blocks, d),
                  run<12>(blocks, d)};
  const double wave_instr = (double)blocks * 4 * kIters * 8;
  const double per_simd = wave_instr / (p.multiProcessorCount * 4);
  printf("clock %d kHz, %d CUs\n", p.clockRate, p.multiProcessorCount);
  for (int i = 0; i < NK; ++i)
    printf("%-9s %.3f ms  %.3f ns per loop-body op per SIMD (%.2f cycles @2.4GHz)\n", names[i], ms[i],
           ms[i] * 1e6 / per_simd, ms[i] * 1e6 / per_simd * 2.4);
  return 0;
}
