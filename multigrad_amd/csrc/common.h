// Shared device helpers for the multigrad_amd gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mg {

constexpr int kWave = 64;  // CDNA wavefront width (never 32)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

// Deterministic block reduction of N values per thread; result valid in thread 0.
// scratch: N * (blockDim.x / 64) floats of LDS.
template <int N, typename T>
__device__ __forceinline__ void block_sum_n(T (&v)[N], T* scratch) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = wave_sum(v[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) scratch[k * nw + wid] = v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
      T s = scratch[k * nw];
      for (int w = 1; w < nw; ++w) s += scratch[k * nw + w];
      v[k] = s;
    }
  }
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// Upper-tail normal probability Q(|z|) = P(Z > |z|) = erfc(|z|/sqrt2)/2, accurate to a
// few ulp *relative* in the far tail (so bin masses far from the mean keep their
// precision; 0.5*(1+erf) loses it).  Shepherd-Laframboise form: with a = |z|/sqrt2 and
// q = (a-2)/(a+2), (1+2a) exp(a^2) erfc(a) is a smooth function of q in [-1, 1); it is
// fitted here by a degree-10 polynomial (coefficients include the factor 1/2).
// One reciprocal + one exp2 per call.
__device__ __forceinline__ float normal_tail(float z) {
  // (clamped: beyond a = 16 exp(-a^2) is 0 and the rational part must stay finite)
  const float a = fminf(fabsf(z) * 0.70710678118654752f, 16.0f);
  const float ap2 = a + 2.0f;
  const float tp1 = fmaf(2.0f, a, 1.0f);
  const float r = fast_rcp(ap2 * tp1);  // 1 / ((a+2)(1+2a))
  const float q = (a - 2.0f) * tp1 * r;
  float p = 0x1.5139fap-14f;
  p = fmaf(p, q, -0x1.8126a8p-14f);
  p = fmaf(p, q, -0x1.6de016p-11f);
  p = fmaf(p, q, 0x1.11743cp-11f);
  p = fmaf(p, q, 0x1.1cb9eep-8f);
  p = fmaf(p, q, -0x1.044460p-8f);
  p = fmaf(p, q, -0x1.bc1ab8p-6f);
  p = fmaf(p, q, 0x1.4ff206p-4f);
  p = fmaf(p, q, -0x1.54081cp-4f);
  p = fmaf(p, q, -0x1.7bf524p-5f);
  p = fmaf(p, q, 0x1.46e80ep-1f);
  // exp(-a^2) = exp2(-z^2 * log2(e) / 2)
  const float e = fast_exp2(z * z * -0.72134752044448170f);
  return p * ap2 * r * e;
}

}  // namespace mg
