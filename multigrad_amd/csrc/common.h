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

// Scaled normal coordinate used by the SMF kernels: w = z * kWScale with
// kWScale = sqrt(log2(e)/2), so that the Gaussian kernel exp(-z^2/2) = exp2(-w^2) costs
// one multiply + one v_exp_f32.
constexpr float kWScale = 0x1.b2da4ep-1f;  // 0.84932180

// Upper-tail normal probability Q(|z|) = P(Z > |z|) = erfc(|z|/sqrt2)/2 from the scaled
// coordinate w, accurate to ~5e-7 *relative* everywhere (including the far tail, where
// 0.5*(1+erf) loses all precision).  With a = |z|/sqrt2 and q = (a-K)/(a+K), K = 2.5,
// erfcx(a) = exp(a^2) erfc(a) is a smooth function of q in [-1, 1): a degree-9 minimax
// polynomial (coefficients fitted offline, they include the factor 1/2).  q is formed
// directly from b = |w| = a*sqrt(log2 e) (homogeneous), so one v_rcp + one v_exp + 13
// VALU per call, branch free, NaN only for NaN input.
__device__ __forceinline__ float normal_tail_w(float w) {
  constexpr float kKs = 0x1.805bf2p+1f;  // K * sqrt(log2 e) = 3.00280602
  // q = (b-K)/(b+K) = 1 - 2K/(b+K): one rcp + one fma, finite for b = inf (q -> 1)
  const float r = fast_rcp(fabsf(w) + kKs);
  const float q = fmaf(-2.0f * kKs, r, 1.0f);
  float p = -0x1.9bba2ap-15f;
  p = fmaf(p, q, 0x1.6288b6p-14f);
  p = fmaf(p, q, 0x1.c3390ap-12f);
  p = fmaf(p, q, -0x1.54b8b8p-10f);
  p = fmaf(p, q, -0x1.05c212p-9f);
  p = fmaf(p, q, 0x1.46f0a8p-6f);
  p = fmaf(p, q, -0x1.001088p-4f);
  p = fmaf(p, q, 0x1.01c172p-3f);
  p = fmaf(p, q, -0x1.7ca898p-3f);
  p = fmaf(p, q, 0x1.afbb3cp-4f);
  return p * fast_exp2(-w * w);
}

// The two factors of Q(|z|) = p(r) * exp2(-w^2), returned unmultiplied so that the
// caller can fold the sign and the accumulation into one fma.  Unlike normal_tail_w the
// polynomial is in r = 1/(|w| + K) itself (no q = 1 - 2Kr step); minimax coefficients
// fitted offline by a linear program (weighted as below), checked in float32 on a
// 4e5-point grid:
//  REL = true : degree 7, K = 3.2 (w units); max *relative* error of the float32 product
//               4e-6 up to w = 9 (1.2e-6 for the fit itself), i.e. tail-accurate: bins
//               fed only by far Gaussian tails keep ~5-6 significant digits.
//  REL = false: degree 5, K = 1.8; max *absolute* error 1.6e-7 (the accuracy class of
//               the float32 erf the reference evaluates).  The fit is weighted by
//               exp2(-w^2), so the far tail is only absolutely accurate.
// Cost: one v_rcp + one v_exp + (DEG + 2) VALU.
template <bool REL>
__device__ __forceinline__ void normal_tail_parts_w(float w, float& p, float& g) {
  if constexpr (REL) {
    const float r = fast_rcp(fabsf(w) + 0x1.99999ap+1f);
    p = -0x1.c816e0p+7f;
    p = fmaf(p, r, 0x1.9741fcp+7f);
    p = fmaf(p, r, -0x1.42955cp+4f);
    p = fmaf(p, r, 0x1.d3aa86p+3f);
    p = fmaf(p, r, 0x1.5e9730p+1f);
    p = fmaf(p, r, 0x1.1b7a3ap+0f);
    p = fmaf(p, r, 0x1.5a604cp-2f);
    p = fmaf(p, r, 0x1.7dececp-18f);
  } else {
    const float r = fast_rcp(fabsf(w) + 0x1.ccccccp+0f);
    p = 0x1.3a12c0p+0f;
    p = fmaf(p, r, -0x1.bacb20p+1f);
    p = fmaf(p, r, 0x1.901deap+1f);
    p = fmaf(p, r, -0x1.0b406ap-7f);
    p = fmaf(p, r, 0x1.b317b2p-2f);
    p = fmaf(p, r, -0x1.428b48p-8f);
  }
  g = fast_exp2(-w * w);
}

// Two halos at once (packed fp32: v_pk_fma/v_pk_mul do both lanes of a pair in one
// issue, the transcendental and bitwise steps stay per element).  Same contract as
// normal_tail_parts_w.
typedef float v2f __attribute__((ext_vector_type(2)));

// The two reciprocals of a pair, one v_rcp each.  (Sharing one v_rcp, 1/a = b/(ab), was a
// compiled-out variant until round 5, when the unmeasured switch was removed.)
__device__ __forceinline__ v2f pair_rcp(float a, float b) {
  v2f r;
  r.x = fast_rcp(a);
  r.y = fast_rcp(b);
  return r;
}

template <bool REL>
__device__ __forceinline__ void normal_tail_parts_w2(v2f w, v2f& p, v2f& g) {
  v2f r;
  if constexpr (REL) {
    constexpr float kK = 0x1.99999ap+1f;
    r = pair_rcp(fabsf(w.x) + kK, fabsf(w.y) + kK);
    p = (v2f)(-0x1.c816e0p+7f);
    p = p * r + 0x1.9741fcp+7f;
    p = p * r + -0x1.42955cp+4f;
    p = p * r + 0x1.d3aa86p+3f;
    p = p * r + 0x1.5e9730p+1f;
    p = p * r + 0x1.1b7a3ap+0f;
    p = p * r + 0x1.5a604cp-2f;
    p = p * r + 0x1.7dececp-18f;
  } else {
    constexpr float kK = 0x1.ccccccp+0f;
    r = pair_rcp(fabsf(w.x) + kK, fabsf(w.y) + kK);
    p = (v2f)(0x1.3a12c0p+0f);
    p = p * r + -0x1.bacb20p+1f;
    p = p * r + 0x1.901deap+1f;
    p = p * r + -0x1.0b406ap-7f;
    p = p * r + 0x1.b317b2p-2f;
    p = p * r + -0x1.428b48p-8f;
  }
  const v2f t = -w * w;
  g.x = fast_exp2(t.x);
  g.y = fast_exp2(t.y);
}

}  // namespace mg
