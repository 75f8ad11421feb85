// Per-element Adam math shared by the stand-alone fused Adam (adam.hip) and the kernels
// that fuse the update into a collective (xgmi.hip: reduce-scatter -> Adam -> all-gather).
// Same expression order everywhere, so every path produces the same bits.
//
// Reference: multigrad/adam.py:52-68 (jax.example_libraries.optimizers.adam) and the
// bound transforms of multigrad/adam.py:202-239 (diagonal dp/du instead of the dense
// jax.jacobian of :174-180).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mg {

constexpr float kPi = 3.14159265358979323846f;

enum BoundKind : int8_t { kNone = 0, kBoth = 1, kLow = 2, kHigh = 3 };

__device__ __forceinline__ float dpdu(float at, float lo, float hi, int8_t k) {
  if (k == kBoth) {
    const float s = (hi - lo) / kPi;
    const float r = at / s;
    return 1.0f / (1.0f + r * r);
  }
  if (k == kLow || k == kHigh) {
    const float q = at / sqrtf(at * at + 4.0f);
    return 0.5f * (k == kLow ? 1.0f + q : 1.0f - q);
  }
  return 1.0f;
}

__device__ __forceinline__ float inv_transform(float u, float lo, float hi, int8_t k) {
  if (k == kBoth) {
    const float mid = (hi + lo) * 0.5f;
    const float s = (hi - lo) / kPi;
    return mid + s * atanf(u / s);
  }
  if (k == kLow) return 0.5f * (2.0f * lo + u + sqrtf(u * u + 4.0f));
  if (k == kHigh) return 0.5f * (2.0f * hi + u - sqrtf(u * u + 4.0f));
  return u;
}

// One Adam step of one coordinate.  H: any struct with lr, b1, b2, eps.  bc1/bc2 are the
// bias corrections 1 - b^(i+1) of the 0-based step i.
template <bool BOUNDED, bool LEGACY, class H>
__device__ __forceinline__ void adam_elem(const H& a, float bc1, float bc2, float g, float& u,
                                          float& m, float& v, float pold, float lo, float hi,
                                          int8_t k, float& pnew) {
  if (BOUNDED) g *= dpdu(LEGACY ? pold : u, lo, hi, k);
  m = (1.0f - a.b1) * g + a.b1 * m;
  v = (1.0f - a.b2) * (g * g) + a.b2 * v;
  const float mhat = m / bc1;
  const float vhat = v / bc2;
  u = u - a.lr * mhat / (sqrtf(vhat) + a.eps);
  pnew = BOUNDED ? inv_transform(u, lo, hi, k) : u;
}

}  // namespace mg
