// Fused Adam for gfx950 (MI355X): bounded-coordinate chain rule + moments + bias
// correction + inverse transform + trajectory write in one HBM pass.
//
// Reference: multigrad/adam.py:52-68 (jax.example_libraries.optimizers.adam) and the
// bound transforms of multigrad/adam.py:202-239, whose dense P x P jax.jacobian
// (:174-180) collapses here to the diagonal dp/du computed in registers.
//
// Per element (i = 0-based step):
//   g_u = g_p * dp/du(at)      (at = u, or p with the legacy Q1 Jacobian)
//   m = (1-b1) g_u + b1 m ;  v = (1-b2) g_u^2 + b2 v
//   u -= lr * (m / (1-b1^(i+1))) / (sqrt(v / (1-b2^(i+1))) + eps)
//   p  = T^-1(u) ; traj[i+1] = p
// The step counter lives in device memory ([step, ticket]); the last workgroup to
// finish advances it, so the kernel is HIP-graph replayable without host arguments
// (eager callers may pass the step instead: no counter traffic at all).
// Memory: 16 B read + 12 B written per unbounded parameter (+8 B read, +4 B written for
// the bounded p output, +4 B for the trajectory) -> HBM-bandwidth bound; float4 lanes.
#include "adam.h"
#include "common.h"

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

namespace mg {

constexpr int kAdamThreads = 256;

struct AdamArgs {
  float* u;
  float* m;
  float* v;
  const float* g;
  float* p;            // bounded output (nullptr: unbounded, p == u)
  const float* lo;
  const float* hi;
  const int8_t* kind;
  int* step;           // [step, ticket]
  float* traj;         // trajectory base (row r at traj + r * traj_stride) or nullptr
  int64_t traj_stride;
  int64_t n;
  int host_step;       // >= 0: the 0-based step, passed by an eager caller; -1: read *step
  float lr, b1, b2, eps;
};

// Small updates (all workgroups finish together) advance the step in a separate
// one-thread kernel instead: ~1000 tickets on one address at the very end serialise in L2
// (20 us for 1.25M parameters vs 7 us of streaming); large updates keep the ticket, whose
// atomics are spread over the kernel and hidden.
constexpr int64_t kTicketMinParams = int64_t(1) << 23;

__global__ void advance_step_kernel(int* step) { step[0] += 1; }

template <bool BOUNDED, bool LEGACY, bool VEC, bool TICKET>
__global__ __launch_bounds__(kAdamThreads) void fused_adam_kernel(AdamArgs a) {
  const int step = a.host_step >= 0
                       ? a.host_step
                       : __hip_atomic_load(a.step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float bc1 = 1.0f - powf(a.b1, (float)(step + 1));
  const float bc2 = 1.0f - powf(a.b2, (float)(step + 1));
  float* trow = a.traj ? a.traj + (int64_t)(step + 1) * a.traj_stride : nullptr;
  const int64_t tid = (int64_t)blockIdx.x * kAdamThreads + threadIdx.x;
  const int64_t nthr = (int64_t)gridDim.x * kAdamThreads;
  if (VEC) {
    const int64_t n4 = a.n >> 2;
    for (int64_t i = tid; i < n4; i += nthr) {
      float4 g = reinterpret_cast<const float4*>(a.g)[i];
      float4 u = reinterpret_cast<float4*>(a.u)[i];
      float4 m = reinterpret_cast<float4*>(a.m)[i];
      float4 v = reinterpret_cast<float4*>(a.v)[i];
      float4 po = make_float4(0.f, 0.f, 0.f, 0.f), lo = po, hi = po;
      char4 k = make_char4(0, 0, 0, 0);
      if (BOUNDED) {
        lo = reinterpret_cast<const float4*>(a.lo)[i];
        hi = reinterpret_cast<const float4*>(a.hi)[i];
        k = reinterpret_cast<const char4*>(a.kind)[i];
        if (LEGACY) po = reinterpret_cast<float4*>(a.p)[i];
      }
      float4 pn;
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.x, u.x, m.x, v.x, po.x, lo.x, hi.x, k.x, pn.x);
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.y, u.y, m.y, v.y, po.y, lo.y, hi.y, k.y, pn.y);
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.z, u.z, m.z, v.z, po.z, lo.z, hi.z, k.z, pn.z);
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.w, u.w, m.w, v.w, po.w, lo.w, hi.w, k.w, pn.w);
      reinterpret_cast<float4*>(a.u)[i] = u;
      reinterpret_cast<float4*>(a.m)[i] = m;
      reinterpret_cast<float4*>(a.v)[i] = v;
      if (BOUNDED) reinterpret_cast<float4*>(a.p)[i] = pn;
      if (trow) reinterpret_cast<float4*>(trow)[i] = pn;
    }
    // scalar tail
    for (int64_t i = (n4 << 2) + tid; i < a.n; i += nthr) {
      float u = a.u[i], m = a.m[i], v = a.v[i], pn;
      const float po = (BOUNDED && LEGACY) ? a.p[i] : 0.f;
      const float lo = BOUNDED ? a.lo[i] : 0.f, hi = BOUNDED ? a.hi[i] : 0.f;
      const int8_t k = BOUNDED ? a.kind[i] : (int8_t)0;
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, a.g[i], u, m, v, po, lo, hi, k, pn);
      a.u[i] = u; a.m[i] = m; a.v[i] = v;
      if (BOUNDED) a.p[i] = pn;
      if (trow) trow[i] = pn;
    }
  } else {
    for (int64_t i = tid; i < a.n; i += nthr) {
      float u = a.u[i], m = a.m[i], v = a.v[i], pn;
      const float po = (BOUNDED && LEGACY) ? a.p[i] : 0.f;
      const float lo = BOUNDED ? a.lo[i] : 0.f, hi = BOUNDED ? a.hi[i] : 0.f;
      const int8_t k = BOUNDED ? a.kind[i] : (int8_t)0;
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, a.g[i], u, m, v, po, lo, hi, k, pn);
      a.u[i] = u; a.m[i] = m; a.v[i] = v;
      if (BOUNDED) a.p[i] = pn;
      if (trow) trow[i] = pn;
    }
  }
  // Advance the device step once every workgroup has read it: each block takes a
  // ticket after its own read of `step`; the last ticket holder publishes step+1.
  if (!TICKET) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = atomicAdd(&a.step[1], 1);
    if (t == (int)gridDim.x - 1) {
      __hip_atomic_store(&a.step[1], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.step[0], step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

void fused_adam(torch::Tensor u, torch::Tensor m, torch::Tensor v, torch::Tensor g,
                c10::optional<torch::Tensor> p, c10::optional<torch::Tensor> lo,
                c10::optional<torch::Tensor> hi, c10::optional<torch::Tensor> kind,
                torch::Tensor step, double lr, double b1, double b2, double eps, bool legacy,
                c10::optional<torch::Tensor> traj, int64_t traj_stride, int64_t host_step) {
  for (auto* t : {&u, &m, &v, &g}) {
    TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kFloat,
                "adam tensors must be contiguous float32 device tensors");
    TORCH_CHECK(t->numel() == u.numel(), "adam tensor size mismatch");
  }
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kInt && step.numel() >= 2,
              "step must be a [2] int32 device tensor");
  const bool bounded = p.has_value() && p->defined() && lo.has_value() && lo->defined();
  AdamArgs a;
  a.u = u.data_ptr<float>();
  a.m = m.data_ptr<float>();
  a.v = v.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.p = nullptr;
  a.lo = a.hi = nullptr;
  a.kind = nullptr;
  if (bounded) {
    TORCH_CHECK(p->numel() == u.numel() && lo->numel() == u.numel() && hi->numel() == u.numel() &&
                kind->numel() == u.numel(), "bounds size mismatch");
    TORCH_CHECK(kind->scalar_type() == at::kChar, "kind must be int8");
    a.p = p->data_ptr<float>();
    a.lo = lo->data_ptr<float>();
    a.hi = hi->data_ptr<float>();
    a.kind = kind->data_ptr<int8_t>();
  }
  a.step = step.data_ptr<int>();
  a.traj = (traj.has_value() && traj->defined()) ? traj->data_ptr<float>() : nullptr;
  a.traj_stride = traj_stride;
  a.n = u.numel();
  a.host_step = (int)host_step;
  a.lr = (float)lr; a.b1 = (float)b1; a.b2 = (float)b2; a.eps = (float)eps;
  bool vec = aligned16(a.u) && aligned16(a.m) && aligned16(a.v) && aligned16(a.g);
  if (bounded) vec = vec && aligned16(a.p) && aligned16(a.lo) && aligned16(a.hi) &&
                     (reinterpret_cast<uintptr_t>(a.kind) & 3) == 0;
  if (a.traj) vec = vec && aligned16(a.traj) && (traj_stride % 4 == 0);
  const int64_t work = vec ? (a.n + 3) / 4 : a.n;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>((work + kAdamThreads - 1) / kAdamThreads, 2048));
  auto stream = at::hip::getCurrentHIPStream();
  // host step: nothing to advance on the device (eager callers keep the count)
  const bool ticket = host_step < 0 && a.n >= kTicketMinParams;
#define MG_ADAM_LAUNCH(B, L, V)                                                              \
  do {                                                                                       \
    if (ticket)                                                                              \
      hipLaunchKernelGGL((fused_adam_kernel<B, L, V, true>), dim3(blocks), dim3(kAdamThreads), \
                         0, stream, a);                                                      \
    else                                                                                     \
      hipLaunchKernelGGL((fused_adam_kernel<B, L, V, false>), dim3(blocks), dim3(kAdamThreads), \
                         0, stream, a);                                                      \
  } while (0)
  if (bounded) {
    if (legacy) { if (vec) MG_ADAM_LAUNCH(true, true, true); else MG_ADAM_LAUNCH(true, true, false); }
    else { if (vec) MG_ADAM_LAUNCH(true, false, true); else MG_ADAM_LAUNCH(true, false, false); }
  } else {
    if (vec) MG_ADAM_LAUNCH(false, false, true); else MG_ADAM_LAUNCH(false, false, false);
  }
#undef MG_ADAM_LAUNCH
  if (!ticket && host_step < 0)
    hipLaunchKernelGGL(advance_step_kernel, dim3(1), dim3(1), 0, stream, a.step);
}

}  // namespace mg
