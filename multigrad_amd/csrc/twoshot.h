// Two-shot reduce-scatter -> Adam -> all-gather over peer memory (see xgmi.hip for the
// protocol), as the work of a range of workgroups: the stand-alone exchange kernel
// (xgmi.hip) and the compute kernels that run the exchange of the previous parameter chunk
// in their first workgroups (smf.hip, "fused exchange": the exchange of chunk c-1 overlaps
// the VJP of chunk c without a second stream or cross-stream events).
#pragma once

#include "adam.h"
#include "common.h"
#include "xgmi.h"

#include <cstring>
#include <stdexcept>
#include <string>

namespace mg {

struct TwoShotArgs {
  XgmiPeers g;          // peers' gradient regions (as mapped in this process)
  XgmiPeers t;          // peers' parameter regions
  XgmiPeers f;          // peers' flag regions
  int rank, size;
  int64_t lo, n;        // owned float range; lo % 4 == 0, n % 4 == 0
  float* u;             // bounded: owned u slice; unbounded: nullptr (u = own parameters)
  float* m;
  float* v;
  const float* blo;     // owned bounds (bounded modes)
  const float* bhi;
  const int8_t* kind;
  float* traj;          // owned trajectory base (row r at traj + r * traj_stride) or null
  int64_t traj_stride;
  int* step;            // device step counter [step, ticket] (read when host_step < 0)
  int host_step;
  unsigned* seq;
  int* err;
  long long ticks;
  float lr, b1, b2, eps;
};

constexpr int kTsThreads = 256;

// MODE 0: plain sum (self-test: theta = sum of the gradients); 1: Adam, unbounded;
// 2: Adam in bounded coordinates; 3: bounded with the reference's legacy Jacobian (Q1);
// 4: reduce-scatter only -- the rank-order sum of the owned slice goes to the local buffer
// `u`, nothing is pushed; 5: all-gather only -- the local slice `u` is pushed into every
// rank's parameter region, nothing is pulled.  (4 and 5 are the device L-BFGS's sharded
// evaluation: gradient to the owned slice, owned slice of the iterate to every rank.)
// The exchange as workgroups [0, nblk) of the calling grid (bid = this workgroup's index in
// that range).  Every workgroup of the range must call it; it returns when this
// workgroup's share is done (the last one returns when every rank's slice has landed).
// `lds`: two ints of LDS for the block-wide flags (lent by the caller: the fused VJP sits at
// exactly 20 KiB so that 8 workgroups fit a CU, and a __shared__ here would add to it).
// LEAN: one element's Adam at a time (scalar loads of its state, scheduling barriers
// between the four), for the bounded modes carried by compute kernels whose launch bounds
// allow 64 VGPRs (the float4 form spilled 43-65 VGPRs there).
template <int MODE, int PB = kXMaxRanks, bool LEAN = false>
__device__ __forceinline__ void twoshot_block(const TwoShotArgs& a, int bid, int nblk, int* lds) {
  static_assert(kXMaxRanks % PB == 0, "peer batches must tile the rank limit");
  static_assert(MODE >= 0 && MODE <= 5, "two-shot mode");
  constexpr bool ADAM = MODE >= 1 && MODE <= 3;
  constexpr bool BOUNDED = MODE == 2 || MODE == 3;
  constexpr bool LEGACY = MODE == 3;
  constexpr bool PULL = MODE != 5;
  constexpr bool PUSH = MODE != 4;
  const unsigned seq = __hip_atomic_load(a.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  const int st = a.host_step >= 0
                     ? a.host_step
                     : __hip_atomic_load(a.step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  char* me = a.f.base[a.rank];
  // my gradient is complete: the VJP's stores to the uncached buffer were acknowledged
  // before that launch ended, and this launch is ordered after it
  if (bid == 0 && (int)threadIdx.x < a.size) uc_signal(ts_gflag(a.f.base[threadIdx.x]) + a.rank, seq);
  const int bad = ts_wait_all(ts_gflag(me), a.size, seq, a.err, a.ticks, lds + 1);
  const float bc1 = 1.0f - powf(a.b1, (float)(st + 1));
  const float bc2 = 1.0f - powf(a.b2, (float)(st + 1));
  float* trow = a.traj ? a.traj + (int64_t)(st + 1) * a.traj_stride : nullptr;
  const float* own = reinterpret_cast<const float*>(a.t.base[a.rank]) + a.lo;
  const int64_t n4 = a.n >> 2;
  const int64_t stride = (int64_t)nblk * kTsThreads;
  for (int64_t i = (int64_t)bid * kTsThreads + threadIdx.x; i < n4; i += stride) {
    const int64_t off = a.lo + 4 * i;
    // the peers' loads are issued PB at a time before their adds (the peer loop is unrolled
    // to the compile-time rank limit), so PB remote round trips overlap instead of running
    // one after another; the sum is taken in rank order either way (same bits for any PB).
    // PB = 8: every load in flight (the stand-alone kernel); PB = 4 keeps the registers of
    // the compute kernels that carry the exchange (fused exchange)
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (PULL) {
#pragma unroll
      for (int q0 = 0; q0 < kXMaxRanks; q0 += PB) {
        float4 hs[PB];
#pragma unroll
        for (int j = 0; j < PB; ++j)
          if (q0 + j < a.size)
            hs[j] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.g.base[q0 + j]) + off);
#pragma unroll
        for (int j = 0; j < PB; ++j) {
          if (q0 + j == 0) {
            g = hs[0];
          } else if (q0 + j < a.size) {
            g.x += hs[j].x; g.y += hs[j].y; g.z += hs[j].z; g.w += hs[j].w;
          }
        }
      }
    } else {
      g = reinterpret_cast<const float4*>(a.u)[i];
    }
    float4 p = g;
    if constexpr (ADAM && LEAN) {
      // one element at a time: scalar loads of its state, a scheduling barrier after each
      const float gs[4] = {g.x, g.y, g.z, g.w};
      float ps[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t e = 4 * i + q;
        float uu = BOUNDED ? a.u[e] : own[e];
        float mm = a.m[e], vv = a.v[e], po = 0.f, lo = 0.f, hi = 0.f;
        int8_t kk = 0;
        if constexpr (BOUNDED) {
          lo = a.blo[e];
          hi = a.bhi[e];
          kk = a.kind[e];
          if (LEGACY) po = own[e];
        }
        float pp;
        adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, gs[q], uu, mm, vv, po, lo, hi, kk, pp);
        if (bad) uu = pp = __builtin_nanf("");
        a.m[e] = mm;
        a.v[e] = vv;
        if constexpr (BOUNDED) a.u[e] = uu;
        if (trow) trow[e] = pp;
        ps[q] = pp;
        __builtin_amdgcn_sched_barrier(0);
      }
      p = make_float4(ps[0], ps[1], ps[2], ps[3]);
    } else if constexpr (ADAM) {
      float4 u = BOUNDED ? reinterpret_cast<const float4*>(a.u)[i]
                         : reinterpret_cast<const float4*>(own)[i];
      float4 m = reinterpret_cast<const float4*>(a.m)[i];
      float4 v = reinterpret_cast<const float4*>(a.v)[i];
      float4 po = make_float4(0.f, 0.f, 0.f, 0.f), lo = po, hi = po;
      char4 k = make_char4(0, 0, 0, 0);
      if constexpr (BOUNDED) {
        lo = reinterpret_cast<const float4*>(a.blo)[i];
        hi = reinterpret_cast<const float4*>(a.bhi)[i];
        k = reinterpret_cast<const char4*>(a.kind)[i];
        if (LEGACY) po = reinterpret_cast<const float4*>(own)[i];
      }
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.x, u.x, m.x, v.x, po.x, lo.x, hi.x, k.x, p.x);
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.y, u.y, m.y, v.y, po.y, lo.y, hi.y, k.y, p.y);
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.z, u.z, m.z, v.z, po.z, lo.z, hi.z, k.z, p.z);
      adam_elem<BOUNDED, LEGACY>(a, bc1, bc2, g.w, u.w, m.w, v.w, po.w, lo.w, hi.w, k.w, p.w);
      if (bad) {
        const float nan = __builtin_nanf("");
        u = make_float4(nan, nan, nan, nan);
        p = u;
      }
      reinterpret_cast<float4*>(a.m)[i] = m;
      reinterpret_cast<float4*>(a.v)[i] = v;
      if constexpr (BOUNDED) reinterpret_cast<float4*>(a.u)[i] = u;
      if (trow) reinterpret_cast<float4*>(trow)[i] = p;
    } else if (bad) {
      const float nan = __builtin_nanf("");
      p = make_float4(nan, nan, nan, nan);
    }
    if constexpr (MODE == 4) reinterpret_cast<float4*>(a.u)[i] = p;
    if constexpr (PUSH) {
      for (int q = 0; q < a.size; ++q)
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.t.base[q]) + off) = p;
    }
  }
  // grid completion: every thread's pushes are acknowledged before its block takes a
  // ticket; the last block publishes "my slice is everywhere" and waits until every
  // peer's slice has landed here
  uc_release();
  __syncthreads();
  int& last = lds[0];
  if (threadIdx.x == 0) {
    const unsigned tk = atomicAdd(ts_ticket(me), 1u);
    last = tk == (unsigned)nblk - 1;
  }
  __syncthreads();
  if (!last) return;
  if (threadIdx.x == 0) __hip_atomic_store(ts_ticket(me), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((int)threadIdx.x < a.size) uc_signal(ts_tflag(a.f.base[threadIdx.x]) + a.rank, seq);
  ts_wait_all(ts_tflag(me), a.size, seq, a.err, a.ticks, lds + 1);
  if (threadIdx.x == 0) {
    __hip_atomic_store(a.seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.host_step < 0) __hip_atomic_store(a.step, st + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}


// The exchange carried by a compute kernel (fused exchange), peers 4 at a time: unbounded
// Adam (mode 1), or bounded (mode 2, or 3 with the legacy Jacobian) in the kernels' separate
// bounded instantiations (XS = 2 in smf.hip), so the unbounded ones keep their registers.
__device__ __forceinline__ void twoshot_block_fused(const TwoShotArgs& a, int bid, int nblk,
                                                    int* lds) {
  twoshot_block<1, 4>(a, bid, nblk, lds);
}
__device__ __forceinline__ void twoshot_block_fused_bounded(const TwoShotArgs& a, int mode,
                                                            int bid, int nblk, int* lds) {
  if (mode == 3) twoshot_block<3, 4, true>(a, bid, nblk, lds);
  else twoshot_block<2, 4, true>(a, bid, nblk, lds);
}

// Packed launch arguments of one exchange (xgmi_twoshot_pack -> the fused kernels' host
// wrappers): the struct, the mode and the workgroup count, as raw bytes.
struct TwoShotPack {
  TwoShotArgs a;
  int mode;
  int blocks;
};

// Stand-alone launch of a packed exchange on `stream` (xgmi.hip): the fallback of the
// compute launches that cannot carry it (e.g. non-uniform bins in the VJP).
void twoshot_launch(const TwoShotPack& P, hipStream_t stream);

// The packed exchange from the bytes of xgmi_twoshot_pack (host side).
inline TwoShotPack twoshot_unpack(const std::string& b) {
  TwoShotPack P;
  if (b.size() != sizeof(P)) throw std::runtime_error("bad packed two-shot exchange");
  std::memcpy(&P, b.data(), sizeof(P));
  return P;
}

}  // namespace mg
