// Device side of the one-shot peer-memory all-reduce (see xgmi.hip for the protocol).
// Shared by the stand-alone all-reduce kernel and by kernels that fuse the exchange into
// their epilogue (smf.hip: slab reduction -> exchange -> loss in one launch).
#pragma once

#include <hip/hip_runtime.h>

namespace mg {

constexpr int kXMaxRanks = 8;
constexpr int kXMaxFloats = 64;
constexpr int kXFlagOff = 0;        // uint32 flags[2][kXMaxRanks]
constexpr int kXDataOff = 256;      // float data[2][kXMaxRanks][kXMaxFloats]
constexpr int64_t kXRegionBytes = kXDataOff + 2 * kXMaxRanks * kXMaxFloats * 4;

struct XgmiPeers {
  char* base[kXMaxRanks];
};

// Ordering without cache maintenance.  Every word a peer reads is in an UNCACHED region
// (hipDeviceMallocUncached: no L2 line is ever allocated for it, on any XCD or GPU), so a
// store is visible to every agent once memory has acknowledged it.  A release is then
// "wait until this thread's stores are acknowledged" (s_waitcnt vmcnt(0); stores count in
// vmcnt on gfx9) and the flag store that follows is a plain system-scope relaxed store;
// an acquire is the polling load itself (relaxed, system scope: it bypasses the caches)
// plus program order.  __threadfence_system() would instead write back and invalidate the
// whole L2 of the GPU (buffer_wbl2 / buffer_inv sc0 sc1) -- on every poll iteration of the
// acquire loads -- stalling this and every other kernel running on the chip.
__device__ __forceinline__ void uc_release() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): all of this thread's stores acknowledged
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ unsigned uc_poll(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void uc_signal(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ unsigned* xflags(char* b) {
  return reinterpret_cast<unsigned*>(b + kXFlagOff);
}
__device__ __forceinline__ float* xdata(char* b) { return reinterpret_cast<float*>(b + kXDataOff); }

// Block-wide in-place SUM of vals[0..n) (n <= 64; vals in shared or global memory,
// written by this block) across `size` ranks.  Every thread of the block must call it.
__device__ __forceinline__ void xgmi_block_allreduce(const XgmiPeers& peers, int rank, int size,
                                                     float* vals, int n, unsigned* seq_ptr,
                                                     int* err, long long timeout_ticks) {
  const int t = threadIdx.x;
  __syncthreads();
  const unsigned seq = *seq_ptr + 1u;
  const int slot = (int)(seq & 1u);
  if (t < n) {
    const float mine = vals[t];
    for (int p = 0; p < size; ++p)
      __hip_atomic_store(xdata(peers.base[p]) + (slot * kXMaxRanks + rank) * kXMaxFloats + t, mine,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  uc_release();
  __syncthreads();
  if (t < size) uc_signal(xflags(peers.base[t]) + slot * kXMaxRanks + rank, seq);
  char* me = peers.base[rank];
  // a peer that never signals (a rank that skipped the call, or is late by more than the
  // timeout) must not yield a silently wrong sum: the error word is raised for the host
  // (checked at the engine's sync points) and the result is poisoned with NaN
  __shared__ int timed_out;
  if (t == 0) timed_out = 0;
  __syncthreads();
  if (t < size) {
    const long long t0 = wall_clock64();
    // after a timeout the protocol is out of step until reset(): fail fast (NaN) instead of
    // waiting out the timeout again in every later call
    const bool dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    while (uc_poll(xflags(me) + slot * kXMaxRanks + t) != seq) {
      if (dead || wall_clock64() - t0 > timeout_ticks) {
        atomicExch(err, 1);
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  asm volatile("" ::: "memory");
  __syncthreads();
  if (t < n) {
    float s = 0.0f;
    for (int q = 0; q < size; ++q)
      s += __hip_atomic_load(xdata(me) + (slot * kXMaxRanks + q) * kXMaxFloats + t,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    vals[t] = timed_out ? __builtin_nanf("") : s;
  }
  __syncthreads();
  if (t == 0) *seq_ptr = seq;
}

}  // namespace mg

namespace mg {

// ---------------------------------------------------------------------------- wide one-shot
// The same push / signal / poll / local-sum protocol for the optimizers' reductions (device
// L-BFGS(-B): the packed inner products of an iteration, the directional derivative of a
// line-search point): up to kXwMax fp64 values per call, values [0, nsum) summed and
// [nsum, nsum + nmax) max-reduced, both in rank order, so every rank holds the same bits.
// Values travel as raw 64-bit words (no fp32 rounding anywhere on the way).
constexpr int kXwMax = 1024;
constexpr int kXwThreads = 256;
constexpr int kXwFlagOff = 0;       // uint32 flags[2][kXMaxRanks]
constexpr int kXwDataOff = 256;     // uint64 data[2][kXMaxRanks][kXwMax]
constexpr int64_t kXwRegionBytes = kXwDataOff + 2LL * kXMaxRanks * kXwMax * 8;

__device__ __forceinline__ unsigned* xwflags(char* b) {
  return reinterpret_cast<unsigned*>(b + kXwFlagOff);
}
__device__ __forceinline__ unsigned long long* xwdata(char* b) {
  return reinterpret_cast<unsigned long long*>(b + kXwDataOff);
}

}  // namespace mg

namespace mg {

// ---------------------------------------------------------------------------- two-shot
// Flag region of the two-shot reduce-scatter / all-gather (one per rank, uncached, IPC
// mapped by every peer): gflag[q] = last step whose gradient rank q has published,
// tflag[q] = last step whose parameter slice rank q has pushed, ticket = grid completion
// counter of the local kernel.
constexpr int kTsGflagOff = 0;
constexpr int kTsTflagOff = 64;
constexpr int kTsTicketOff = 128;
constexpr int64_t kTsFlagBytes = 256;

__device__ __forceinline__ unsigned* ts_gflag(char* b) {
  return reinterpret_cast<unsigned*>(b + kTsGflagOff);
}
__device__ __forceinline__ unsigned* ts_tflag(char* b) {
  return reinterpret_cast<unsigned*>(b + kTsTflagOff);
}
__device__ __forceinline__ unsigned* ts_ticket(char* b) {
  return reinterpret_cast<unsigned*>(b + kTsTicketOff);
}

// Threads t < size of the calling block wait until flag[t] >= seq (monotonic sequence
// numbers, wrap-safe difference); returns 1 (and raises *err) on a timeout -- at once when
// *err is already raised (a protocol out of step until reset(): no second timeout).  Every
// thread of the block must call it.  `to`: one int of LDS (the caller's, so a kernel that
// carries the exchange can lend it from its own LDS instead of growing its footprint).
__device__ __forceinline__ int ts_wait_all(unsigned* flags, int size, unsigned seq, int* err,
                                           long long timeout_ticks, int* to_lds) {
  int& to = *to_lds;
  if (threadIdx.x == 0) to = 0;
  __syncthreads();
  if ((int)threadIdx.x < size) {
    const long long t0 = wall_clock64();
    const bool dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    while ((int)(uc_poll(flags + threadIdx.x) - seq) < 0) {
      if (dead || wall_clock64() - t0 > timeout_ticks) {
        atomicExch(err, 1);
        to = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  asm volatile("" ::: "memory");
  __syncthreads();
  return to;
}

}  // namespace mg
