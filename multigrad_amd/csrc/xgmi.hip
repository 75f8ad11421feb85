// One-shot all-reduce for tiny fp32 vectors over peer GPU memory (xGMI), SURVEY §5.8.3.
//
// The per-step sumstat all-reduce of the engine moves K <= 64 floats: it is pure
// latency.  RCCL's small-message path runs a ring/tree protocol; on a fully connected
// xGMI node every GPU can instead write its K values straight into every peer's inbox
// and read the W inboxes locally:
//
//   rank r, call seq (slot = seq & 1):
//     for every rank p:  inbox_p[slot][r][:] = x        (remote stores, system scope)
//     fence; for every rank p:  flag_p[slot][r] = seq    (release, system scope)
//     wait until flag_r[slot][q] == seq for every q      (acquire, local polling)
//     x = sum_q inbox_r[slot][q][:]   in rank order      (bitwise identical on all ranks)
//
// Two slots suffice: a rank can only start call seq+2 after every peer has signalled
// seq+1, i.e. after every peer finished reading the slot of call seq.  The sequence
// number lives in device memory, so the kernel is HIP-graph replayable.  Each rank's
// region is allocated uncached (hipDeviceMallocUncached) so remote stores and local
// polling see each other without cache maintenance, exported with hipIpcGetMemHandle and
// mapped by the peers with hipIpcOpenMemHandle.  A bounded wait (wall clock) turns a
// protocol error into an error flag instead of a hung GPU.
//
// Used for tiny device all-reduces after a start-up self-test passes on every rank
// (multigrad_amd/parallel/xgmi.py; MULTIGRAD_ALLREDUCE=rccl disables it); verified with two
// processes sharing one GPU (tests/test_xgmi_gpu.py).
#include "common.h"

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstring>
#include <string>
#include <vector>

namespace mg {

constexpr int kXMaxRanks = 8;
constexpr int kXMaxFloats = 64;
constexpr int kXFlagOff = 0;        // uint32 flags[2][kXMaxRanks]
constexpr int kXDataOff = 256;      // float data[2][kXMaxRanks][kXMaxFloats]
constexpr int64_t kXRegionBytes = kXDataOff + 2 * kXMaxRanks * kXMaxFloats * 4;

struct XgmiPeers {
  char* base[kXMaxRanks];
};

__device__ __forceinline__ unsigned* xflags(char* b) {
  return reinterpret_cast<unsigned*>(b + kXFlagOff);
}
__device__ __forceinline__ float* xdata(char* b) { return reinterpret_cast<float*>(b + kXDataOff); }

__global__ __launch_bounds__(64) void xgmi_oneshot_kernel(XgmiPeers peers, int rank, int size,
                                                         float* __restrict__ x, int n,
                                                         unsigned* __restrict__ seq_ptr,
                                                         int* __restrict__ err,
                                                         long long timeout_ticks) {
  const int t = threadIdx.x;
  const unsigned seq = *seq_ptr + 1u;
  const int slot = (int)(seq & 1u);
  const float mine = t < n ? x[t] : 0.0f;
  for (int p = 0; p < size; ++p)
    if (t < n)
      __hip_atomic_store(xdata(peers.base[p]) + (slot * kXMaxRanks + rank) * kXMaxFloats + t, mine,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  __syncthreads();
  if (t < size)
    __hip_atomic_store(xflags(peers.base[t]) + slot * kXMaxRanks + rank, seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  char* me = peers.base[rank];
  if (t < size) {
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(xflags(me) + slot * kXMaxRanks + t, __ATOMIC_ACQUIRE,
                             __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      if (wall_clock64() - t0 > timeout_ticks) {
        atomicExch(err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __threadfence_system();
  __syncthreads();
  if (t < n) {
    float s = 0.0f;
    for (int q = 0; q < size; ++q)
      s += __hip_atomic_load(xdata(me) + (slot * kXMaxRanks + q) * kXMaxFloats + t,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    x[t] = s;
  }
  if (t == 0) *seq_ptr = seq;
}

static void xcheck(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

// Allocate and zero this rank's region; returns its device address.
int64_t xgmi_alloc() {
  void* p = nullptr;
  xcheck(hipExtMallocWithFlags(&p, kXRegionBytes, hipDeviceMallocUncached), "hipExtMallocWithFlags");
  xcheck(hipMemset(p, 0, kXRegionBytes), "hipMemset");
  xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return reinterpret_cast<int64_t>(p);
}

pybind11::bytes xgmi_handle(int64_t base) {
  hipIpcMemHandle_t h;
  xcheck(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base)), "hipIpcGetMemHandle");
  return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
}

int64_t xgmi_open(pybind11::bytes handle) {
  std::string s = handle;
  hipIpcMemHandle_t h;
  TORCH_CHECK(s.size() == sizeof(h), "bad IPC handle size");
  std::memcpy(&h, s.data(), sizeof(h));
  void* p = nullptr;
  xcheck(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  return reinterpret_cast<int64_t>(p);
}

void xgmi_close(int64_t ptr) { (void)hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr)); }
void xgmi_free(int64_t ptr) { (void)hipFree(reinterpret_cast<void*>(ptr)); }

// In-place SUM of the fp32 vector x (n <= 64) across `size` ranks; peers[r] is rank r's
// region as mapped in this process (our own region at peers[rank]).
void xgmi_allreduce(torch::Tensor x, std::vector<int64_t> peers, int64_t rank, torch::Tensor seq,
                    torch::Tensor err, double timeout_s) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == at::kFloat, "x: contiguous fp32 device");
  TORCH_CHECK(x.numel() >= 1 && x.numel() <= kXMaxFloats, "one-shot all-reduce takes 1..64 floats");
  const int size = (int)peers.size();
  TORCH_CHECK(size >= 1 && size <= kXMaxRanks && rank >= 0 && rank < size, "bad rank/size");
  TORCH_CHECK(seq.is_cuda() && seq.scalar_type() == at::kInt && err.is_cuda() &&
              err.scalar_type() == at::kInt, "seq/err: int32 device");
  XgmiPeers p;
  for (int r = 0; r < kXMaxRanks; ++r) p.base[r] = r < size ? reinterpret_cast<char*>(peers[r]) : nullptr;
  const long long ticks = (long long)(timeout_s * 1e8);  // wall_clock64: 100 MHz
  hipLaunchKernelGGL(xgmi_oneshot_kernel, dim3(1), dim3(64), 0, at::hip::getCurrentHIPStream(), p,
                     (int)rank, size, x.data_ptr<float>(), (int)x.numel(),
                     reinterpret_cast<unsigned*>(seq.data_ptr<int>()), err.data_ptr<int>(), ticks);
}

}  // namespace mg
