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
#include "xgmi.h"

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>

#include <cstring>
#include <string>
#include <vector>

namespace mg {

__global__ __launch_bounds__(64) void xgmi_oneshot_kernel(XgmiPeers peers, int rank, int size,
                                                         float* __restrict__ x, int n,
                                                         unsigned* __restrict__ seq_ptr,
                                                         int* __restrict__ err,
                                                         long long timeout_ticks) {
  __shared__ float v[kXMaxFloats];
  if (threadIdx.x < n) v[threadIdx.x] = x[threadIdx.x];
  xgmi_block_allreduce(peers, rank, size, v, n, seq_ptr, err, timeout_ticks);
  if (threadIdx.x < n) x[threadIdx.x] = v[threadIdx.x];
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

// Re-zero this rank's region (flags and inboxes); the caller has drained every kernel
// and synchronised with the peers before and after (OneShotAllReduce.reset).
void xgmi_zero(int64_t base) {
  xcheck(hipMemset(reinterpret_cast<void*>(base), 0, kXRegionBytes), "hipMemset");
  xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
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
