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
#include "adam.h"
#include "common.h"
#include "twoshot.h"
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

// Wide one-shot (xgmi.h): in-place all-reduce of x[0, nsum + nmax) fp64, [0, nsum) summed
// and the rest max-reduced, in rank order.  One workgroup; the protocol (two slots, the
// sequence number in device memory, bounded waits that NaN-poison the result) is the one of
// xgmi_oneshot_kernel.
__global__ __launch_bounds__(kXwThreads) void xgmi_oneshot_wide_kernel(
    XgmiPeers peers, int rank, int size, double* __restrict__ x, int nsum, int nmax,
    unsigned* __restrict__ seq_ptr, int* __restrict__ err, long long timeout_ticks) {
  const int t = threadIdx.x;
  const int n = nsum + nmax;
  const unsigned seq = *seq_ptr + 1u;
  const int slot = (int)(seq & 1u);
  for (int i = t; i < n; i += kXwThreads) {
    const unsigned long long bits = (unsigned long long)__double_as_longlong(x[i]);
    for (int p = 0; p < size; ++p)
      __hip_atomic_store(xwdata(peers.base[p]) + (int64_t)(slot * kXMaxRanks + rank) * kXwMax + i,
                         bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  uc_release();
  __syncthreads();
  if (t < size) uc_signal(xwflags(peers.base[t]) + slot * kXMaxRanks + rank, seq);
  char* me = peers.base[rank];
  __shared__ int timed_out;
  if (t == 0) timed_out = 0;
  __syncthreads();
  if (t < size) {
    const long long t0 = wall_clock64();
    const bool dead = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    while (uc_poll(xwflags(me) + slot * kXMaxRanks + t) != seq) {
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
  for (int i = t; i < n; i += kXwThreads) {
    double s = 0.0;
    for (int q = 0; q < size; ++q) {
      const double v = __longlong_as_double((long long)__hip_atomic_load(
          xwdata(me) + (int64_t)(slot * kXMaxRanks + q) * kXwMax + i, __ATOMIC_RELAXED,
          __HIP_MEMORY_SCOPE_SYSTEM));
      if (q == 0) s = v;
      else if (i < nsum) s += v;
      else s = v > s ? v : s;
    }
    x[i] = timed_out ? __builtin_nan("") : s;
  }
  __syncthreads();
  if (t == 0) *seq_ptr = seq;
}

static void xcheck(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

// Allocate and zero an uncached region of `bytes` (default: the one-shot region); returns
// its device address.  Uncached (MTYPE UC): remote stores/loads over xGMI and local
// accesses see each other without any cache maintenance.
int64_t xgmi_alloc(int64_t bytes) {
  if (bytes <= 0) bytes = kXRegionBytes;
  void* p = nullptr;
  xcheck(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached), "hipExtMallocWithFlags");
  xcheck(hipMemset(p, 0, (size_t)bytes), "hipMemset");
  xcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return reinterpret_cast<int64_t>(p);
}

// A float32 tensor aliasing `numel` floats at `ptr` on the current device (the caller
// keeps the region alive for the tensor's lifetime).
torch::Tensor xgmi_tensor(int64_t ptr, int64_t numel) {
  int dev = 0;
  xcheck(hipGetDevice(&dev), "hipGetDevice");
  auto opts = torch::TensorOptions().dtype(torch::kFloat32).device(torch::kCUDA, dev);
  return torch::from_blob(reinterpret_cast<void*>(ptr), {numel}, [](void*) {}, opts);
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
void xgmi_zero(int64_t base, int64_t bytes) {
  if (bytes <= 0) bytes = kXRegionBytes;
  xcheck(hipMemset(reinterpret_cast<void*>(base), 0, (size_t)bytes), "hipMemset");
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

// In-place fp64 all-reduce of x[0, nsum + nmax) over the ranks of `peers` (wide one-shot
// regions, xgmi_alloc(xgmi_wide_region_bytes())): [0, nsum) summed, the rest max-reduced.
void xgmi_allreduce_wide(torch::Tensor x, int64_t nsum, int64_t nmax, std::vector<int64_t> peers,
                         int64_t rank, torch::Tensor seq, torch::Tensor err, double timeout_s) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous() && x.scalar_type() == at::kDouble,
              "x: contiguous fp64 device");
  TORCH_CHECK(nsum >= 0 && nmax >= 0 && nsum + nmax >= 1 && nsum + nmax <= kXwMax &&
              nsum + nmax <= x.numel(), "wide one-shot all-reduce takes 1..1024 values");
  const int size = (int)peers.size();
  TORCH_CHECK(size >= 1 && size <= kXMaxRanks && rank >= 0 && rank < size, "bad rank/size");
  TORCH_CHECK(seq.is_cuda() && seq.scalar_type() == at::kInt && err.is_cuda() &&
              err.scalar_type() == at::kInt, "seq/err: int32 device");
  XgmiPeers p;
  for (int r = 0; r < kXMaxRanks; ++r) p.base[r] = r < size ? reinterpret_cast<char*>(peers[r]) : nullptr;
  const long long ticks = (long long)(timeout_s * 1e8);
  hipLaunchKernelGGL(xgmi_oneshot_wide_kernel, dim3(1), dim3(kXwThreads), 0,
                     at::hip::getCurrentHIPStream(), p, (int)rank, size, x.data_ptr<double>(),
                     (int)nsum, (int)nmax, reinterpret_cast<unsigned*>(seq.data_ptr<int>()),
                     err.data_ptr<int>(), ticks);
}

int64_t xgmi_wide_region_bytes() { return kXwRegionBytes; }

// PCI bus id of the current device: ranks that report the same id (and host) share one GPU
// and size their peer-memory exchange grids so that every rank's exchange workgroups can
// be resident at once (parallel/xgmi.py).
std::string device_pci_bus_id() {
  int dev = 0;
  xcheck(hipGetDevice(&dev), "hipGetDevice");
  char buf[64] = {0};
  xcheck(hipDeviceGetPCIBusId(buf, (int)sizeof(buf) - 1, dev), "hipDeviceGetPCIBusId");
  return std::string(buf);
}


// ============================================================================ two-shot
// Reduce-scatter -> Adam -> all-gather of the dense gradient over peer memory, ONE launch
// per optimizer step (reference multigrad/multigrad.py:531-532, the P-float
// gradient Allreduce, plus the Adam update of multigrad/adam.py:52-68).
//
// Every rank holds three uncached, IPC-exported regions: its gradient g_r (written by the
// VJP), its parameter vector theta_r (read by the forward) and a flag region.  Rank r owns
// the float range [lo_r, lo_r + n_r) (1/W of the vector, ZeRO-1 optimizer state).  One
// call on rank r, step seq:
//
//   block 0:  gflag_q[r] = seq on every rank q          (my gradient is complete)
//   all blocks: wait gflag_r[q] >= seq for every q
//   for each float4 of the owned range:                  (grid-stride, 16 B per access)
//       g = g_0 + g_1 + ... + g_{W-1}   (peer loads over xGMI, FIXED rank order)
//       Adam on (u, m, v) of the slice  (adam.h: the same bits as csrc/adam.hip)
//       theta_q[i] = p for every rank q (peer stores over xGMI = the all-gather)
//       trajectory row (owned slice)
//   last block (grid ticket): tflag_q[r] = seq on every q, wait tflag_r[q] >= seq for all q
//
// The pulls (peer -> me) and pushes (me -> peer) run on all W-1 links of the fully
// connected node at once: each link carries P/W floats of gradient and P/W floats of
// parameters in each direction, where a single ring pushes (W-1)/W * P floats per phase
// through ONE outgoing link per GPU.
// The kernel returns only when every rank's slice has landed everywhere, so the next
// forward reads complete parameters with no further synchronisation, and no rank can
// overwrite its gradient (next VJP) while a peer still reads it.  The sequence number
// lives in device memory (graph replayable); bounded waits raise err and NaN-poison the
// owned slice instead of hanging.
template <int MODE>
__global__ __launch_bounds__(kTsThreads) void xgmi_twoshot_kernel(TwoShotArgs a) {
  __shared__ int lds[2];
  twoshot_block<MODE>(a, blockIdx.x, gridDim.x, lds);
}

static XgmiPeers peers_of(const std::vector<int64_t>& v) {
  XgmiPeers p;
  for (int r = 0; r < kXMaxRanks; ++r) p.base[r] = r < (int)v.size() ? reinterpret_cast<char*>(v[r]) : nullptr;
  return p;
}

static float* opt_ptr(const c10::optional<torch::Tensor>& t, int64_t numel, const char* name) {
  if (!t.has_value() || !t->defined() || t->numel() == 0) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->is_contiguous() && t->scalar_type() == at::kFloat, name,
              ": contiguous fp32 device tensor");
  TORCH_CHECK(numel < 0 || t->numel() >= numel, name, " too small");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, name, " must be 16-byte aligned");
  return t->data_ptr<float>();
}

// Launch arguments of one two-shot step (see above).  mode: 0 sum, 1 Adam, 2 bounded
// Adam, 3 bounded legacy, 4 reduce-scatter into u, 5 all-gather of u (twoshot.h).  scalars: [host_step, lr, b1, b2, eps, timeout_s, traj_stride
// (, max_blocks)]; returns the packed arguments with the mode and the workgroup count.
static TwoShotPack twoshot_args(std::vector<int64_t> gbufs, std::vector<int64_t> tbufs,
                                std::vector<int64_t> flags, int64_t rank, int64_t lo, int64_t n,
                                int64_t total, int64_t mode, c10::optional<torch::Tensor> u,
                                c10::optional<torch::Tensor> m, c10::optional<torch::Tensor> v,
                                c10::optional<torch::Tensor> blo, c10::optional<torch::Tensor> bhi,
                                c10::optional<torch::Tensor> kind, c10::optional<torch::Tensor> traj,
                                torch::Tensor step, torch::Tensor seq, torch::Tensor err,
                                std::vector<double> scalars) {
  const int size = (int)gbufs.size();
  TORCH_CHECK(size >= 1 && size <= kXMaxRanks && (int)tbufs.size() == size && (int)flags.size() == size,
              "two-shot: 1..8 ranks, one region of each kind per rank");
  TORCH_CHECK(rank >= 0 && rank < size, "bad rank");
  TORCH_CHECK(lo >= 0 && n >= 0 && lo % 4 == 0 && n % 4 == 0 && lo + n <= total,
              "owned range must be float4 aligned and inside the vector");
  TORCH_CHECK(mode >= 0 && mode <= 5, "bad mode");
  TORCH_CHECK(scalars.size() == 7 || scalars.size() == 8,
              "scalars: host_step, lr, b1, b2, eps, timeout_s, traj_stride[, max_blocks]");
  TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kInt && step.numel() >= 2, "step: [2] int32 device");
  TORCH_CHECK(seq.is_cuda() && seq.scalar_type() == at::kInt && err.is_cuda() && err.scalar_type() == at::kInt,
              "seq/err: int32 device");
  TwoShotPack P;
  TwoShotArgs& a = P.a;
  a.g = peers_of(gbufs);
  a.t = peers_of(tbufs);
  a.f = peers_of(flags);
  a.rank = (int)rank;
  a.size = size;
  a.lo = lo;
  a.n = n;
  a.u = opt_ptr(u, n, "u");
  a.m = opt_ptr(m, n, "m");
  a.v = opt_ptr(v, n, "v");
  a.blo = opt_ptr(blo, n, "lo");
  a.bhi = opt_ptr(bhi, n, "hi");
  a.kind = nullptr;
  if (kind.has_value() && kind->defined() && kind->numel()) {
    TORCH_CHECK(kind->is_cuda() && kind->scalar_type() == at::kChar && kind->numel() >= n, "kind: int8 [n]");
    TORCH_CHECK((reinterpret_cast<uintptr_t>(kind->data_ptr()) & 3) == 0, "kind must be 4-byte aligned");
    a.kind = kind->data_ptr<int8_t>();
  }
  a.traj = opt_ptr(traj, -1, "traj");
  a.traj_stride = (int64_t)scalars[6];
  TORCH_CHECK(a.traj_stride % 4 == 0, "trajectory stride must keep float4 alignment");
  if (mode >= 1 && mode <= 3) TORCH_CHECK(a.m && a.v, "Adam modes need m and v");
  if (mode == 2 || mode == 3)
    TORCH_CHECK(a.u && a.blo && a.bhi && a.kind, "bounded modes need u and the bounds");
  if (mode >= 4) TORCH_CHECK(a.u, "reduce-scatter / all-gather modes need the local slice u");
  a.step = step.data_ptr<int>();
  a.host_step = (int)scalars[0];
  a.lr = (float)scalars[1];
  a.b1 = (float)scalars[2];
  a.b2 = (float)scalars[3];
  a.eps = (float)scalars[4];
  a.ticks = (long long)(scalars[5] * 1e8);
  a.seq = reinterpret_cast<unsigned*>(seq.data_ptr<int>());
  a.err = err.data_ptr<int>();
  const int64_t n4 = n / 4;
  // grid cap: 1024 by default; a smaller cap (scalars[7]) leaves the CUs to the compute
  // kernels an exchange on a side stream overlaps (the grid-stride loop covers any size)
  const int64_t cap = scalars.size() == 8 && scalars[7] >= 1 ? std::min<int64_t>((int64_t)scalars[7], 1024) : 1024;
  P.mode = (int)mode;
  P.blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n4 + kTsThreads - 1) / kTsThreads, cap));
  return P;
}

// One two-shot step (see above), launched on the current stream.
void xgmi_twoshot(std::vector<int64_t> gbufs, std::vector<int64_t> tbufs, std::vector<int64_t> flags,
                  int64_t rank, int64_t lo, int64_t n, int64_t total, int64_t mode,
                  c10::optional<torch::Tensor> u, c10::optional<torch::Tensor> m,
                  c10::optional<torch::Tensor> v, c10::optional<torch::Tensor> blo,
                  c10::optional<torch::Tensor> bhi, c10::optional<torch::Tensor> kind,
                  c10::optional<torch::Tensor> traj, torch::Tensor step, torch::Tensor seq,
                  torch::Tensor err, std::vector<double> scalars) {
  const TwoShotPack P = twoshot_args(gbufs, tbufs, flags, rank, lo, n, total, mode, u, m, v, blo,
                                     bhi, kind, traj, step, seq, err, scalars);
  twoshot_launch(P, at::hip::getCurrentHIPStream());
}

void twoshot_launch(const TwoShotPack& P, hipStream_t stream) {
  switch (P.mode) {
    case 0: hipLaunchKernelGGL(xgmi_twoshot_kernel<0>, dim3(P.blocks), dim3(kTsThreads), 0, stream, P.a); break;
    case 1: hipLaunchKernelGGL(xgmi_twoshot_kernel<1>, dim3(P.blocks), dim3(kTsThreads), 0, stream, P.a); break;
    case 2: hipLaunchKernelGGL(xgmi_twoshot_kernel<2>, dim3(P.blocks), dim3(kTsThreads), 0, stream, P.a); break;
    case 3: hipLaunchKernelGGL(xgmi_twoshot_kernel<3>, dim3(P.blocks), dim3(kTsThreads), 0, stream, P.a); break;
    case 4: hipLaunchKernelGGL(xgmi_twoshot_kernel<4>, dim3(P.blocks), dim3(kTsThreads), 0, stream, P.a); break;
    default: hipLaunchKernelGGL(xgmi_twoshot_kernel<5>, dim3(P.blocks), dim3(kTsThreads), 0, stream, P.a); break;
  }
}

// A packed exchange launched on its own on the current stream (the last chunk's exchange
// of a fused-exchange step when no further compute launch carries it).
void xgmi_twoshot_launch_packed(std::string packed) {
  twoshot_launch(twoshot_unpack(packed), at::hip::getCurrentHIPStream());
}

// The same step's arguments packed as bytes, for a compute launch that runs the exchange
// in its first workgroups (smf.hip fused exchange: smf_forward / smf_vjp ``exchange``);
// Adam modes only.  The tensors must stay alive until that launch is enqueued.
pybind11::bytes xgmi_twoshot_pack(std::vector<int64_t> gbufs, std::vector<int64_t> tbufs,
                                  std::vector<int64_t> flags, int64_t rank, int64_t lo, int64_t n,
                                  int64_t total, int64_t mode, c10::optional<torch::Tensor> u,
                                  c10::optional<torch::Tensor> m, c10::optional<torch::Tensor> v,
                                  c10::optional<torch::Tensor> blo, c10::optional<torch::Tensor> bhi,
                                  c10::optional<torch::Tensor> kind, c10::optional<torch::Tensor> traj,
                                  torch::Tensor step, torch::Tensor seq, torch::Tensor err,
                                  std::vector<double> scalars) {
  TORCH_CHECK(mode >= 1 && mode <= 3, "a fused exchange is an Adam step (mode 1..3)");
  const TwoShotPack P = twoshot_args(gbufs, tbufs, flags, rank, lo, n, total, mode, u, m, v, blo,
                                     bhi, kind, traj, step, seq, err, scalars);
  return pybind11::bytes(reinterpret_cast<const char*>(&P), sizeof(P));
}

int64_t xgmi_twoshot_flag_bytes() { return kTsFlagBytes; }


// ============================================================================ all-to-all-v
// Pull-mode all-to-all-v over peer memory: the setup-time re-partition of a data-parallel
// shard by parameter owner (parallel/alltoall.py, Comm.all_to_all_v).  Every rank has packed
// its send rows by destination into an exported region; rank r reads source q's segment for
// r (q's send displacement of r, C[q][r] 32-bit words) straight over the q<->r xGMI link and
// writes it at r's receive displacement of q.  All W-1 incoming links are busy at once
// (blockIdx.y walks the sources), where a ring would push every byte through one link per
// hop.  Host barriers bracket the launch (every sender's packing is complete before it,
// every pull after it), so no device flags are involved; the caller verifies per-segment
// checksums before trusting the result.
struct A2aSegs {
  const uint32_t* src[kXMaxRanks];
  int64_t n[kXMaxRanks];
  int64_t dst[kXMaxRanks];
};

constexpr int kA2aThreads = 256;
constexpr int kA2aUnroll = 4;

__global__ __launch_bounds__(kA2aThreads) void xgmi_a2a_pull_kernel(A2aSegs s,
                                                                    uint32_t* __restrict__ out) {
  const int q = blockIdx.y;
  const uint32_t* __restrict__ src = s.src[q];
  uint32_t* __restrict__ dst = out + s.dst[q];
  const int64_t n = s.n[q];
  const int64_t S = (int64_t)gridDim.x * kA2aThreads;
  int64_t i = (int64_t)blockIdx.x * kA2aThreads + threadIdx.x;
  // kA2aUnroll independent remote loads in flight per thread before the stores
  for (; i + (kA2aUnroll - 1) * S < n; i += kA2aUnroll * S) {
    uint32_t v[kA2aUnroll];
#pragma unroll
    for (int k = 0; k < kA2aUnroll; ++k) v[k] = src[i + k * S];
#pragma unroll
    for (int k = 0; k < kA2aUnroll; ++k) dst[i + k * S] = v[k];
  }
  for (; i < n; i += S) dst[i] = src[i];
}

// out[dst_offs[q] : + counts[q]] = words at src_ptrs[q] (peer addresses, already offset to the
// segment), for every source q; counts / offsets in 32-bit words.  Launched on the current
// stream; the caller synchronises.
void xgmi_a2a_pull(std::vector<int64_t> src_ptrs, std::vector<int64_t> counts,
                   std::vector<int64_t> dst_offs, torch::Tensor out) {
  const int nsrc = (int)src_ptrs.size();
  TORCH_CHECK(nsrc >= 1 && nsrc <= kXMaxRanks && (int)counts.size() == nsrc &&
              (int)dst_offs.size() == nsrc, "all-to-all pull: 1..8 sources, one count/offset each");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.element_size() == 4,
              "all-to-all pull: contiguous 32-bit device output");
  A2aSegs s;
  int64_t nmax = 0;
  for (int q = 0; q < kXMaxRanks; ++q) {
    s.src[q] = q < nsrc ? reinterpret_cast<const uint32_t*>(src_ptrs[q]) : nullptr;
    s.n[q] = q < nsrc ? counts[q] : 0;
    s.dst[q] = q < nsrc ? dst_offs[q] : 0;
    if (q < nsrc) {
      TORCH_CHECK(counts[q] >= 0 && dst_offs[q] >= 0 && dst_offs[q] + counts[q] <= out.numel(),
                  "all-to-all pull: segment ", q, " outside the output");
      TORCH_CHECK(counts[q] == 0 || (src_ptrs[q] != 0 && (src_ptrs[q] & 3) == 0),
                  "all-to-all pull: segment ", q, " has no 4-byte aligned source");
      nmax = std::max(nmax, counts[q]);
    }
  }
  if (nmax == 0) return;
  const int64_t per = (int64_t)kA2aThreads * kA2aUnroll;
  const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((nmax + per - 1) / per, 2048));
  hipLaunchKernelGGL(xgmi_a2a_pull_kernel, dim3(gx, nsrc), dim3(kA2aThreads), 0,
                     at::hip::getCurrentHIPStream(), s,
                     reinterpret_cast<uint32_t*>(out.data_ptr()));
}

}  // namespace mg
