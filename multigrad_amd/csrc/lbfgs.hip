// Vector kernels for the device L-BFGS (SPMD, optionally sharded across ranks).
//
// Reference: multigrad/bfgs.py drives scipy's compiled L-BFGS-B on the root rank with
// two pickled broadcasts per function evaluation.  The device L-BFGS keeps the history
// (S, Y) on the GPU -- sharded 1/W per rank for 1e7-1e8 parameters -- and needs, per
// iteration, the 2m x 3 dot products [S; Y] . [s_new, y_new, g] (new row/column of
// S^T Y and Y^T Y plus S^T g, Y^T g for the compact inverse-Hessian product).  They are
// computed in ONE pass over the history by `multi_dot` (fp32 per-lane accumulation,
// fp64 fixed-order block and slab reductions: deterministic), and all-reduced across
// ranks as one small RCCL message.  The search direction d = -(gamma g + sum_i c_i H_i)
// is one fused pass (`lincomb`).
#include "common.h"

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <vector>

namespace mg {

constexpr int kDotThreads = 256;
constexpr int kRowGroup = 8;   // history rows per block (blockIdx.y)
constexpr int kMaxCols = 4;    // right-hand vectors

struct RowPtrs {
  const float* p[kMaxCols];
};

// VEC: float4 lanes (rows and vectors 16-byte aligned, lda % 4 == 0); the n % 4 tail is
// taken by the scalar loop.  Measured at 20 rows x 3 vectors x 1e7: 529 us scalar.
template <int NC, bool VEC>
__global__ __launch_bounds__(kDotThreads) void multi_dot_kernel(
    const float* __restrict__ A, int64_t lda, int nrows, RowPtrs B, int nc, int64_t n,
    double* __restrict__ partial) {
  const int r0 = blockIdx.y * kRowGroup;
  float acc[kRowGroup][NC];
#pragma unroll
  for (int i = 0; i < kRowGroup; ++i)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[i][c] = 0.0f;
  const int64_t tid = (int64_t)blockIdx.x * kDotThreads + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * kDotThreads;
  int64_t j0 = 0;
  if constexpr (VEC) {
    const int64_t n4 = n >> 2;
    for (int64_t j = tid; j < n4; j += stride) {
      float4 b[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c)
        b[c] = c < nc ? reinterpret_cast<const float4*>(B.p[c])[j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int i = 0; i < kRowGroup; ++i) {
        if (r0 + i < nrows) {
          const float4 a = reinterpret_cast<const float4*>(A + (int64_t)(r0 + i) * lda)[j];
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            float t = acc[i][c];
            t = fmaf(a.x, b[c].x, t);
            t = fmaf(a.y, b[c].y, t);
            t = fmaf(a.z, b[c].z, t);
            t = fmaf(a.w, b[c].w, t);
            acc[i][c] = t;
          }
        }
      }
    }
    j0 = n4 << 2;
  }
  for (int64_t j = j0 + tid; j < n; j += stride) {
    float b[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) b[c] = c < nc ? B.p[c][j] : 0.0f;
#pragma unroll
    for (int i = 0; i < kRowGroup; ++i) {
      if (r0 + i < nrows) {
        const float a = A[(int64_t)(r0 + i) * lda + j];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[i][c] = fmaf(a, b[c], acc[i][c]);
      }
    }
  }
  __shared__ double scratch[kRowGroup * NC * (kDotThreads / kWave)];
  double v[kRowGroup * NC];
#pragma unroll
  for (int i = 0; i < kRowGroup; ++i)
#pragma unroll
    for (int c = 0; c < NC; ++c) v[i * NC + c] = (double)acc[i][c];
  block_sum_n<kRowGroup * NC>(v, scratch);
  if (threadIdx.x == 0) {
    double* out = partial + ((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * kRowGroup * NC;
#pragma unroll
    for (int k = 0; k < kRowGroup * NC; ++k) out[k] = v[k];
  }
}

// out[r, c] = sum over the column blocks of the partials: one workgroup per output, each
// thread a fixed strided subset, then the fixed shuffle/LDS tree -> deterministic.  (One
// thread per output walking all 1024 partials took 193 us per call.)
__global__ __launch_bounds__(kDotThreads) void multi_dot_reduce_kernel(
    const double* __restrict__ partial, int nblk_x, int ngroups, int nrows, int nc, int ncp,
    double* __restrict__ out) {
  const int t = blockIdx.x;
  const int r = t / nc, c = t % nc;
  const int g = r / kRowGroup, i = r % kRowGroup;
  double s[1] = {0.0};
  for (int b = threadIdx.x; b < nblk_x; b += kDotThreads)
    s[0] += partial[((int64_t)b * ngroups + g) * kRowGroup * ncp + i * ncp + c];
  __shared__ double scratch[kDotThreads / kWave];
  block_sum_n<1>(s, scratch);
  if (threadIdx.x == 0) out[t] = s[0];
}

// y = alpha * x + sum_i coef[i] * H[i, :]   (coef in device memory, nrows <= 64)
__global__ __launch_bounds__(256) void lincomb_kernel(const float* __restrict__ H, int64_t ldh,
                                                      int nrows, const float* __restrict__ coef,
                                                      float alpha, const float* __restrict__ x,
                                                      int64_t n, float* __restrict__ y) {
  __shared__ float c[64];
  if (threadIdx.x < nrows) c[threadIdx.x] = coef[threadIdx.x];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
    float acc = x ? alpha * x[j] : 0.0f;
    for (int i = 0; i < nrows; ++i) acc = fmaf(c[i], H[(int64_t)i * ldh + j], acc);
    y[j] = acc;
  }
}

static int dot_blocks(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + kDotThreads - 1) / kDotThreads, 1024));
}

// A: [nrows, lda] row-major rows; B: list of nc (<= 4) vectors; out [nrows, nc] fp64.
void multi_dot(torch::Tensor A, int64_t nrows, std::vector<torch::Tensor> B, int64_t n,
               torch::Tensor out, torch::Tensor workspace) {
  const int64_t nc = (int64_t)B.size();
  TORCH_CHECK(A.is_cuda() && out.is_cuda() && workspace.is_cuda(), "device tensors");
  TORCH_CHECK(A.scalar_type() == at::kFloat, "fp32 vectors");
  TORCH_CHECK(out.scalar_type() == at::kDouble && workspace.scalar_type() == at::kDouble, "fp64 out");
  TORCH_CHECK(A.dim() == 2 && A.stride(1) == 1, "A must be row-major 2-d");
  TORCH_CHECK(nrows >= 1 && nrows <= A.size(0) && nc >= 1 && nc <= kMaxCols, "bad shape");
  TORCH_CHECK(n <= A.size(1), "n too large");
  TORCH_CHECK(out.numel() >= nrows * nc, "out too small");
  RowPtrs rp;
  for (int c = 0; c < kMaxCols; ++c) rp.p[c] = nullptr;
  for (int64_t c = 0; c < nc; ++c) {
    TORCH_CHECK(B[c].is_cuda() && B[c].scalar_type() == at::kFloat && B[c].is_contiguous() &&
                B[c].numel() >= n, "B vectors: contiguous fp32 device, >= n");
    rp.p[c] = B[c].data_ptr<float>();
  }
  const int bx = dot_blocks(n);
  const int gy = (int)((nrows + kRowGroup - 1) / kRowGroup);
  const int ncp = (int)nc <= 1 ? 1 : (nc <= 2 ? 2 : 4);
  TORCH_CHECK(workspace.numel() >= (int64_t)bx * gy * kRowGroup * ncp, "workspace too small");
  auto stream = at::hip::getCurrentHIPStream();
  const float* a = A.data_ptr<float>();
  double* ws = workspace.data_ptr<double>();
  dim3 grid(bx, gy);
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  bool vec = al16(a) && A.stride(0) % 4 == 0;
  for (int64_t c = 0; c < nc; ++c) vec = vec && al16(rp.p[c]);
#define MG_DOT(NCV)                                                                         \
  do {                                                                                      \
    if (vec)                                                                                \
      hipLaunchKernelGGL((multi_dot_kernel<NCV, true>), grid, dim3(kDotThreads), 0, stream, a, \
                         A.stride(0), (int)nrows, rp, (int)nc, n, ws);                      \
    else                                                                                    \
      hipLaunchKernelGGL((multi_dot_kernel<NCV, false>), grid, dim3(kDotThreads), 0, stream, a, \
                         A.stride(0), (int)nrows, rp, (int)nc, n, ws);                      \
  } while (0)
  if (ncp == 1) MG_DOT(1);
  else if (ncp == 2) MG_DOT(2);
  else MG_DOT(4);
#undef MG_DOT
  const int tot = (int)(nrows * nc);
  hipLaunchKernelGGL(multi_dot_reduce_kernel, dim3(tot), dim3(kDotThreads), 0, stream, ws, bx, gy,
                     (int)nrows, (int)nc, ncp, out.data_ptr<double>());
}

int64_t multi_dot_workspace(int64_t nrows, int64_t n) {
  return (int64_t)dot_blocks(n) * ((nrows + kRowGroup - 1) / kRowGroup) * kRowGroup * kMaxCols;
}

void lincomb(torch::Tensor H, int64_t nrows, torch::Tensor coef, double alpha,
             c10::optional<torch::Tensor> x, int64_t n, torch::Tensor y) {
  TORCH_CHECK(H.is_cuda() && coef.is_cuda() && y.is_cuda(), "device tensors");
  TORCH_CHECK(H.scalar_type() == at::kFloat && coef.scalar_type() == at::kFloat &&
              y.scalar_type() == at::kFloat, "fp32");
  TORCH_CHECK(H.dim() == 2 && H.stride(1) == 1 && nrows <= H.size(0) && nrows <= 64 &&
              coef.numel() >= nrows && n <= H.size(1) && y.numel() >= n, "bad shapes");
  const float* xp = nullptr;
  if (x.has_value() && x->defined()) {
    TORCH_CHECK(x->is_cuda() && x->scalar_type() == at::kFloat && x->numel() >= n, "bad x");
    xp = x->data_ptr<float>();
  }
  auto stream = at::hip::getCurrentHIPStream();
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 2048));
  hipLaunchKernelGGL(lincomb_kernel, dim3(blocks), dim3(256), 0, stream, H.data_ptr<float>(),
                     H.stride(0), (int)nrows, coef.data_ptr<float>(), (float)alpha, xp, n,
                     y.data_ptr<float>());
}

}  // namespace mg
