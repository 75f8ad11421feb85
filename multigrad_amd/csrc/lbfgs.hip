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

template <int NC>
__global__ __launch_bounds__(kDotThreads) void multi_dot_kernel(
    const float* __restrict__ A, int64_t lda, int nrows, RowPtrs B, int nc, int64_t n,
    double* __restrict__ partial) {
  const int r0 = blockIdx.y * kRowGroup;
  float acc[kRowGroup][NC];
#pragma unroll
  for (int i = 0; i < kRowGroup; ++i)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[i][c] = 0.0f;
  const int64_t stride = (int64_t)gridDim.x * kDotThreads;
  for (int64_t j = (int64_t)blockIdx.x * kDotThreads + threadIdx.x; j < n; j += stride) {
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

// out[r, c] = sum over column blocks (fixed order) of the partials.
__global__ void multi_dot_reduce_kernel(const double* __restrict__ partial, int nblk_x, int ngroups,
                                        int nrows, int nc, int ncp, double* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nrows * nc) return;
  const int r = t / nc, c = t % nc;
  const int g = r / kRowGroup, i = r % kRowGroup;
  double s = 0.0;
  for (int b = 0; b < nblk_x; ++b) s += partial[((int64_t)b * ngroups + g) * kRowGroup * ncp + i * ncp + c];
  out[t] = s;
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
  if (ncp == 1) hipLaunchKernelGGL(multi_dot_kernel<1>, grid, dim3(kDotThreads), 0, stream, a, A.stride(0), (int)nrows, rp, (int)nc, n, ws);
  else if (ncp == 2) hipLaunchKernelGGL(multi_dot_kernel<2>, grid, dim3(kDotThreads), 0, stream, a, A.stride(0), (int)nrows, rp, (int)nc, n, ws);
  else hipLaunchKernelGGL(multi_dot_kernel<4>, grid, dim3(kDotThreads), 0, stream, a, A.stride(0), (int)nrows, rp, (int)nc, n, ws);
  const int tot = (int)(nrows * nc);
  hipLaunchKernelGGL(multi_dot_reduce_kernel, dim3((tot + 255) / 256), dim3(256), 0, stream, ws, bx, gy,
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
