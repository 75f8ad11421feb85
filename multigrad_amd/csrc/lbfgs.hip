// Vector kernels for the device L-BFGS (SPMD, optionally sharded across ranks).
//
// Reference: multigrad/bfgs.py drives scipy's compiled L-BFGS-B on the root rank with
// two pickled broadcasts per function evaluation.  The device L-BFGS keeps the history
// (S, Y) on the GPU -- sharded 1/W per rank for 1e7-1e8 parameters -- and needs, per
// iteration, the 2m x 3 dot products [S; Y] . [s_new, y_new, g] (new row/column of
// S^T Y and Y^T Y plus S^T g, Y^T g for the compact inverse-Hessian product).  They are
// computed in ONE pass over the history by `multi_dot` (fp32 per-lane accumulation,
// fp64 fixed-order block and slab reductions: deterministic), and all-reduced across
// ranks as one device all-reduce (optim/_reduce.py: the wide one-shot peer-memory kernel,
// else RCCL).  The search direction d = -(gamma g + sum_i c_i H_i)
// is one fused pass (`lincomb`).
#include "common.h"

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <vector>

namespace mg {

constexpr int kDotThreads = 256;
constexpr int kDotWaves = kDotThreads / kWave;
constexpr int kMaxCols = 4;    // right-hand vectors
constexpr int kDotMaxBlocks = 2048;

struct RowPtrs {
  const float* p[kMaxCols];
};

// SPLIT (>= 4 rows): the 4 waves of a workgroup take the same float4 chunks of the NC
// right-hand vectors and RPW rows each (wave w: rows r0 + w RPW ..), so a chunk of the
// vectors comes from HBM once and reaches the other waves from the caches, while each row
// is read once; about 60 VGPRs at 6 rows x 3 vectors (8 waves per SIMD).  (Round 4 had
// thread-private groups of 8 rows in separate workgroups, which re-read the vectors from
// HBM for every group: 4.0 TB/s at 23 rows x 3 vectors x 1e7.)
// Not SPLIT (1-3 rows): every thread takes all RPW rows of its own chunks.
// Row indices past nrows are clamped to the last row (their sums are never read), so the
// loads of a chunk carry no branches and are all in flight before the FMAs.  fp32 partial
// sums per lane, then fp64 reductions in a fixed order (wave shuffles, LDS, the per-output
// reduce kernel): deterministic.
template <int NC, int RPW, bool SPLIT, bool VEC>
__global__ __launch_bounds__(kDotThreads) void multi_dot_kernel(
    const float* __restrict__ A, int64_t lda, int nrows, RowPtrs B, int64_t n,
    double* __restrict__ partial) {
  constexpr int RB = SPLIT ? kDotWaves * RPW : RPW;  // rows per workgroup
  constexpr int TPB = SPLIT ? kWave : kDotThreads;    // threads per chunk set
  const int wid = threadIdx.x / kWave;
  const int lane = threadIdx.x % kWave;
  const int r0 = blockIdx.y * RB + (SPLIT ? wid * RPW : 0);
  const float* rows[RPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) rows[i] = A + (int64_t)min(r0 + i, nrows - 1) * lda;
  float acc[RPW][NC];
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[i][c] = 0.0f;
  const int64_t tid = (int64_t)blockIdx.x * TPB + (SPLIT ? lane : (int)threadIdx.x);
  const int64_t stride = (int64_t)gridDim.x * TPB;
  int64_t j0 = 0;
  if constexpr (VEC) {
    const int64_t n4 = n >> 2;
    for (int64_t j = tid; j < n4; j += stride) {
      float4 b[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) b[c] = reinterpret_cast<const float4*>(B.p[c])[j];
      float4 a[RPW];
#pragma unroll
      for (int i = 0; i < RPW; ++i) a[i] = reinterpret_cast<const float4*>(rows[i])[j];
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          float t = acc[i][c];
          t = fmaf(a[i].x, b[c].x, t);
          t = fmaf(a[i].y, b[c].y, t);
          t = fmaf(a[i].z, b[c].z, t);
          t = fmaf(a[i].w, b[c].w, t);
          acc[i][c] = t;
        }
      }
    }
    j0 = n4 << 2;
  }
  for (int64_t j = j0 + tid; j < n; j += stride) {
    float b[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) b[c] = B.p[c][j];
#pragma unroll
    for (int i = 0; i < RPW; ++i) {
      const float a = rows[i][j];
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[i][c] = fmaf(a, b[c], acc[i][c]);
    }
  }
  constexpr int K = RPW * NC;
  double* out = partial + ((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * RB * NC;
  if constexpr (SPLIT) {
    // each wave owns its rows: wave reductions, lane 0 writes
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const double v = wave_sum((double)acc[k / NC][k % NC]);
      if (lane == 0) out[wid * K + k] = v;
    }
  } else {
    __shared__ double scratch[8 * kDotWaves];
#pragma unroll
    for (int k0 = 0; k0 < K; k0 += 8) {
      double v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = k0 + j < K ? (double)acc[(k0 + j) / NC][(k0 + j) % NC] : 0.0;
      block_sum_n<8>(v, scratch);
      if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k0 + j < K) out[k0 + j] = v[j];
      }
      __syncthreads();
    }
  }
}

// out[r, c] = sum over the column blocks of the partials: one workgroup per output, each
// thread a fixed strided subset, then the fixed shuffle/LDS tree -> deterministic.  (One
// thread per output walking all 1024 partials took 193 us per call.)
__global__ __launch_bounds__(kDotThreads) void multi_dot_reduce_kernel(
    const double* __restrict__ partial, int nblk_x, int ngroups, int rb, int nc,
    double* __restrict__ out) {
  const int t = blockIdx.x;
  const int r = t / nc, c = t % nc;
  const int g = r / rb, i = r % rb;
  double s[1] = {0.0};
  for (int b = threadIdx.x; b < nblk_x; b += kDotThreads)
    s[0] += partial[((int64_t)b * ngroups + g) * rb * nc + i * nc + c];
  __shared__ double scratch[kDotThreads / kWave];
  block_sum_n<1>(s, scratch);
  if (threadIdx.x == 0) out[t] = s[0];
}

// y = alpha * x + sum_i coef[i] * H[i, :]   (coef in device memory, nrows <= kLincombRows)
constexpr int kLincombRows = 256;
__global__ __launch_bounds__(256) void lincomb_kernel(const float* __restrict__ H, int64_t ldh,
                                                      int nrows, const float* __restrict__ coef,
                                                      float alpha, const float* __restrict__ x,
                                                      int64_t n, float* __restrict__ y) {
  __shared__ float c[kLincombRows];
  for (int i = threadIdx.x; i < nrows; i += blockDim.x) c[i] = coef[i];
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
    float acc = x ? alpha * x[j] : 0.0f;
    for (int i = 0; i < nrows; ++i) acc = fmaf(c[i], H[(int64_t)i * ldh + j], acc);
    y[j] = acc;
  }
}

// rows per wave (SPLIT, >= 4 rows) or per thread (1-3 rows)
static int dot_rpw(int64_t nrows) {
  if (nrows < kDotWaves) return (int)nrows;
  const int64_t per = (nrows + kDotWaves - 1) / kDotWaves;
  return per <= 2 ? 2 : (per <= 4 ? 4 : (per <= 6 ? 6 : 8));
}
static int dot_rows_per_block(int64_t nrows) {
  return nrows < kDotWaves ? (int)nrows : kDotWaves * dot_rpw(nrows);
}

// Grid: the chunk count, capped at what the GPU holds resident at once (the occupancy of
// the instantiation times the CU count), so no workgroup starts after the first wave of
// workgroups has finished (a grid-stride loop with a late tail).
template <int NC, int RPW, bool SPLIT>
static void launch_dot(int64_t n, int gy, hipStream_t stream, bool vec, const float* a, int64_t lda,
                       int nrows, const RowPtrs& rp, double* ws, int* bx_out) {
  auto kv = multi_dot_kernel<NC, RPW, SPLIT, true>;
  auto ks = multi_dot_kernel<NC, RPW, SPLIT, false>;
  static int cap = 0;
  if (cap == 0) {
    int dev = 0, cus = 0, per = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kv, kDotThreads, 0);
    cap = std::max(1, std::min(kDotMaxBlocks, std::max(1, cus) * std::max(1, per)));
  }
  const int64_t tpb = SPLIT ? kWave : kDotThreads;
  const int64_t chunks = vec ? (n >> 2) : n;
  const int bx = (int)std::max<int64_t>(1, std::min<int64_t>((chunks + tpb - 1) / tpb, cap));
  *bx_out = bx;
  dim3 grid(bx, gy);
  if (vec)
    hipLaunchKernelGGL(kv, grid, dim3(kDotThreads), 0, stream, a, lda, nrows, rp, n, ws);
  else
    hipLaunchKernelGGL(ks, grid, dim3(kDotThreads), 0, stream, a, lda, nrows, rp, n, ws);
}

template <int NC>
static void launch_dot_nc(int64_t nrows, int64_t n, int gy, hipStream_t stream, bool vec,
                          const float* a, int64_t lda, const RowPtrs& rp, double* ws, int* bx) {
  const int r = (int)nrows;
  switch (dot_rpw(nrows) + (nrows < kDotWaves ? 100 : 0)) {
    case 101: launch_dot<NC, 1, false>(n, gy, stream, vec, a, lda, r, rp, ws, bx); break;
    case 102: launch_dot<NC, 2, false>(n, gy, stream, vec, a, lda, r, rp, ws, bx); break;
    case 103: launch_dot<NC, 3, false>(n, gy, stream, vec, a, lda, r, rp, ws, bx); break;
    case 2: launch_dot<NC, 2, true>(n, gy, stream, vec, a, lda, r, rp, ws, bx); break;
    case 4: launch_dot<NC, 4, true>(n, gy, stream, vec, a, lda, r, rp, ws, bx); break;
    case 6: launch_dot<NC, 6, true>(n, gy, stream, vec, a, lda, r, rp, ws, bx); break;
    default: launch_dot<NC, 8, true>(n, gy, stream, vec, a, lda, r, rp, ws, bx); break;
  }
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
  const int rb = dot_rows_per_block(nrows);
  const int gy = (int)((nrows + rb - 1) / rb);
  TORCH_CHECK(workspace.numel() >= (int64_t)kDotMaxBlocks * gy * rb * nc, "workspace too small");
  auto stream = at::hip::getCurrentHIPStream();
  const float* a = A.data_ptr<float>();
  double* ws = workspace.data_ptr<double>();
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  bool vec = al16(a) && A.stride(0) % 4 == 0;
  for (int64_t c = 0; c < nc; ++c) vec = vec && al16(rp.p[c]);
  int bx = 1;
  const int64_t lda = A.stride(0);
  switch (nc) {
    case 1: launch_dot_nc<1>(nrows, n, gy, stream, vec, a, lda, rp, ws, &bx); break;
    case 2: launch_dot_nc<2>(nrows, n, gy, stream, vec, a, lda, rp, ws, &bx); break;
    case 3: launch_dot_nc<3>(nrows, n, gy, stream, vec, a, lda, rp, ws, &bx); break;
    default: launch_dot_nc<4>(nrows, n, gy, stream, vec, a, lda, rp, ws, &bx); break;
  }
  const int tot = (int)(nrows * nc);
  hipLaunchKernelGGL(multi_dot_reduce_kernel, dim3(tot), dim3(kDotThreads), 0, stream, ws, bx, gy,
                     rb, (int)nc, out.data_ptr<double>());
}

int64_t multi_dot_workspace(int64_t nrows, int64_t n) {
  // any call with at most nrows rows fits (rows per block * groups grows with nrows)
  int64_t most = 0;
  for (int64_t r = 1; r <= nrows; ++r) {
    const int64_t rb = dot_rows_per_block(r);
    most = std::max(most, ((r + rb - 1) / rb) * rb);
  }
  (void)n;
  return (int64_t)kDotMaxBlocks * most * kMaxCols;
}

void lincomb(torch::Tensor H, int64_t nrows, torch::Tensor coef, double alpha,
             c10::optional<torch::Tensor> x, int64_t n, torch::Tensor y) {
  TORCH_CHECK(H.is_cuda() && coef.is_cuda() && y.is_cuda(), "device tensors");
  TORCH_CHECK(H.scalar_type() == at::kFloat && coef.scalar_type() == at::kFloat &&
              y.scalar_type() == at::kFloat, "fp32");
  TORCH_CHECK(H.dim() == 2 && H.stride(1) == 1 && nrows <= H.size(0) && nrows <= kLincombRows &&
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
