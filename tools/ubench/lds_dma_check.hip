// Semantics check of the primitives the pipelined-update forward relies on (gfx950):
// global_load_lds dword / dwordx4 with an immediate offset (moves both the global and the
// LDS address), a per-lane gather into LDS, and raw buffer loads / stores with SGPR offsets.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <utility>
#include <vector>

constexpr int kWave = 64;
template <int I>
__device__ __forceinline__ void chunk(const float* src, float* dst, int lane) {
  constexpr int base = (I / 4) * 1024;
  __builtin_amdgcn_global_load_lds(src + base + lane * 4, dst + base, 16, (I % 4) * 1024, 0);
}
template <int R>
__device__ __forceinline__ void row(const float* src, float* dst, int lane) {
  constexpr int base = (R * kWave / 1024) * 1024;
  __builtin_amdgcn_global_load_lds(src + base + lane, dst + base, 4, (R * kWave - base) * 4, 0);
}
template <int NR, int... I, int... R>
__device__ void stage(const float* s, float* d, int lane, std::integer_sequence<int, I...>,
                      std::integer_sequence<int, R...>) {
  (chunk<I>(s, d, lane), ...);
  (row<(NR / 4) * 4 + R>(s, d, lane), ...);
}

__global__ void k(const float* src, const int* idx, const float* gat, float* out, float* out2) {
  constexpr int NR = 22, NRow = NR + 2;
  __shared__ __attribute__((aligned(16))) float ub[4 * NRow * kWave];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* u = ub + w * NRow * kWave;
  const float* s = src + (blockIdx.x * 4 + w) * NR * kWave;
  stage<NR>(s, u, lane, std::make_integer_sequence<int, NR / 4>{}, std::make_integer_sequence<int, NR % 4>{});
  const float* gp = gat + idx[lane];
  __builtin_amdgcn_global_load_lds(gp, u + NR * kWave, 4, 0, 0);
  __builtin_amdgcn_global_load_lds(gp + 1, u + (NR + 1) * kWave, 4, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  float* o = out + (blockIdx.x * 4 + w) * NRow * kWave;
  for (int r = 0; r < NRow; ++r) o[r * kWave + lane] = u[r * kWave + lane];
  // buffer load / store with SGPR offsets
  auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(s), (short)0, 0x7fffffff, 0x00020000);
  auto rd = __builtin_amdgcn_make_buffer_rsrc(out2 + (blockIdx.x * 4 + w) * NR * kWave, (short)0, 0x7fffffff, 0x00020000);
  for (int r = 0; r < NR; ++r) {
    unsigned v = __builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, r * 256, 0);
    __builtin_amdgcn_raw_buffer_store_b32(v, rd, lane * 4, r * 256, 0);
  }
}

int main() {
  constexpr int NR = 22, NRow = 24, NW = 8 * 4;
  std::vector<float> src(NW * NR * kWave), gat(4096);
  std::vector<int> idx(kWave);
  for (size_t i = 0; i < src.size(); ++i) src[i] = (float)i;
  for (size_t i = 0; i < gat.size(); ++i) gat[i] = 0.5f * (float)i;
  for (int l = 0; l < kWave; ++l) idx[l] = (l * 37 % 64) * 2 + 100;
  float *ds, *dg, *dout, *dout2;
  int* di;
  hipMalloc(&ds, src.size() * 4); hipMalloc(&dg, gat.size() * 4); hipMalloc(&di, 256);
  hipMalloc(&dout, NW * NRow * kWave * 4); hipMalloc(&dout2, src.size() * 4);
  hipMemcpy(ds, src.data(), src.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dg, gat.data(), gat.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(di, idx.data(), 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(8), dim3(256), 0, 0, ds, di, dg, dout, dout2);
  std::vector<float> out(NW * NRow * kWave), out2(src.size());
  hipMemcpy(out.data(), dout, out.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(out2.data(), dout2, out2.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0, bad2 = 0;
  for (int w = 0; w < NW; ++w)
    for (int r = 0; r < NRow; ++r)
      for (int l = 0; l < kWave; ++l) {
        float want = r < NR ? src[(w * NR + r) * kWave + l] : gat[idx[l] + (r - NR)];
        float got = out[(w * NRow + r) * kWave + l];
        if (got != want && bad++ < 10) printf("dma w%d r%d l%d got %g want %g\n", w, r, l, got, want);
      }
  for (size_t i = 0; i < src.size(); ++i)
    if (out2[i] != src[i] && bad2++ < 10) printf("buf %zu got %g want %g\n", i, out2[i], src[i]);
  printf("lds_dma_check: dma mismatches %d, buffer mismatches %d\n", bad, bad2);
  return bad || bad2;
}
