// Host-side native runtime pieces: data sharding/schedule construction.
//
// The reference has no native runtime (its data "loader" is np.array_split on every
// rank, tests/smf_example/smf_grad_descent.py:28).  For population-structured models the
// device kernels need a static schedule that cuts the population-sorted halo array
// into workgroup tiles at population boundaries; building it is an O(J) sequential
// scan over population counts (5e6 populations for the 1e7-parameter benchmark), done
// once per data shard in C++.
#include <torch/extension.h>

#include <algorithm>
#include <cstring>
#include <cstdint>
#include <tuple>
#include <vector>

namespace mg {

struct TileRec {
  int64_t h0, h1;
  int32_t p0, p1;
  int32_t slot;
  int32_t pad;
};
static_assert(sizeof(TileRec) == 32, "tile record must be 32 bytes");

// counts: int64 [J] halos per population (halos sorted by population).
// breaks: sorted population indices where a tile must end (chunk boundaries); J is implied.
// Returns (tiles int64 [T,4], giant int32 [G,3] = {pop, slot_begin, slot_end},
//          chunk_tiles int64 [C+1] tile offsets per chunk, chunk_giant int64 [C+1], nslots).
std::tuple<torch::Tensor, torch::Tensor, torch::Tensor, torch::Tensor, int64_t>
build_tiles(torch::Tensor counts, std::vector<int64_t> breaks, int64_t tile_halos,
            int64_t tile_pops) {
  TORCH_CHECK(counts.device().is_cpu() && counts.scalar_type() == at::kLong, "counts: int64 CPU");
  TORCH_CHECK(tile_halos >= 1 && tile_pops >= 1, "bad tile limits");
  auto c = counts.contiguous();
  const int64_t* cnt = c.data_ptr<int64_t>();
  const int64_t J = c.numel();
  std::vector<int64_t> brk;
  for (auto b : breaks)
    if (b > 0 && b < J) brk.push_back(b);
  std::sort(brk.begin(), brk.end());
  brk.erase(std::unique(brk.begin(), brk.end()), brk.end());
  brk.push_back(J);

  std::vector<TileRec> tiles;
  std::vector<int32_t> giant;
  std::vector<int64_t> chunk_tiles{0}, chunk_giant{0};
  int64_t nslots = 0;
  int64_t h = 0;
  size_t bi = 0;
  int64_t tp0 = 0, th0 = 0;  // open tile start
  auto close_tile = [&](int64_t p_end, int64_t h_end) {
    if (p_end > tp0) tiles.push_back({th0, h_end, (int32_t)tp0, (int32_t)p_end, -1, 0});
    tp0 = p_end;
    th0 = h_end;
  };
  for (int64_t p = 0; p < J; ++p) {
    const int64_t n = cnt[p];
    TORCH_CHECK(n >= 0, "negative population count");
    if (n > tile_halos) {
      // giant population: close the open tile, emit partial tiles of tile_halos each
      close_tile(p, h);
      const int64_t s0 = nslots;
      for (int64_t off = 0; off < n; off += tile_halos) {
        tiles.push_back({h + off, h + std::min(n, off + tile_halos), (int32_t)p, (int32_t)(p + 1),
                         (int32_t)nslots++, 0});
      }
      giant.insert(giant.end(), {(int32_t)p, (int32_t)s0, (int32_t)nslots});
      h += n;
      tp0 = p + 1;
      th0 = h;
    } else {
      if (h + n - th0 > tile_halos || p + 1 - tp0 > tile_pops) close_tile(p, h);
      h += n;
    }
    if (p + 1 == brk[bi]) {
      close_tile(p + 1, h);
      chunk_tiles.push_back((int64_t)tiles.size());
      chunk_giant.push_back((int64_t)giant.size() / 3);
      ++bi;
    }
  }
  if (J == 0) {
    chunk_tiles.push_back(0);
    chunk_giant.push_back(0);
  }
  auto t = torch::empty({(int64_t)tiles.size(), 4}, torch::kLong);
  if (!tiles.empty()) std::memcpy(t.data_ptr<int64_t>(), tiles.data(), tiles.size() * sizeof(TileRec));
  auto g = torch::empty({(int64_t)giant.size() / 3, 3}, torch::kInt);
  if (!giant.empty()) std::memcpy(g.data_ptr<int32_t>(), giant.data(), giant.size() * sizeof(int32_t));
  auto ct = torch::tensor(chunk_tiles, torch::kLong);
  auto cg = torch::tensor(chunk_giant, torch::kLong);
  return {t, g, ct, cg, nslots};
}

// Counting sort of population ids -> (order int64 [N], counts int64 [J]); stable, O(N+J).
std::tuple<torch::Tensor, torch::Tensor> sort_by_population(torch::Tensor pop, int64_t npop) {
  TORCH_CHECK(pop.device().is_cpu() && pop.scalar_type() == at::kInt, "pop: int32 CPU");
  auto p = pop.contiguous();
  const int32_t* pp = p.data_ptr<int32_t>();
  const int64_t N = p.numel();
  auto counts = torch::zeros({npop}, torch::kLong);
  int64_t* cnt = counts.data_ptr<int64_t>();
  for (int64_t i = 0; i < N; ++i) {
    TORCH_CHECK(pp[i] >= 0 && pp[i] < npop, "population id out of range");
    ++cnt[pp[i]];
  }
  std::vector<int64_t> off(npop + 1, 0);
  for (int64_t j = 0; j < npop; ++j) off[j + 1] = off[j] + cnt[j];
  auto order = torch::empty({N}, torch::kLong);
  int64_t* o = order.data_ptr<int64_t>();
  for (int64_t i = 0; i < N; ++i) o[off[pp[i]]++] = i;
  return {order, counts};
}

}  // namespace mg
