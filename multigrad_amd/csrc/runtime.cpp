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
#include <queue>
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


// ---------------------------------------------------------------------------------
// Lane schedule ("lanes" layout): one 64-wide wavefront processes a *group* of 64
// population slots, one slot per lane, each lane walking its own slot's halos serially.
// The halos of a group are stored interleaved (halo j of lane l at base + 64 j + l), so
// every load is fully coalesced, a lane loads its (a, sigma) once per slot instead of
// once per halo, and -- because a lane owns a whole population -- per-population sums
// need no cross-lane segmentation at all.  To keep the lanes of a wave busy for the
// same number of iterations, slots are sorted by halo count (descending) inside windows
// of `window` consecutive populations (windows keep the gradient scatter local), then cut
// into groups of 64; a group runs max(len) iterations and shorter lanes are padded with
// a sentinel.  Populations with more than `lmax` halos are split into parts of <= lmax
// halos ("virtual" slots); their per-part gradient partials are summed in a fixed order
// by the finalize kernel.
//
// counts: int64 [J] halos per population (halos sorted by population, CPU).
// breaks: population indices where a chunk ends (windows never straddle a chunk).
// Returns (slot_pop int32 [S] (-1: empty), slot_src int64 [S] (first halo in the sorted
//          array), slot_len int32 [S], slot_part int32 [S] (partial index or -1),
//          group_base int64 [G+1] (offset of the group in the interleaved array; the last
//          entry is its total length), group_len int32 [G], chunk_groups int64 [C+1],
//          giant int32 [P,3] = {pop, part_begin, part_end}, chunk_giant int64 [C+1],
//          fwd_order int32 [G]: each chunk's groups longest first, for the forward,
//          slot_pidx int32 [S]: internal parameter-unit index per slot (-1: empty),
//          perm int32 [J]: internal unit index -> population).
// order_counts (optional, int64 [J]): counts that decide the population order inside a
// window (default: counts); pass the cross-rank sums so that all ranks agree on it.
std::vector<torch::Tensor> build_lanes(torch::Tensor counts, std::vector<int64_t> breaks,
                                       int64_t window, int64_t lmax,
                                       c10::optional<torch::Tensor> order_counts) {
  TORCH_CHECK(counts.device().is_cpu() && counts.scalar_type() == at::kLong, "counts: int64 CPU");
  TORCH_CHECK(window >= 1 && lmax >= 1, "bad lane-schedule limits");
  constexpr int64_t kLanes = 64;
  auto c = counts.contiguous();
  const int64_t* cnt = c.data_ptr<int64_t>();
  const int64_t J = c.numel();
  torch::Tensor oc = c;
  if (order_counts.has_value() && order_counts->defined()) {
    oc = order_counts->contiguous();
    TORCH_CHECK(oc.device().is_cpu() && oc.scalar_type() == at::kLong && oc.numel() == J,
                "order_counts: int64 CPU [J]");
  }
  const int64_t* key = oc.data_ptr<int64_t>();
  std::vector<int64_t> brk;
  for (auto b : breaks)
    if (b > 0 && b < J) brk.push_back(b);
  std::sort(brk.begin(), brk.end());
  brk.erase(std::unique(brk.begin(), brk.end()), brk.end());
  brk.push_back(J);

  std::vector<int64_t> off(J + 1, 0);
  for (int64_t p = 0; p < J; ++p) {
    TORCH_CHECK(cnt[p] >= 0, "negative population count");
    off[p + 1] = off[p] + cnt[p];
  }
  struct Item {
    int64_t key, len, pop, part, src;
  };
  std::vector<int32_t> slot_pop, slot_len, slot_part, giant;
  std::vector<int64_t> slot_src, group_base{0}, chunk_groups{0}, chunk_giant{0};
  std::vector<int32_t> group_len, fwd_order;
  std::vector<Item> items;
  int64_t nparts = 0;
  int64_t p = 0;
  // groups of the current chunk before emission: 64 slots each
  struct Slot {
    int32_t pop, len, part;
    int64_t src;
  };
  std::vector<Slot> cslots;
  std::vector<int64_t> cglen;
  for (size_t bi = 0; bi < brk.size(); ++bi) {
    const int64_t pend = brk[bi];
    cslots.clear();
    cglen.clear();
    for (int64_t w0 = p; w0 < pend; w0 += window) {
      const int64_t w1 = std::min(pend, w0 + window);
      items.clear();
      for (int64_t q = w0; q < w1; ++q) {
        const int64_t n = cnt[q];
        if (n > lmax) {
          const int64_t k = (n + lmax - 1) / lmax;
          for (int64_t i = 0; i < k; ++i)
            items.push_back({key[q], std::min(lmax, n - i * lmax), q, i, off[q] + i * lmax});
          // partial indices are contiguous per split population, in population order
          giant.insert(giant.end(), {(int32_t)q, (int32_t)nparts, (int32_t)(nparts + k)});
          nparts += k;
        } else {
          items.push_back({key[q], n, q, -1, off[q]});
        }
      }
      // order by the *ordering* counts (the global ones under data parallelism, so every
      // rank derives the same population order), lengths are the local counts
      std::stable_sort(items.begin(), items.end(), [](const Item& a, const Item& b) {
        return a.key > b.key;
      });
      const size_t n_items = items.size();
      const size_t padded = (n_items + kLanes - 1) / kLanes * kLanes;
      for (size_t i = 0; i < padded; i += kLanes) {
        int64_t glen = 0;
        for (size_t l = 0; l < (size_t)kLanes; ++l) {
          if (i + l < n_items) {
            const Item& it = items[i + l];
            // part i -> -1-i; whole population -> 0 (mapped to global indices below)
            cslots.push_back({(int32_t)it.pop, (int32_t)it.len, -1 - (int32_t)it.part, it.src});
            glen = std::max(glen, it.len);
          } else {
            cslots.push_back({-1, 0, 0, 0});
          }
        }
        cglen.push_back(glen);
      }
    }
    // Groups are stored in creation (= window) order, so that the VJP's gradient writes
    // and parameter reads of one window of populations stay together.  The forward
    // visits them through fwd_order, longest first: a grid-stride over that order hands
    // every wavefront groups of nearly equal length in each round (static LPT balance).
    const int64_t gbase = (int64_t)group_len.size();
    std::vector<int64_t> order(cglen.size());
    for (size_t g = 0; g < order.size(); ++g) order[g] = (int64_t)g;
    std::stable_sort(order.begin(), order.end(),
                     [&](int64_t a, int64_t b) { return cglen[a] > cglen[b]; });
    for (int64_t g : order) fwd_order.push_back((int32_t)(gbase + g));
    for (size_t g = 0; g < cglen.size(); ++g) {
      for (int64_t l = 0; l < kLanes; ++l) {
        const Slot& sl = cslots[g * kLanes + l];
        slot_pop.push_back(sl.pop);
        slot_len.push_back(sl.len);
        slot_src.push_back(sl.src);
        slot_part.push_back(sl.pop < 0 ? -1 : sl.part);
      }
      group_len.push_back((int32_t)cglen[g]);
      group_base.push_back(group_base.back() + cglen[g] * kLanes);
    }
    p = pend;
    chunk_groups.push_back((int64_t)group_len.size());
    chunk_giant.push_back((int64_t)giant.size() / 3);
  }
  // part fix-up: slot_part held -1 - part_index_within_pop (or -1 - (-1) = 0 for whole
  // populations); map to the global partial index giant[pop].part_begin + i.
  {
    std::vector<int32_t> part_begin(J, -1);
    for (size_t g = 0; g < giant.size(); g += 3) part_begin[giant[g]] = giant[g + 1];
    for (size_t s = 0; s < slot_pop.size(); ++s) {
      const int32_t q = slot_pop[s];
      if (q < 0 || part_begin[q] < 0) {
        slot_part[s] = -1;
      } else {
        slot_part[s] = part_begin[q] + (-1 - slot_part[s]);
      }
    }
  }
  // Internal parameter order: populations by first appearance in (window-ordered) slot
  // order.  Lanes of a group then hold consecutive internal indices, so parameter reads
  // and gradient writes in internal order are coalesced; with global ordering counts the
  // order is identical on every rank.
  std::vector<int32_t> slot_pidx(slot_pop.size(), -1), perm, pidx_of(J, -1);
  perm.reserve(J);
  for (size_t s2 = 0; s2 < slot_pop.size(); ++s2) {
    const int32_t q = slot_pop[s2];
    if (q < 0) continue;
    if (pidx_of[q] < 0) {
      pidx_of[q] = (int32_t)perm.size();
      perm.push_back(q);
    }
    slot_pidx[s2] = pidx_of[q];
  }
  TORCH_CHECK((int64_t)perm.size() == J, "every population needs a slot");
  auto i32 = [](const std::vector<int32_t>& v) {
    auto t = torch::empty({(int64_t)v.size()}, torch::kInt);
    if (!v.empty()) std::memcpy(t.data_ptr<int32_t>(), v.data(), v.size() * sizeof(int32_t));
    return t;
  };
  auto i64 = [](const std::vector<int64_t>& v) {
    auto t = torch::empty({(int64_t)v.size()}, torch::kLong);
    if (!v.empty()) std::memcpy(t.data_ptr<int64_t>(), v.data(), v.size() * sizeof(int64_t));
    return t;
  };
  return {i32(slot_pop), i64(slot_src), i32(slot_len), i32(slot_part), i64(group_base),
          i32(group_len), i64(chunk_groups), i32(giant).reshape({-1, 3}), i64(chunk_giant),
          i32(fwd_order), i32(slot_pidx), i32(perm)};
}


// Static LPT (longest processing time first) assignment of the lanes groups [g0, g1) of
// fwd_order to `nwaves` persistent wavefronts: groups in decreasing cost order go to
// the currently least-loaded wave (binary heap).  A group costs its length in halo rows
// plus `overhead` (parameter gather + residual stores, in halo-row units).  Round-robin
// over the longest-first order is within a few % of this when every wave takes ~10+
// groups (one GPU), but loses ~20% at 2-3 groups per wave (a population-owner shard on
// each of 8 GPUs).  Returns (order [g1-g0] int32: group ids wave by wave,
// wave_start [nwaves+1] int32).
std::vector<torch::Tensor> lpt_waves(torch::Tensor group_len, torch::Tensor fwd_order,
                                     int64_t g0, int64_t g1, int64_t nwaves, double overhead) {
  TORCH_CHECK(group_len.device().is_cpu() && group_len.scalar_type() == at::kInt, "group_len: int32 CPU");
  TORCH_CHECK(fwd_order.device().is_cpu() && fwd_order.scalar_type() == at::kInt, "fwd_order: int32 CPU");
  TORCH_CHECK(nwaves >= 1 && g0 >= 0 && g0 <= g1 && g1 <= fwd_order.numel(), "bad LPT request");
  auto gl = group_len.contiguous();
  auto fo = fwd_order.contiguous();
  const int32_t* len = gl.data_ptr<int32_t>();
  const int32_t* ord = fo.data_ptr<int32_t>();
  std::vector<int32_t> items(ord + g0, ord + g1);
  std::stable_sort(items.begin(), items.end(),
                   [&](int32_t a, int32_t b) { return len[a] > len[b]; });
  using Load = std::pair<double, int64_t>;  // (load, wave): min-heap, ties -> lower wave
  std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
  for (int64_t w = 0; w < nwaves; ++w) heap.push({0.0, w});
  std::vector<std::vector<int32_t>> lists(nwaves);
  for (int32_t g : items) {
    Load l = heap.top();
    heap.pop();
    lists[l.second].push_back(g);
    l.first += (double)len[g] + overhead;
    heap.push(l);
  }
  auto order = torch::empty({g1 - g0}, torch::kInt);
  auto start = torch::empty({nwaves + 1}, torch::kInt);
  int32_t* o = order.data_ptr<int32_t>();
  int32_t* st = start.data_ptr<int32_t>();
  int64_t pos = 0;
  for (int64_t w = 0; w < nwaves; ++w) {
    st[w] = (int32_t)pos;
    for (int32_t g : lists[w]) o[pos++] = g;
  }
  st[nwaves] = (int32_t)pos;
  return {order, start};
}

}  // namespace mg
