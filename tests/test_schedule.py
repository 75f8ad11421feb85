"""Host-side schedules for the SMF kernels (runtime.cpp vs its Python mirror, and the
invariants the kernels rely on).  CPU only."""
import numpy as np
import pytest
import torch

from multigrad_amd.ops import _ext
from multigrad_amd.ops._schedule import build_lanes_py, build_tiles_py


def _counts(J, seed=0):
    rng = np.random.default_rng(seed)
    c = torch.tensor(rng.poisson(27, J), dtype=torch.int64)
    if J > 20:
        c[3] = 5000   # split into parts
        c[11] = 0     # empty population
        c[J - 1] = 130
    return c


@pytest.mark.parametrize("J,window,lmax,breaks", [(2000, 256, 100, [500, 501, 1500]),
                                                   (3000, 4096, 4096, []), (1, 64, 10, []),
                                                   (0, 64, 10, [])])
def test_lanes_schedule_invariants(J, window, lmax, breaks):
    counts = _counts(J)
    (pop, src, ln, part, base, glen, cg, giant, cgi, ford, spidx, perm) = build_lanes_py(
        counts, breaks, window, lmax)
    nchunks = len(sorted({b for b in breaks if 0 < b < J})) + 1
    assert len(cg) == nchunks + 1 and len(cgi) == nchunks + 1
    ng = glen.numel()
    assert pop.numel() == 64 * ng and base.numel() == ng + 1
    # every halo of every population is covered exactly once
    off = np.concatenate([[0], np.cumsum(counts.numpy())])
    cover = np.zeros(int(off[-1]), dtype=np.int64)
    for s in range(pop.numel()):
        q = int(pop[s])
        if q < 0:
            assert int(ln[s]) == 0
            continue
        a = int(src[s])
        assert off[q] <= a and a + int(ln[s]) <= off[q + 1]
        cover[a:a + int(ln[s])] += 1
        assert int(ln[s]) <= lmax
    assert (cover == 1).all()
    # every population has a slot (so its gradient is written), parts are contiguous
    seen = set(int(q) for q in pop.tolist() if q >= 0)
    assert seen == set(range(J))
    for q, p0, p1 in giant.tolist():
        assert counts[q] > lmax and p1 - p0 == -(-int(counts[q]) // lmax)
        assert sorted(int(part[s]) for s in range(pop.numel()) if int(pop[s]) == q) == list(range(p0, p1))
    # groups are stored in window order; the forward order is a per-chunk permutation,
    # longest group first
    starts = [0] + sorted({b for b in breaks if 0 < b < J})
    for c in range(len(cg) - 1):
        a, b = int(cg[c]), int(cg[c + 1])
        assert sorted(ford[a:b].tolist()) == list(range(a, b))
        lens = glen[ford[a:b].long()]
        assert (lens[:-1] >= lens[1:]).all()
        firsts = [int(pop[64 * g]) for g in range(a, b) if int(pop[64 * g]) >= 0]
        wins = [(q - starts[c]) // window for q in firsts]
        assert wins == sorted(wins)
    # internal order: a permutation of the populations, chunk-aligned, and consistent with
    # the slots (first appearance order)
    assert sorted(perm.tolist()) == list(range(J))
    for s_ in range(pop.numel()):
        if int(pop[s_]) >= 0:
            assert int(perm[int(spidx[s_])]) == int(pop[s_])
        else:
            assert int(spidx[s_]) == -1
    bounds = [0] + sorted({b for b in breaks if 0 < b < J}) + [J]
    for c in range(len(bounds) - 1):
        chunk = perm[bounds[c]:bounds[c + 1]].tolist()
        assert all(bounds[c] <= q < bounds[c + 1] for q in chunk)
    # group length = longest lane, groups never mix chunks
    for g in range(ng):
        assert int(glen[g]) == int(ln[64 * g:64 * g + 64].max())
        assert int(base[g + 1] - base[g]) == 64 * int(glen[g])
    for c in range(nchunks):
        qs = [int(q) for q in pop[64 * int(cg[c]):64 * int(cg[c + 1])].tolist() if q >= 0]
        if qs:
            assert max(qs) < (sorted({b for b in breaks if 0 < b < J}) + [J])[c]


@pytest.mark.skipif(not _ext.available(), reason="native extension not built")
@pytest.mark.parametrize("J,window,lmax,breaks", [(2000, 256, 100, [500, 501, 1500]),
                                                   (3000, 4096, 4096, []), (0, 64, 10, [])])
def test_native_schedules_match_python(J, window, lmax, breaks):
    counts = _counts(J, seed=1)
    a = _ext.ext().build_lanes(counts, breaks, window, lmax)
    b = build_lanes_py(counts, breaks, window, lmax)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    glob = counts * 3 + torch.arange(J) % 5  # e.g. cross-rank sums
    a = _ext.ext().build_lanes(counts, breaks, window, lmax, glob)
    b = build_lanes_py(counts, breaks, window, lmax, glob)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    ta = _ext.ext().build_tiles(counts, breaks, 2048, 2048)
    tb = build_tiles_py(counts, breaks, 2048, 2048)
    for x, y in zip(ta[:4], tb[:4]):
        assert torch.equal(torch.as_tensor(x), torch.as_tensor(y))
    assert int(ta[4]) == int(tb[4])


def test_internal_order_is_rank_independent():
    """Two ranks with different local counts but the same ordering (global) counts get
    the same internal parameter order."""
    rng = np.random.default_rng(4)
    J = 3000
    l0 = torch.tensor(rng.poisson(14, J), dtype=torch.int64)
    l1 = torch.tensor(rng.poisson(14, J), dtype=torch.int64)
    l1[7] = 9000  # split into parts on one rank only
    glob = l0 + l1
    p0 = build_lanes_py(l0, [1000], 256, 4096, glob)[-1]
    p1 = build_lanes_py(l1, [1000], 256, 4096, glob)[-1]
    assert torch.equal(p0, p1)


def test_lane_classes_group_narrow_populations():
    """PopulationShard.set_lane_classes: populations of one class share 64-lane groups, so
    1% narrow populations scattered over the catalog put about 1% of the groups (plus at
    most one mixed group per window) on the per-edge path instead of ~47% (every group with
    one narrow lane).  The order inside a class stays by halo count."""
    from multigrad_amd.models.population import make_population_data
    data = make_population_data(num_params=2 * 20_000, num_halos=540_000, seed=3, device="cpu")
    sh = data["shard"]
    rng = np.random.default_rng(1)
    cls = torch.tensor(rng.random(sh.npop) < 0.01, dtype=torch.int64)

    def mixed_and_narrow():
        sp = sh.slot_pop.long()
        c = torch.where(sp >= 0, cls[sp.clamp(min=0)], torch.zeros(1, dtype=torch.int64))
        g = c.reshape(-1, 64)
        occupied = (sp.reshape(-1, 64) >= 0)
        narrow = g.amax(1) > 0
        mixed = narrow & ((g == 0) & occupied).any(1)
        return int(narrow.sum()), int(mixed.sum()), g.shape[0]

    n0, _, G = mixed_and_narrow()
    assert n0 > 0.3 * G  # without classes: a large share of groups hold a narrow lane
    assert sh.set_lane_classes(cls)
    assert not sh.set_lane_classes(cls)  # unchanged
    sh.set_chunks(sh.chunk_pops)
    n1, mixed, G1 = mixed_and_narrow()
    windows = -(-sh.npop // sh._lane_window)
    assert mixed <= windows and n1 <= int(cls.sum()) // 64 + 2 * windows, (n1, mixed, windows)
    assert sh.set_lane_classes(None)
    sh.set_chunks(sh.chunk_pops)
    assert mixed_and_narrow()[0] == n0


@pytest.mark.parametrize("J,breaks,window", [(5000, [], 4096), (20000, [7000, 13001], 4096),
                                             (3000, [1000], 256), (130, [], 64), (1, [], 64)])
def test_lanes_schedule_torch_builder_matches_native(J, breaks, window):
    """The sort-and-scatter lanes builder (run on the GPU for re-layouts during a fit) gives
    exactly the host builder's schedule: slots, groups, forward order, internal order."""
    from multigrad_amd.ops._ext import ext
    from multigrad_amd.ops._schedule import build_lanes_py, build_lanes_torch
    g = torch.Generator().manual_seed(J)
    cnt = torch.randint(0, 60, (J,), generator=g)
    cls = (torch.rand(J, generator=g) < 0.05).long()
    for key in (None, cnt + (cls << 40), cnt * 3 + 1):
        try:
            ref = ext().build_lanes(cnt.long(), breaks, window, 4096, key)
        except ImportError:
            ref = build_lanes_py(cnt, breaks, window, 4096, key)
        got = build_lanes_torch(cnt, breaks, window, 4096, key)
        assert got is not None
        for a, b in zip(ref, got):
            assert torch.equal(a.cpu().to(b.dtype), b.cpu())
    big = cnt.clone()
    big[0] = 5000  # a split population: the host builder's job
    assert build_lanes_torch(big, breaks, window, 4096) is None
