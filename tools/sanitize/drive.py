"""Drive the ASan/UBSan host runtime (build/asan/_C_host_asan.so) over randomized and
edge-case inputs and compare every output with the regular extension's.  Run under
LD_PRELOAD=libasan.so (tests/test_sanitize_host.py does)."""
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def load_asan():
    path = os.path.join(ROOT, "build", "asan", "_C_host_asan.so")
    spec = importlib.util.spec_from_file_location("_C_host_asan", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def same(a, b):
    if isinstance(a, (list, tuple)):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            same(x, y)
    elif torch.is_tensor(a):
        assert torch.equal(a, b), (a, b)
    else:
        assert a == b, (a, b)


def main():
    A = load_asan()
    from multigrad_amd.ops import build  # noqa: F401  (ensure the package imports)
    import multigrad_amd._C as R
    g = torch.Generator().manual_seed(0)
    cases = 0
    for J in (1, 2, 63, 64, 65, 1000, 5000):
        for dist in ("poisson", "zeros", "heavy"):
            if dist == "poisson":
                counts = torch.poisson(torch.full((J,), 20.0), generator=g).to(torch.int64)
            elif dist == "zeros":
                counts = torch.zeros(J, dtype=torch.int64)
                counts[::7] = 3
            else:
                counts = torch.randint(0, 5, (J,), generator=g, dtype=torch.int64)
                counts[J // 2] = 9000  # a population split into parts
            breaks = sorted({int(b) for b in torch.randint(0, J + 1, (3,), generator=g)})
            for window, lmax in ((4096, 4096), (16, 100), (1, 1)):
                oc = counts + torch.randint(0, 3, (J,), generator=g, dtype=torch.int64)
                same(A.build_lanes(counts, breaks, window, lmax, oc),
                     R.build_lanes(counts, breaks, window, lmax, oc))
                same(A.build_lanes(counts, breaks, window, lmax),
                     R.build_lanes(counts, breaks, window, lmax))
                cases += 2
            same(A.build_tiles(counts, breaks, 2048, 2048), R.build_tiles(counts, breaks, 2048, 2048))
            same(A.build_tiles(counts, breaks, 64, 7), R.build_tiles(counts, breaks, 64, 7))
            out = R.build_lanes(counts, breaks, 4096, 4096)
            group_len, fwd_order = out[5], out[9]
            ng = group_len.numel()
            for nw in (1, 3, 4096):
                for g0, g1 in ((0, ng), (0, ng // 2), (ng // 2, ng)):
                    same(A.lpt_waves(group_len, fwd_order, g0, g1, nw, 3.0),
                         R.lpt_waves(group_len, fwd_order, g0, g1, nw, 3.0))
                    cases += 1
            pop = torch.randint(0, J, (5000,), generator=g, dtype=torch.int32)
            same(A.sort_by_population(pop, J), R.sort_by_population(pop, J))
            cases += 3
    print(f"sanitized host runtime: {cases} cases clean")


if __name__ == "__main__":
    main()
