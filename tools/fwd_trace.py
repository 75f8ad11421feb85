"""Per-wave timeline of one lanes-forward launch (needs the -DMG_FWD_TRACE variant):
dispatch skew (spread of wave start times), work, and tail (spread of end times).
Usage: python tools/fwd_trace.py --so variants/trace/_C.so [--params P --halos N]"""
import argparse
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", required=True)
    ap.add_argument("--params", type=int, default=1_250_000)
    ap.add_argument("--halos", type=int, default=1 << 24)
    ap.add_argument("--shuffle", action="store_true",
                    help="hand the static LPT lists to the waves in a random order")
    a = ap.parse_args()
    import torch
    spec = importlib.util.spec_from_file_location("multigrad_amd._C", a.so)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["multigrad_amd._C"] = mod
    if a.shuffle:
        lpt = mod.lpt_waves

        def shuffled(*args):
            order, start = lpt(*args)
            nw = start.numel() - 1
            perm = torch.randperm(nw, generator=torch.Generator().manual_seed(7))
            lens = (start[1:] - start[:-1])[perm]
            lists = [order[start[w]:start[w + 1]] for w in perm.tolist()]
            new_start = torch.zeros_like(start)
            new_start[1:] = torch.cumsum(lens, 0)
            return torch.cat(lists), new_start
        mod.lpt_waves = shuffled
    from multigrad_amd.models.population import make_population_data
    from multigrad_amd.ops import smf as S
    dev = torch.device("cuda", 0)
    data = make_population_data(a.params, a.halos, seed=1, device=dev)
    shard, bins = data["shard"], data["bins"]
    th = data["guess"].reshape(-1, 2)[shard.perm].reshape(-1).contiguous()
    out = torch.zeros(bins.nbp, device=dev)
    nblk = shard.fwd_rows(shard.n, bins.nb, True, bins.rel_tail, resid=True)
    slab = torch.zeros(nblk * bins.nbp, device=dev)
    for _ in range(3):
        S.smf_forward_into(th, shard, bins, True, out, slab=slab, resid=True, order="internal")
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    S.smf_forward_into(th, shard, bins, True, out, slab=slab, resid=True, order="internal")
    e1.record()
    torch.cuda.synchronize()
    tr = mod.smf_fwd_trace()[: nblk * 4].double()
    t0 = tr[:, 0].min()
    st, en, ng = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0, tr[:, 2]  # 100 MHz -> us
    q = torch.tensor([0.0, 0.5, 0.9, 0.99, 1.0], dtype=torch.float64)
    print(f"launch {e0.elapsed_time(e1) * 1e3:.1f} us; waves {tr.shape[0]}; groups/wave "
          f"mean {ng.mean():.2f} max {ng.max():.0f}")
    print("start quantiles us", [round(float(v), 1) for v in torch.quantile(st, q)])
    print("end   quantiles us", [round(float(v), 1) for v in torch.quantile(en, q)])
    print("busy  quantiles us", [round(float(v), 1) for v in torch.quantile(en - st, q)])


if __name__ == "__main__":
    main()
