"""Per-wave timeline of the PIPELINED lanes forward (the fused VJP + Adam update of the
previous step, then the forward: the owner-shard step's main launch), with a fit of each
wave's busy time to its work: busy = a * rows + b * groups + c.  ``b`` is what one more lane
group costs a wave beyond its rows (the group transition: staged residual / moment loads,
the theta gather and the residual stores), the price of finer work units.

Needs the -DMG_FWD_TRACE variant (VARIANT_DIR=abvar bash tools/build_variant.sh trace
-DMG_FWD_TRACE=1).  Usage: python tools/fwd_trace_step.py --so abvar/trace/_C.so
[--params P --halos N --steps K]"""
import argparse
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", required=True)
    ap.add_argument("--params", type=int, default=1_250_000)
    ap.add_argument("--halos", type=int, default=1 << 24)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    os.environ["MULTIGRAD_AUTOTUNE"] = "off"
    import torch
    spec = importlib.util.spec_from_file_location("multigrad_amd._C", a.so)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["multigrad_amd._C"] = mod
    from multigrad_amd.models.population import PopulationSMFModel, make_population_data
    dev = torch.device("cuda", 0)
    data = make_population_data(a.params, a.halos, seed=1234, device=dev)
    model = PopulationSMFModel(aux_data=data)
    model.set_target_from_truth()
    eng = model.fused_engine(graph=False)
    eng.setup(data["guess"], nsteps=a.steps + 2, learning_rate=0.01, history="full")
    assert eng.pipeline, "the trace is of the pipelined (update + forward) launch"
    eng.steps(a.steps)
    torch.cuda.synchronize()
    shard = data["shard"]
    nblk = shard.fwd_blocks(shard.n, data["bins"].nb, True, data["bins"].rel_tail)
    nw = nblk * 4
    tr = mod.smf_fwd_trace()[:nw].double()
    order, start, queues = shard.fwd_schedule(None, nblk)
    assert queues is None and start is not None, "static LPT lists expected at this size"
    order, start = order.cpu().long(), start.cpu().long()
    glen = shard.group_len.cpu().double()
    rows = torch.zeros(nw, dtype=torch.float64)
    ngr = (start[1:] - start[:-1]).double()
    for w in range(nw):
        rows[w] = glen[order[start[w]:start[w + 1]]].sum()
    t0 = tr[:, 0].min()
    st, en = (tr[:, 0] - t0) / 100.0, (tr[:, 1] - t0) / 100.0  # 100 MHz -> us
    busy = en - st
    assert torch.equal(tr[:, 2], ngr), "trace group counts differ from the LPT lists"
    X = torch.stack([rows, ngr, torch.ones_like(rows)], 1)
    coef = torch.linalg.lstsq(X, busy.unsqueeze(1)).solution.squeeze(1)
    pred = X @ coef
    r2 = 1.0 - float(((busy - pred) ** 2).sum() / ((busy - busy.mean()) ** 2).sum())
    q = torch.tensor([0.0, 0.5, 0.9, 0.99, 1.0], dtype=torch.float64)
    out = {
        "params": a.params, "halos": a.halos, "waves": nw, "groups": int(ngr.sum()),
        "groups_per_wave": round(float(ngr.mean()), 3),
        "rows_per_group": round(float(rows.sum() / ngr.sum()), 2),
        "end_q_us": [round(float(v), 2) for v in torch.quantile(en, q)],
        "busy_q_us": [round(float(v), 2) for v in torch.quantile(busy, q)],
        "fit_us": {"per_row": round(float(coef[0]), 4), "per_group": round(float(coef[1]), 3),
                   "const": round(float(coef[2]), 3), "r2": round(r2, 4)},
        "busy_by_groups": {int(k): round(float(busy[ngr == k].mean()), 2)
                           for k in torch.unique(ngr).tolist()},
        "rows_by_groups": {int(k): round(float(rows[ngr == k].mean()), 1)
                           for k in torch.unique(ngr).tolist()},
    }
    # where the late waves are: by XCD (workgroups are dealt round-robin over the 8 XCDs, so
    # block b % 8 names the XCD group), by wave slot in the workgroup, and by start time
    blk = torch.arange(nw) // 4
    out["end_by_xcd_us"] = {int(x): [round(float(en[blk % 8 == x].mean()), 2),
                                     round(float(en[blk % 8 == x].max()), 2)] for x in range(8)}
    out["end_by_wave_slot_us"] = {int(s): round(float(en[torch.arange(nw) % 4 == s].mean()), 2)
                                  for s in range(4)}
    late = en >= torch.quantile(en, torch.tensor(0.9, dtype=torch.float64))
    out["late_waves"] = {"n": int(late.sum()), "mean_rows": round(float(rows[late].mean()), 1),
                         "mean_groups": round(float(ngr[late].mean()), 2),
                         "mean_start_us": round(float(st[late].mean()), 2),
                         "all_mean_rows": round(float(rows.mean()), 1)}
    # the same CU's waves: 4 workgroups of 4 waves per CU at this occupancy; block b and
    # b + 8 k share an XCD, the CU inside it is not observable from the block index, so the
    # per-block spread (max - min end of a workgroup's 4 waves) stands in for it
    eb = en.reshape(-1, 4)
    out["block_end_spread_q_us"] = [round(float(v), 2) for v in
                                    torch.quantile(eb.max(1).values - eb.min(1).values, q)]
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
