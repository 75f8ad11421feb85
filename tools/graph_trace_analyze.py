"""Replay vs eager launches of the same engine step, from rocprofv3 kernel traces
(tools/graph_trace.sh): per kernel the mean duration, the idle gap before it (end of the
previous dispatch -> its start), the queue ids, and the step period.

    python tools/graph_trace_analyze.py <kernel_trace.csv> [<kernel_trace.csv> ...]
"""
import csv
import statistics as st
import sys


def short(name: str) -> str:
    n = name.split("(")[0]
    for key in ("smf_fwd_lanes_kernel", "smf_epilogue_kernel", "smf_fwd_kernel",
                "smf_vjp_tiles_kernel", "fused_adam", "smf_vjp_lanes_kernel", "xgmi"):
        if key in n:
            return n.replace("void ", "").replace("mg::", "")
    return None


def analyze(path: str, last: int = 400):
    rows = [r for r in csv.DictReader(open(path)) if short(r["Kernel_Name"])]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-last:]
    per = {}
    prev_end = None
    fwd_starts = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        d = per.setdefault(k, {"dur": [], "gap": [], "queues": set()})
        d["dur"].append((e - s) / 1e3)
        if prev_end is not None:
            d["gap"].append((s - prev_end) / 1e3)
        d["queues"].add(r["Queue_Id"])
        prev_end = e
        if "fwd" in k:
            fwd_starts.append(s)
    period = [(b - a) / 1e3 for a, b in zip(fwd_starts, fwd_starts[1:])]
    out = {"file": path, "dispatches": len(rows),
           "step_period_us": round(st.median(period), 2) if period else None}
    for k, d in per.items():
        out[k] = {"n": len(d["dur"]), "dur_us_median": round(st.median(d["dur"]), 2),
                  "gap_before_us_median": round(st.median(d["gap"]), 2) if d["gap"] else None,
                  "gap_before_us_p90": round(sorted(d["gap"])[int(0.9 * (len(d["gap"]) - 1))], 2)
                  if d["gap"] else None,
                  "queues": sorted(d["queues"])}
    return out


if __name__ == "__main__":
    import json
    for p in sys.argv[1:]:
        print(json.dumps(analyze(p)), flush=True)
