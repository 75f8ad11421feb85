"""Per-kernel means of rocprofv3 --pmc counter CSVs (tools/pmc_r5.sh) and derived shares.

Usage: python tools/pmc_summary.py <dir> [name filter ...] -> a markdown table on stdout."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
filters = sys.argv[2:] or ["mg::"]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "set*_counter_collection.csv"))):
    per_dispatch = {}
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if not any(x in name for x in filters):
            continue
        short = name.split("(")[0].replace("void ", "")
        key = (short, r["Dispatch_Id"])
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
        per_dispatch[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    for (short, _), us in per_dispatch.items():
        dur[short].append(us)


def mean(x):
    return sum(x) / len(x) if x else float("nan")


SIMDS, XCDS = 1024, 8
print("| kernel | µs | VALU instr (waves) | trans | VALU active / SIMD cycles | dep. wait / wave cycles | clock GHz | HBM rd+wr MB |")
print("|---|---|---|---|---|---|---|---|")
for k, c in sorted(vals.items(), key=lambda kv: -mean(dur[kv[0]])):
    m = {n: mean(v) for n, v in c.items()}
    us = mean(dur[k])
    gui = m.get("GRBM_GUI_ACTIVE", float("nan"))
    cyc = gui / XCDS  # shader-clock cycles of the dispatch (per XCD)
    ghz = cyc / (us * 1e3) if us > 0 else float("nan")
    valu_share = 4 * m.get("SQ_ACTIVE_INST_VALU", float("nan")) / SIMDS / cyc
    dep = m.get("SQ_WAIT_INST_ANY", float("nan")) / m.get("SQ_WAVE_CYCLES", float("nan"))
    mb = (m.get("TCC_EA0_RDREQ_sum", 0) + m.get("TCC_EA0_WRREQ_sum", 0)) * 64 / 1e6
    print(f"| `{k[:60]}` | {us:.1f} | {m.get('SQ_INSTS_VALU', float('nan')):.3g} | "
          f"{m.get('SQ_INSTS_VALU_TRANS_F32', float('nan')):.3g} | {valu_share:.2f} | {dep:.2f} | "
          f"{ghz:.2f} | {mb:.0f} |")
