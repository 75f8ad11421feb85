"""Instruction census of one kernel in a device .s file: per basic block, counts of VALU /
transcendental / packed / SALU / memory instructions; the hottest loop is the block with
a backward branch and the most VALU.  Usage: python tools/isa_census.py file.s REGEX"""
import re
import sys
from collections import Counter

TRANS = ("v_exp_f32", "v_log_f32", "v_rcp_f32", "v_rsq_f32", "v_sqrt_f32", "v_sin_f32", "v_cos_f32")


def kernel_lines(path, pat):
    lines = open(path).read().split("\n")
    rx = re.compile(pat)
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^[A-Za-z_][\w.]*:", l) and rx.search(l.split(":")[0]):
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i]
    raise SystemExit("kernel not found")


def census(block):
    c = Counter()
    for l in block:
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
            continue
        op = t[0]
        if op.startswith("v_"):
            c["valu"] += 1
            if op.startswith(TRANS):
                c["trans"] += 1
            if op.startswith("v_pk_"):
                c["pk"] += 1
            c[op] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
            c[op] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "ds_", "scratch_")):
            c["mem"] += 1
            c[op] += 1
    return c


def main():
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    blocks, cur, name = [], [], "entry"
    for l in lines:
        if re.match(r"^\.LBB\d+_\d+:", l):
            blocks.append((name, cur))
            name, cur = l.split(":")[0], []
        else:
            cur.append(l)
    blocks.append((name, cur))
    tot = census(lines)
    print("kernel total:", {k: tot[k] for k in ("valu", "trans", "pk", "salu", "mem")})
    for name, b in blocks:
        c = census(b)
        if c["valu"] < 20:
            continue
        loop = any(name in l for l in b if "s_cbranch" in l or "s_branch" in l)
        print(f"{name} loop={loop} valu={c['valu']} trans={c['trans']} pk={c['pk']} salu={c['salu']} mem={c['mem']}")
        top = [(k, v) for k, v in c.most_common() if k not in ("valu", "trans", "pk", "salu", "mem")][:24]
        print("   ", " ".join(f"{k}:{v}" for k, v in top))


if __name__ == "__main__":
    main()
