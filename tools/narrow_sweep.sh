#!/bin/bash
# Headline bench over the share of narrow populations (bin width > 0.5 sigma: outside the
# Euler-Maclaurin forward's range), the in-tree build against variants/<name>/_C.so
# (e.g. round 3's deferral list: tools/build_variant.sh defer1 -DMG_LANES_DEFER=1),
# alternating on one box, then one rocprofv3 kernel trace per share with the in-tree build.
#   bash tools/narrow_sweep.sh <variant> [fractions...]      -> gpurun_out/narrow/
set -u
name=$1; shift
fracs=${*:-0 0.01 0.1 1.0}
out=gpurun_out/narrow
mkdir -p $out
cp multigrad_amd/_C.so /tmp/_C_base.so
restore() { cp /tmp/_C_base.so multigrad_amd/_C.so; }
trap restore EXIT
for f in $fracs; do
  for v in base $name; do
    if [ $v = base ]; then restore; else cp variants/$v/_C.so multigrad_amd/_C.so; fi
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --narrow-frac $f \
      > $out/${v}_$f.json 2> $out/${v}_$f.err || { echo "bench $v $f failed"; exit 1; }
    echo "$v narrow=$f $(grep -o '"value": [0-9.]*' $out/${v}_$f.json) $(grep -o '"per_edge_groups": \[[0-9, ]*\]' $out/${v}_$f.json)"
  done
done
restore
for f in $fracs; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$f -o run -- \
    python3 bench.py --steps 20 --warmup 5 --narrow-frac $f --no-count-launches \
    > $out/prof_$f.json 2> $out/prof_$f.err || { echo "rocprof $f failed"; exit 1; }
done
echo done
