#!/bin/bash
# Headline bench over the share of narrow populations (bin width > 0.5 sigma: outside the
# Euler-Maclaurin forward's range), the in-tree build against variants/<name>/_C.so
# (e.g. round 3's deferral list: tools/build_variant.sh defer1 -DMG_LANES_DEFER=1),
# alternating on one box, then one rocprofv3 kernel trace per share with the in-tree build.
#   [STEPS=200] bash tools/narrow_sweep.sh <variant> [fractions...]   -> gpurun_out/narrow/
set -u
export TMPDIR=/tmp
name=$1; shift
steps=${STEPS:-200}
fracs=${*:-0 0.01 0.1 1.0}
out=gpurun_out/narrow
mkdir -p $out
cp multigrad_amd/_C.so /tmp/_C_base.so
restore() { cp /tmp/_C_base.so multigrad_amd/_C.so; }
trap restore EXIT
for f in $fracs; do
  for v in base $name; do
    if [ $v = base ]; then restore; else cp variants/$v/_C.so multigrad_amd/_C.so; fi
    timeout -k 10 300 python3 bench.py --steps $steps --warmup 5 --narrow-frac $f \
      > $out/${v}_$f.json 2> $out/${v}_$f.err || { echo "bench $v $f failed"; exit 1; }
    echo "$v narrow=$f $(grep -o '"value": [0-9.]*' $out/${v}_$f.json) $(grep -o '"per_edge_groups": \[[0-9, ]*\]' $out/${v}_$f.json)"
  done
done
restore
for f in $fracs; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$f -o run -- \
    python3 bench.py --steps $steps --warmup 5 --narrow-frac $f --no-count-launches \
    > $out/prof_$f.json 2> $out/prof_$f.err || { echo "rocprof $f failed"; exit 1; }
  # keep the per-kernel statistics and the trace of the last 120 kernels (the timed steps)
  for t in $(find $out/prof_$f -name '*kernel_trace.csv'); do
    { head -1 $t; tail -120 $t; } > ${t%.csv}_tail.csv && rm -f $t
  done
  find $out/prof_$f -type f ! -name '*kernel_stats.csv' ! -name '*_tail.csv' -delete
done
echo done
