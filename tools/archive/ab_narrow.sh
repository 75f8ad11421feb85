#!/bin/bash
# Alternating same-box A/B of the headline bench (in-tree _C.so vs variants/<v>/_C.so for each
# variant) at given narrow-population fractions:
#   bash tools/ab_narrow.sh "<variants>" "<fractions>" [steps] [reps]   -> stdout lines
set -u
variants=$1; fracs=$2; steps=${3:-200}; reps=${4:-2}
mkdir -p gpurun_out/ab
cp multigrad_amd/_C.so /tmp/_C_base.so
restore() { cp /tmp/_C_base.so multigrad_amd/_C.so; }
trap restore EXIT
for f in $fracs; do
  for r in $(seq $reps); do
    for v in base $variants; do
      if [ $v = base ]; then restore; else cp variants/$v/_C.so multigrad_amd/_C.so; fi
      o=gpurun_out/ab/${v}_${f}_$r.json
      timeout -k 10 300 python3 bench.py --steps $steps --warmup 5 --narrow-frac $f \
        --no-count-launches > $o 2> ${o%.json}.err || { echo "bench $v $f failed"; exit 1; }
      echo "$v narrow=$f rep=$r $(grep -o '"value": [0-9.]*' $o) $(grep -o '"ms_per_step": [0-9.]*' $o)"
    done
  done
done
