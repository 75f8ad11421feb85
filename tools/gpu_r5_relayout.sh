#!/bin/bash
# Round 5: re-layout of the lane groups during a fit -- GPU tests, then 2000-step benches
# whose narrow populations start wide and cross the Euler-Maclaurin limit (~step 100):
# re-layout on, off, and the per-edge kernel forced; per-100-step phase rates.
set -o pipefail
O=gpurun_out/r5_relayout
mkdir -p $O
export MULTIGRAD_PROGRESS=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_relayout_during_fit_matches_static_layout" \
  "tests/test_kernels_gpu.py::test_relayout_checkpoint_resumes_in_setup_layout" \
  "tests/test_kernels_gpu.py::test_narrow_populations_get_their_own_lane_groups" \
  "tests/test_kernels_gpu.py::test_per_edge_kernel_mode_matches_em_kernel" \
  > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
A="--steps 2000 --warmup 5 --narrow-frac 0.01 --narrow-guess -0.64 --phase-steps 100 --no-count-launches"
timeout -k 10 300 python -u bench.py $A > $O/relayout_on.json 2> $O/on.err || { tail -20 $O/on.err; exit 1; }
MULTIGRAD_RELAYOUT=0 timeout -k 10 300 python -u bench.py $A > $O/relayout_off.json 2> $O/off.err || { tail -20 $O/off.err; exit 1; }
MULTIGRAD_RELAYOUT=0 MULTIGRAD_PER_EDGE_SHARE=0 timeout -k 10 300 python -u bench.py $A > $O/per_edge_kernel.json 2> $O/pe.err || { tail -20 $O/pe.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 5 --narrow-frac 0.01 --phase-steps 100 --no-count-launches > $O/narrow_at_start.json 2> $O/ns.err || { tail -20 $O/ns.err; exit 1; }
for f in $O/*.json; do python -c "
import json; d=json.load(open('$f'))
print('$f', d['value'], [p['ms_per_step'] for p in d['phases']], [p['per_edge_share'] for p in d['phases']], d['config']['relayouts'])"; done
