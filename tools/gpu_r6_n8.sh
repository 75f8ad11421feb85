#!/bin/bash
# Round 6: 8 processes sharing one MI355X, hashed input re-partitioned by owner at setup
# (rehearsal of the driver's N=8 run), with set-up tracing to find where a rank stalls.
set -o pipefail
O=gpurun_out/r6_n8
mkdir -p $O
GPU_MAX_HW_QUEUES=${HWQ:-4} MULTIGRAD_TRACE=1 NPROC=8 PLACEMENT=repartition timeout -k 10 400 bash tools/bench_2rank.sh --steps 20 --warmup 5 --no-count-launches \
  > $O/bench_n8.json 2> $O/bench_n8.err; rc=$?
grep -v "amdgpu.ids\|socket.cpp" $O/bench_n8.err | tail -60
echo "rc=$rc"
[ $rc -eq 0 ] && python -c "
import json; d=json.loads([l for l in open('$O/bench_n8.json') if l.startswith('{')][-1])
print(8, 'value', d['value'], 'loss', d['loss_last'], 'setup', d['setup_s'], d['config']['autotune'])"
exit $rc
