#!/bin/bash
# torch_replay_repro.py (quick set: the failing schedules) under runtime settings that
# separate ordering races from allocator effects
for e in "BASE=1" "AMD_SERIALIZE_KERNEL=3" "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "REPRO_SYNC=stream" "PYTORCH_HIP_ALLOC_CONF=expandable_segments:True"; do
  echo "== $e"
  env REPRO_QUICK=1 $e timeout -k 10 200 python3 tools/dbg/torch_replay_repro.py 2>&1 | grep -v amdgpu.ids || exit 1
done
