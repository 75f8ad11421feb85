#!/bin/bash
# PMC counters for the SMF kernels (kernel-trace only; no sys/runtime trace with --pmc).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
mkdir -p "$R/gpurun_out/pmc"
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$R/gpurun_out/pmc" -o set$i -- python3 "$R/tools/kernel_bench.py" --iters 3 "$@" > "$R/gpurun_out/pmc/log$i.txt" 2>&1 || exit $?
done
echo done
