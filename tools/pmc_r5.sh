#!/bin/bash
# Round 5: PMC counters (kernel-trace only, one pass per counter set) of the headline step's
# kernels and of the per-rank proxy of the 8-GPU hashed step (tiles layout, 1/8 of the halos).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/pmc_r5
mkdir -p "$O"
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/head" -o set$i -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --no-count-launches > "$O/head_log$i.txt" 2>&1 || exit $?
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/proxy" -o set$i -- \
    python3 "$R/bench.py" --params 10000000 --halos 16777216 --layout tiles --steps 20 --warmup 3 \
    --no-count-launches > "$O/proxy_log$i.txt" 2>&1 || exit $?
done
echo done
