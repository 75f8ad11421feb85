#!/bin/bash
# Round 5: PMC counters of the pipelined headline step, unbounded vs --bounds both (kernel-trace
# only, one pass per counter set): where the bounded update's extra time goes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/pmc_bounded
mkdir -p "$O"
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  for b in none both; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/$b" -o set$i -- \
      python3 "$R/bench.py" --steps 10 --warmup 3 --bounds $b --no-count-launches > "$O/${b}_log$i.txt" 2>&1 || exit $?
  done
done
python3 $R/tools/pmc_summary.py $O/none smf_fwd_lanes > $O/none_table.md
python3 $R/tools/pmc_summary.py $O/both smf_fwd_lanes > $O/both_table.md
cat $O/none_table.md $O/both_table.md
