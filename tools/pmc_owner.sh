#!/bin/bash
# Round 5: PMC counters of the 8-GPU owner-shard proxy (1/8 of params and halos on one GPU).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/pmc_owner
mkdir -p "$O"
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/owner" -o set$i -- \
    python3 "$R/bench.py" --params 1250000 --halos 16777216 --steps 20 --warmup 3 --no-count-launches > "$O/log$i.txt" 2>&1 || exit $?
done
python3 $R/tools/pmc_summary.py $O/owner smf_ > $O/table.md
cat $O/table.md
