#!/bin/bash
# Round 6: PMC counters of the SMF fused step (forward + step kernel) in the reference's GD
# benchmark at 1e8 halos, kernel-trace only, one pass per counter set.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/r6_pmc_smf2
mkdir -p "$O"
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/gd1e8" -o set$i -- \
    python3 "$R/benchmarks/smf_gd_benchmark.py" --num-halos 100000000 --num-steps 100 > "$O/log$i.txt" 2>&1 || exit $?
done
cd "$R"
python tools/pmc_summary.py $O/gd1e8 "smf2_fwd" "smf2_step" | head -10
