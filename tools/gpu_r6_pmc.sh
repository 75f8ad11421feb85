#!/bin/bash
# Round 6: PMC counters of the headline forward with and without the two-term EM groups
# (clock, bytes, VALU per halo of each candidate), kernel-trace only, one
# pass per counter set; then every BASELINE config on this tree.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
O=$R/gpurun_out/r6_pmc
mkdir -p "$O"
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/em2" -o set$i -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --no-count-launches > "$O/em2_log$i.txt" 2>&1 || exit $?
  MULTIGRAD_EXT_SO=$R/abvar/em2off/_C.so timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$O/em2off" -o set$i -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --no-count-launches > "$O/em2off_log$i.txt" 2>&1 || exit $?
done
cd "$R"
python tools/pmc_summary.py $O/em2 "smf_fwd_lanes" "smf_epilogue" | head -8
python tools/pmc_summary.py $O/em2off "smf_fwd_lanes" "smf_epilogue" | head -8
timeout -k 10 900 python -u benchmarks/configs.py --which toy adam1e6 adam1e7 adam1e8 lbfgs lbfgsb --steps 200 \
  > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
grep '^{' $O/configs.log | cut -c1-250
