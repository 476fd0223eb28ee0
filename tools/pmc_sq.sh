#!/bin/bash
# SQ-level counters for chosen kernels of the attention path (one pass each).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KR=${KREGEX:-"node_scores|linear_mfma|stats_team|attn_team|keysum_partial|agg_kernel"}
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAVES" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set --kernel-include-regex "$KR" --output-format csv -d $OUT/pmc_sq_$i -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 --rhs-plain-reps 2 > $OUT/pmc_sq_$i.log 2>&1
  rc=$?; echo "set $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
