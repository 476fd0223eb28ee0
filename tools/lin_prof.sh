#!/bin/bash
# Kernel trace + SQ/TCC counters of the projection micro-benchmark.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lin_trace -o run -- python3 $R/tools/linear_bench.py > $OUT/lin_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
grep -E "linear" $OUT/lin_trace/run_kernel_stats.csv | cut -c1-200
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "linear_" --output-format csv -d $OUT/pmc_lin_$i -o run -- \
    python3 $R/tools/linear_bench.py > $OUT/pmc_lin_$i.log 2>&1
  rc=$?; echo "set $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 $R/tools/pmc_table.py $OUT/pmc_lin_*/run_counter_collection.csv
