#!/bin/bash
# SQ counters of the MFMA projection (tools/linear_bench.py), one pass per set.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-include-regex "linear_mfma" --output-format csv -d $OUT/pmc_lin_$i -o run -- \
    python3 $R/tools/linear_bench.py > $OUT/pmc_lin_$i.log 2>&1
  rc=$?; echo "set $i rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
python3 $R/tools/pmc_table.py $OUT/pmc_lin_1/run_counter_collection.csv $OUT/pmc_lin_2/run_counter_collection.csv
