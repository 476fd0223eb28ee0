#!/bin/bash
# Sweep of the persistent aggregation grid (GNPDE_AGG_BPC workgroups per CU; 0 = one pass, not persistent).
mkdir -p gpurun_out
make -C graph-neural-pde_amd -j16 > gpurun_out/make.log 2>&1 || exit 1
for b in ${BPCS:-0 2 3 4 6 8}; do
  GNPDE_AGG_BPC=$b timeout -k 10 300 python tools/k1_bench.py >> gpurun_out/k1_grid.log 2>gpurun_out/k1_grid_err_$b.log
  rc=$?; echo "bpc $b rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
cat gpurun_out/k1_grid.log
