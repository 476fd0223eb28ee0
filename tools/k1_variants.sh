#!/bin/bash
mkdir -p gpurun_out
make -C graph-neural-pde_amd -j16 > gpurun_out/make.log 2>&1 || exit 1
for v in ${VARIANTS:-0 1 2 3 4 5}; do
  GNPDE_AGG_VARIANT=$v timeout -k 10 300 python tools/k1_bench.py >> gpurun_out/k1_variants.log 2>gpurun_out/k1_err_$v.log
  rc=$?; echo "variant $v rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done
cat gpurun_out/k1_variants.log
