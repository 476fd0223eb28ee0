#!/bin/bash
# projection waves sweep + bf16 BLEND geometry A/B
set -u
mkdir -p gpurun_out
OUT=gpurun_out/kern_sweep.log; : > $OUT
for w in 1024 2048 3072 4096 6144 8192; do
  GNPDE_LIN_WAVES=$w timeout -k 10 120 python3 tools/linear_bench.py >> $OUT 2>/dev/null; rc=$?
  case $rc in 124|134|137|139) echo "linear rc=$rc"; exit $rc;; esac
done
GNPDE_LINEAR=1 timeout -k 10 120 python3 tools/linear_bench.py >> $OUT 2>/dev/null
for v in 0 9 0 9; do
  K1_C=${K1_C:-168} GNPDE_AGG_VARIANT=$v timeout -k 10 200 python3 tools/bf16_k1_bench.py >> $OUT 2>&1; rc=$?
  case $rc in 124|134|137|139) echo "bf16 rc=$rc"; exit $rc;; esac
done
cat $OUT
