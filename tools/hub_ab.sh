#!/bin/bash
# A/B of the hub-row combine: in-launch (default) vs the separate fixup kernels
# (GNPDE_HUB_FIXUP=1), alternated on one box: K1 stage timings, one
# cached-graph odeint call and the attention RHS micro-benchmark.
# Output: gpurun_out/k1s_<v>.log, ov_<v>.log, ab_attn_<v>.log
set -u
mkdir -p gpurun_out
for v in 0 1 0 1; do
  GNPDE_HUB_FIXUP=$v timeout -k 10 120 python tools/k1_stage_bench.py > gpurun_out/k1s_$v.log 2>&1 || exit 1
  grep "^{" gpurun_out/k1s_$v.log
done
for v in 0 1; do
  GNPDE_HUB_FIXUP=$v OV_WARM_STEPS=10 timeout -k 10 120 python tools/odeint_overhead.py > gpurun_out/ov_$v.log 2>&1 || exit 1
  echo "fixup=$v $(grep '^{' gpurun_out/ov_$v.log | cut -c1-90)"
done
for v in 0 1; do
  GNPDE_HUB_FIXUP=$v ATT_MODES=reference:1 timeout -k 10 120 python tools/attn_bench.py > gpurun_out/ab_attn_$v.log 2>&1 || exit 1
  echo "fixup=$v $(grep '^{' gpurun_out/ab_attn_$v.log)"
done
