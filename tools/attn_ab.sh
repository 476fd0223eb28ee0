#!/bin/bash
# A/B of the in-launch long-group statistics combine (default) against the
# separate fixup pass (GNPDE_HUB_FIXUP=1) on the attention RHS micro-benchmark,
# alternated on one box.  Output: gpurun_out/ab_attn_<v>_<i>.log
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0 1; do
    GNPDE_HUB_FIXUP=$v ATT_MODES=${ATT_MODES:-reference:1,per_edge:1} timeout -k 10 120 python tools/attn_bench.py \
      > gpurun_out/ab_attn_${v}_$i.log 2>&1 || exit 1
    grep "^{" gpurun_out/ab_attn_${v}_$i.log | sed "s/^/fixup=$v /"
  done
done
