#!/bin/bash
# Kernel traces of the attention RHS workloads (tools/pmc_run.py attn:*, the solve's
# node numbering): per-kernel mean durations -> gpurun_out/$TAG/attn_*_summary.txt
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-attnprof}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for w in ${WL:-attn:reference_norm1 attn:per_edge_norm0 attn:per_edge_norm1}; do
  f=${w//:/_}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$f -o run -- \
    python3 $R/tools/pmc_run.py $w --reps 20 > $OUT/$f.log 2>&1 || { echo "$w failed"; tail -5 $OUT/$f.log; exit 1; }
  t=$(find $OUT/$f -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/trace_summary.py $t --top 12 > $OUT/${f}_summary.txt
  rm -rf $OUT/$f
  echo "== $w"; cat $OUT/${f}_summary.txt
done
