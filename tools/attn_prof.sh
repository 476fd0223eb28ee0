#!/bin/bash
# Kernel-level profile of the attention RHS micro-benchmark (tools/attn_bench.py).
# Usage: TAG=x tools/attn_prof.sh  -> gpurun_out/attn_$TAG/ (kernel stats) + attn_$TAG.log
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-a}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/attn_$TAG -o run -- \
  python3 $R/tools/attn_bench.py > $OUT/attn_$TAG.log 2>&1
rc=$?; echo "attn prof rc=$rc"; cat $OUT/attn_$TAG.log | grep '^{'; exit $rc
