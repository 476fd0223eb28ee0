#!/bin/bash
# Kernel timeline of one training step (tools/train_trace.py under rocprofv3): the
# last SPAN ms -> gpurun_out/$TAG/train_timeline.txt (the raw trace is deleted).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-trainprof}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/train_trace.py > $OUT/train.log 2>&1 || { echo "trace failed"; tail -5 $OUT/train.log; exit 1; }
t=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline.py $t ${SPAN:-5} > $OUT/train_timeline.txt
python3 $R/tools/trace_summary.py $t --top 16 > $OUT/train_summary.txt
rm -rf $OUT/trace
cat $OUT/train_summary.txt
