#!/bin/bash
# Kernel timeline of one headline solve (tools/solve_trace.py under rocprofv3).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-solveprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/solve_trace.py > $OUT/solve.log 2>&1 || { echo "trace failed"; tail -5 $OUT/solve.log; exit 1; }
t=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline.py $t > $OUT/solve_timeline.txt
rm -rf $OUT/trace
head -12 $OUT/solve_timeline.txt; tail -4 $OUT/solve_timeline.txt
