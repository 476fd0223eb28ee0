#!/bin/bash
# Kernel timelines of one G-arxiv dopri5 solve (tools/dopri5_trace.py under
# rocprofv3) for the product library and the A/B variants named in $LIBS
# (paths of libgnpde*.so, GNPDE_LIB), plus the wall-clock dopri5 line of each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-d5tl}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
LIBS=${LIBS:-"$R/graph-neural-pde_amd/gnpde/libgnpde.so"}
i=0
for L in $LIBS; do
  n=$(basename $L .so)
  GNPDE_LIB=$L timeout -k 10 200 python3 $R/tools/dopri5_prof.py --reps 5 > $OUT/${n}_wall.txt 2>&1 || { echo "wall $n failed"; tail -5 $OUT/${n}_wall.txt; exit 1; }
  echo "$n: $(tail -1 $OUT/${n}_wall.txt)"
  GNPDE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$n -o run -- \
    python3 $R/tools/dopri5_trace.py > $OUT/${n}_trace.log 2>&1 || { echo "trace $n failed"; tail -5 $OUT/${n}_trace.log; exit 1; }
  t=$(find $OUT/trace_$n -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/timeline.py $t > $OUT/${n}_timeline.txt
  rm -rf $OUT/trace_$n
  tail -2 $OUT/${n}_timeline.txt
  i=$((i+1))
done
