#!/bin/bash
# Kernel timelines of one G-arxiv dopri5 solve (tools/dopri5_trace.py under
# rocprofv3) and the wall-clock dopri5 line for each spec in $SPECS
# ("name@path-of-libgnpde.so@ENV=V,ENV2=W", as tools/c2_prof.sh; default: the product).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-d5tl}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SPECS=${SPECS:-"product"}
for S in $SPECS; do
  IFS='@' read -r n L E <<< "$S"
  L=${L:-$R/graph-neural-pde_amd/gnpde/libgnpde.so}
  case $L in /*) ;; *) L=$R/$L ;; esac
  ENVS="GNPDE_LIB=$L ${E//,/ }"
  env $ENVS timeout -k 10 200 python3 $R/tools/dopri5_prof.py --reps 5 > $OUT/${n}_wall.txt 2>&1 || { echo "wall $n failed"; tail -5 $OUT/${n}_wall.txt; exit 1; }
  echo "$n: $(tail -1 $OUT/${n}_wall.txt)"
  env $ENVS timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$n -o run -- \
    python3 $R/tools/dopri5_trace.py > $OUT/${n}_trace.log 2>&1 || { echo "trace $n failed"; tail -5 $OUT/${n}_trace.log; exit 1; }
  t=$(find $OUT/trace_$n -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/timeline.py $t > $OUT/${n}_timeline.txt
  rm -rf $OUT/trace_$n
  tail -1 $OUT/${n}_timeline.txt
done
