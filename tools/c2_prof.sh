#!/bin/bash
# configs[1] (Cora-sized transformer, dopri5) per-kernel summary of one solve under
# rocprofv3 --kernel-trace for each spec in $SPECS, plus the wall-clock per-step time
# (tools/dopri5_prof.py --c2).  A spec is "name@path-of-libgnpde.so@ENV=V,ENV2=W"
# (path and environment optional): A/B variants of the library and of the knobs.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-c2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SPECS=${SPECS:-"product"}
for S in $SPECS; do
  IFS='@' read -r n L E <<< "$S"
  L=${L:-$R/graph-neural-pde_amd/gnpde/libgnpde.so}
  case $L in /*) ;; *) L=$R/$L ;; esac
  ENVS="GNPDE_LIB=$L ${E//,/ }"
  env $ENVS timeout -k 10 200 python3 $R/tools/dopri5_prof.py --c2 --reps 10 > $OUT/${n}_wall.txt 2>&1 || { echo "wall $n failed"; tail -5 $OUT/${n}_wall.txt; exit 1; }
  echo "$n: $(tail -1 $OUT/${n}_wall.txt)"
  [ "${WALL_ONLY:-0}" = 1 ] && continue
  env $ENVS timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$n -o run -- \
    python3 $R/tools/dopri5_trace.py --c2 > $OUT/${n}_trace.log 2>&1 || { echo "trace $n failed"; tail -5 $OUT/${n}_trace.log; exit 1; }
  t=$(find $OUT/trace_$n -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/timeline.py $t --summary > $OUT/${n}_summary.txt
  rm -rf $OUT/trace_$n
  head -6 $OUT/${n}_summary.txt
done
