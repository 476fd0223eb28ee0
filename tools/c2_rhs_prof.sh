#!/bin/bash
# Per-kernel summary of configs[1]'s transformer RHS (tools/c2_rhs_prof.py) under
# rocprofv3 --kernel-trace for each spec in $SPECS ("name@lib@ENV=V,..." as tools/c2_prof.sh).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-c2rhs}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SPECS=${SPECS:-"product"}
for S in $SPECS; do
  IFS='@' read -r n L E <<< "$S"
  L=${L:-$R/graph-neural-pde_amd/gnpde/libgnpde.so}
  case $L in /*) ;; *) L=$R/$L ;; esac
  ENVS="GNPDE_LIB=$L ${E//,/ }"
  env $ENVS timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$n -o run -- \
    python3 $R/tools/c2_rhs_prof.py > $OUT/${n}_trace.log 2>&1 || { echo "trace $n failed"; tail -5 $OUT/${n}_trace.log; exit 1; }
  t=$(find $OUT/trace_$n -name "*kernel_trace.csv" | head -1)
  python3 $R/tools/timeline.py $t --summary > $OUT/${n}_summary.txt
  rm -rf $OUT/trace_$n
  echo "== $n"; head -8 $OUT/${n}_summary.txt
done
