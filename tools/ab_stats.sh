#!/bin/bash
# A/B of the reference statistics kernel over variants (tools/stats_probe.py per library)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-abstats}
mkdir -p $OUT
for r in 1 2; do
  for lib in $R/${VDIR:-variants}/libgnpde_*.so; do
    echo -n "$(basename $lib) " >> $OUT/ab.txt
    GNPDE_LIB=$lib timeout -k 10 120 python3 $R/tools/stats_probe.py >> $OUT/ab.txt 2>> $OUT/ab.err || exit 1
  done
done
cat $OUT/ab.txt
