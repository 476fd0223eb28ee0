#!/bin/bash
# A/B of the Laplacian K1 builds named in $LIBS (GNPDE_LIB paths): the headline rk4
# line (bench.py without the attention / training / G-rmat / CPU legs) and the
# dopri5 wall time of each, twice in alternation.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ablap}
mkdir -p $OUT
cd $R
for rep in 1 2; do
  for L in $LIBS; do
    n=$(basename $L .so)
    GNPDE_LIB=$L timeout -k 10 300 python3 bench.py --no-attention --no-train --no-grmat --no-cpu-baseline \
      --steps 20 --warmup 5 > $OUT/${n}_bench$rep.log 2>&1 || { echo "bench $n failed"; tail -5 $OUT/${n}_bench$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], 'value', d['value'], 'launch_ms', d['roofline']['launch_ms'], 'plain', d['rhs_plain']['rhs_ms'])" $OUT/${n}_bench$rep.log $n
    GNPDE_LIB=$L timeout -k 10 200 python3 tools/dopri5_prof.py --reps 5 > $OUT/${n}_d5_$rep.txt 2>&1 || { echo "dopri5 $n failed"; exit 1; }
    echo "$n $(tail -1 $OUT/${n}_d5_$rep.txt)"
  done
done
