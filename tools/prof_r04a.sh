#!/bin/bash
# dopri5 kernel traces (G-arxiv laplacian and the configs[1] transformer shape)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=gpurun_out/r04prof
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/dopri5_prof.py > $OUT/wall.txt 2>&1 || exit $?
timeout -k 10 120 python3 tools/dopri5_prof.py --c2 >> $OUT/wall.txt 2>&1 || exit $?
cat $OUT/wall.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/lap -o run -- python3 tools/dopri5_prof.py --reps 3 > $OUT/lap.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2 -o run -- python3 tools/dopri5_prof.py --reps 3 --c2 > $OUT/c2.log 2>&1 || exit $?
for d in lap c2; do
  f=$(find $OUT/$d -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_summary.py $f --top 30 > $OUT/${d}_summary.txt
  cp $(find $OUT/$d -name "*kernel_stats.csv" | head -1) $OUT/${d}_kernel_stats.csv
  rm -rf $OUT/$d
done
cat $OUT/lap_summary.txt $OUT/c2_summary.txt
