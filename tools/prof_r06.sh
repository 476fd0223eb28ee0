#!/bin/bash
# Round-6 profile session on one MI355X:
#   1. per-workload PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs) of
#      tools/pmc_run.py -> profiles/traffic.json (tools/pmc_reduce.py), the
#      counter bytes bench.py divides by its live launch / RHS times;
#   2. kernel trace + stats of the default bench command (the rocprof summary
#      whose averages must agree with the bench line's HIP-event times);
#   3. the default bench line itself.
# Every GPU step has its own time limit; the script stops at the first fault.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r06z}
OUT=$R/gpurun_out/$TAG
WL=${WORKLOADS:-"lap dopri5 grmat attn:reference_norm1 attn:reference_norm0 attn:per_edge_norm0 attn:per_edge_norm1 blend_bf16 blend_fp32"}
STEPS=${STEPS:-"pmc trace bench"}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
fatal() { [ "$1" != 0 ]; }
if [[ " $STEPS " == *" pmc "* ]]; then
  for w in $WL; do
    f=${w//:/_}
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/${f}_$ctr -o run -- \
        python3 $R/tools/pmc_run.py $w > $OUT/${f}.json 2> $OUT/${f}_$ctr.err
      rc=$?; echo "pmc $w $ctr rc=$rc"; if fatal $rc; then tail -5 $OUT/${f}_$ctr.err; exit $rc; fi
      # the counter CSV may sit one directory level down (rocprofv3 per-host/pid naming)
      c=$(find $OUT/${f}_$ctr -name 'run_counter_collection.csv' | head -1)
      [ -n "$c" ] && [ "$c" != "$OUT/${f}_$ctr/run_counter_collection.csv" ] && cp "$c" $OUT/${f}_$ctr/run_counter_collection.csv
    done
  done
  cd $R && python3 tools/pmc_reduce.py $TAG $OUT $OUT/traffic.json > $OUT/reduce.log 2>&1; echo "reduce rc=$?"; tail -12 $OUT/reduce.log
  cd /tmp
fi
if [[ " $STEPS " == *" trace "* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline > $OUT/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"; tail -c 300 $OUT/trace.log; echo; if fatal $rc; then exit $rc; fi
  # keep the per-kernel stats and a summary; the full trace is too large to merge back
  t=$(find $OUT/trace -name '*kernel_trace.csv' | head -1)
  st=$(find $OUT/trace -name '*kernel_stats.csv' | head -1)
  [ -n "$st" ] && cp "$st" $OUT/kernel_stats.csv
  [ -n "$t" ] && python3 $R/tools/trace_summary.py "$t" --top 40 > $OUT/trace_summary.txt
  rm -rf $OUT/trace
fi
if [[ " $STEPS " == *" bench "* ]]; then
  cd $R
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 600 $OUT/bench.log
fi
