#!/bin/bash
# Profile session: kernel trace + stats of the full bench, PMC passes (FETCH_SIZE,
# WRITE_SIZE separately) over K1 and the attention kernels, then the plain bench line.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02e}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_trace -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $OUT/prof_${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -c 300 $OUT/prof_${TAG}_trace.log; echo; if fatal $rc; then exit $rc; fi
KRE='agg_kernel|keysum|key_proj|node_scores|seg_softmax|linear_|stats_|attn_'
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex "$KRE" --output-format csv \
    -d $OUT/prof_${TAG}_pmc_$ctr -o run -- python3 $R/bench.py --no-cpu-baseline --no-grmat --steps 5 --warmup 2 \
    --rhs-plain-reps 5 > $OUT/prof_${TAG}_pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; if fatal $rc; then exit $rc; fi
done
cd $R
timeout -k 10 600 python3 bench.py > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 400 $OUT/bench.log
