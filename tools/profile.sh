#!/bin/bash
# rocprofv3 passes over bench.py: kernel trace + stats, then one PMC pass per
# counter (FETCH_SIZE / WRITE_SIZE cannot share a pass on gfx950).
# Usage: TAG=r01 tools/profile.sh   (outputs under gpurun_out/prof_$TAG*)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r01}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
BARGS=${BENCH_ARGS:---no-cpu-baseline}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_trace -o run -- \
  python3 $R/bench.py $BARGS > $OUT/prof_${TAG}_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -3 $OUT/prof_${TAG}_trace.log; if fatal $rc; then exit $rc; fi
for ctr in ${PMCS-FETCH_SIZE WRITE_SIZE}; do
  timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-include-regex "${KREGEX:-agg_kernel}" --output-format csv \
    -d $OUT/prof_${TAG}_pmc_$ctr -o run -- python3 $R/bench.py --no-cpu-baseline --no-attention --steps 5 --warmup 2 --rhs-plain-reps 5 \
    > $OUT/prof_${TAG}_pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; tail -2 $OUT/prof_${TAG}_pmc_$ctr.log; if fatal $rc; then exit $rc; fi
done
find $OUT -name "*.csv" -newer $OUT/prof_${TAG}_trace.log -o -name "*stats*.csv" | head -20
