#!/bin/bash
# Quick GPU session: the fused-attention and attention/stage parity tests, the
# default bench line, then (STEPS includes trace) a kernel trace of the bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r03f1}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_flash.py tests/test_gpu_parity.py -x -q --timeout 120 \
  --timeout-method thread -k "${PYK:-flash or attention or stage}" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
[ $rc = 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 300 $OUT/bench.log
[ $rc = 0 ] || exit $rc
if [ "${TRACE:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/trace.log 2>&1
  rc=$?; echo "trace rc=$rc"; tail -c 200 $OUT/trace.log
fi
