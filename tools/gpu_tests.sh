#!/bin/bash
# GPU test session: the -m gpu suite (one process, per-test time limits), smoke(),
# then a short bench line.  Stops at the first failing step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-tests}
mkdir -p $OUT
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
[ $rc = 0 ] || exit $rc
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 1500 $OUT/bench.log
fi
