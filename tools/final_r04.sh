#!/bin/bash
# Closing GPU session of round 4: the GPU suite, smoke(), the driver-form bench line
# (fresh fractions from profiles/traffic.json) and the training / attention lines.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r04final}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $OUT/bench.json; [ $rc = 0 ] || exit $rc
