#!/bin/bash
# Training-path check: the backward GPU tests, then the bench's training and
# block-forward lines (no G-rmat, no CPU baseline) with a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-train}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_backward.py tests/test_gpu_grad_golden.py -x -q --timeout 120 \
  --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-grmat --no-cpu-baseline --no-attention > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 $OUT/bench.log
