#!/bin/bash
# Dense-output instantiation + degree kernels: adaptive GPU tests, dopri5 and preprocessing
# kernel traces.  Stops after a crash or time limit of any step.
OUT=gpurun_out/r05k2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_adaptive.py \
  tests/test_gpu_blocks.py > $OUT/t.log 2>&1
rc=$?
tail -2 $OUT/t.log
case $rc in 124|137|134|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o dopri5 -- \
  python3 $GRAFT_REPO_ROOT/tools/dopri5_prof.py --reps 5 > $GRAFT_REPO_ROOT/$OUT/dp.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o prep -- \
  python3 $GRAFT_REPO_ROOT/tools/prep_prof.py > $GRAFT_REPO_ROOT/$OUT/pp.log 2>&1 || exit $?
timeout -k 10 200 python3 $GRAFT_REPO_ROOT/tools/dopri5_prof.py --reps 5 > $GRAFT_REPO_ROOT/$OUT/d.log 2>&1
grep solve $GRAFT_REPO_ROOT/$OUT/d.log
