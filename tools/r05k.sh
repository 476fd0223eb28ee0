#!/bin/bash
# Round-5 Krylov-step validation: GPU tests touching the adaptive solvers, then a
# kernel trace of the G-arxiv dopri5 solve (tools/dopri5_prof.py).  Stops after a
# crash or time limit of any step.
OUT=gpurun_out/r05k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread \
  tests/test_gpu_adaptive.py tests/test_gpu_adjoint.py tests/test_gpu_blocks.py tests/test_gpu_parity.py \
  tests/test_gpu_backward.py tests/test_abi.py > $OUT/t.log 2>&1
rc=$?
tail -3 $OUT/t.log
case $rc in 124|137|134|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o dopri5 -- \
  python3 $GRAFT_REPO_ROOT/tools/dopri5_prof.py --reps 5 > $GRAFT_REPO_ROOT/$OUT/dp.log 2>&1
