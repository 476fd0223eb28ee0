#!/bin/bash
# Round-3 closing session on one MI355X: the whole -m gpu suite + smoke + bench
# (tools/gpu_tests.sh), the training-step timing, then the PMC traffic table of the
# current library (tools/prof_r03.sh, pmc step only).  Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
TAG=r03t bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python3 tools/train_trace.py > gpurun_out/r03t/train.log 2>&1 || exit $?
tail -1 gpurun_out/r03t/train.log
TAG=r03q STEPS=pmc bash tools/prof_r03.sh
