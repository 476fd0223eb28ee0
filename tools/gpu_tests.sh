#!/bin/bash
# GPU test session: the listed test files (default: all -m gpu), then optionally the bench.
# Usage: FILES="tests/a.py tests/b.py" PYTEST_K="bf16 or blend" BENCH=1 tools/gpu_tests.sh
set -u
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ -n "${PYTEST_K:-}" ]; then KARG=(-k "$PYTEST_K"); else KARG=(); fi
timeout -k 10 1100 python -u -m pytest ${FILES:-tests} -m gpu -q -ra --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -25 gpurun_out/gpu_tests.log; if fatal $rc; then exit $rc; fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench.log
fi
