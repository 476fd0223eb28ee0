#!/bin/bash
# One GPU session: smoke, the whole GPU suite, the default bench line.
set -u
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; if fatal $rc; then exit $rc; fi
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -ra --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -12 gpurun_out/gpu_tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 4000 gpurun_out/bench.log
