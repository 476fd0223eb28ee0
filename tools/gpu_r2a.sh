#!/bin/bash
# Round-2 first GPU session: smoke, the new GPU tests, the whole GPU suite, the bench.
set -u
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; if fatal $rc; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_blocks.py tests/test_gpu_sharded.py -v -ra --timeout 300 --timeout-method thread > gpurun_out/gpu_new.log 2>&1; rc=$?
echo "new tests rc=$rc"; tail -15 gpurun_out/gpu_new.log; if fatal $rc; then exit $rc; fi
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -ra --timeout 200 --timeout-method thread --deselect tests/test_gpu_sharded.py --deselect tests/test_gpu_blocks.py -x > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -8 gpurun_out/gpu_tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
