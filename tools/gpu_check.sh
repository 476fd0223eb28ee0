#!/bin/bash
# One GPU session: smoke -> gpu tests -> bench.  Stops at the first crash-like
# exit (abort/segv/timeout); plain test failures do not stop the later steps.
set -u
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
# libgnpde.so is built in the container (make -C graph-neural-pde_amd) and travels with the tree
STEPS="${STEPS:-smoke tests bench}"
for s in $STEPS; do
  case $s in
    smoke) timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$? ;;
    tests) timeout -k 10 1200 python -u -m pytest tests -m gpu -q -ra --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1; rc=$? ;;
    bench) timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$? ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  echo "step $s rc=$rc"
  tail -5 gpurun_out/$([ $s = tests ] && echo gpu_tests || echo $s).log
  if fatal $rc; then echo "fatal exit in step $s; stopping"; exit $rc; fi
done
