set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_layout.py -v --timeout 200 --timeout-method thread > gpurun_out/layout_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -12 gpurun_out/layout_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_layout.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench_layout.log
case $rc in 124|134|137|139) exit $rc;; esac
GNPDE_NODE_ORDER=none timeout -k 10 600 python bench.py --no-cpu-baseline --no-attention > gpurun_out/bench_nolayout.log 2>&1; rc=$?
echo "bench none rc=$rc"; tail -c 1500 gpurun_out/bench_nolayout.log
