set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_layout.py -q --timeout 300 --timeout-method thread > gpurun_out/sharded_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/sharded_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 400 python tools/stripe_bench.py > gpurun_out/stripe_default.log 2>&1 || exit 1
grep '^{' gpurun_out/stripe_default.log
