set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py -q --timeout 200 --timeout-method thread > gpurun_out/layout_tests.log 2>&1; rc=$?
echo "layout tests rc=$rc"; tail -3 gpurun_out/layout_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
GNPDE_NODE_ORDER=none timeout -k 10 400 python tools/stripe_bench.py > gpurun_out/stripes_none.log 2>&1 || exit 1
GNPDE_LAYOUT_MIN_MB=0 timeout -k 10 400 python tools/stripe_bench.py > gpurun_out/stripes_deg.log 2>&1 || exit 1
grep '^{' gpurun_out/stripes_none.log; echo ---; grep '^{' gpurun_out/stripes_deg.log
