set -u
GNPDE_LINEAR=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "linear" -q --timeout 120 --timeout-method thread > gpurun_out/lin3_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/lin3_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
for w in 2048 3072 4096; do
  GNPDE_LINEAR=3 GNPDE_LIN_WAVES=$w timeout -k 10 120 python tools/linear_bench.py || exit 1
done
for e in 0 1; do for w in 1024 2048; do
  GNPDE_LIN_EARLY=$e GNPDE_LIN_WAVES=$w timeout -k 10 120 python tools/linear_bench.py || exit 1
done; done
timeout -k 10 300 python tools/reorder_bench.py
