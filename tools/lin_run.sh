set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "linear or per_edge or attention" -q --timeout 120 --timeout-method thread > gpurun_out/lin_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/lin_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
for v in 2 0; do for w in 1024 2048 3072 4096; do
  GNPDE_LINEAR=$v GNPDE_LIN_WAVES=$w timeout -k 10 120 python tools/linear_bench.py || exit 1
done; done
LIN_K=80 LIN_N=256 timeout -k 10 120 python tools/linear_bench.py
GNPDE_LINEAR=2 LIN_K=80 LIN_N=256 timeout -k 10 120 python tools/linear_bench.py
