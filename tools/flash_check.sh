set -u
mkdir -p gpurun_out/r03f
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_flash.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "flash or attention or stage" > gpurun_out/r03f/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03f/pytest.log
[ $rc = 0 ] || exit $rc
TAG=r03f PROF=1 ROUNDS=2 bash tools/variants_ab.sh
