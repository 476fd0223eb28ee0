set -u
mkdir -p gpurun_out/r03f1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_flash.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "flash or attention or stage" > gpurun_out/r03f1/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r03f1/pytest.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-grmat --no-train --no-cpu-baseline > gpurun_out/r03f1/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 400 gpurun_out/r03f1/bench.log
