set -u
OUT=gpurun_out/r06f; mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_dense_fold.py tests/test_gpu_adaptive.py tests/test_gpu_endtoend.py -x -q --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
[ $rc = 0 ] || exit $rc
for f in 1 0 1; do
  GNPDE_DENSE_FOLD=$f timeout -k 10 200 python3 tools/bench_part.py dopri5 5 > $OUT/dopri5_fold$f.json 2>&1; rc=$?
  echo "dopri5 fold=$f rc=$rc"; tail -c 900 $OUT/dopri5_fold$f.json; echo
  [ $rc = 0 ] || exit $rc
done
