#!/bin/bash
# Projection check: the linear / attention parity tests, tools/linear_bench.py at the
# attention shape (and K = 64 / 16), the per-edge attention RHS lines, with a trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-lin}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_flash.py tests/test_gpu_backward.py -x -q \
  --timeout 120 --timeout-method thread -k "linear or attention or flash or transformer" > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc = 0 ] || exit $rc
for k in 128 64 16; do
  LIN_K=$k timeout -k 10 120 python3 tools/linear_bench.py >> $OUT/lin.jsonl 2>> $OUT/lin.err || exit 1
done
cat $OUT/lin.jsonl
cd /tmp && export TMPDIR=/tmp
ATT_MODES=per_edge:0,per_edge:1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/attn_ab.py > $OUT/attn.log 2>&1; rc=$?
echo "attn rc=$rc"; grep '^{' $OUT/attn.log
