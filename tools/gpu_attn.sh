#!/bin/bash
# Attention session: parity tests of the attention paths, the reference-mode
# piece bench, and a kernel trace of it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02e}
OUT=$R/gpurun_out
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest ${FILES:-tests/test_gpu_parity.py} -m gpu -q -ra --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/attn_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -8 $OUT/attn_tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u tools/attn_ref_bench.py > $OUT/attn_ref_${TAG}.jsonl 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 1500 $OUT/attn_ref_${TAG}.jsonl; if fatal $rc; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_attn_${TAG} -o run -- \
  python3 $R/tools/attn_ref_bench.py > $OUT/prof_attn_${TAG}.log 2>&1; rc=$?
echo "trace rc=$rc"
f=$(find $OUT/prof_attn_${TAG} -name "*kernel_stats.csv" | head -1); python3 $R/tools/kstats.py "$f" 30
if [ -n "${SWEEP_TILES:-}" ]; then
  cd $R
  for t in $SWEEP_TILES; do
    GNPDE_KEYSUM_TILES=$t timeout -k 10 200 python -u tools/attn_ref_bench.py > $OUT/attn_tiles_$t.jsonl 2>&1; rc=$?
    echo "tiles $t rc=$rc $(tail -c 400 $OUT/attn_tiles_$t.jsonl)"; if fatal $rc; then exit $rc; fi
  done
fi
