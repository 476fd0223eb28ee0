#!/bin/bash
# A/B session: GPU tests, then the attention piece bench and the headline bench
# under each knob setting in AB (space-separated VAR=VALUE or "base").
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest ${FILES:-tests} -m gpu -q -ra --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/ab_tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; tail -6 $OUT/ab_tests.log; if fatal $rc; then exit $rc; fi
fi
for kv in ${AB:-base}; do
  if [ "$kv" = base ]; then envs=(); else envs=(env "$kv"); fi
  tag=${kv//\//_}
  "${envs[@]}" timeout -k 10 200 python -u tools/attn_ref_bench.py > $OUT/ab_attn_$tag.jsonl 2>&1; rc=$?
  echo "attn[$kv] rc=$rc $(tail -1 $OUT/ab_attn_$tag.jsonl)"; if fatal $rc; then exit $rc; fi
  if [ "${HEADLINE:-1}" = 1 ]; then
    "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-grmat --no-train --no-attention > $OUT/ab_bench_$tag.log 2>&1; rc=$?
    echo "bench[$kv] rc=$rc $(tail -1 $OUT/ab_bench_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["launch_ms"], d.get("rhs_plain",{}).get("rhs_ms"))' 2>&1)"
    if fatal $rc; then exit $rc; fi
  fi
done
