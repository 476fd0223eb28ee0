#!/bin/bash
# The whole GPU suite, then one bench line without the CPU baseline.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -ra --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -6 gpurun_out/gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1; rc=$?
echo "bench rc=$rc"
python - <<'PY'
import json
d = [json.loads(l) for l in open("gpurun_out/bench_quick.log") if l.startswith('{"metric"')][-1]
print("value", d["value"], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
if "attention" in d:
    print({k: v["rhs_ms"] for k, v in d["attention"].items() if isinstance(v, dict)})
    print("blend", d["blend_c162"]["fp32"]["ms_per_step"], d["blend_c162"]["bf16"]["ms_per_step"])
if "grmat" in d:
    print("grmat", d["grmat"]["one_gpu"]["value"])
PY
