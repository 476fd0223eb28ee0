#!/bin/bash
# the headline K1 (G-arxiv fused rk4 stage, in-degree numbering) with
# the XCD-aware work mapping (GNPDE_XCD_REMAP, experiment build of csrc/rhs.hip:
# variants/libgnpde_xcd.so) — per remap value: the kernel's mean duration
# (rocprofv3 --kernel-trace --stats of tools/pmc_run.py lap) and its counter bytes
# (FETCH_SIZE, WRITE_SIZE in separate passes, tools/pmc_reduce.py) -> $OUT/xcd_ab.jsonl
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-xcd}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
L=$R/variants/libgnpde_xcd.so
for v in ${REMAPS:-0 1 8 32}; do
  D=$OUT/remap$v
  mkdir -p $D
  GNPDE_LIB=$L GNPDE_XCD_REMAP=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
    python3 $R/tools/pmc_run.py lap > $D/trace.log 2>&1 || { echo "trace $v failed"; tail -5 $D/trace.log; exit 1; }
  st=$(find $D/trace -name '*kernel_stats.csv' | head -1); cp "$st" $D/kernel_stats.csv; rm -rf $D/trace
  for ctr in FETCH_SIZE WRITE_SIZE; do
    GNPDE_LIB=$L GNPDE_XCD_REMAP=$v timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $D/lap_$ctr -o run -- \
      python3 $R/tools/pmc_run.py lap > $D/lap.json 2> $D/lap_$ctr.err || { echo "pmc $v $ctr failed"; tail -5 $D/lap_$ctr.err; exit 1; }
    c=$(find $D/lap_$ctr -name 'run_counter_collection.csv' | head -1)
    [ -n "$c" ] && [ "$c" != "$D/lap_$ctr/run_counter_collection.csv" ] && cp "$c" $D/lap_$ctr/run_counter_collection.csv
  done
  (cd $R && GNPDE_LIB=$L python3 tools/pmc_reduce.py xcd$v $D $D/traffic.json > $D/reduce.log 2>&1)
  python3 - "$v" "$D" >> $OUT/xcd_ab.jsonl <<'PY'
import csv, json, sys
v, d = sys.argv[1], sys.argv[2]
name = "agg_kernel<4, 32, 1, 4, 2, 1, gnpde::PlainWeights, float>"
us = None
for r in csv.DictReader(open(d + "/kernel_stats.csv")):
    if name in r["Name"]:
        us = float(r["AverageNs"]) / 1e3
t = json.load(open(d + "/traffic.json"))["workloads"]["lap"]["kernels"]
b = [k["bytes"] for k in t if name in k["kernel"]]
print(json.dumps({"xcd_remap": int(v), "k1_stage_us": us, "k1_stage_counter_bytes": b[0] if b else None,
                  "compulsory_bytes": 270388224, "refetch": round(b[0] / 270388224, 3) if b else None}))
PY
  tail -1 $OUT/xcd_ab.jsonl
done
