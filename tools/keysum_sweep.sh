#!/bin/bash
# Kernel times of the reference-mode key-sum chain for several tile counts
# (GNPDE_KEYSUM_TILES), from rocprofv3 kernel traces of tools/attn_ref_bench.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
cd /tmp && export TMPDIR=/tmp
for t in ${TILES:-256 512 1024}; do
  GNPDE_KEYSUM_TILES=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_$t -o run -- \
    python3 $R/tools/attn_ref_bench.py > $OUT/ks_$t.log 2>&1; rc=$?
  echo "tiles $t rc=$rc"; if fatal $rc; then exit $rc; fi
  python3 - "$OUT/ks_$t" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("keysum", "key_proj", "node_scores", "seg_softmax", "stats_fixup", "RefDst")):
        print("   %-60s %8.2f us" % (n.split("(")[0][-60:], float(r["AverageNs"]) / 1e3))
PY
done
