#!/bin/bash
# Kernel times of the reference-mode attention chain under several knob settings,
# from rocprofv3 kernel traces of tools/attn_ref_bench.py.
#   ENVS="GNPDE_KEYSUM_TILES=256 GNPDE_KEYSUM_BLOCK=512,GNPDE_KEYSUM_TILES=512" tools/keysum_sweep.sh
# (one run per space-separated entry; commas join several variables; TILES="a b" is
# shorthand for GNPDE_KEYSUM_TILES=a GNPDE_KEYSUM_TILES=b)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
ENVS=${ENVS:-}
for t in ${TILES:-}; do ENVS="$ENVS GNPDE_KEYSUM_TILES=$t"; done
cd /tmp && export TMPDIR=/tmp
i=0
for e in ${ENVS:-base}; do
  i=$((i + 1))
  if [ "$e" = base ]; then envs=(); else envs=(env ${e//,/ }); fi
  "${envs[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ks_$i -o run -- \
    python3 $R/tools/attn_ref_bench.py > $OUT/ks_$i.log 2>&1; rc=$?
  echo "[$e] rc=$rc"; if fatal $rc; then exit $rc; fi
  python3 - "$OUT/ks_$i" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("keysum", "key_proj", "node_scores", "seg_softmax", "stats_fixup", "RefDst")):
        print("   %-60s %8.2f us" % (n.split("(")[0][-60:], float(r["AverageNs"]) / 1e3))
PY
done
