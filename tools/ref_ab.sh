#!/bin/bash
# Reference-attention pieces per variant library: tools/stats_probe.py (item
# classes of the CSC statistics) and tools/attn_ref_bench.py (every piece and the
# whole RHS), once per variants/libgnpde_*.so.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-refab}
mkdir -p $OUT
cd $R
for lib in variants/libgnpde_*.so; do
  for sc in tools/stats_probe.py tools/attn_ref_bench.py; do
    echo "{\"lib\": \"$lib\", \"script\": \"$sc\"}" >> $OUT/ab.jsonl
    GNPDE_LIB=$R/$lib timeout -k 10 180 python3 $sc >> $OUT/ab.jsonl 2> $OUT/ab.err; rc=$?
    [ $rc = 0 ] || { echo "$lib $sc rc=$rc"; tail -5 $OUT/ab.err; exit $rc; }
  done
done
cat $OUT/ab.jsonl
