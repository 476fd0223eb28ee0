#!/bin/bash
# A/B of variant libraries (variants/libgnpde_*.so, make -C graph-neural-pde_amd variant ...):
# tools/attn_ab.py (or $AB_SCRIPT) once per library, ROUNDS times in alternation.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p $OUT
cd $R
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${VDIR:-variants}/libgnpde_*.so; do
    if [ "${PROF:-0}" = 1 ] && [ $r = 1 ]; then
      n=$(basename $lib .so)
      (cd /tmp && export TMPDIR=/tmp && GNPDE_LIB=$R/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats \
        --output-format csv -d $OUT/prof_$n -o run -- python3 $R/${AB_SCRIPT:-tools/attn_ab.py} >> $OUT/ab.jsonl \
        2> $OUT/ab.err); rc=$?
    else
      GNPDE_LIB=$R/$lib timeout -k 10 180 python3 ${AB_SCRIPT:-tools/attn_ab.py} >> $OUT/ab.jsonl 2> $OUT/ab.err; rc=$?
    fi
    [ $rc = 0 ] || { echo "$lib rc=$rc"; tail -5 $OUT/ab.err; exit $rc; }
    tail -1 $OUT/ab.jsonl
  done
done
