#!/bin/bash
# A/B of the attention RHS over the product library and variants/libgnpde_*.so
# (make -C graph-neural-pde_amd variant VNAME=... VFLAGS=...; VDIR= another directory of them):
#   MODES=per_edge:0 TAG=r04d bash tools/ab_attn.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 200 python3 $R/tools/attn_ab.py --tag product --modes ${MODES:-per_edge:0} >> $OUT/ab.jsonl 2>>$OUT/ab.err || exit 1
for lib in $R/${VDIR:-variants}/libgnpde_*.so; do
  [ -e "$lib" ] || continue
  v=$(basename $lib .so)
  GNPDE_LIB=$lib timeout -k 10 200 python3 $R/tools/attn_ab.py --tag ${v#libgnpde_} --modes ${MODES:-per_edge:0} \
    >> $OUT/ab.jsonl 2>>$OUT/ab.err || exit 1
done
cat $OUT/ab.jsonl
