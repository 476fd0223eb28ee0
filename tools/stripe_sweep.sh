#!/bin/bash
# Narrow-row K1 sweep (column stripes of G-arxiv): geometry variants x chunk x plan order.
set -u
mkdir -p gpurun_out
OUT=gpurun_out/stripe_sweep.log; : > $OUT
for cfg in "0 256 lpt" "0 256 rows" "0 128 lpt" "0 64 lpt" "0 64 rows" "6 256 lpt" "7 256 lpt" "8 256 lpt" "7 128 rows" "6 64 rows"; do
  set -- $cfg
  GNPDE_AGG_VARIANT=$1 GNPDE_CHUNK=$2 GNPDE_PLAN_ORDER=$3 STRIPE_RMAT=0 timeout -k 10 200 python3 tools/stripe_bench.py > /tmp/s.log 2>&1
  rc=$?; echo "cfg $cfg rc=$rc"
  grep '^{' /tmp/s.log | sed "s/^/{\"cfg\": \"$cfg\", \"r\": /; s/$/}/" >> $OUT
  case $rc in 124|134|137|139) exit $rc;; esac
done
cat $OUT
