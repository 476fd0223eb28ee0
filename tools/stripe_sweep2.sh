#!/bin/bash
# Plan order x narrow geometry for the column stripes (G-arxiv, and G-rmat at 8 ranks).
set -u
mkdir -p gpurun_out
OUT=gpurun_out/stripe_sweep2.log; : > $OUT
for cfg in "0 lpt" "0 classes" "0 hubs" "6 classes" "8 classes" "6 hubs"; do
  set -- $cfg
  GNPDE_AGG_VARIANT=$1 GNPDE_PLAN_ORDER=$2 STRIPE_RMAT=${RMAT:-0} timeout -k 10 250 python3 tools/stripe_bench.py > /tmp/s.log 2>&1
  rc=$?; echo "cfg $cfg rc=$rc"
  grep '^{' /tmp/s.log | sed "s/^/{\"cfg\": \"$cfg\", \"r\": /; s/$/}/" >> $OUT
  case $rc in 124|134|137|139) exit $rc;; esac
done
cat $OUT
