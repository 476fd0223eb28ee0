#!/bin/bash
# K1 with and without the XCD-contiguous workgroup remap (GNPDE_XCD_REMAP).
for r in 0 1; do GNPDE_XCD_REMAP=$r timeout -k 10 200 python tools/k1_stage_bench.py | sed "s/^/remap $r /" || exit 1; done
