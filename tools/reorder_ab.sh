set -u
ORDER_ONLY=1 timeout -k 10 300 python tools/reorder_bench.py || exit 1
GNPDE_PLAN_ORDER=rows timeout -k 10 300 python tools/reorder_bench.py || exit 1
K1_C=162 REORDER=none,rand,deg,rcm timeout -k 10 300 python tools/reorder_bench.py
