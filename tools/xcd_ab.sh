set -u
for r in 0 8 32 128; do
  GNPDE_XCD_REMAP=$r REORDER=deg,rcm,bfs timeout -k 10 300 python tools/reorder_bench.py | sed "s/^/xcd=$r /" || exit 1
done
