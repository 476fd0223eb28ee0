set -u
for v in 0 2 3 4; do
  GNPDE_AGG_VARIANT=$v REORDER=deg timeout -k 10 300 python tools/reorder_bench.py | sed "s/^/variant=$v /" || exit 1
done
for c in 192 256 320; do
  GNPDE_CHUNK=$c REORDER=deg timeout -k 10 300 python tools/reorder_bench.py | sed "s/^/chunk=$c /" || exit 1
done
