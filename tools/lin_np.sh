set -u
for w in 2048 6000 12000; do
  GNPDE_LIN_WAVES=$w timeout -k 10 120 python tools/linear_bench.py || exit 1
done
