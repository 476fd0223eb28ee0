set -u
for i in 1 2; do for v in 0 10 11; do
  GNPDE_AGG_VARIANT=$v K1_C=168 timeout -k 10 300 python tools/bf16_k1_bench.py || exit 1
done; done
