set -u
for c in 256 128 192 384 512; do
  GNPDE_CHUNK=$c K1_C=168 timeout -k 10 300 python tools/bf16_k1_bench.py | sed "s/^/chunk=$c /" || exit 1
done
for o in classes lpt; do
  GNPDE_PLAN_ORDER=$o K1_C=168 timeout -k 10 300 python tools/bf16_k1_bench.py | sed "s/^/order=$o /" || exit 1
done
