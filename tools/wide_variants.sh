set -u
mkdir -p gpurun_out
for v in 3 4 2; do
  GNPDE_AGG_VARIANT=$v timeout -k 10 400 python tools/stripe_bench.py > gpurun_out/wide_v$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/wide_v$v.log | grep -E '"world": (1|2),' | sed "s/^/v$v /"
done
