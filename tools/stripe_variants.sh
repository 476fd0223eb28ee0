set -u
mkdir -p gpurun_out
for v in 6 7 8; do
  GNPDE_AGG_VARIANT=$v timeout -k 10 400 python tools/stripe_bench.py > gpurun_out/stripe_v$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/stripe_v$v.log | grep -v '"world": 1,' | sed "s/^/v$v /"
done
