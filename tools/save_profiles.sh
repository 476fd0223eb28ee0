#!/bin/bash
# Copy one profile run's summaries from gpurun_out/ (scratch) into profiles/ (tracked).
# Usage: tools/save_profiles.sh TAG   (expects gpurun_out/prof_TAG_* and gpurun_out/bench.log)
set -eu
TAG=$1
cp gpurun_out/prof_${TAG}_trace/run_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  f=gpurun_out/prof_${TAG}_pmc_$c/run_counter_collection.csv
  [ -f $f ] && cp $f profiles/${TAG}_pmc_$c.csv
done
grep '^{"metric"' gpurun_out/bench.log | tail -1 > profiles/${TAG}_bench.json
ls -la profiles/ | grep $TAG
