set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/train_prof -o run -- python3 $R/tools/train_bench.py > $R/gpurun_out/train_prof.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' $R/gpurun_out/train_prof.log
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("/root/repo/gpurun_out/train_prof/run_kernel_stats.csv")))
for r in rows[:22]:
    print(r["Name"][:100], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), r["Percentage"][:5])
PY
