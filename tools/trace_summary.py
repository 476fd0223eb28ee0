"""Summarise a rocprofv3 kernel trace (kernel_trace.csv): per kernel name the count,
total and mean duration (us), and the wall span of the traced kernels; optional
name filter.  python tools/trace_summary.py TRACE.csv [--top 25]"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    agg = defaultdict(lambda: [0, 0.0])
    t_min, t_max = None, None
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name") or r.get("KernelName")
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            a = agg[name]
            a[0] += 1
            a[1] += (e - s) / 1e3
            t_min = s if t_min is None else min(t_min, s)
            t_max = e if t_max is None else max(t_max, e)
    tot = sum(v[1] for v in agg.values())
    print("kernels %d, busy %.1f us, span %.1f us" % (sum(v[0] for v in agg.values()), tot, (t_max - t_min) / 1e3))
    for name, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print("%8.1f us %5d x %8.2f  %s" % (us, n, us / n, name[:150]))


if __name__ == "__main__":
    main()
