#!/usr/bin/env python
"""Kernel timeline of a rocprofv3 kernel trace: the window between the last two
marker kernels (dot_final_kernel) when there are two, else the last `span` ms
before the final kernel; kernels in start order with the idle gap before each.
python tools/timeline.py <run_kernel_trace.csv> [span_ms] [--summary]
--summary: per kernel name in the window, calls / total / average duration."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
args = [a for a in sys.argv[2:] if not a.startswith("--")]
span = float(args[0]) if args else 5.0
summary = "--summary" in sys.argv
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# a marker pair (dot_final_kernel, tools/train_trace.py): the window between the last two
mk = [i for i, e in enumerate(ev) if "dot_final_kernel" in e[2]]
if len(mk) >= 2:
    ev = ev[mk[-2]:mk[-1] + 1]
else:
    t_end = ev[-1][1]
    ev = [e for e in ev if e[0] >= t_end - span * 1e6]
if summary:
    agg = {}
    for s, e, n in ev:
        a = agg.setdefault(n[:110], [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    for n, (c, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print("%9.1f us %5d x %8.2f  %s" % (tot, c, tot / c, n))
prev = ev[0][0]
busy = 0
for s, e, n in (ev if not summary else []):
    gap = max(0, s - prev)
    print("%8.1f gap %6.1f dur %7.1f  %s" % ((s - ev[0][0]) / 1e3, gap / 1e3, (e - s) / 1e3, n[:100]))
    busy += e - s
    prev = max(prev, e)
if summary:
    busy = sum(e - s for s, e, _ in ev)
    prev = max(e for _, e, _ in ev)
print("window %.1f us, busy %.1f us" % ((prev - ev[0][0]) / 1e3, busy / 1e3))
