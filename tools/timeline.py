#!/usr/bin/env python
"""Kernel timeline of a rocprofv3 kernel trace: the window between the last two
marker kernels (dot_final_kernel) when there are two, else the last `span` ms
before the final kernel; kernels in start order with the idle gap before each.
python tools/timeline.py <run_kernel_trace.csv> [span_ms]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
span = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# a marker pair (dot_final_kernel, tools/train_trace.py): the window between the last two
mk = [i for i, e in enumerate(ev) if "dot_final_kernel" in e[2]]
if len(mk) >= 2:
    ev = ev[mk[-2]:mk[-1] + 1]
else:
    t_end = ev[-1][1]
    ev = [e for e in ev if e[0] >= t_end - span * 1e6]
prev = ev[0][0]
busy = 0
for s, e, n in ev:
    gap = max(0, s - prev)
    print("%8.1f gap %6.1f dur %7.1f  %s" % ((s - ev[0][0]) / 1e3, gap / 1e3, (e - s) / 1e3, n[:100]))
    busy += e - s
    prev = max(prev, e)
print("window %.1f us, busy %.1f us" % ((prev - ev[0][0]) / 1e3, busy / 1e3))
