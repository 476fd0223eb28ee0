#!/usr/bin/env python
"""Print the kernel sequence (duration, gap) after the first kernel matching a
pattern in a rocprofv3 kernel_trace.csv: tools/trace_seq.py <csv> <pattern> [count] [skip]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
pat, cnt = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 10
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
hits = [i for i, r in enumerate(rows) if pat in r['Kernel_Name']]
i0 = hits[min(skip, len(hits) - 1)]
prev = None
tot = 0
for r in rows[i0:i0 + cnt]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    name = r['Kernel_Name'].replace('gnpde::', '').replace('HIP_vector_type<int, 4u>', 'int4')
    print("%-70s %8.2f us  gap %6s" % (name[:70], (e - s) / 1e3, "%.2f" % ((s - prev) / 1e3) if prev else '-'))
    tot += e - s
    prev = e
print("sum of durations: %.2f us" % (tot / 1e3))
