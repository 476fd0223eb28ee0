#!/usr/bin/env python
"""Print a rocprofv3 kernel_stats.csv compactly: tools/kstats.py <csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:n]:
    name = r['Name'].replace('HIP_vector_type<int, 4u>', 'int4').replace('gnpde::', '')
    print("%-80s %6s %10.1f %9.2f %6.2f" % (name[:80], r['Calls'], float(r['TotalDurationNs']) / 1e3,
                                          float(r['AverageNs']) / 1e3, float(r['Percentage'])))
