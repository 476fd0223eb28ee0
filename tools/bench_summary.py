#!/usr/bin/env python
"""Summary of a bench line and (optionally) the rocprofv3 kernel stats of the same
session: python tools/bench_summary.py gpurun_out/<tag>"""
import csv
import json
import os
import sys

d = sys.argv[1]
line = [x for x in open(os.path.join(d, "bench.log")) if x.startswith("{")][-1]
b = json.loads(line)
print("value %.1f RHS/s  ms/step %.4f  rhs_ms %.4f  overhead %.4f  frac %s" % (
    b["value"], b["ms_per_step"], b["rhs_ms"], b.get("solve_overhead_ms", 0), b["roofline"].get("frac")))
if b.get("rhs_plain"):
    print("plain rhs_ms", b["rhs_plain"]["rhs_ms"])
for k, v in (b.get("attention") or {}).items():
    if isinstance(v, dict):
        print("attention %-16s rhs_ms %.4f eager %.4f frac %s" % (k, v["rhs_ms"], v["rhs_ms_eager"], v.get("frac")))
bl = b.get("blend_c162")
if bl:
    print("blend fp32 %.4f bf16 %.4f ms/step" % (bl["fp32"]["ms_per_step"], bl["bf16"]["ms_per_step"]))
for k in ("block_forward", "train_rk4"):
    if b.get(k):
        print(k, {kk: vv for kk, vv in b[k].items() if kk != "config"})
g = (b.get("grmat") or {}).get("one_gpu")
if g:
    print("grmat %.1f RHS/s %.3f ms/step" % (g["value"], g["ms_per_step"]))
st = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(st):
    rows = list(csv.DictReader(open(st)))
    for r in rows[:int(os.environ.get("TOP", 30))]:
        print("%-110s %6s %9.1f us" % (r["Name"][:110], r["Calls"], float(r["AverageNs"]) / 1000))
