#!/usr/bin/env python
"""Per-kernel HBM roofline from one profile session (tools/prof_r02.sh):

  tools/roofline_table.py TAG [--k1-json profiles/k1_traffic.json]

Reads gpurun_out/prof_TAG_trace/run_kernel_trace.csv (durations, no counters)
and the two PMC passes gpurun_out/prof_TAG_pmc_{FETCH,WRITE}_SIZE; groups
launches by (kernel, grid size) — one instantiation serves several workloads —
and writes profiles/TAG_roofline.json + a markdown table on stdout:
traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes; MI355X_MICROARCH.md §HBM:
FETCH_SIZE counts half the bytes of 16-B-per-lane reads, WRITE_SIZE is exact
for 16-B stores; both count Infinity-Cache hits), rate = traffic / mean
duration, frac = rate / 8 TB/s.  With --k1-json also refreshes the K1
per-launch traffic bench.py reads (G-arxiv, C = 128)."""
import collections
import csv
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8000.0


def short(name):
    m = re.match(r"(?:void )?(?:gnpde::)?([\w:]+)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    tag = sys.argv[1]
    out_dir = os.path.join(ROOT, "gpurun_out")
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(out_dir, "prof_%s_trace" % tag, "run_kernel_trace.csv"))):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
        dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(out_dir, "prof_%s_pmc_%s" % (tag, c), "run_counter_collection.csv")
        for r in csv.DictReader(open(p)):
            ctr[(short(r["Kernel_Name"]), int(r["Grid_Size"]))][c].append(float(r["Counter_Value"]) * 1024)
    table = []
    for key in sorted(ctr, key=lambda k: -statistics.mean(dur.get(k, [0]))):
        f, w = ctr[key].get("FETCH_SIZE"), ctr[key].get("WRITE_SIZE")
        if not f or not w or key not in dur:
            continue
        us = statistics.mean(dur[key])
        traffic = 2 * statistics.mean(f) + statistics.mean(w)
        rate = traffic / (us * 1e-6) / 1e9
        table.append({"kernel": key[0], "grid": key[1], "launches_traced": len(dur[key]), "mean_us": round(us, 2),
                      "fetch_bytes_x2": round(2 * statistics.mean(f)), "write_bytes": round(statistics.mean(w)),
                      "traffic_bytes": round(traffic), "GBs": round(rate, 1), "frac": round(rate / PEAK, 4)})
    js = {"tag": tag, "method": "traffic = 2*FETCH_SIZE + WRITE_SIZE per launch (KiB->bytes), mean duration from the "
                                "kernel trace of the same bench command, frac = traffic/duration/8 TB/s",
          "kernels": table}
    with open(os.path.join(ROOT, "profiles", "%s_roofline.json" % tag), "w") as fh:
        json.dump(js, fh, indent=1)
    print("| kernel | grid | launches | mean µs | traffic MB | GB/s | frac |")
    print("|---|---|---|---|---|---|---|")
    for t in table:
        print("| %s | %d | %d | %.1f | %.1f | %.0f | %.3f |" % (t["kernel"], t["grid"], t["launches_traced"], t["mean_us"],
                                                               t["traffic_bytes"] / 1e6, t["GBs"], t["frac"]))
    if "--k1-json" in sys.argv:
        path = sys.argv[sys.argv.index("--k1-json") + 1]
        k1 = {"nodes": 169343, "edges": 1200000, "dim": 128, "tag": tag,
              "method": "2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes), per launch"}
        for t in table:
            if t["kernel"] == "agg_kernel<4, 32, 1, 4, 2, 1, gnpde::PlainWeights, float>":
                k1["fused_step_launch"] = {"kernel": t["kernel"], "grid": t["grid"], "hbm_bytes": t["traffic_bytes"],
                                           "mean_us": t["mean_us"]}
            if t["kernel"] == "agg_kernel<4, 32, 1, 4, 2, 0, gnpde::PlainWeights, float>":
                k1["plain_launch"] = {"kernel": t["kernel"], "grid": t["grid"], "hbm_bytes": t["traffic_bytes"],
                                      "mean_us": t["mean_us"]}
        with open(path, "w") as fh:
            json.dump(k1, fh, indent=1)


if __name__ == "__main__":
    main()
