#!/usr/bin/env python
"""Per-kernel HBM traffic of the tools/pmc_run.py workloads -> profiles/traffic.json.

  tools/pmc_reduce.py TAG DIR [OUT.json]   (default profiles/traffic.json)

DIR holds, per workload W (':' written as '_'), W.json (the runner's JSON line)
and the two rocprofv3 passes W_FETCH_SIZE/run_counter_collection.csv and
W_WRITE_SIZE/run_counter_collection.csv.  Traffic per dispatch = 2*FETCH_SIZE +
WRITE_SIZE (KiB -> bytes; MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the
bytes of 16-B-per-lane reads, WRITE_SIZE is exact for 16-B stores; both count
Infinity-Cache hits, so they bound HBM traffic from above).

Per workload: every kernel (name, grid) with its dispatch count and mean bytes
per dispatch; for attention workloads also the bytes of one RHS evaluation =
the bytes of every kernel dispatched after the workload's marker divided by
the evaluations.  bench.py reads
the result to turn its live launch / RHS times into counter-based fractions."""
import collections
import csv
import glob
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    m = re.match(r"(?:void )?(?:gnpde::)?([\w:]+)(<[^()]*>)?", name)
    s = (m.group(1) + (m.group(2) or "")) if m else name[:80]
    return s.replace("gnpde::", "").replace("HIP_vector_type<int, 4u>", "int4")


def counters(path):
    """(kernel, grid) -> bytes of every dispatch after the workload's marker (the
    last dot kernel, tools/pmc_run.py)."""
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "dot_final_kernel" in r["Kernel_Name"]]
    start = marks[-1] + 1 if marks else 0
    acc = collections.defaultdict(list)
    for r in rows[start:]:
        acc[(short(r["Kernel_Name"]), int(r["Grid_Size"]))].append(float(r["Counter_Value"]) * 1024)
    return acc


def main():
    tag, d = sys.argv[1], sys.argv[2]
    sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
    from gnpde import _lib
    out = {"tag": tag, "build_id": _lib.source_hash(),
           "method": "per dispatch 2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes), separate rocprofv3 --pmc passes of "
                     "tools/pmc_run.py WORKLOAD, dispatches after its marker; per_rhs_bytes = bytes of every "
                     "dispatch / evaluations", "workloads": {}}
    for mp in sorted(glob.glob(os.path.join(d, "*.json"))):
        w = os.path.basename(mp)[:-5]
        lines = [ln for ln in open(mp).read().splitlines() if ln.startswith("{")]
        if not lines:
            continue
        meta = json.loads(lines[-1])
        f = os.path.join(d, w + "_FETCH_SIZE", "run_counter_collection.csv")
        wr = os.path.join(d, w + "_WRITE_SIZE", "run_counter_collection.csv")
        if not (os.path.exists(f) and os.path.exists(wr)):
            continue
        fc, wc = counters(f), counters(wr)
        ks = []
        for key, fv in fc.items():
            wv = wc.get(key, [0.0])
            ks.append({"kernel": key[0], "grid": key[1], "count": len(fv), "fetch_bytes_x2": 2 * statistics.mean(fv),
                       "write_bytes": statistics.mean(wv), "bytes": 2 * statistics.mean(fv) + statistics.mean(wv)})
        ks.sort(key=lambda k: -k["bytes"] * k["count"])
        ent = {"meta": meta, "kernels": ks}
        if "rhs" in meta:
            n = meta["rhs"]
            ent["per_rhs_bytes"] = sum(k["bytes"] * k["count"] for k in ks) / n
            ent["per_rhs_kernels"] = ["%s x%g" % (k["kernel"], k["count"] / n) for k in ks]
        if "steps" in meta:
            n = meta["steps"]
            ent["per_step_bytes"] = sum(k["bytes"] * k["count"] for k in ks) / n
            ent["per_step_kernels"] = ["%s x%g" % (k["kernel"], k["count"] / n) for k in ks]
        out["workloads"][meta["workload"]] = ent
        print("%-24s" % meta["workload"], ", ".join("%s x%d %.1f MB" % (k["kernel"][:50], k["count"], k["bytes"] / 1e6)
                                                   for k in ks[:6]))
    path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "traffic.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
