#!/usr/bin/env python
"""Per-launch HBM traffic of the K1 kernels from rocprofv3 PMC passes.

  tools/traffic.py <FETCH_SIZE counter_collection.csv> <WRITE_SIZE csv> N E C [out.json]

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the
bytes of a wide coalesced (16 B/lane) read -> x2; WRITE_SIZE is exact for
16-B stores.  Both counters are in KiB.  Launches are grouped by kernel symbol;
the stage (true) and plain (false) K1 instantiations are reported separately.
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return acc


def main():
    fetch, write = per_kernel(sys.argv[1]), per_kernel(sys.argv[2])
    N, E, C = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    out = {"nodes": N, "edges": E, "dim": C, "method": "2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes)"}
    for name, fv in fetch.items():
        if "agg_kernel" not in name:
            continue
        wv = write.get(name, [0.0])
        tag = "fused_step_launch" if (", true," in name or ", 1, gnpde::PlainWeights" in name) else "plain_launch"
        f = sum(fv) / len(fv) * 1024
        w = sum(wv) / len(wv) * 1024
        out[tag] = {"kernel": name.split("(")[0], "fetch_bytes_raw": f, "write_bytes": w, "hbm_bytes": 2 * f + w,
                    "launches": len(fv)}
    js = json.dumps(out, indent=1)
    print(js)
    if len(sys.argv) > 6:
        open(sys.argv[6], "w").write(js + "\n")


if __name__ == "__main__":
    main()
