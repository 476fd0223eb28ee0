#!/usr/bin/env python
"""A/B timing of the transformer RHS (bench.bench_attention's workloads): one JSON
line per (mode, norm) with the graph-replayed RHS time in the solve's numbering
and in the user numbering.  Run once per library (GNPDE_LIB=... for a variant):

  tools/attn_ab.py [--tag NAME] [--modes reference:1,per_edge:0,per_edge:1] [--reps 50]

(--modes defaults to $ATT_MODES when set: tools/variants_ab.sh, tools/lin_check.sh.)
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--tag", default=os.environ.get("GNPDE_LIB", "product"))
    p.add_argument("--modes", default=os.environ.get("ATT_MODES", "reference:1,per_edge:0,per_edge:1"))
    p.add_argument("--reps", type=int, default=50)
    a = p.parse_args()
    from gnpde import synthetic
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ei, _ = synthetic.rw_graph(169343, 1200000, seed=0, device=dev)
    x = synthetic.features(1, 169343, 128, seed=1, device=dev)
    for mn in a.modes.split(","):
        mode, norm = mn.split(":")
        func = bench.attention_func(mode, int(norm), 128, dev)
        func.edge_index = ei
        func.graph_for(x)
        xs, lay = bench.solve_numbering(func, x)
        best = {}
        for name, (xx, ll) in (("layout", (xs, lay)), ("user", (x, None))):
            ts = [bench._time_rhs(func, xx, ll, a.reps)[1] for _ in range(3)]
            best[name] = round(min(ts), 4)
        print(json.dumps({"tag": a.tag, "mode": mode, "norm": int(norm), "rhs_ms": best}), flush=True)


if __name__ == "__main__":
    main()
