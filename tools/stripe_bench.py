#!/usr/bin/env python
"""Per-rank work of the column-striped layout (gnpde.dist.ColumnShardedLaplacian)
measured on ONE GPU: rk4 steps of the full graph at the stripe widths C/N of
N = 1, 2, 4, 8 ranks (the stripes need no communication, so a rank's step time
is this).  Prints one JSON line per (graph, width): ms per rk4 step and the
implied strong-scaling speed-up t(C) / t(C/N)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

import gnpde  # noqa: E402
from gnpde import integrator as integ, synthetic  # noqa: E402

OPT = {'block': 'constant', 'function': 'laplacian', 'add_source': False, 'no_alpha_sigmoid': False,
       'max_nfe': 10 ** 9, 'multi_modal': False}


def step_ms(func, x, steps, h=0.25):
    dev = x.device

    def run(n):
        t = torch.tensor([0.0, n * h], device=dev)
        return gnpde.odeint(func, x, t, method='rk4', options={'step_size': h})[1]
    with torch.no_grad():
        run(max(integ.GRAPH_MIN_STEPS, 2 * integ.GRAPH_BLOCK))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(steps)
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def main():
    dev = torch.device("cuda", 0)
    graphs = [("G-arxiv", synthetic.ARXIV_N, synthetic.ARXIV_E, 128, 50)]
    if os.environ.get("STRIPE_RMAT", "1") == "1":
        graphs.append(("G-rmat", 2_000_000, 20_000_000, 256, 10))
    for name, N, E, C, steps in graphs:
        ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
        base = None
        for world in (1, 2, 4, 8):
            c = C // world
            x = synthetic.features(1, N, c, seed=1, device=dev)
            func = gnpde.LaplacianODEFunc(c, c, dict(OPT, hidden_dim=c), dev).to(dev)
            func.edge_index, func.edge_weight = ei, w
            ms = step_ms(func, x, steps)
            base = ms if base is None else base
            print(json.dumps({"graph": name, "world": world, "cols_per_rank": c, "ms_per_step": round(ms, 4),
                              "implied_speedup": round(base / ms, 3),
                              "variant": os.environ.get("GNPDE_AGG_VARIANT", "0")}), flush=True)
            del func, x
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
