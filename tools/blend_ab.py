#!/usr/bin/env python
"""The bench's BLEND lines (configs[3] shape, C = 162, fp32 and bf16 rk4 steps on
G-arxiv) for the library GNPDE_LIB points at (A/B of variant builds): one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    import gnpde
    from gnpde import _lib, synthetic
    dev = torch.device("cuda", 0)
    N, E = synthetic.ARXIV_N, synthetic.ARXIV_E
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, 128, seed=1, device=dev)
    func = gnpde.LaplacianODEFunc(128, 128, dict(bench.LAP_OPT, hidden_dim=128), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    with torch.no_grad():
        g = func.graph_for(x)
    r = bench.bench_blend(g, dev)
    out = {"lib": os.path.basename(os.environ.get("GNPDE_LIB", _lib.LIB_PATH)),
           "fp32": r["fp32"]["ms_per_step"], "bf16": r["bf16"]["ms_per_step"], "ok": r["check"]["ok"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
