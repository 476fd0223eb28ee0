#!/usr/bin/env python
"""Host-side cost of the headline solve (bench.rk4_solve, G-arxiv, 20 rk4 steps,
replayed block graphs): cProfile over 50 solves, top functions by own time."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    import gnpde
    from gnpde import synthetic
    dev = torch.device("cuda", 0)
    C = 128
    ei, w = synthetic.rw_graph(synthetic.ARXIV_N, synthetic.ARXIV_E, seed=0, device=dev)
    x = synthetic.features(1, synthetic.ARXIV_N, C, seed=1, device=dev)
    func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    with torch.no_grad():
        for _ in range(4):
            bench.rk4_solve(func, x, 20, 0.25, dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            bench.rk4_solve(func, x, 20, 0.25, dev)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print("host issue per solve %.1f us; with GPU %.1f us" % ((t1 - t0) / 50 * 1e6, (t2 - t0) / 50 * 1e6))
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(50):
            bench.rk4_solve(func, x, 20, 0.25, dev)
        pr.disable()
        torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
