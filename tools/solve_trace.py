#!/usr/bin/env python
"""The bench's headline solve (G-arxiv rk4, 20 steps, replayed block graphs)
between two markers (gnpde_dot_f64: dot_final_kernel) for a kernel timeline of
one timed solve (tools/timeline.py, tools/train_prof.sh's pattern)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    import gnpde
    from gnpde import ops, synthetic
    dev = torch.device("cuda", 0)
    C = 128
    ei, w = synthetic.rw_graph(synthetic.ARXIV_N, synthetic.ARXIV_E, seed=0, device=dev)
    x = synthetic.features(1, synthetic.ARXIV_N, C, seed=1, device=dev)
    func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    mk = torch.ones(64, device=dev)
    with torch.no_grad():
        bench.rk4_solve(func, x, 5, 0.25, dev)
        for _ in range(3):
            bench.rk4_solve(func, x, 20, 0.25, dev)
        torch.cuda.synchronize()
        ops.dot(mk, mk)
        bench.rk4_solve(func, x, 20, 0.25, dev)
        ops.dot(mk, mk)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
