#!/usr/bin/env python
"""One timed G-arxiv dopri5 solve (ogbn-arxiv best_params T / tol_scale, the bench's
dopri5 line) between two marker kernels (gnpde_dot_f64: dot_final_kernel), for a
kernel timeline of the solve under rocprofv3 --kernel-trace (tools/timeline.py).
  python tools/dopri5_trace.py [--first-step H]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--first-step", type=float, default=None)
    a = p.parse_args()
    import bench
    import gnpde
    from gnpde import ops, synthetic
    dev = torch.device("cuda", 0)
    C = 128
    ei, w = synthetic.rw_graph(synthetic.ARXIV_N, synthetic.ARXIV_E, seed=0, device=dev)
    x = synthetic.features(1, synthetic.ARXIV_N, C, seed=1, device=dev)
    func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    T, ts = bench.ARXIV_DOPRI5
    t = torch.tensor([0.0, T], dtype=torch.float32, device=dev)
    kw = dict(method='dopri5', rtol=1e-9 * ts, atol=1e-7 * ts)
    if a.first_step:
        kw['options'] = {'first_step': a.first_step}
    mk = torch.ones(64, device=dev)
    with torch.no_grad():
        for _ in range(3):
            gnpde.odeint(func, x, t, **kw)
        torch.cuda.synchronize()
        ops.dot(mk, mk)
        gnpde.odeint(func, x, t, **kw)
        ops.dot(mk, mk)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
