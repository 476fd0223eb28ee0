#!/usr/bin/env python
"""Micro-benchmark of K1 (plain RHS and fused rk4 step) on G-arxiv; prints one
JSON line.  Used to compare lane-geometry variants (GNPDE_AGG_VARIANT)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

import gnpde  # noqa: E402
from gnpde import integrator as gi, ops, synthetic  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    N = int(os.environ.get("K1_N", synthetic.ARXIV_N))
    E = int(os.environ.get("K1_E", synthetic.ARXIV_E))
    C = int(os.environ.get("K1_C", 128))
    dev = torch.device("cuda", 0)
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, device=dev)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9,
           'multi_modal': False}
    func = gnpde.LaplacianODEFunc(C, C, opt, dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    with torch.no_grad():
        g = func.graph_for(x)
        wc = func.csr_weights(g, w, 'w')
        alpha = func.alpha_train.detach()
        out = torch.empty_like(x)
        t_rhs = timeit(lambda: ops.spmm_rhs(g, wc, x, alpha=alpha, out=out.view(-1, C)), 50)
        ws = gi._Workspace()
        t_step = timeit(lambda: gi._fused_step('rk4', func, 0.0, 0.25, 0.25, x, ws), 20)
        t_step_unfused = timeit(lambda: gi._fixed_step('rk4', func, 0.0, 0.25, 0.25, x, gi._Combine()), 10)
    print(json.dumps({"variant": int(os.environ.get("GNPDE_AGG_VARIANT", "0")),
                      "bpc": os.environ.get("GNPDE_AGG_BPC", "auto"), "N": N, "E": E, "C": C,
                      "rhs_us": round(t_rhs, 2), "rk4_fused_us": round(t_step, 1),
                      "rk4_unfused_us": round(t_step_unfused, 1),
                      "rhs_GBs": round((4 * E * C + 8 * N * C + 8 * E + 4 * (N + 1)) / t_rhs / 1e3, 1)}))


if __name__ == "__main__":
    main()
