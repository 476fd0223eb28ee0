#!/usr/bin/env python
"""Locality experiment: the G-arxiv K1 (plain RHS and fused rk4 step) on the same
graph under different node numberings (an isomorphic relabelling; the work is
identical, only which gathered rows sit close in time changes).
REORDER = none | rand | rcm | deg (in-degree descending) | bfs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from scipy.sparse.csgraph import reverse_cuthill_mckee, breadth_first_order  # noqa: E402
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


def numbering(kind, ei, N):
    src, dst = ei[0, 0].cpu().numpy(), ei[0, 1].cpu().numpy()
    if kind == "rand":
        return np.random.default_rng(5).permutation(N)
    A = sp.coo_matrix((np.ones(src.shape[0], np.int8), (src, dst)), shape=(N, N)).tocsr()
    S = (A + A.T).tocsr()
    if kind == "rcm":
        order = reverse_cuthill_mckee(S, symmetric_mode=True)
    elif kind == "deg":
        order = np.argsort(-np.bincount(dst, minlength=N), kind="stable")
    elif kind == "bfs":
        order, _ = breadth_first_order(S, int(np.argmax(np.bincount(dst, minlength=N))), directed=False)
        rest = np.setdiff1d(np.arange(N), order)
        order = np.concatenate([order, rest])
    else:
        return np.arange(N)
    new_id = np.empty(N, np.int64)
    new_id[order] = np.arange(N)
    return new_id


def main():
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, int(os.environ.get("K1_C", 128))
    dev = torch.device("cuda", 0)
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, device=dev)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9,
           'multi_modal': False}
    for kind in os.environ.get("REORDER", "none,rand,deg,rcm,bfs").split(","):
        new_id = torch.from_numpy(numbering(kind, ei, N)).to(dev)
        order_only = os.environ.get("ORDER_ONLY", "0") == "1"
        eik = ei if order_only else new_id[ei]
        func = gnpde.LaplacianODEFunc(C, C, opt, dev).to(dev)
        func.edge_index, func.edge_weight = eik, w
        with torch.no_grad():
            g = func.graph_for(x)
            if order_only:
                # same numbering, K1 items re-sorted: length class, then the rank of the row
                pl = g.csr.plan
                it = pl.items[:pl.n_items * 4].view(-1, 4)
                ln = (it[:, 2] - it[:, 1]).long().clamp(min=1)
                cls = -torch.floor(torch.log2(ln.double())).long()
                key = cls * (N + 1) + new_id[it[:, 0].long()]
                it.copy_(it[torch.argsort(key, stable=True)])
            wc = func.csr_weights(g, w, 'w')
            alpha = func.alpha_train.detach()
            out = torch.empty_like(x)
            t_rhs = timeit(lambda: ops.spmm_rhs(g, wc, x, alpha=alpha, out=out.view(-1, C)), 50)
            ws = gi._Workspace()
            t_step = timeit(lambda: gi._fused_step('rk4', func, 0.0, 0.25, 0.25, x, ws), 20)
        print(json.dumps({"reorder": kind, "order_only": order_only, "C": C, "rhs_us": round(t_rhs, 2), "rk4_fused_us": round(t_step, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
