#!/usr/bin/env python
"""One rank per GPU under torch.distributed.run (RCCL): a dopri5 solve of the
G-arxiv Laplacian in feature-column stripes (gnpde.dist.ColumnShardedLaplacian,
the global error norm as one all-reduce per step, columns all-gathered at the
end) against the unsharded solve of the same ODE on this rank's GPU.  Prints one
JSON line: world size, accepted+rejected steps of both, max relative difference."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    import gnpde
    from gnpde import dist as gd, synthetic
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    alpha = torch.zeros((), device=dev)
    t = torch.tensor([0.0, 2.0], device=dev)
    tol = dict(rtol=1e-5, atol=1e-7)
    with torch.no_grad():
        opt = {'block': 'constant', 'function': 'laplacian', 'add_source': False, 'no_alpha_sigmoid': False,
               'max_nfe': 10 ** 9, 'multi_modal': False, 'hidden_dim': C}
        func = gnpde.LaplacianODEFunc(C, C, opt, dev).to(dev)
        func.edge_index, func.edge_weight = ei, w
        gnpde.odeint(func, x, t, method='dopri5', **tol)  # warm-up: CSR, plans, step graphs
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        y1 = gnpde.odeint(func, x, t, method='dopri5', **tol)[1]
        torch.cuda.synchronize()
        el1 = time.perf_counter() - t0
        n1 = gnpde.integrator.odeint.last_n_steps
        sh = gd.ColumnShardedLaplacian(ei, w, N, C, alpha)
        xl = sh.split(x)
        gnpde.odeint(sh, xl, t, method='dopri5', options={'norm': sh.global_rms_norm}, **tol)  # warm-up
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        yl = gnpde.odeint(sh, xl, t, method='dopri5', options={'norm': sh.global_rms_norm}, **tol)[1]
        full = sh.gather(yl)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        n = gnpde.integrator.odeint.last_n_steps
    rel = float((full - y1).abs().max() / y1.abs().max())
    if dist.get_rank() == 0:
        print(json.dumps({"check": "dopri5 column-striped solve (global_rms_norm all-reduce) vs unsharded",
                          "world": dist.get_world_size(), "backend": dist.get_backend(), "graph": "G-arxiv",
                          "steps_sharded": n, "steps_unsharded": n1, "max_rel_diff": rel,
                          "ms_sharded": round(el * 1e3, 3), "ms_unsharded": round(el1 * 1e3, 3),
                          "columns_per_rank": sh.c1 - sh.c0, "ok": bool(n == n1 and rel < 1e-5)}))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
