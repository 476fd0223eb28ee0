#!/usr/bin/env python
"""One timed G-arxiv dopri5 solve (ogbn-arxiv best_params T / tol_scale, the bench's
dopri5 line) between two marker kernels (gnpde_dot_f64: dot_final_kernel), for a
kernel timeline of the solve under rocprofv3 --kernel-trace (tools/timeline.py).
  python tools/dopri5_trace.py [--first-step H] [--c2]"""
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
    p.add_argument("--c2", action="store_true", help="configs[1]'s transformer solve (tools/dopri5_prof.py)")
    a = p.parse_args()
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import dopri5_prof
    import gnpde
    from gnpde import ops
    func, x, t, kw = dopri5_prof.problem(a.c2)
    dev = x.device
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
