#!/usr/bin/env python
"""bf16-storage K1 (plain RHS) on G-arxiv at C = K1_C (default 128): one JSON
line with the launch time; compare GNPDE_BF16_VEC / GNPDE_AGG_VARIANT settings."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

import gnpde  # noqa: E402
from gnpde import ops, synthetic  # noqa: E402


def main():
    N, E = synthetic.ARXIV_N, synthetic.ARXIV_E
    C = int(os.environ.get("K1_C", 128))
    reps = 40
    dev = torch.device("cuda", 0)
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, device=dev).to(torch.bfloat16)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9,
           'multi_modal': False}
    func = gnpde.LaplacianODEFunc(C, C, opt, dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    with torch.no_grad():
        for _ in range(3):
            func(None, x)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            func(None, x)
        e.record()
        torch.cuda.synchronize()
    rhs_us = s.elapsed_time(e) / reps * 1e3
    # rk4 steps through the integrator (fused stages, graph replay), as bench.py's blend_c162
    steps = 40
    with torch.no_grad():
        t = torch.tensor([0.0, 0.25 * steps], device=dev)
        gnpde.odeint(func, x, t, method='rk4', options={'step_size': 0.25})
        torch.cuda.synchronize()
        s.record()
        gnpde.odeint(func, x, t, method='rk4', options={'step_size': 0.25})
        e.record()
        torch.cuda.synchronize()
    print(json.dumps({"C": C, "dtype": "bf16", "vec": os.environ.get("GNPDE_BF16_VEC", "default"),
                      "variant": os.environ.get("GNPDE_AGG_VARIANT", "0"), "rhs_us": round(rhs_us, 1),
                      "rk4_step_ms": round(s.elapsed_time(e) / steps, 4)}))


if __name__ == "__main__":
    main()
