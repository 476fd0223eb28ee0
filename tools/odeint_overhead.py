#!/usr/bin/env python
"""Host-side overhead of one gnpde.odeint call on G-arxiv (rk4, 50 steps, cached
step graphs): wall time vs the GPU time inside the replays, the host time to
return (GPU still busy), and a cProfile of the call's Python side."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

import gnpde  # noqa: E402
from gnpde import integrator as gi, synthetic  # noqa: E402


def main():
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    steps = int(os.environ.get("OV_STEPS", 50))
    dev = torch.device("cuda", 0)
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, device=dev)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': False, 'no_alpha_sigmoid': False,
           'max_nfe': 10 ** 9, 'multi_modal': False}
    func = gnpde.LaplacianODEFunc(C, C, opt, dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    h = 0.25

    def call():
        t = torch.tensor([0.0, steps * h], dtype=torch.float32, device=dev)
        return gnpde.odeint(func, x, t, method='rk4', options={'step_size': h})[1]

    r = {}
    warm = int(os.environ.get("OV_WARM_STEPS", 0))
    with torch.no_grad():
        if warm:  # bench.py's order: one warm-up call of `warm` steps, then the timed call
            t = torch.tensor([0.0, warm * h], dtype=torch.float32, device=dev)
            gnpde.odeint(func, x, t, method='rk4', options={'step_size': h})
        else:
            for _ in range(3):
                call()
        torch.cuda.synchronize()
        ev = []
        gi.replay_events = ev
        t0 = time.perf_counter()
        call()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        gi.replay_events = None
        r["wall_ms"] = round((t2 - t0) * 1e3, 3)
        r["host_return_ms"] = round((t1 - t0) * 1e3, 3)
        r["replay_gpu_ms"] = round(sum(s.elapsed_time(e) for s, e, _ in ev), 3)
        r["replays"] = [(n, round(s.elapsed_time(e), 3)) for s, e, n in ev]
        r["gaps_ms"] = [round(ev[i][1].elapsed_time(ev[i + 1][0]), 3) for i in range(len(ev) - 1)]
        pr = cProfile.Profile()
        pr.enable()
        call()
        pr.disable()
        torch.cuda.synchronize()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(json.dumps(r), flush=True)
    print(s.getvalue())


if __name__ == "__main__":
    main()
