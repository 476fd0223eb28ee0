#!/usr/bin/env python
"""One workload of the bench, run alone so that a rocprofv3 --pmc pass over it
can be attributed per kernel and per RHS evaluation (tools/pmc_reduce.py):

  tools/pmc_run.py WORKLOAD [--reps N]

WORKLOAD: lap (G-arxiv rk4, fused K1 stages + plain K1 launches), grmat
(configs[4] graph rk4), dopri5 (replays of one captured G-arxiv dopri5 step), attn:<mode>_norm<k> (the transformer RHS of
bench.bench_attention, eager), blend_fp32 / blend_bf16 (C = 162 rk4 steps).
Setup (graph, plans, cached weights) and two warm-up evaluations run first,
then a marker (one gnpde_dot_f64, used by no workload), then the N measured
evaluations: the reducer counts only dispatches after the marker.  Prints one JSON line: the workload and how many
RHS evaluations of each kind ran (the reducer divides by them)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("workload")
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    import gnpde
    from gnpde import synthetic
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    wl, reps, warm = a.workload, a.reps, 2
    meta = {"workload": wl, "reps": reps, "warm": warm}
    from gnpde import ops
    mk = torch.ones(64, device=dev)

    def marker():
        # the measured region starts after the last dot_final_kernel (gnpde_dot_f64 runs in no workload)
        torch.cuda.synchronize()
        ops.dot(mk, mk)
        torch.cuda.synchronize()
    with torch.no_grad():
        if wl in ("lap", "grmat"):
            N, E, C = (169343, 1200000, 128) if wl == "lap" else (2000000, 20000000, 256)
            ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
            x = synthetic.features(1, N, C, seed=1, device=dev)
            func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
            func.edge_index, func.edge_weight = ei, w
            steps = reps if wl == "lap" else max(2, reps // 4)
            bench.rk4_solve(func, x, warm, 0.25, dev)
            marker()
            bench.rk4_solve(func, x, steps, 0.25, dev)
            meta.update({"nodes": N, "edges": E, "dim": C, "rk4_steps": steps, "fused_launches": 4 * steps})
            if wl == "lap":
                # plain K1 launches on the numbering the solve ran in (as bench.py's rhs_plain)
                lay = func.node_layout(x)
                gp, xp = (lay.graph, lay.to_internal(x)) if lay is not None else (func.graph_for(x), x)
                wc = func.csr_weights(gp, w, 'w')
                out = torch.empty_like(x).view(-1, C)
                for _ in range(reps):
                    ops.spmm_rhs(gp, wc, xp, alpha=func.alpha_train.detach(), out=out)
                meta["plain_launches"] = reps
        elif wl.startswith("attn:"):
            mode, norm = wl[5:].rsplit("_norm", 1)
            ei, w = synthetic.rw_graph(169343, 1200000, seed=0, device=dev)
            x = synthetic.features(1, 169343, 128, seed=1, device=dev)
            func = bench.attention_func(mode, int(norm), 128, dev)
            func.edge_index = ei
            func.graph_for(x)
            # the numbering a solve runs the RHS in (bench.bench_attention)
            x, lay = bench.solve_numbering(func, x)
            func._layout = lay
            for _ in range(warm):
                func(None, x)
            marker()
            for _ in range(reps):
                func(None, x)
            func._layout = None
            meta["node_order"] = "degree" if lay is not None else "none"
            meta.update({"nodes": 169343, "edges": 1200000, "dim": 128, "heads": 2, "attention_dim": 32,
                         "rhs": reps})
        elif wl == "dopri5":
            # the bench's dopri5 line (G-arxiv, ogbn-arxiv best_params): warm solves, then `reps`
            # replays of one captured step (6 RHS launches + error reduction + device controller)
            import gnpde.integrator as integ
            ei, w = synthetic.rw_graph(169343, 1200000, seed=0, device=dev)
            x = synthetic.features(1, 169343, 128, seed=1, device=dev)
            func = gnpde.LaplacianODEFunc(128, 128, dict(bench.LAP_OPT, hidden_dim=128), dev).to(dev)
            func.edge_index, func.edge_weight = ei, w
            T, ts = bench.ARXIV_DOPRI5
            t = torch.tensor([0.0, T], dtype=torch.float32, device=dev)
            for _ in range(3):
                gnpde.odeint(func, x, t, method='dopri5', rtol=1e-9 * ts, atol=1e-7 * ts)
            g = integ.adaptive_step_graph(func)
            marker()
            for _ in range(reps):
                g.replay()
            meta.update({"nodes": 169343, "edges": 1200000, "dim": 128, "steps": reps, "rhs_per_step": 6})
        elif wl.startswith("blend_"):
            dt = torch.bfloat16 if wl == "blend_bf16" else torch.float32
            ei, w = synthetic.rw_graph(169343, 1200000, seed=0, device=dev)
            func = bench.blend_func(dev)
            func.edge_index = ei
            x = synthetic.features(1, 169343, 162, seed=3, device=dev).to(dt)
            for n in (warm, reps):
                if n == reps:
                    marker()
                t = torch.tensor([0.0, 0.25 * n], device=dev)
                gnpde.odeint(func, x, t, method='rk4', options={'step_size': 0.25})
            meta.update({"nodes": 169343, "edges": 1200000, "dim": 162, "rk4_steps": reps, "fused_launches": 4 * reps})
        else:
            raise SystemExit("unknown workload %r" % wl)
        torch.cuda.synchronize()
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
