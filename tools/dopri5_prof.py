"""dopri5 on G-arxiv (ogbn-arxiv best_params T / tol_scale) through the fused adaptive
step: per-solve and per-step wall times, with the initial-step selection included and
excluded (first_step given), for rocprofv3 kernel traces of the step.
  python tools/dopri5_prof.py [--reps 5] [--c2]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def problem(c2):
    import gnpde
    from gnpde import synthetic
    dev = torch.device("cuda", 0)
    if c2:
        N, E, C = 2708, 13264, 80
    else:
        N, E, C = 169343, 1200000, 128
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    if c2:
        opt = {'hidden_dim': C, 'heads': 8, 'attention_dim': 128, 'attention_norm_idx': 1,
               'attention_type': 'scaled_dot', 'function': 'transformer', 'add_source': False,
               'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False, 'mix_features': False,
               'square_plus': False, 'beltrami': False}
        func = gnpde.ODEFuncTransformerAtt(C, C, opt, dev).to(dev).eval()
        gen = torch.Generator(device=dev)
        gen.manual_seed(11)
        with torch.no_grad():
            for lin in (func.multihead_att_layer.Q, func.multihead_att_layer.K):
                lin.weight.copy_(torch.randn(128, C, generator=gen, device=dev) * 0.03)
                lin.bias.copy_(torch.randn(128, generator=gen, device=dev) * 0.03)
        func.edge_index = ei
        T, ts = bench.CORA_DOPRI5
    else:
        func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
        func.edge_index, func.edge_weight = ei, w
        T, ts = bench.ARXIV_DOPRI5
    t = torch.tensor([0.0, T], dtype=torch.float32, device=dev)
    kw = dict(method='dopri5', rtol=1e-9 * ts, atol=1e-7 * ts)
    return func, x, t, kw


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--c2", action="store_true")
    a = p.parse_args()
    func, x, t, kw = problem(a.c2)
    import gnpde
    import gnpde.integrator as integ
    with torch.no_grad():
        gnpde.odeint(func, x, t, **kw)
        steps = integ.odeint.last_n_steps
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            gnpde.odeint(func, x, t, **kw)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / a.reps
        h0 = 0.5  # a fixed first step: the step loop alone
        gnpde.odeint(func, x, t, options={'first_step': h0}, **kw)
        steps1 = integ.odeint.last_n_steps
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            gnpde.odeint(func, x, t, options={'first_step': h0}, **kw)
        torch.cuda.synchronize()
        el1 = (time.perf_counter() - t0) / a.reps
    print("solve %.3f ms, %d steps (%.3f ms/step); first_step given: %.3f ms, %d steps (%.3f ms/step)" %
          (el * 1e3, steps, el * 1e3 / steps, el1 * 1e3, steps1, el1 * 1e3 / steps1), flush=True)


if __name__ == "__main__":
    main()
