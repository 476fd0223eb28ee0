"""Diagnostic: the three adaptive-adjoint backward paths on the test_gpu_adjoint case."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import numpy as np
import torch
import gnpde
from gnpde import integrator as gi

DEV = "cuda"
OPT = {'self_loop_weight': 1, 'add_source': False, 'hidden_dim': 6, 'block': 'constant', 'function': 'laplacian',
       'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False}


def run(method, add_source, mode, tol=1e-3):
    N, E, C = 3000, 24000, 32
    rng = np.random.default_rng(6)
    ei = torch.from_numpy(rng.integers(0, N, size=(1, 2, E))).to(DEV)
    ei[:, 1, :300] = 5
    w = torch.from_numpy(rng.uniform(0.05, 0.5, size=(1, E)).astype(np.float32)).to(DEV)
    x = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
    x0 = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
    R = torch.from_numpy(rng.standard_normal((2, 1, N, C)).astype(np.float32)).to(DEV)
    t = torch.tensor([0.0, 0.7, 2.0], device=DEV)
    func = gnpde.LaplacianODEFunc(C, C, dict(OPT, hidden_dim=C, add_source=add_source), DEV).to(DEV)
    with torch.no_grad():
        func.alpha_train.fill_(0.3)
        func.beta_train.fill_(-0.4)
    func.edge_index, func.edge_weight = ei, w
    if add_source:
        func.x0 = x0
    gi.FUSED_ADJOINT = mode != 'autograd'
    gi.FUSED_ADAPTIVE_ADJOINT = mode == 'fused'
    xt = x.clone().requires_grad_(True)
    func.nfe = 0
    z = gi.odeint_adjoint(func, xt, t, rtol=tol * 1e-2, atol=tol, method='dopri5', adjoint_method=method)
    nf = func.nfe
    (z[1:] * R).sum().backward()
    return xt.grad.double().cpu(), float(func.alpha_train.grad), func.nfe - nf, gi._OdeintAdjoint.last_path


for method in ("dopri5", "adaptive_heun"):
    res = {m: run(method, False, m) for m in ("fused", "direct", "autograd")}
    ref = res["autograd"][0]
    for m, (g, a, n, p) in res.items():
        print(method, m, p, "nfe", n, "alpha", a, "x relerr", float((g - ref).abs().max() / ref.abs().max()), flush=True)

print("---- step logs (dopri5)")
from gnpde.adjoint_adaptive import AdaptiveAdjoint
logs = []
o1 = gi._RKAdaptive._step
def s1(self, y0, f0, t0, dt):
    logs.append(("ref", float(t0), float(dt)))
    return o1(self, y0, f0, t0, dt)
gi._RKAdaptive._step = s1
o2 = AdaptiveAdjoint._step
def s2(self, mid):
    logs.append(("fused", float(self.scale)))
    return o2(self, mid)
AdaptiveAdjoint._step = s2
o3 = AdaptiveAdjoint._ratio
def s3(self, *a):
    r = o3(self, *a)
    logs.append(("ratio", r))
    return r
AdaptiveAdjoint._ratio = s3
for m in ("fused", "autograd"):
    logs.clear()
    run("dopri5", False, m)
    print(m, logs)
