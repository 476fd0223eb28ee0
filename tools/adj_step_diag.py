"""Diagnostic: one fused adjoint step against integrator._RKAdaptive._step of the direct augmented RHS."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import numpy as np
import torch
import gnpde
from gnpde import integrator as gi, ops
from gnpde.adjoint_adaptive import AdaptiveAdjoint

DEV = "cuda"
OPT = {'self_loop_weight': 1, 'add_source': False, 'hidden_dim': 6, 'block': 'constant', 'function': 'laplacian',
       'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False}
N, E, C = 3000, 24000, 32
rng = np.random.default_rng(6)
ei = torch.from_numpy(rng.integers(0, N, size=(1, 2, E))).to(DEV)
w = torch.from_numpy(rng.uniform(0.05, 0.5, size=(1, E)).astype(np.float32)).to(DEV)
y = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
a = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
func = gnpde.LaplacianODEFunc(C, C, dict(OPT, hidden_dim=C), DEV).to(DEV)
with torch.no_grad():
    func.alpha_train.fill_(0.3)
func.edge_index, func.edge_weight = ei, w
params = (func.alpha_train,)
ny = y.numel()
for method in ("dopri5", "bosh3", "adaptive_heun"):
  with torch.no_grad():
    ans = torch.stack([y, y])
    aug = gi._laplacian_aug(func, params, y.shape, ny, ans)
    z0 = torch.cat([y.reshape(-1), a.reshape(-1), torch.zeros(1, device=DEV)])
    f0 = aug(0.0, z0)
    dt = 0.05
    solver = gi._RKAdaptive(aug, z0, 1e-5, 1e-3, gi._Combine(), method=method)
    y1, f1, err, k = solver._step(z0, f0, torch.tensor(0.0, dtype=torch.float64), torch.tensor(dt, dtype=torch.float64))
    # fused
    A = AdaptiveAdjoint(func, params, method, 1e-5, 1e-3)
    A._setup(y)
    b = A.bufs
    b['Y'][0].copy_(y); b['Y'][1].copy_(a)
    A._rhs(b['Y'], ops.Stage(f_out=b['K0'][0]), ops.Stage(f_out=b['K0'][1]), 2, A._beta_slot(0))
    print(method, "f0 y", float((b['K0'][0].reshape(-1) - f0[:ny]).abs().max()), "f0 a", float((b['K0'][1].reshape(-1) - f0[ny:2*ny]).abs().max()))
    A.scale.fill_(dt)
    A._step(True)
    r = A._read()
    P = A.plan
    Y1 = b['Y1']
    print(method, "y1 y", float((Y1[0].reshape(-1) - y1[:ny]).abs().max()), "y1 a", float((Y1[1].reshape(-1) - y1[ny:2*ny]).abs().max()),
          "scale", float(y1[:2*ny].abs().max()))
    kn = b['K%d' % P.ns]
    print(method, "f1 y", float((kn[0].reshape(-1) - f1[:ny]).abs().max()), "f1 a", float((kn[1].reshape(-1) - f1[ny:2*ny]).abs().max()))
    for j in range(1, P.ns + 1):
        if ('K%d' % j) in b:
            kj = b['K%d' % j]
            print(method, "k%d" % j, float((kj[0].reshape(-1) - k[j][:ny]).abs().max()), float((kj[1].reshape(-1) - k[j][ny:2*ny]).abs().max()))
    tol = 1e-3 + 1e-5 * torch.max(z0.abs(), y1.abs())
    q = (err / tol)[:2*ny].double()
    print(method, "e2 y", r[0], float((q[:ny] ** 2).sum()), "e2 a", r[1], float((q[ny:] ** 2).sum()))
    print(method, "kalpha", [A.one_minus_sig * r[2 + j] for j in range(1, P.ns + 1)], [float(kk[-1]) for kk in k[1:]])
