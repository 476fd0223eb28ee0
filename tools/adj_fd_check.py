"""Diagnostic: the alpha_train gradient of a Laplacian rk4 solve by finite differences
of the loss (central, two step sizes) against direct backprop and the continuous adjoint."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import numpy as np
import torch
import gnpde
from gnpde import integrator as gi

DEV = "cuda"
OPT = {'self_loop_weight': 1, 'add_source': True, 'hidden_dim': 16, 'block': 'constant', 'function': 'laplacian',
       'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False}
N, E, C = 1500, 12000, 16
rng = np.random.default_rng(8)
ei = torch.from_numpy(rng.integers(0, N, size=(1, 2, E))).to(DEV)
w = torch.from_numpy(rng.uniform(0.05, 0.3, size=(1, E)).astype(np.float32)).to(DEV)
x = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
x0 = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
R = torch.from_numpy(rng.standard_normal((1, 1, N, C)).astype(np.float32)).to(DEV)
t = torch.tensor([0.0, 1.0], device=DEV)
h = 0.05
func = gnpde.LaplacianODEFunc(C, C, OPT, DEV).to(DEV)
func.edge_index, func.edge_weight, func.x0 = ei, w, x0
with torch.no_grad():
    func.beta_train.fill_(-0.4)


def loss(a):
    with torch.no_grad():
        func.alpha_train.fill_(a)
        z = gi.odeint(func, x, t, method='rk4', options={'step_size': h})
        return float((z[1:].double() * R.double()).sum())


for eps in (1e-2, 5e-3, 2e-3):
    print("FD eps", eps, (loss(0.3 + eps) - loss(0.3 - eps)) / (2 * eps))
with torch.no_grad():
    func.alpha_train.fill_(0.3)
xt = x.clone().requires_grad_(True)
func.alpha_train.grad = None
z = gi.odeint(func, xt, t, method='rk4', options={'step_size': h})
(z[1:] * R).sum().backward()
print("direct", float(func.alpha_train.grad))
for fused in (True, False):
    gi.FUSED_ADJOINT = fused
    xt = x.clone().requires_grad_(True)
    func.alpha_train.grad = None
    z = gi.odeint_adjoint(func, xt, t, method='rk4', options={'step_size': h}, adjoint_method='rk4',
                          adjoint_options={'step_size': h})
    (z[1:] * R).sum().backward()
    print("adjoint fused" if fused else "adjoint restated", float(func.alpha_train.grad))
# the same with float64 autograd of a torch restatement (eager, no gnpde kernels)
src, dst = ei[0, 0], ei[0, 1]
def f64(y, a, b):
    ax = torch.zeros_like(y).index_add(0, src, w[0].double()[:, None] * y[dst])
    return torch.sigmoid(a) * (ax - y) + b * x0[0].double()
a = torch.tensor(0.3, dtype=torch.float64, device=DEV, requires_grad=True)
b = torch.tensor(-0.4, dtype=torch.float64, device=DEV)
y = x[0].double()
n = int(round(1.0 / h))
for _ in range(n):
    k1 = f64(y, a, b); k2 = f64(y + h * k1 / 3, a, b); k3 = f64(y + h * (k2 - k1 / 3), a, b)
    k4 = f64(y + h * (k1 - k2 + k3), a, b)
    y = y + h * (k1 + 3 * k2 + 3 * k3 + k4) / 8
(y * R[0, 0].double()).sum().backward()
print("fp64 torch autograd", float(a.grad))
