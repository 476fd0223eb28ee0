"""GPU parity of backprop through adaptive solves of the Laplacian as one autograd node
(gnpde.adaptive_backprop: Cora's / Citeseer's training path, src/best_params.py:1-2 —
block attention, dopri5, adjoint False): the fused forward (stage plan in the K1
epilogues, each accepted step's stage inputs kept) and its discrete adjoint (transposed
stages over the CSC with the alpha rows, one SDDMM over every stage for the weights)
against the restated torchdiffeq loop with autograd through every RHS and stage
combination (GNPDE_ADAPTIVE_BACKPROP=0) on the same inputs.

Both differentiate the SAME discrete map (the accepted steps and the dense output; the
step sizes are constants, as torchdiffeq's no_grad controller makes them) when they take
the same steps: the tests pass ``first_step`` (the initial-step selection's fp32 rounding
is not what is under test) and assert equal step counts, then gradients within 1e-5 of
the largest.  torchdiffeq is absent: parity with the reference's own autograd is through
the RHS gradients it is pinned to (tests/test_gpu_grad_golden.py)."""
import numpy as np
import pytest
import torch

import gnpde
from gnpde import integrator as gi

pytestmark = pytest.mark.gpu
DEV = "cuda"

OPT = {'self_loop_weight': 1, 'add_source': False, 'hidden_dim': 6, 'block': 'constant', 'function': 'laplacian',
       'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False}


def relerr(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _run(fused, monkeypatch, method, add_source, t, first_step, tol=1e-4):
    N, E, C = 2500, 20000, 32
    rng = np.random.default_rng(91)
    ei = torch.from_numpy(rng.integers(0, N, size=(1, 2, E))).to(DEV)
    ei[:, 0, :400] = 3  # hub row (CSR split plan)
    ei[:, 1, 400:800] = 8  # hub column (CSC split plan)
    w = torch.from_numpy(rng.uniform(0.05, 0.3, size=(1, E)).astype(np.float32)).to(DEV)
    x = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
    x0 = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
    R = torch.from_numpy(rng.standard_normal((len(t), 1, N, C)).astype(np.float32)).to(DEV)
    monkeypatch.setattr(gi, "ADAPTIVE_BACKPROP", fused)
    func = gnpde.LaplacianODEFunc(C, C, dict(OPT, hidden_dim=C, add_source=add_source), DEV).to(DEV)
    with torch.no_grad():
        func.alpha_train.fill_(0.35)
        func.beta_train.fill_(-0.25)
    wt = w.clone().requires_grad_(True)
    func.edge_index, func.edge_weight = ei, wt
    if add_source:
        func.x0 = x0
    xt = x.clone().requires_grad_(True)
    func.nfe = 0
    tt = torch.tensor(t, device=DEV)
    z = gnpde.odeint(func, xt, tt, method=method, rtol=tol * 1e-2, atol=tol, options={'first_step': first_step})
    path = gi.odeint.last_path
    steps = gi.odeint.last_n_steps
    (z * R).sum().backward()
    return dict(z=z.detach(), x=xt.grad, alpha=func.alpha_train.grad, beta=func.beta_train.grad, w=wt.grad,
                nfe=func.nfe, steps=steps, path=path)


@pytest.mark.parametrize("method", ["dopri5", "adaptive_heun", "bosh3"])
@pytest.mark.parametrize("add_source", [False, True])
def test_adaptive_backprop_vs_restated_autograd(method, add_source, monkeypatch):
    """Outputs at an interior time (dense output) and at the end; gradients of x, alpha,
    beta and the edge weights."""
    t = [0.0, 0.55, 1.6]
    a = _run(True, monkeypatch, method, add_source, t, 0.05)
    b = _run(False, monkeypatch, method, add_source, t, 0.05)
    assert a['path'] == 'fused_backprop' and b['path'] == 'restated'
    assert a['steps'] == b['steps'] and a['nfe'] == b['nfe'], (a['steps'], b['steps'], a['nfe'], b['nfe'])
    assert relerr(a['z'], b['z']) <= 1e-5
    for k in ('x', 'alpha', 'w') + (('beta',) if add_source else ()):
        assert relerr(a[k], b[k]) <= 1e-5, (k, relerr(a[k], b[k]))
    if not add_source:
        assert float(a['beta'].abs().max()) == 0.0


def test_cora_attention_block_training_step(monkeypatch):
    """AttODEblock at Cora's best_params shape (heads 8, attention_dim 128, norm_idx 1,
    add_source, dopri5, backprop) on a small graph: the block's training step through the
    fused node against the restated loop — x, alpha / beta and the attention layer's Q / K
    gradients (the weights' SDDMM feeding the attention backward)."""
    N, E, C = 1500, 9000, 40
    rng = np.random.default_rng(93)
    ei = torch.from_numpy(rng.integers(0, N, size=(1, 2, E))).to(DEV)
    x = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
    gout = torch.from_numpy(rng.standard_normal((1, N, C)).astype(np.float32)).to(DEV)
    opt = dict(OPT, hidden_dim=C, block='attention', function='laplacian', heads=8, attention_dim=64,
               attention_norm_idx=1, attention_type='scaled_dot', add_source=True, adjoint=False, method='dopri5',
               step_size=1, tol_scale=500.0, self_loop_weight=1.0, data_norm='rw', leaky_relu_slope=0.2,
               reweight_attention=False, square_plus=False, mix_features=False, beltrami=False, augment=False,
               max_iters=100, max_nfe=2000)
    data = gnpde.GraphData()
    data.new_graph(ei, N)
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(gi, "ADAPTIVE_BACKPROP", fused)
        torch.manual_seed(0)
        blk = gnpde.AttODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0.0, 2.0], device=DEV))
        blk = blk.to(DEV).train()
        g = torch.Generator(device=DEV)
        g.manual_seed(5)
        with torch.no_grad():
            for lin in (blk.multihead_att_layer.Q, blk.multihead_att_layer.K):
                lin.weight.copy_(torch.randn(lin.weight.shape, generator=g, device=DEV) * 0.05)
            blk.odefunc.alpha_train.fill_(0.3)
            blk.odefunc.beta_train.fill_(0.2)
        xi = x.clone().requires_grad_(True)
        blk.set_x0(xi)
        z = blk(xi, data)
        assert gi.odeint.last_path == ('fused_backprop' if fused else 'restated')
        n = gi.odeint.last_n_steps
        (z * gout).sum().backward()
        lay = blk.multihead_att_layer
        res[fused] = (z.detach(), xi.grad, blk.odefunc.alpha_train.grad, blk.odefunc.beta_train.grad,
                      lay.Q.weight.grad, lay.K.weight.grad, n)
    a, b = res[True], res[False]
    assert a[6] == b[6], (a[6], b[6])
    for name, u, v in zip(("z", "x", "alpha", "beta", "Q", "K"), a[:6], b[:6]):
        assert u is not None and v is not None, name
        assert relerr(u, v) <= 1e-5, (name, relerr(u, v))
