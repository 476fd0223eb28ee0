"""GPU gradients of the RHS and the attention against
torch float64 autograd of a plain-torch restatement of the reference formulas
(function_laplacian_diffusion.py:39-77, function_transformer_attention.py:
218-267 incl. the fork's global-key-sum scaled_dot, utils.py:116-127).

Tolerance: max|g - g_ref| / max|g_ref| <= 1e-4 per gradient (fp32 kernels with
fp32/fp64 accumulation against fp64 autograd).
"""
import numpy as np
import pytest
import torch

import gnpde
from gnpde import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
GTOL = 1e-4

OPT = {'self_loop_weight': 1, 'leaky_relu_slope': 0.2, 'heads': 2, 'attention_norm_idx': 0, 'add_source': False,
       'hidden_dim': 6, 'block': 'constant', 'function': 'laplacian', 'augment': False, 'adjoint': False,
       'tol_scale': 1, 'time': 1, 'method': 'euler', 'no_alpha_sigmoid': False, 'reweight_attention': False,
       'step_size': 1, 'beltrami': False, 'attention_type': 'scaled_dot', 'square_plus': False, 'max_nfe': 100000,
       'data_norm': 'rw', 'max_iters': 1000, 'multi_modal': False, 'mix_features': False, 'attention_dim': 16}


def relerr(a, b, floor=1e-30):
    """max|a - b| / max(max|b|, floor).  ``floor``: the scale of a gradient that is
    mathematically zero by softmax shift invariance (a q bias under destination
    groups, a k bias under source groups), where fp32 noise meets an fp64 zero."""
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), floor))


BIAS_OF = {"bq": 1, "bk": 3}  # index of the weight matrix whose gradient scale bounds the bias noise


# ---------------------------------------------------------------- torch fp64 restatement (test oracle)
def t_aggregate(ei, w, x):
    """sum_{e: src=i} w_e x[dst]  per batch element (function_laplacian_diffusion.py:39-58)."""
    B, N, C = x.shape
    out = []
    for b in range(B):
        src, dst = ei[b, 0], ei[b, 1]
        out.append(torch.zeros(N, C, dtype=x.dtype, device=x.device).index_add(0, src, w[b][:, None] * x[b][dst]))
    return torch.stack(out)


def t_softmax(s, idx, N):
    """utils.softmax (src/utils.py:116-127) for s [E,H] grouped by idx [E]."""
    m = torch.full((N, s.shape[1]), -float('inf'), dtype=s.dtype, device=s.device)
    m = m.index_reduce(0, idx, s.detach(), 'amax', include_self=True)
    e = torch.exp(s - m[idx])
    den = torch.zeros(N, s.shape[1], dtype=s.dtype, device=s.device).index_add(0, idx, e)
    return e / (den[idx] + 1e-16)


def t_attention(x, ei, Wq, bq, Wk, bk, H, norm_idx, mode):
    """[B,E,H] attention: fork scaled_dot (mode 'reference': q_src . sum_e' k_dst(e') / sqrt dk)
    or per-edge scaled_dot (q_src . k_dst / sqrt dk)."""
    B, N, C = x.shape
    att_dim = Wq.shape[0]
    dk = att_dim // H
    q = (x @ Wq.t() + bq).view(B, N, H, dk)
    k = (x @ Wk.t() + bk).view(B, N, H, dk)
    outs = []
    for b in range(B):
        src, dst = ei[b, 0], ei[b, 1]
        if mode == 'reference':
            S = k[b][dst].sum(0)                               # [H, dk]
            s = (q[b][src] * S[None]).sum(-1) / dk ** 0.5      # [E, H]
        else:
            s = (q[b][src] * k[b][dst]).sum(-1) / dk ** 0.5
        outs.append(t_softmax(s, ei[b, norm_idx], N))
    return torch.stack(outs)


def t_rhs(x, ei, w, alpha, beta=None, x0=None):
    f = torch.sigmoid(alpha) * (t_aggregate(ei, w, x) - x)
    return f if x0 is None else f + beta * x0


def graph(seed, N, E, B=1, hub=True):
    rng = np.random.default_rng(seed)
    ei = rng.integers(0, N, size=(B, 2, E))
    if hub:
        ei[:, 0, :min(E // 5, 400)] = 3          # a hub source group
        ei[:, 1, E // 5:E // 5 + min(E // 5, 400)] = 7  # a hub destination group
    return torch.from_numpy(ei).to(DEV)


def qk_params(seed, C, att, scale=0.2):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(*sh, generator=g) * scale).to(DEV) for sh in ((att, C), (att,), (att, C), (att,))]


# ---------------------------------------------------------------- Laplacian RHS: edge weights
def test_laplacian_edge_weight_gradient_sddmm():
    N, E, C = 900, 7000, 40
    ei = graph(1, N, E)
    torch.manual_seed(1)
    x = torch.randn(1, N, C, device=DEV)
    w = torch.rand(1, E, device=DEV)
    R = torch.randn(1, N, C, device=DEV)
    func = gnpde.LaplacianODEFunc(C, C, dict(OPT, hidden_dim=C), DEV).to(DEV)
    with torch.no_grad():
        func.alpha_train.fill_(0.4)
    wt = w.clone().requires_grad_(True)
    xt = x.clone().requires_grad_(True)
    func.edge_index, func.edge_weight = ei, wt
    (func(0, xt) * R).sum().backward()
    w64 = w.double().requires_grad_(True)
    x64 = x.double().requires_grad_(True)
    a64 = torch.tensor(0.4, dtype=torch.float64, device=DEV, requires_grad=True)
    (t_rhs(x64, ei, w64, a64) * R.double()).sum().backward()
    assert relerr(wt.grad, w64.grad) <= GTOL
    assert relerr(xt.grad, x64.grad) <= GTOL
    assert relerr(func.alpha_train.grad, a64.grad) <= GTOL


def test_laplacian_attention_mean_gradient():
    """block='attention': w = attention_weights.mean(2); the SDDMM gradient lands on every head / H."""
    N, E, C, H = 500, 4000, 16, 4
    ei = graph(2, N, E, B=2)
    torch.manual_seed(2)
    x = torch.randn(2, N, C, device=DEV)
    att = torch.rand(2, E, H, device=DEV)
    R = torch.randn(2, N, C, device=DEV)
    func = gnpde.LaplacianODEFunc(C, C, dict(OPT, hidden_dim=C, block='attention'), DEV).to(DEV)
    at = att.clone().requires_grad_(True)
    func.edge_index, func.attention_weights = ei, at
    (func(0, x) * R).sum().backward()
    a64 = att.double().requires_grad_(True)
    (t_rhs(x.double(), ei, a64.mean(2), torch.tensor(0.0, dtype=torch.float64, device=DEV)) * R.double()).sum() \
        .backward()
    assert relerr(at.grad, a64.grad) <= GTOL


# ---------------------------------------------------------------- transformer RHS: attention backward
@pytest.mark.parametrize("mode,norm_idx", [("reference", 1), ("reference", 0), ("per_edge", 0), ("per_edge", 1)])
@pytest.mark.parametrize("H,att", [(2, 16), (1, 8), (4, 32)])
def test_transformer_rhs_gradients(mode, norm_idx, H, att):
    N, E, C, B = 600, 5000, 24, 2
    ei = graph(3 + H, N, E, B=B)
    torch.manual_seed(3)
    x = torch.randn(B, N, C, device=DEV)
    x0 = torch.randn(B, N, C, device=DEV)
    R = torch.randn(B, N, C, device=DEV)
    Wq, bq, Wk, bk = qk_params(4, C, att, scale=0.3 if mode == 'per_edge' else 0.05)
    opt = dict(OPT, hidden_dim=C, heads=H, attention_dim=att, function='transformer', attention_norm_idx=norm_idx,
               attention_score_mode=mode, add_source=True)
    func = gnpde.ODEFuncTransformerAtt(C, C, opt, DEV).to(DEV)
    lay = func.multihead_att_layer
    with torch.no_grad():
        for p, v in ((lay.Q.weight, Wq), (lay.Q.bias, bq), (lay.K.weight, Wk), (lay.K.bias, bk)):
            p.copy_(v)
        func.alpha_train.fill_(0.3)
        func.beta_train.fill_(0.6)
    func.edge_index, func.x0 = ei, x0
    xt = x.clone().requires_grad_(True)
    (func(0, xt) * R).sum().backward()

    p64 = [t.double().requires_grad_(True) for t in (x, Wq, bq, Wk, bk)]
    a64 = torch.tensor(0.3, dtype=torch.float64, device=DEV, requires_grad=True)
    attn = t_attention(p64[0], ei, *p64[1:], H, norm_idx, mode)
    f64 = t_rhs(p64[0], ei, attn.mean(2), a64, 0.6, x0.double())
    (f64 * R.double()).sum().backward()
    got = [xt.grad, lay.Q.weight.grad, lay.Q.bias.grad, lay.K.weight.grad, lay.K.bias.grad, func.alpha_train.grad]
    want = [p.grad for p in p64] + [a64.grad]
    uniform = mode == 'reference' and norm_idx == 0
    for name, gg, ww in zip(("x", "Wq", "bq", "Wk", "bk", "alpha"), got, want):
        if uniform and name in ("Wq", "bq", "Wk", "bk"):
            # fork scaled_dot under source-grouped softmax: the attention is 1/outdeg for any Q, K
            assert float(ww.abs().max()) < 1e-9 and float(gg.abs().max()) == 0.0, name
            continue
        floor = float(want[BIAS_OF[name]].abs().max()) if name in BIAS_OF else 1e-30
        assert relerr(gg, ww, floor) <= GTOL, (name, relerr(gg, ww, floor))


# ---------------------------------------------------------------- blocks: training through the integrator
def test_attention_block_training_gradients():
    """AttODEblock in training mode (euler, 3 steps): gradients of Q/K, alpha and the input."""
    N, E, C, H, att = 400, 3000, 16, 2, 16
    ei = graph(5, N, E, hub=False)
    torch.manual_seed(5)
    x = torch.randn(1, N, C, device=DEV)
    R = torch.randn(1, N, C, device=DEV)
    opt = dict(OPT, hidden_dim=C, heads=H, attention_dim=att, block='attention', attention_norm_idx=1,
               method='euler', step_size=1.0 / 3.0)
    blk = gnpde.AttODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).train()
    Wq, bq, Wk, bk = qk_params(6, C, att, scale=0.1)
    lay = blk.multihead_att_layer
    with torch.no_grad():
        for p, v in ((lay.Q.weight, Wq), (lay.Q.bias, bq), (lay.K.weight, Wk), (lay.K.bias, bk)):
            p.copy_(v)
        blk.odefunc.alpha_train.fill_(0.2)
    data = gnpde.GraphData()
    data.new_graph(ei, N)
    xt = x.clone().requires_grad_(True)
    (blk(xt, data) * R).sum().backward()

    eo, wo = blk.odefunc.edge_index, blk.odefunc.edge_weight  # after self loops + rw normalisation
    p64 = [t.double().requires_grad_(True) for t in (x, Wq, bq, Wk, bk)]
    a64 = torch.tensor(0.2, dtype=torch.float64, device=DEV, requires_grad=True)
    w = t_attention(p64[0], eo, *p64[1:], H, 1, 'reference').mean(2)
    y = p64[0]
    for _ in range(3):
        y = y + (1.0 / 3.0) * t_rhs(y, eo, w, a64)
    (y * R.double()).sum().backward()
    got = [xt.grad, lay.Q.weight.grad, lay.Q.bias.grad, lay.K.weight.grad, lay.K.bias.grad,
           blk.odefunc.alpha_train.grad]
    want = [p.grad for p in p64] + [a64.grad]
    for name, gg, ww in zip(("x", "Wq", "bq", "Wk", "bk", "alpha"), got, want):
        floor = float(want[BIAS_OF[name]].abs().max()) if name in BIAS_OF else 1e-30
        assert relerr(gg, ww, floor) <= GTOL, (name, relerr(gg, ww, floor))


def test_mixed_block_gamma_gradient():
    N, E, C, H, att = 300, 2500, 12, 1, 8
    ei = graph(7, N, E, hub=False)
    torch.manual_seed(7)
    x = torch.randn(1, N, C, device=DEV)
    R = torch.randn(1, N, C, device=DEV)
    opt = dict(OPT, hidden_dim=C, heads=H, attention_dim=att, block='mixed', attention_norm_idx=0,
               attention_score_mode='per_edge', method='euler', step_size=0.5)
    blk = gnpde.MixedODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).train()
    Wq, bq, Wk, bk = qk_params(8, C, att, scale=0.3)
    lay = blk.multihead_att_layer
    with torch.no_grad():
        for p, v in ((lay.Q.weight, Wq), (lay.Q.bias, bq), (lay.K.weight, Wk), (lay.K.bias, bk)):
            p.copy_(v)
        blk.gamma.fill_(0.3)
    data = gnpde.GraphData()
    data.new_graph(ei, N)
    (blk(x, data) * R).sum().backward()

    eo, wo = blk.odefunc.edge_index, blk.odefunc.edge_weight
    p64 = [t.double().requires_grad_(True) for t in (Wq, bq, Wk, bk)]
    g64 = torch.tensor([0.3], dtype=torch.float64, device=DEV, requires_grad=True)
    s = torch.sigmoid(g64)
    w = t_attention(x.double(), eo, *p64, H, 0, 'per_edge').mean(2) * (1 - s) + wo.double() * s
    a = torch.tensor(0.0, dtype=torch.float64, device=DEV)
    y = x.double()
    for _ in range(2):
        y = y + 0.5 * t_rhs(y, eo, w, a)
    (y * R.double()).sum().backward()
    assert relerr(blk.gamma.grad, g64.grad) <= GTOL
    assert relerr(lay.Q.weight.grad, p64[0].grad) <= GTOL
    assert relerr(lay.K.bias.grad, p64[3].grad, float(p64[2].grad.abs().max())) <= GTOL  # zero: source groups


def test_backward_is_bit_reproducible():
    N, E, C, H, att = 700, 6000, 32, 2, 16
    ei = graph(9, N, E)
    torch.manual_seed(9)
    x = torch.randn(1, N, C, device=DEV)
    R = torch.randn(1, N, C, device=DEV)
    opt = dict(OPT, hidden_dim=C, heads=H, attention_dim=att, function='transformer', attention_norm_idx=1)
    grads = []
    for _ in range(2):
        func = gnpde.ODEFuncTransformerAtt(C, C, opt, DEV).to(DEV)
        torch.manual_seed(10)
        for p in func.multihead_att_layer.parameters():
            torch.nn.init.normal_(p, std=0.05)
        func.edge_index = ei
        xt = x.clone().requires_grad_(True)
        (func(0, xt) * R).sum().backward()
        grads.append((xt.grad.clone(), func.multihead_att_layer.Q.weight.grad.clone()))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


# ---------------------------------------------------------------- adjoint integration
@pytest.mark.parametrize("method,step,tol", [("rk4", 0.05, 1e-7), ("dopri5", None, 1e-7),
                                             ("adaptive_heun", None, 1e-5)])
def test_adjoint_matches_direct_backprop(method, step, tol):
    """odeint_adjoint (torchdiffeq semantics) against backprop through the solver:
    gradients of y0 and of the RHS parameters (alpha_train, beta_train)."""
    N, E, C = 500, 4000, 16
    ei = graph(11, N, E)
    torch.manual_seed(11)
    x = torch.randn(1, N, C, device=DEV)
    x0 = torch.randn(1, N, C, device=DEV)
    w = torch.rand(1, E, device=DEV)
    R = torch.randn(1, N, C, device=DEV)
    t = torch.tensor([0.0, 0.5, 1.0], device=DEV)
    opts = {} if step is None else {'step_size': step}
    res = []
    for integ in (gnpde.integrator.odeint, gnpde.integrator.odeint_adjoint):
        func = gnpde.LaplacianODEFunc(C, C, dict(OPT, hidden_dim=C, add_source=True), DEV).to(DEV)
        with torch.no_grad():
            func.alpha_train.fill_(0.5)
            func.beta_train.fill_(-0.3)
        func.edge_index, func.edge_weight, func.x0 = ei, w, x0
        xt = x.clone().requires_grad_(True)
        z = integ(func, xt, t, rtol=tol, atol=tol * 1e-2, method=method, options=dict(opts))
        (z[1:] * R).sum().backward()
        res.append((xt.grad, func.alpha_train.grad, func.beta_train.grad))
    for gd, ga in zip(*res):
        assert relerr(ga, gd) <= 1e-3, relerr(ga, gd)


@pytest.mark.parametrize("adjoint_method", ["rk4", "adaptive_heun"])
def test_constant_block_adjoint_training(adjoint_method):
    """ConstantODEblock with opt['adjoint']: the block routes through odeint_adjoint with
    adjoint_method / adjoint_step_size (block_constant.py:34-44) and trains alpha;
    adaptive_heun is the reference's default adjoint_method (run_GNN.py:334)."""
    N, E, C = 300, 2500, 8
    ei = graph(12, N, E, hub=False)
    torch.manual_seed(12)
    x = torch.randn(1, N, C, device=DEV)
    opt = dict(OPT, hidden_dim=C, adjoint=True, adjoint_method=adjoint_method, adjoint_step_size=0.1, method='rk4',
               step_size=0.1, tol_scale_adjoint=1000.0)
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).train()
    assert blk.train_integrator is gnpde.integrator.odeint_adjoint
    data = gnpde.GraphData()
    data.new_graph(ei, N)
    xt = x.clone().requires_grad_(True)
    (blk(xt, data) ** 2).sum().backward()
    assert xt.grad is not None and torch.isfinite(xt.grad).all()
    assert blk.odefunc.alpha_train.grad is not None and float(blk.odefunc.alpha_train.grad) != 0.0


@pytest.mark.parametrize("n", [1, 7, 4096, 1000003, 21675904])
def test_dot_f64_vs_torch_and_deterministic(n):
    """gnpde_dot_f64 (the alpha / beta gradient reductions): fp64 accumulation
    of fp32 products, fixed order — equal to torch's fp64 sum to 1e-12 relative
    and bit-identical run to run (also on an unaligned view: scalar path)."""
    gen = torch.Generator(device=DEV)
    gen.manual_seed(n)
    a = torch.randn(n + 1, generator=gen, device=DEV)
    b = torch.randn(n + 1, generator=gen, device=DEV)
    for x, y in ((a[:n], b[:n]), (a[1:], b[1:])):
        got = ops.dot(x, y)
        want = (x.double() * y.double()).sum()
        assert abs(float(got - want)) <= 1e-12 * max(1.0, float((x.double() * y.double()).abs().sum()))
        assert torch.equal(ops.dot(x, y), got)


@pytest.mark.parametrize("method", ["euler", "midpoint", "rk4"])
@pytest.mark.parametrize("add_source,no_sig", [(False, False), (True, False), (True, True)])
def test_fused_fixed_grid_backward_matches_autograd(method, add_source, no_sig):
    """integrator._LaplacianFixedGridFn (the discrete adjoint of a fixed-grid
    Laplacian solve as one autograd node) against autograd through every RHS
    and stage combination (GNPDE_FUSED_BACKWARD=0): gradients to the state,
    alpha_train and beta_train, with output times inside the grid."""
    import gnpde.integrator as integ
    from gnpde import synthetic
    N, E, C = 3000, 24000, 64
    ei, w = synthetic.rw_graph(N, E, seed=5, device=DEV)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': add_source, 'no_alpha_sigmoid': no_sig,
           'max_nfe': 10 ** 6, 'multi_modal': False}
    func = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
    with torch.no_grad():
        func.alpha_train.fill_(0.4)
        func.beta_train.fill_(0.3)
    func.edge_index, func.edge_weight = ei, w
    gen = torch.Generator(device=DEV)
    gen.manual_seed(3)
    x = torch.randn(1, N, C, generator=gen, device=DEV)
    func.x0 = torch.randn(1, N, C, generator=gen, device=DEV)
    g1, g2 = torch.randn(2, 1, N, C, generator=gen, device=DEV)
    t = torch.tensor([0.0, 0.5, 1.0], device=DEV)
    res = []
    for fused in (True, False):
        integ.FUSED_BACKWARD = fused
        try:
            xi = x.clone().requires_grad_(True)
            func.alpha_train.grad = func.beta_train.grad = None
            func.nfe = 0
            y = gnpde.odeint(func, xi, t, method=method, options={'step_size': 0.25})
            ((y[1] * g1).sum() + (y[2] * g2).sum()).backward()
            res.append((y.detach(), xi.grad, func.alpha_train.grad.clone(), None if func.beta_train.grad is None
                        else func.beta_train.grad.clone(), func.nfe))
        finally:
            integ.FUSED_BACKWARD = True
    (yf, gxf, gaf, gbf, nf), (ye, gxe, gae, gbe, ne) = res
    assert nf == ne  # the backward's recomputed stages are not counted as RHS evaluations
    assert (yf - ye).abs().max() / ye.abs().max() < 1e-5
    assert (gxf - gxe).abs().max() / gxe.abs().max() < 1e-5
    assert abs(float(gaf - gae)) <= 1e-5 * max(1.0, abs(float(gae)))
    if add_source:
        assert abs(float(gbf - gbe)) <= 1e-5 * max(1.0, abs(float(gbe)))


def test_fused_fixed_grid_backward_full_size_garxiv():
    """The discrete-adjoint node on the full G-arxiv graph (hub rows split into
    chunk items over the CSC): two rk4 steps, gradients to x and alpha_train
    against autograd through every RHS call."""
    import gnpde.integrator as integ
    from gnpde import synthetic
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 64
    ei, w = synthetic.rw_graph(N, E, seed=0, device=DEV)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': False, 'no_alpha_sigmoid': False,
           'max_nfe': 10 ** 6, 'multi_modal': False}
    func = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
    func.edge_index, func.edge_weight = ei, w
    x = synthetic.features(1, N, C, seed=1, device=DEV)
    gout = synthetic.features(1, N, C, seed=2, device=DEV)
    t = torch.tensor([0.0, 0.5], device=DEV)
    res = []
    for fused in (True, False):
        integ.FUSED_BACKWARD = fused
        try:
            xi = x.clone().requires_grad_(True)
            func.alpha_train.grad = None
            y = gnpde.odeint(func, xi, t, method='rk4', options={'step_size': 0.25})[1]
            (y * gout).sum().backward()
            res.append((xi.grad, func.alpha_train.grad.clone()))
        finally:
            integ.FUSED_BACKWARD = True
    (gxf, gaf), (gxe, gae) = res
    assert (gxf - gxe).abs().max() / gxe.abs().max() < 1e-5
    assert abs(float(gaf - gae)) <= 1e-5 * max(1.0, abs(float(gae)))


def test_fused_backward_reads_its_forward_state():
    """two forwards with different x0, alpha AND graph
    weights (a new edge_weight tensor on the same edge_index) before ONE
    backward — each backward uses the operands of its own forward, so the summed
    gradient equals the gradients taken one at a time."""
    from gnpde import synthetic
    N, E, C = 2000, 16000, 32
    ei, w = synthetic.rw_graph(N, E, seed=8, device=DEV)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': True, 'no_alpha_sigmoid': False,
           'max_nfe': 10 ** 6, 'multi_modal': False}
    func = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
    func.edge_index, func.edge_weight = ei, w
    gen = torch.Generator(device=DEV)
    gen.manual_seed(9)
    xs = [torch.randn(1, N, C, generator=gen, device=DEV) for _ in range(2)]
    x0s = [torch.randn(1, N, C, generator=gen, device=DEV) for _ in range(2)]
    gs = [torch.randn(1, N, C, generator=gen, device=DEV) for _ in range(2)]
    alphas = [0.4, -0.3]
    wts = [w, w * (0.5 + torch.rand(w.shape, generator=gen, device=DEV))]
    t = torch.tensor([0.0, 0.5], device=DEV)

    def fwd(k):
        with torch.no_grad():
            func.alpha_train.fill_(alphas[k])
        func.x0 = x0s[k]
        func.edge_weight = wts[k]
        xi = xs[k].clone().requires_grad_(True)
        return xi, gnpde.odeint(func, xi, t, method='rk4', options={'step_size': 0.125})[1]

    one_at_a_time = []
    for k in range(2):
        func.alpha_train.grad = func.beta_train.grad = None
        xi, y = fwd(k)
        (y * gs[k]).sum().backward()
        one_at_a_time.append((xi.grad.clone(), func.alpha_train.grad.clone(), func.beta_train.grad.clone()))
    func.alpha_train.grad = func.beta_train.grad = None
    (xa, ya), (xb, yb) = fwd(0), fwd(1)  # the second forward changes x0 and alpha before any backward
    ((ya * gs[0]).sum() + (yb * gs[1]).sum()).backward()
    assert torch.equal(xa.grad, one_at_a_time[0][0])
    assert torch.equal(xb.grad, one_at_a_time[1][0])
    ga = one_at_a_time[0][1] + one_at_a_time[1][1]
    gb = one_at_a_time[0][2] + one_at_a_time[1][2]
    assert abs(float(func.alpha_train.grad - ga)) <= 1e-6 * max(1.0, abs(float(ga)))
    assert abs(float(func.beta_train.grad - gb)) <= 1e-6 * max(1.0, abs(float(gb)))


@pytest.mark.parametrize("add_source", [False, True])
def test_fused_backward_in_node_layout_equals_user_numbering(monkeypatch, add_source):
    """A training solve large enough for the in-degree numbering (ops.NodeLayout):
    the adjoint's last launch stores the input gradient straight into the caller's
    numbering (the stage's out_rows) and the x0 gradient joins in place.  Against
    the same solve with the numbering switched off: x gradients bit-identical
    (every row keeps its edges and their order), alpha within fp64 summation order,
    beta's gradient None without add_source (it is not on the path)."""
    from gnpde import synthetic
    N, E, C = 40000, 320000, 128
    ei, w = synthetic.rw_graph(N, E, seed=11, device=DEV)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(12)
    x = torch.randn(1, N, C, generator=gen, device=DEV)
    gout = torch.randn(2, 1, N, C, generator=gen, device=DEV)
    t = torch.tensor([0.0, 0.5], device=DEV)
    res = []
    for on in (True, False):
        monkeypatch.setattr(ops, "LAYOUT_MIN_ROWS", 32768 if on else 1 << 40)
        monkeypatch.setattr(ops, "LAYOUT_MIN_BYTES", 1 << 20)
        opt = dict(OPT, hidden_dim=C, add_source=add_source)
        func = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
        func.edge_index, func.edge_weight = ei, w
        with torch.no_grad():
            func.alpha_train.fill_(0.3)
            func.beta_train.fill_(0.2)
        func.x0 = x * 0.5
        assert (func.node_layout(x) is not None) == on
        xi = x.clone().requires_grad_(True)
        sol = gnpde.odeint(func, xi, t, method='rk4', options={'step_size': 0.125})
        (sol * gout).sum().backward()  # both output times: sol[0]'s gradient joins x's
        res.append((sol.detach(), xi.grad, func.alpha_train.grad, func.beta_train.grad))
    (s1, gx1, ga1, gb1), (s0, gx0, ga0, gb0) = res
    assert torch.equal(s1, s0)
    assert torch.equal(gx1, gx0)
    assert abs(float(ga1 - ga0)) <= 1e-6 * max(1.0, abs(float(ga0)))
    if add_source:
        assert abs(float(gb1 - gb0)) <= 1e-6 * max(1.0, abs(float(gb0)))
    else:
        assert gb1 is None and gb0 is None
