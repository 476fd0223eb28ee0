"""Host-side logic of the drop-in layer, on CPU: registry, constructor/attribute
contract, state_dict keys, the no-fallback guarantee, graph normalisation
(intended semantics, pinned by the reference's KATs) and the bundled
integrator's control logic (with a torch stage combiner injected — the product
path always combines on the GPU)."""
import numpy as np
import pytest
import torch

import gnpde
import gnpde_oracle as O
from gnpde import integrator as gode
from gnpde import utils as gu

OPT = {'self_loop_weight': 1, 'leaky_relu_slope': 0.2, 'heads': 2, 'attention_norm_idx': 0, 'add_source': False,
       'hidden_dim': 6, 'block': 'constant', 'function': 'laplacian', 'augment': False, 'adjoint': False,
       'tol_scale': 1, 'time': 1, 'method': 'euler', 'no_alpha_sigmoid': False, 'reweight_attention': False,
       'step_size': 1, 'beltrami': False, 'attention_type': 'scaled_dot', 'square_plus': False, 'max_nfe': 1000,
       'data_norm': 'rw', 'max_iters': 1000, 'multi_modal': False, 'mix_features': False, 'attention_dim': 16}


def test_registry_matches_reference_names():
    assert gnpde.set_function(dict(OPT, function='laplacian')) is gnpde.LaplacianODEFunc
    assert gnpde.set_function(dict(OPT, function='transformer')) is gnpde.ODEFuncTransformerAtt
    assert gnpde.set_block(dict(OPT, block='constant')) is gnpde.ConstantODEblock
    assert gnpde.set_block(dict(OPT, block='attention')) is gnpde.AttODEblock
    assert gnpde.set_block(dict(OPT, block='mixed')) is gnpde.MixedODEblock
    assert gnpde.set_block(dict(OPT, block='hard_attention')) is gnpde.HardAttODEblock
    with pytest.raises(NotImplementedError):
        gnpde.set_block(dict(OPT, block='rewire_attention'))
    with pytest.raises(NotImplementedError):
        gnpde.set_function(dict(OPT, function='GAT'))
    from gnpde.model_configurations import BlockNotDefined, FunctionNotDefined
    with pytest.raises(BlockNotDefined):
        gnpde.set_block(dict(OPT, block='nope'))
    with pytest.raises(FunctionNotDefined):
        gnpde.set_function(dict(OPT, function='nope'))


def test_state_dict_keys_match_reference_layout():
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], OPT, None, t=torch.tensor([0, 1]))
    keys = set(blk.state_dict().keys())
    for k in ('odefunc.alpha_train', 'odefunc.beta_train', 'odefunc.w', 'odefunc.d', 'odefunc.alpha_sc',
              'odefunc.beta_sc', 'reg_odefunc.odefunc.alpha_train'):
        assert k in keys
    tr = gnpde.ODEFuncTransformerAtt(6, 6, OPT, None)
    keys = set(tr.state_dict().keys())
    for k in ('multihead_att_layer.Q.weight', 'multihead_att_layer.K.bias', 'multihead_att_layer.V.weight',
              'multihead_att_layer.Wout.weight', 'alpha_train'):
        assert k in keys
    assert float(tr.multihead_att_layer.Q.weight[0, 0].detach()) == pytest.approx(1e-5)


def test_attention_block_contract():
    blk = gnpde.AttODEblock(gnpde.LaplacianODEFunc, [], dict(OPT, block='attention'), None,
                            t=torch.tensor([0, 1]))
    assert isinstance(blk.multihead_att_layer, gnpde.SpGraphTransAttentionLayer)
    assert blk.test_integrator is gnpde.odeint and blk.atol == 1e-7 and blk.rtol == 1e-9


def test_mixed_block_contract():
    """test/test_block_mixed.py:57-66: gamma initialised to 0, Laplacian odefunc, attention layer."""
    blk = gnpde.MixedODEblock(gnpde.LaplacianODEFunc, [], dict(OPT, block='mixed', heads=1), None,
                              t=torch.tensor([0, 1]))
    assert isinstance(blk.odefunc, gnpde.LaplacianODEFunc)
    assert blk.gamma.item() == 0.0 and tuple(blk.gamma.shape) == (1,)
    assert isinstance(blk.multihead_att_layer, gnpde.SpGraphTransAttentionLayer)
    assert 'gamma' in blk.state_dict() and 'multihead_att_layer.Q.weight' in blk.state_dict()


def test_hard_attention_block_contract():
    opt = dict(OPT, block='hard_attention', att_samp_pct=0.5)
    blk = gnpde.HardAttODEblock(gnpde.LaplacianODEFunc, [], opt, None, t=torch.tensor([0, 1]))
    assert isinstance(blk.multihead_att_layer, gnpde.SpGraphTransAttentionLayer)
    tr = gnpde.HardAttODEblock(gnpde.ODEFuncTransformerAtt, [], dict(opt, function='transformer'), None,
                               t=torch.tensor([0, 1]))
    assert not hasattr(tr, 'multihead_att_layer')  # uses the odefunc's layer (:21-23, :29)
    with pytest.raises(AssertionError):
        gnpde.HardAttODEblock(gnpde.LaplacianODEFunc, [], dict(opt, att_samp_pct=0.0), None, t=torch.tensor([0, 1]))


def test_no_cpu_fallback():
    func = gnpde.LaplacianODEFunc(2, 2, dict(OPT, hidden_dim=2), None)
    func.edge_index = torch.tensor([[[0, 1, 2, 1], [1, 0, 1, 2]]])
    func.edge_weight = torch.ones(1, 4)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        func(0, torch.ones(1, 3, 2))
    with pytest.raises(RuntimeError, match="ROCm device"):
        gnpde.odeint(lambda t, y: y, torch.ones(3), torch.tensor([0., 1.]), method='euler')


def test_unsupported_settings_raise():
    for bad in (dict(mix_features=True), dict(square_plus=True), dict(multi_modal=True),
                dict(beltrami=True, attention_type='exp_kernel')):
        with pytest.raises(NotImplementedError):
            gnpde.ODEFuncTransformerAtt(6, 6, dict(OPT, **bad), None)


def test_max_nfe_guard():
    func = gnpde.LaplacianODEFunc(2, 2, dict(OPT, hidden_dim=2, max_nfe=3), None)
    func.nfe = 4
    with pytest.raises(gnpde.MaxNFEException):
        func(0, torch.ones(1, 3, 2))


@pytest.mark.parametrize("self_loop", [0, 0.3, 1, 3.2])
@pytest.mark.parametrize("norm_dim", [0, 1])
def test_get_rw_adj_kat(self_loop, norm_dim):
    """test/test_utils.py:62-79 against gnpde.utils (torch, intended semantics)."""
    from sklearn.preprocessing import normalize
    edge = torch.tensor([[[0, 2, 2, 1], [1, 0, 1, 2]]])
    ei, w = gu.get_rw_adj(edge, norm_dim=norm_dim, fill_value=self_loop, num_nodes=3)
    got = O.to_dense(ei[0].numpy(), w[0].numpy(), 3)
    base = O.to_dense(edge[0].numpy(), np.ones(4), 3)
    assert np.allclose(got, normalize(base + np.identity(3) * self_loop, norm='l1', axis=0 if norm_dim == 1 else 1))


def test_gcn_norm_kat():
    edge = torch.tensor([[[0, 1, 2, 1], [1, 0, 1, 2]]])
    ei, w = gu.gcn_norm_fill_val(edge, fill_value=1, num_nodes=3)
    aug = O.to_dense(edge[0].numpy(), np.ones(4), 3) + np.identity(3)
    deg = np.sqrt(aug.sum(axis=1))
    assert np.allclose(O.to_dense(ei[0].numpy(), w[0].numpy(), 3), aug / deg[:, None] / deg[None, :])


def test_add_remaining_self_loops_matches_oracle():
    rng = np.random.default_rng(0)
    ei = rng.integers(0, 9, size=(2, 2, 30))
    ei[:, 1, :5] = ei[:, 0, :5]  # some existing loops
    w = rng.uniform(size=(2, 30)).astype(np.float32)
    oe, ow = O.add_remaining_self_loops(ei, w, 0.5, 9)
    for b in range(2):
        te, tw = gu.add_remaining_self_loops(torch.from_numpy(ei[b:b + 1]), torch.from_numpy(w[b:b + 1]), 0.5, 9)
        assert np.array_equal(te[0].numpy(), oe[b]) and np.allclose(tw[0].numpy(), ow[b])
    if oe[0].shape[1] != oe[1].shape[1]:
        with pytest.raises(ValueError, match="equal counts"):
            gu.add_remaining_self_loops(torch.from_numpy(ei), torch.from_numpy(w), 0.5, 9)


def test_utils_softmax_matches_oracle():
    rng = np.random.default_rng(1)
    src = rng.standard_normal((2, 100, 3))
    idx = rng.integers(0, 12, size=(2, 100))
    got = gu.softmax(torch.from_numpy(src), torch.from_numpy(idx)).numpy()
    assert np.abs(got - O.edge_softmax(src, idx)).max() < 1e-14


# ---------------------------------------------------------------- integrator control logic
def test_fixed_grid_constructor():
    t = torch.tensor([0.0, 1.0])
    assert gode.fixed_grid(t, 0.1).tolist() == pytest.approx(O.fixed_grid(0, 1, 0.1).tolist())
    assert len(gode.fixed_grid(torch.tensor([0.0, 3.0]), 0.25)) == 13


@pytest.mark.parametrize("method,tol", [("euler", 0.02), ("midpoint", 2e-3), ("rk4", 1e-6)])
def test_fixed_solvers_linear_ode(method, tol):
    f = lambda t, y: -y  # noqa: E731
    y0 = torch.ones(4, dtype=torch.float64)
    out = gode.odeint(f, y0, torch.tensor([0.0, 1.0], dtype=torch.float64), method=method,
                      options=dict(step_size=0.1), combine=gode._torch_combine)
    assert out.shape == (2, 4)
    assert torch.allclose(out[1], torch.full((4,), np.exp(-1.0), dtype=torch.float64), atol=tol)


def test_rk4_matches_oracle_integrator():
    rng = np.random.default_rng(2)
    A = rng.standard_normal((5, 5)) * 0.3
    f_np = lambda t, y: y @ A.T  # noqa: E731
    f_t = lambda t, y: y @ torch.from_numpy(A).T  # noqa: E731
    y0 = rng.standard_normal(5)
    want = O.odeint_fixed(f_np, y0, 0.0, 2.0, "rk4", 0.25)
    got = gode.odeint(f_t, torch.from_numpy(y0), torch.tensor([0.0, 2.0]), method='rk4',
                      options=dict(step_size=0.25), combine=gode._torch_combine)[1].numpy()
    assert np.allclose(got, want, rtol=1e-12, atol=1e-12)


def test_dopri5_accuracy_and_step_control():
    f = lambda t, y: -2.0 * y  # noqa: E731
    y0 = torch.ones(3, dtype=torch.float64)
    out = gode.odeint(f, y0, torch.tensor([0.0, 0.5, 1.0]), method='dopri5', rtol=1e-9, atol=1e-10,
                      combine=gode._torch_combine)
    assert torch.allclose(out[1], torch.full((3,), np.exp(-1.0), dtype=torch.float64), atol=1e-8)
    assert torch.allclose(out[2], torch.full((3,), np.exp(-2.0), dtype=torch.float64), atol=1e-8)
    n_tight = gode.odeint.last_n_steps
    gode.odeint(f, y0, torch.tensor([0.0, 1.0]), method='dopri5', rtol=1e-4, atol=1e-5, combine=gode._torch_combine)
    assert gode.odeint.last_n_steps < n_tight


@pytest.mark.parametrize("method", list(gode.ADAPTIVE_METHODS))
@pytest.mark.parametrize("tol", [1e-3, 1e-6])
def test_adaptive_solvers_match_oracle_restatement(method, tol):
    """The integrator's adaptive loop (tableau, controller, non-FSAL handling, dense
    output) against the oracle's independent float64 restatement: identical step
    sequence, values to rounding; the oracle itself converges to the exact flow."""
    import scipy.linalg
    rng = np.random.default_rng(5)
    A = rng.standard_normal((6, 6)) * 0.5
    y0 = rng.standard_normal(6)
    ts = [0.0, 0.3, 1.0, 2.5]
    want, n_want = O.odeint_adaptive(lambda t, y: y @ A.T, y0, ts, method, tol, tol * 0.1)
    got = gode.odeint(lambda t, y: y @ torch.from_numpy(A).T, torch.from_numpy(y0),
                      torch.tensor(ts, dtype=torch.float64), method=method, rtol=tol, atol=tol * 0.1,
                      combine=gode._torch_combine).numpy()
    assert gode.odeint.last_n_steps == n_want
    assert np.abs(got - want).max() <= 1e-12
    exact = np.stack([scipy.linalg.expm(A * t) @ y0 for t in ts])
    if tol == 1e-6:
        assert np.abs(want - exact).max() <= 2e-3


def test_unknown_method_raises():
    with pytest.raises(NotImplementedError):
        gode.odeint(lambda t, y: y, torch.ones(2), torch.tensor([0., 1.]), method='implicit_adams',
                    combine=gode._torch_combine)


# ---------------------------------------------------------------- K2 edge-block plan (host C++, no GPU)
@pytest.mark.parametrize("eb", [8, 32, 64])
def test_seg_plan_build_tiles_edges(eb):
    """gnpde_seg_plan_build: items and chunks tile every edge once, whole-group
    items hold consecutive whole groups within eb edges, chunks split only
    groups longer than eb, and heavy lists exactly those groups."""
    import ctypes
    from gnpde import _lib
    rng = np.random.default_rng(eb)
    deg = rng.integers(0, 12, size=3000)
    deg[rng.integers(0, 3000, size=40)] = rng.integers(eb + 1, 5 * eb, size=40)
    deg[:5] = 0
    rp = np.zeros(len(deg) + 1, np.int32)
    rp[1:] = np.cumsum(deg)
    R, nnz = len(deg), int(rp[-1])
    cap_i, cap_c, cap_h = R, nnz // eb + R + 1, nnz // eb + 2
    items, chunks, heavy = (np.zeros((c, 4), np.int32) for c in (cap_i, cap_c, cap_h))
    ni, nc, nh = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.call("gnpde_seg_plan_build", rp.ctypes.data, R, eb, items.ctypes.data, cap_i, chunks.ctypes.data, cap_c,
              heavy.ctypes.data, cap_h, ctypes.byref(ni), ctypes.byref(nc), ctypes.byref(nh))
    it, ch, hv = items[:ni.value], chunks[:nc.value], heavy[:nh.value]
    spans = np.concatenate([it[:, :2], ch[:, :2]])
    spans = spans[np.argsort(spans[:, 0])]
    assert spans[0, 0] == 0 and spans[-1, 1] == nnz and (spans[1:, 0] == spans[:-1, 1]).all()
    assert ((spans[:, 1] - spans[:, 0]) <= eb).all() and ((spans[:, 1] - spans[:, 0]) > 0).all()
    starts = set(rp.tolist())
    assert all(b in starts and e in starts for b, e in it[:, :2])
    assert (it[:, 2] == -1).all() and (rp[it[:, 3]] == it[:, 0]).all()
    assert sorted(hv[:, 0].tolist()) == np.nonzero(deg > eb)[0].tolist()
    assert (ch[:, 2] == np.arange(len(ch))).all()
    for g, first, n, _ in hv:
        assert (ch[first:first + n, 3] == g).all() and ch[first, 0] == rp[g] and ch[first + n - 1, 1] == rp[g + 1]
    # greedy packing: no two consecutive whole-group items could have been merged
    for a, b in zip(it[:-1], it[1:]):
        if a[1] == b[0]:
            first_len = rp[b[3] + 1] - b[0]
            assert a[1] - a[0] + first_len > eb


def test_reference_statistics_plan_hub_chunks():
    """gnpde.ops.build_seg_plan(long_items=True) (host only; the plan of the
    reference statistics, ABI 4): groups over seg_long_max() edges become
    seg_long_max()-edge HUB CHUNK items {e_begin, e_end, slot, hub} at the front
    (longest hub first, chunks of a hub consecutive and tiling it), the hub table
    {group, first_slot, n_chunks, 0} indexes them, groups of eb+1..seg_long_max()
    edges are LONG items {.., -2, group} longest first, the rest whole-group items;
    every edge is covered once."""
    from gnpde import ops
    L = ops.seg_long_max()
    eb = 64
    rng = np.random.default_rng(5)
    deg = rng.integers(0, 20, size=4000)
    deg[[7, 100, 2500]] = [3 * L + 17, L + 1, 5 * L]  # hubs
    deg[[11, 12]] = [L, eb + 1]                      # long items at both ends of the range
    rp = np.zeros(len(deg) + 1, np.int32)
    rp[1:] = np.cumsum(deg)
    plan = ops.build_seg_plan(torch.from_numpy(rp), eb, long_items=True)
    it = plan.items.numpy().reshape(-1, 4)[:plan.n_items]
    hv = plan.heavy.numpy().reshape(-1, 4)[:plan.n_heavy]
    nh, nl = plan.n_hub, plan.n_long
    assert plan.n_chunk == 0 and plan.n_slots == nh
    assert hv[:, 0].tolist() == [2500, 7, 100]  # longest hub first
    assert (hv[:, 3] == 0).all() and hv[:, 2].tolist() == [5, 4, 2]
    for k, (grp, first, nch, _) in enumerate(hv):
        ch = it[first:first + nch]
        assert (ch[:, 2] == np.arange(first, first + nch)).all() and (ch[:, 3] == k).all()
        assert ch[0, 0] == rp[grp] and ch[-1, 1] == rp[grp + 1] and (ch[1:, 0] == ch[:-1, 1]).all()
        assert ((ch[:, 1] - ch[:, 0]) <= L).all()
    assert hv[0, 1] == 0 and (hv[1:, 1] == hv[:-1, 1] + hv[:-1, 2]).all() and hv[-1, 1] + hv[-1, 2] == nh
    lg = it[nh:nh + nl]
    ln = lg[:, 1] - lg[:, 0]
    assert (lg[:, 2] == -2).all() and (ln > eb).all() and (ln <= L).all() and (np.diff(ln) <= 0).all()
    assert {11, 12} <= set(lg[:, 3].tolist())
    sh = it[nh + nl:]
    assert (sh[:, 2] == -1).all() and ((sh[:, 1] - sh[:, 0]) <= eb).all()
    spans = it[:, :2][np.argsort(it[:, 0], kind="stable")]
    assert spans[0, 0] == 0 and spans[-1, 1] == rp[-1] and (spans[1:, 0] == spans[:-1, 1]).all()


def test_rk4_adjoint_reformulation_is_the_same_algebra():
    """The rk4 adjoint launches (integrator._LaplacianFixedGridFn.backward) form
    gk2 from gk3, gk1 from gk2 and carry g in the running sum, so that each launch
    reads few rows; restated with the (A^T - I) applications as free vectors, the
    combinations equal the textbook adjoint of the 3/8 rule (float64)."""
    rng = np.random.default_rng(3)
    g, v, u3, u2, u1 = (rng.standard_normal(50) for _ in range(5))
    a, dt = 0.37, 0.25
    c8, ad = dt / 8.0, dt * a
    u4 = c8 * v
    # textbook
    gk3 = 3 * c8 * g + ad * u4
    gk2 = 3 * c8 * g - ad * u4 + ad * u3
    gk1 = c8 * g + ad * u4 - ad / 3 * u3 + ad / 3 * u2
    g_new = g + a * (u4 + u3 + u2 + u1)
    # as launched (coefficients without a, times the device scale a)
    gk3_l = 3 * c8 * g + a * (dt * c8) * v
    gk2_l = gk3_l + a * dt * u3 + a * (-2.0 * dt * c8) * v
    gk1_l = gk2_l / 3.0 + a * (dt / 3.0) * u2 + a * (4.0 * dt * c8 / 3.0) * v + a * (-2.0 * dt / 3.0) * u3
    acc = g + a * u2 + a * c8 * v + a * u3
    g_new_l = acc + a * u1
    for x, y in ((gk3, gk3_l), (gk2, gk2_l), (gk1, gk1_l), (g_new, g_new_l)):
        assert np.allclose(x, y, rtol=1e-13, atol=1e-13)


# ---------------------------------------------------------------- ODE-block module layout (reference state_dict)
@pytest.mark.parametrize("block,extra", [("constant", {}), ("attention", {}), ("mixed", dict(heads=1)),
                                         ("hard_attention", dict(att_samp_pct=0.5))])
def test_block_builds_two_odefuncs_like_reference(block, extra):
    """src/base_classes.py:40,43 wraps a first ODEFunc in reg_odefunc; the block then
    builds its own (src/block_constant.py:11, block_transformer_attention.py:11,
    block_mixed.py:12, block_transformer_hard_attention.py:11).  A reference
    state_dict whose two copies differ loads so that the integrated RHS is odefunc.*."""
    opt = dict(OPT, block=block, **extra)
    cls = gnpde.set_block(opt)
    blk = cls(gnpde.LaplacianODEFunc, [], opt, None, t=torch.tensor([0, 1]))
    assert blk.odefunc is not blk.reg_odefunc.odefunc
    sd = blk.state_dict()
    assert 'odefunc.alpha_train' in sd and 'reg_odefunc.odefunc.alpha_train' in sd
    sd = {k: v.clone() for k, v in sd.items()}
    sd['odefunc.alpha_train'].fill_(0.7)
    sd['reg_odefunc.odefunc.alpha_train'].fill_(-3.0)
    sd['odefunc.beta_train'].fill_(0.2)
    blk.load_state_dict(sd)
    assert blk.odefunc.alpha_train.item() == pytest.approx(0.7)
    assert blk.reg_odefunc.odefunc.alpha_train.item() == pytest.approx(-3.0)
    # the solver integrates self.odefunc (src/block_constant.py:31 in eval): spy integrator
    seen = []

    def spy(func, y, t, **kw):
        seen.append(func)
        return torch.stack([y, y], 0)

    blk.eval()
    blk.test_integrator = spy
    blk.odefunc.attention_weights = torch.ones(1, 4)
    blk._integrate(torch.ones(1, 3, 6), {'step_size': 1})
    assert seen == [blk.odefunc]


def test_reset_graph_data_sets_both_copies_and_fp32():
    """reset_graph_data (src/base_classes.py:86-89) hands the same graph to both copies;
    set_x0 (:53-55) both x0s; the weights are fp32 whatever the state dtype."""
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], OPT, None, t=torch.tensor([0, 1]))
    data = gnpde.GraphData()
    data.new_graph(torch.tensor([[[0, 2, 2, 1], [1, 0, 1, 2]]]), 3)
    blk.reset_graph_data(data, torch.bfloat16)
    assert blk.odefunc.edge_weight.dtype == torch.float32
    assert blk.reg_odefunc.odefunc.edge_index is blk.odefunc.edge_index
    assert blk.reg_odefunc.odefunc.edge_weight is blk.odefunc.edge_weight
    blk.set_x0(torch.ones(1, 3, 6))
    assert blk.odefunc.x0 is not None and blk.reg_odefunc.odefunc.x0 is not None


def test_tensor_key_is_identity_not_address():
    """the derived-data caches must not confuse a freed tensor with a
    new one allocated at the same address."""
    from gnpde._cache import _tensor_key
    a = torch.zeros(4)
    ka = _tensor_key(a)
    b = torch.zeros(4)
    assert ka != _tensor_key(b) and ka == _tensor_key(a)
    a.add_(1)
    assert ka != _tensor_key(a)


@pytest.mark.parametrize("method", list(gode.ADAPTIVE_METHODS))
@pytest.mark.parametrize("tol", [1e-3, 1e-7])
def test_fused_adaptive_plan_matches_the_tableau_loop(method, tol):
    """The fused adaptive step (integrator._AdaptivePlan: each stage input, y1 and the
    error estimate formed in the RHS epilogues from the operands the plan picks, the
    error norm from per-row terms, dense output as two stage passes) against the
    tableau loop (_RKAdaptive) in float64 on CPU: the same step sequence and the same
    values to rounding, several output times inside one step included."""
    from host_stage import HostLinearRHS
    rng = np.random.default_rng(7)
    C = 6
    A = torch.from_numpy(rng.standard_normal((C, C)) * 0.7)
    y0 = torch.from_numpy(rng.standard_normal((1, 40, C)))
    ts = torch.tensor([0.0, 0.01, 0.02, 0.3, 1.0, 2.5], dtype=torch.float64)
    want = gode.odeint(lambda t, y: y @ A.T, y0, ts, method=method, rtol=tol, atol=tol * 0.1,
                       combine=gode._torch_combine)
    n_want = gode.odeint.last_n_steps
    f = HostLinearRHS(A)
    with torch.no_grad():  # the fused paths are the no-grad ones
        got = gode.odeint(f, y0, ts, method=method, rtol=tol, atol=tol * 0.1, combine=gode._Combine())
    assert gode.odeint.last_n_steps == n_want
    assert float((got - want).abs().max()) <= 1e-11 * max(1.0, float(want.abs().max()))
    P = gode._adaptive_plan(method)
    assert f.nfe == 2 + P.ns * n_want  # f0, the initial-step probe, then len(alpha) per step
    assert f.n_stage == P.ns * n_want  # every stage through the fused epilogue


def test_fused_adaptive_plan_dopri5_operands():
    """dopri5's plan: every stage input from the launch's own input (no y0 read), the
    error's first six terms precomputed by the launch that forms y1 (a second
    output), so the FSAL launch reads only that partial and y0; k5 is stored only on
    steps that may cross an output time (dense output)."""
    P = gode._adaptive_plan('dopri5')
    assert P.fsal and P.ns == 6
    assert all(L['next'][0] == 'X' for L in P.launches[:5])
    assert P.launches[4]['epart'] is not None and P.launches[5]['err'][0] == 'E'
    assert P.reads[5] == set()
    assert P.store == {1, 2, 3, 4, 6} and P.store_mid == {5}


def test_krylov_plan_dopri5_coefficients():
    """_KrylovPlan (the affine dopri5 step in the basis u_p = (dt L)^p f0): y1's
    coefficients are the exponential's 1/(p+1)! through the method's order, the
    error combination vanishes below the embedded order (exact zeros, no
    cancellation left to the fp32 sums), f1 = sum_p B[6][p] u_p is the stage
    derivative at y1 (FSAL: B[6] = [1] + G[:6] shifted)."""
    import math
    K = gode._KrylovPlan(gode._adaptive_plan('dopri5'))
    for p in range(5):
        assert abs(K.G[p] - 1.0 / math.factorial(p + 1)) < 1e-15
    assert K.G[6] == 0.0
    assert K.Eps[:4] == [0.0, 0.0, 0.0, 0.0] and all(K.Eps[p] != 0.0 for p in (4, 5, 6))
    assert K.Bn[0] == 1.0 and all(abs(K.Bn[p + 1] - K.G[p]) < 1e-15 for p in range(6))
    y1, (ft, fcf), (et, ecf) = K.last_launch_terms()
    assert [p for p, _ in et] == [4, 5] and ecf == K.Eps[6]
    assert len({p for p, _ in y1} | {p for p, _ in ft}) <= 6  # u_0 .. u_5: the stage's operand table


@pytest.mark.parametrize("tol", [1e-3, 1e-7])
def test_krylov_step_matches_stage_step(monkeypatch, tol):
    """The fused dopri5 solve of an affine RHS with the Krylov step (default) and
    with the stage-combination plan (GNPDE_KRYLOV_STEP=0): the same accepted step
    sequence and the same values to fp64 rounding, dense outputs included."""
    from host_stage import HostLinearRHS
    rng = np.random.default_rng(11)
    C = 5
    A = torch.from_numpy(rng.standard_normal((C, C)) * 0.9)
    y0 = torch.from_numpy(rng.standard_normal((1, 30, C)))
    ts = torch.tensor([0.0, 0.05, 0.7, 2.0], dtype=torch.float64)
    runs = []
    for kry in (True, False):
        monkeypatch.setattr(gode, "KRYLOV_STEP", kry)
        f = HostLinearRHS(A)
        with torch.no_grad():
            got = gode.odeint(f, y0, ts, method='dopri5', rtol=tol, atol=tol * 0.1, combine=gode._Combine())
        runs.append((got, gode.odeint.last_n_steps, f.nfe))
    (a, na, fa), (b, nb, fb) = runs
    assert na == nb and fa == fb
    assert float((a - b).abs().max()) <= 1e-11 * max(1.0, float(b.abs().max()))


def test_krylov_step_selection():
    """The Krylov step is taken for an affine RHS under dopri5 (FSAL, every k kept);
    bosh3 (its k2 not kept), the non-FSAL pairs, a non-affine RHS and
    GNPDE_KRYLOV_STEP=0 keep the stage plan."""
    from host_stage import HostLinearRHS
    A = torch.eye(3, dtype=torch.float64)
    y0 = torch.zeros(1, 4, 3, dtype=torch.float64)
    comb = gode._Combine()

    def solver(method, func):
        return gode._RKAdaptiveFused(func, y0, 1e-6, 1e-8, comb, method=method)
    assert solver('dopri5', HostLinearRHS(A)).krylov is not None
    for m in ('bosh3', 'fehlberg2', 'adaptive_heun'):
        assert solver(m, HostLinearRHS(A)).krylov is None, m

    class NotAffine(HostLinearRHS):
        affine = False
    assert solver('dopri5', NotAffine(A)).krylov is None
    old = gode.KRYLOV_STEP
    try:
        gode.KRYLOV_STEP = False
        assert solver('dopri5', HostLinearRHS(A)).krylov is None
    finally:
        gode.KRYLOV_STEP = old


@pytest.mark.parametrize("method", ["dopri5", "bosh3"])
def test_dense_fold_table_matches_host_interpolant(method):
    """The folded dense output's basis table (integrator._RKAdaptiveFused._dense_table, ABI 8
    dense_m) evaluated at a step's theta and dt — the combination the K1 epilogue forms
    (csrc dense_coefs) — equals the interpolant the separate pass forms (_interp_into's
    Krylov branch: y0, the u_p and f1 = sum_p f1_p u_p + fcf f'), coefficient by coefficient,
    and reproduces torchdiffeq's quartic on random u_p (a float64 restatement of the oracle's
    _interp_fit on the same step)."""
    P = gode._adaptive_plan(method)
    K = gode._krylov_plan(P)
    ns = K.ns
    rng = np.random.default_rng(7)
    u = [rng.standard_normal(5) for _ in range(ns + 1)]  # u_0 .. u_ns (u_ns = (dt L) u_{ns-1})
    y0 = rng.standard_normal(5)
    fp = u[ns - 1] + u[ns]  # f' of the last launch (f_lin = 1)
    y1t, (ft, fcf), _ = K.last_launch_terms()
    fake = gode._RKAdaptiveFused.__new__(gode._RKAdaptiveFused)
    fake.krylov, fake.plan = K, P
    keys = ["u%d" % p for p in range(ns)]
    table = fake._dense_table(keys, ft, fcf)
    for theta, dt in ((0.3, 0.7), (0.85, 1.9), (1.0, 0.25)):
        x2, x3, x4 = theta ** 2, theta ** 3, theta ** 4
        cy0 = 1 - 11 * x2 + 18 * x3 - 8 * x4
        cy1 = -5 * x2 + 14 * x3 - 8 * x4
        cym = 16 * x2 - 32 * x3 + 16 * x4
        cf0 = dt * (theta - 4 * x2 + 5 * x3 - 2 * x4)
        cf1 = dt * (x2 - 3 * x3 + 2 * x4)
        w = [cy0 + cy1 + cym, dt * cy1, dt * cym, cf0, cf1]
        coef = lambda key: sum(wm * c for wm, c in zip(w, table.get(key, [0.0] * 5)))  # noqa: E731
        dense = coef('base') * y0 + sum(coef(k) * u[p] for p, k in enumerate(keys)) + coef('f') * fp
        # the host pass: y1, y_mid and f1 from the u_p, then the quartic
        y1 = y0 + dt * sum(K.G[p] * u[p] for p in range(ns))
        f1 = sum(c * u[p] for p, c in ft) + fcf * fp
        ymid = y0 + dt * (sum(K.Mu[p] * u[p] for p in range(ns)) + P.c_mid[ns] * f1)
        want = cy0 * y0 + cy1 * y1 + cym * ymid + cf0 * u[0] + cf1 * f1
        assert np.allclose(dense, want, rtol=1e-12, atol=1e-12)
        # torchdiffeq's _interp_fit form (oracle.odeint_adaptive): the same polynomial
        p4 = 2 * dt * (f1 - u[0]) - 8 * (y1 + y0) + 16 * ymid
        p3 = dt * (5 * u[0] - 3 * f1) + 18 * y0 + 14 * y1 - 32 * ymid
        p2 = dt * (f1 - 4 * u[0]) - 11 * y0 - 5 * y1 + 16 * ymid
        quartic = y0 + theta * (dt * u[0]) + x2 * p2 + x3 * p3 + x4 * p4
        assert np.allclose(dense, quartic, rtol=1e-12, atol=1e-12)
