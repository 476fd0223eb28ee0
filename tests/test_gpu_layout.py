"""GPU: the integrator's locality numbering of the state (ops.NodeLayout).

A fixed-grid solve on a large graph runs in the graph's in-degree numbering
(gathered rows together at the front of the state) and permutes back once at
the end.  Every output row is summed over the same edges in the same order as
in the user numbering, so the result must be BIT-identical to the solve with
the layout disabled — checked here for euler / midpoint / rk4, add_source,
a batch of two graphs, the zero-padded width (C = 162) and a bf16 state — and
the layout must actually have been used (its graph built, its x0 buffer filled)."""
import pytest
import torch

import gnpde
from gnpde import ops, synthetic
from test_gpu_parity import DEV, OPT

pytestmark = pytest.mark.gpu


def _func(N, E, C, B, add_source, seed=0):
    eis, ws = [], []
    for b in range(B):
        ei, w = synthetic.rw_graph(N, E, seed=seed + b, device=DEV)
        eis.append(ei)
        ws.append(w)
    ei, w = torch.cat(eis, 0), torch.cat(ws, 0)
    opt = dict(OPT, hidden_dim=C, add_source=add_source)
    func = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
    with torch.no_grad():
        func.alpha_train.fill_(0.3)
        func.beta_train.fill_(0.7)
    func.edge_index, func.edge_weight = ei, w
    return func


def _solve(func, x, method, steps, h, order):
    saved = ops.NODE_ORDER
    ops.NODE_ORDER = order
    try:
        with torch.no_grad():
            t = torch.tensor([0.0, steps * h], device=DEV)
            return gnpde.odeint(func, x, t, method=method, options={'step_size': h})
    finally:
        ops.NODE_ORDER = saved


@pytest.mark.parametrize("method,steps", [("euler", 3), ("midpoint", 2), ("rk4", 9)])
@pytest.mark.parametrize("add_source", [False, True])
def test_layout_solve_bit_identical(method, steps, add_source):
    N, E, C = 40000, 300000, 128
    func = _func(N, E, C, 1, add_source)
    x = synthetic.features(1, N, C, seed=3, device=DEV)
    if add_source:
        func.x0 = synthetic.features(1, N, C, seed=4, device=DEV)
    ref = _solve(func, x, method, steps, 0.1, "none")
    got = _solve(func, x, method, steps, 0.1, "degree")
    assert func._layout is None  # released after the solve
    assert getattr(func._graph, '_layout', None) is not None  # ... and it was used
    if add_source:
        assert getattr(func, '_x0_buf_layout', None) is not None
    assert torch.equal(got, ref)
    # a second solve replays the captured steps of the layout graph: same bits again
    assert torch.equal(_solve(func, x, method, steps, 0.1, "degree"), ref)


def test_layout_batched_padded_and_bf16():
    N, E = 36000, 250000
    for C, dtype in ((162, torch.float32), (128, torch.bfloat16)):
        func = _func(N, E, C, 2, True, seed=11)
        x = synthetic.features(2, N, C, seed=5, device=DEV).to(dtype)
        func.x0 = synthetic.features(2, N, C, seed=6, device=DEV).to(dtype)
        ref = _solve(func, x, "rk4", 7, 0.2, "none")
        got = _solve(func, x, "rk4", 7, 0.2, "degree")
        assert torch.equal(got, ref), (C, dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layout_blend_transformer_bit_identical(dtype):
    """configs[3] shape: the transformer RHS with the fork's scaled_dot under
    source-grouped softmax (1/outdeg weights), C = 162 (zero-padded width)."""
    N, E, C = 60000, 450000, 162  # >= 16 MB in bf16 too (ops.LAYOUT_MIN_BYTES)
    ei, _ = synthetic.rw_graph(N, E, seed=31, device=DEV)
    opt = dict(OPT, hidden_dim=C, heads=2, attention_dim=32, attention_norm_idx=0, attention_type='scaled_dot',
               function='transformer', mix_features=False, square_plus=False, beltrami=False)
    func = gnpde.ODEFuncTransformerAtt(C, C, opt, DEV).to(DEV).eval()
    func.edge_index = ei
    x = synthetic.features(1, N, C, seed=8, device=DEV).to(dtype)
    lay = func.node_layout(x)
    assert lay is not None
    ref = _solve(func, x, "rk4", 7, 0.25, "none")
    got = _solve(func, x, "rk4", 7, 0.25, "degree")
    assert torch.equal(got, ref)
    # other attention types keep the user numbering
    opt2 = dict(opt, attention_norm_idx=1, attention_type='cosine_sim')
    f2 = gnpde.ODEFuncTransformerAtt(C, C, opt2, DEV).to(DEV).eval()
    f2.edge_index = ei
    assert f2.node_layout(x) is None


@pytest.mark.parametrize("mode,norm_idx", [("per_edge", 0), ("per_edge", 1), ("reference", 1)])
def test_layout_attention_scores(mode, norm_idx):
    """the scaled_dot score modes run fixed-grid solves in the
    in-degree numbering too, within the suite's 1e-5 of the user numbering (7e-6
    measured for per-edge norm_idx 1 over 7 rk4 steps: the softmax of scores in the
    tens amplifies last-bit differences; 1e-6 for one RHS): the fork's key sum
    (fp64 row tiles) and the destination statistics (packed CSC blocks) sum in
    another order, and in the fused per-edge kernel a row that shares its wavefront
    with a hub chunk accumulates per head (the items pair up differently in the
    other numbering's plan).  The fork's scores sum the keys of all E edges (q . S with
    S ~ E |k|): at the per-edge cases' weight scale they reach ~1e4 and the softmax is
    a hard arg-max whose choice a last-bit difference flips, so a solve is chaotic in
    either numbering (its single RHS is still bit-equal: tools/layout_diag.py); its
    weights are scaled so the scores stay O(1)."""
    N, E, C, h, att = 60000, 450000, 128, 2, 32
    wscale = 1e-3 if mode == "reference" else 0.1
    ei, _ = synthetic.rw_graph(N, E, seed=32, device=DEV)
    opt = dict(OPT, hidden_dim=C, heads=h, attention_dim=att, attention_norm_idx=norm_idx,
               attention_type='scaled_dot', attention_score_mode=mode, function='transformer', mix_features=False,
               square_plus=False, beltrami=False)
    func = gnpde.ODEFuncTransformerAtt(C, C, opt, DEV).to(DEV).eval()
    gen = torch.Generator(device=DEV)
    gen.manual_seed(9)
    with torch.no_grad():
        for lin in (func.multihead_att_layer.Q, func.multihead_att_layer.K):
            lin.weight.copy_(torch.randn(att, C, generator=gen, device=DEV) * wscale)
            lin.bias.copy_(torch.randn(att, generator=gen, device=DEV) * wscale)
        func.alpha_train.fill_(0.3)
    func.edge_index = ei
    x = synthetic.features(1, N, C, seed=8, device=DEV)
    assert func.node_layout(x) is not None
    ref = _solve(func, x, "rk4", 7, 0.25, "none")
    got = _solve(func, x, "rk4", 7, 0.25, "degree")
    assert getattr(func._graph, '_layout', None) is not None
    assert float((got - ref).abs().max() / ref.abs().max()) <= 1e-5
    # one RHS in either numbering
    x_int, lay = func.node_layout(x).to_internal(x), func.node_layout(x)
    with torch.no_grad():
        f_user = func(None, x)
        func._layout = lay
        try:
            f_int = func(None, x_int)
        finally:
            func._layout = None
    f_back = lay.to_user(f_int)
    assert float((f_back - f_user).abs().max() / f_user.abs().max()) <= 1e-6


def test_node_layout_structure():
    N, E = 40000, 300000
    func = _func(N, E, 128, 2, False, seed=21)
    x = synthetic.features(2, N, 128, seed=3, device=DEV)
    g = func.graph_for(x)
    lay = func.node_layout(x)
    assert lay is g.node_layout
    R = 2 * N
    ar = torch.arange(R, device=DEV)
    assert torch.equal(lay.new_id[lay.order], ar) and torch.equal(lay.order[lay.new_id], ar)
    # batch elements keep their row ranges; in-degree non-increasing inside each
    assert torch.equal(lay.order.view(2, N) // N, torch.arange(2, device=DEV).view(2, 1).expand(2, N))
    deg = g.indeg.long()[lay.order].view(2, N)
    assert bool((deg[:, 1:] <= deg[:, :-1]).all())
    # the relabelled graph has the same in-degree multiset, renumbered
    assert torch.equal(lay.graph.indeg.long(), g.indeg.long()[lay.order])
    y = torch.randn(2, N, 128, device=DEV)
    assert torch.equal(lay.to_user(lay.to_internal(y)), y)
    # small states are not renumbered
    small = _func(2000, 12000, 64, 1, False)
    assert small.node_layout(torch.zeros(1, 2000, 64, device=DEV)) is None


def test_layout_column_stripes_bit_identical():
    """gnpde.dist.ColumnShardedLaplacian (the multi-GPU headline layout) solves its
    stripe in the same numbering as the unsharded run: a world of one (gloo
    group, no collective on the fixed-grid path), layout on vs off vs the
    unsharded LaplacianODEFunc — all bit-identical."""
    import random
    import torch.distributed as dist
    from gnpde import dist as gd
    N, E, C = 40000, 300000, 128
    ei, w = synthetic.rw_graph(N, E, seed=41, device=DEV)
    x = synthetic.features(1, N, C, seed=9, device=DEV)
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % random.randint(20000, 40000), rank=0,
                                world_size=1)
    try:
        alpha = torch.tensor(0.3, device=DEV)
        sh = gd.ColumnShardedLaplacian(ei, w, N, C, alpha)
        assert sh.node_layout(sh.split(x)) is not None
        ref = _solve(sh, sh.split(x), "rk4", 9, 0.1, "none")
        got = _solve(sh, sh.split(x), "rk4", 9, 0.1, "degree")
        assert sh._layout is None and sh._lay_ops is not None
        assert torch.equal(got, ref)
        func = _func(N, E, C, 1, False, seed=41)
        assert torch.equal(_solve(func, x, "rk4", 9, 0.1, "degree"), ref)
    finally:
        if own:
            dist.destroy_process_group()
