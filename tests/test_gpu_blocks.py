"""GPU: ODE blocks end to end — the reference's module layout (two ODEFunc
copies), graph normalisation (rw and gcn) on the device, bf16 state, and the
integrator's captured-graph cache across solves, graphs and forwards
(a replay must never read a buffer the module has since rebuilt).

Tolerances: fp32 1e-5 relative (north star); bf16 state 2e-2 against the fp32
oracle (SURVEY §8(d) parity gate for C4)."""
import numpy as np
import pytest
import torch

import gnpde
import gnpde_oracle as O
from test_gpu_parity import DEV, OPT, RTOL, T, _prep_oracle, rel

pytestmark = pytest.mark.gpu


def _graph(N, E, seed):
    rng = np.random.default_rng(seed)
    ei = rng.integers(0, N, size=(1, 2, E))
    ei[0, 0, :600] = 7  # a hub row: split plan, in-launch combine
    return ei, rng


def test_block_state_dict_two_copies_rhs_uses_odefunc():
    """A reference state_dict whose odefunc.* and reg_odefunc.odefunc.* differ:
    the integration uses odefunc.* (src/block_constant.py:31) and
    odefunc.nfe + reg_odefunc.odefunc.nfe (GNN.getNFE, src/base_classes.py:174-176)
    counts every RHS evaluation once."""
    N, E, C = 1500, 9000, 32
    ei, rng = _graph(N, E, 101)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    opt = dict(OPT, hidden_dim=C, method='euler', step_size=0.1, add_source=True)
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).eval()
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    sd['odefunc.alpha_train'].fill_(0.4)
    sd['odefunc.beta_train'].fill_(0.3)
    sd['reg_odefunc.odefunc.alpha_train'].fill_(-2.0)
    sd['reg_odefunc.odefunc.beta_train'].fill_(5.0)
    blk.load_state_dict(sd)
    data = gnpde.GraphData()
    data.new_graph(T(ei), N)
    blk.set_x0(T(x))
    with torch.no_grad():
        z = blk(T(x), data)
    eo, wo = _prep_oracle(ei, N)
    f = lambda t, y: O.laplacian_rhs(eo, y, x, 0.4, 0.3, edge_weight=wo, add_source=True)  # noqa: E731
    assert rel(z, O.odeint_fixed(f, x, 0.0, 1.0, 'euler', 0.1)) <= RTOL
    assert blk.odefunc.nfe + blk.reg_odefunc.odefunc.nfe == 10


@pytest.mark.parametrize("norm", ["rw", "gcn"])
@pytest.mark.parametrize("method,step", [("euler", 0.2), ("rk4", 0.25)])
def test_constant_block_data_norm_vs_oracle(norm, method, step):
    """ConstantODEblock with data_norm rw / gcn (src/base_classes.py:73-82; gcn =
    src/utils.py:177-194, KAT test/test_function_laplacian_diffusion.py:73-85)."""
    N, E, C = 2708, 10556, 80
    ei, rng = _graph(N, E, 102)
    ei[0, 1, :50] = ei[0, 0, :50]  # existing self loops keep their weight
    w = rng.uniform(0.2, 2.0, size=(1, E)).astype(np.float32)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    opt = dict(OPT, hidden_dim=C, method=method, step_size=step, data_norm=norm, self_loop_weight=1.0)
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).eval()
    with torch.no_grad():
        blk.odefunc.alpha_train.fill_(0.6)
    data = gnpde.GraphData()
    data.new_graph(T(ei), N, edge_attr=T(w))
    with torch.no_grad():
        z = blk(T(x), data)
    if norm == "rw":
        eis, ws = O.get_rw_adj(ei, edge_weight=w, norm_dim=1, fill_value=1.0, num_nodes=N)
    else:
        eis, ws = O.gcn_norm_fill_val(ei, edge_weight=w, fill_value=1.0, num_nodes=N)
    eo, wo = np.stack(eis, 0), np.stack(ws, 0)
    got_w = blk.odefunc.edge_weight.double().cpu().numpy()
    assert np.array_equal(blk.odefunc.edge_index.cpu().numpy(), eo)
    assert np.abs(got_w - wo).max() <= 1e-6 * np.abs(wo).max()
    f = lambda t, y: O.laplacian_rhs(eo, y, None, 0.6, 0.0, edge_weight=wo)  # noqa: E731
    assert rel(z, O.odeint_fixed(f, x, 0.0, 1.0, method, step)) <= RTOL


@pytest.mark.parametrize("C", [64, 162])
def test_constant_block_bf16_state_vs_oracle(C):
    """bf16 state through the block (configs[3] storage): fp32 weights from
    reset_graph_data, bf16 K1, fixed-grid fused stages."""
    N, E = 3000, 20000
    ei, rng = _graph(N, E, 103)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    opt = dict(OPT, hidden_dim=C, method='rk4', step_size=0.25)
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).eval()
    data = gnpde.GraphData()
    data.new_graph(T(ei), N)
    with torch.no_grad():
        z = blk(T(x).to(torch.bfloat16), data)
    assert z.dtype == torch.bfloat16 and blk.odefunc.edge_weight.dtype == torch.float32
    eo, wo = _prep_oracle(ei, N)
    f = lambda t, y: O.laplacian_rhs(eo, y, None, 0.0, 0.0, edge_weight=wo)  # noqa: E731
    xb = T(x).to(torch.bfloat16).double().cpu().numpy()
    assert rel(z, O.odeint_fixed(f, xb, 0.0, 1.0, 'rk4', 0.25)) <= 2e-2


def test_graph_cache_survives_solve_on_another_graph():
    """rk4 on graph A captures; a dopri5 solve on graph B makes
    the module rebuild its CSR and weights; rk4 on A again must not replay
    graphs that read B's (or freed) buffers.  Bitwise against eager solves."""
    import gnpde.integrator as integ
    N, E, C = 2500, 15000, 32
    eiA, rng = _graph(N, E, 104)
    eiB = rng.integers(0, N, size=(1, 2, E))
    x = T(rng.standard_normal((1, N, C)).astype(np.float32))
    opt = dict(OPT, hidden_dim=C, max_nfe=10 ** 7)
    (eA, wA), (eB, wB) = _prep_oracle(eiA, N), _prep_oracle(eiB, N)
    t = torch.tensor([0.0, 1.0], device=DEV)
    func = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
    ref = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
    tA, tB = (T(eA), T(wA).float()), (T(eB), T(wB).float())

    def rk4(f, graph):
        with torch.no_grad():
            return gnpde.odeint(f, x, t, method='rk4', options={'step_size': 0.0625, 'gnpde_graph': graph})[1]

    func.edge_index, func.edge_weight = tA
    first = rk4(func, True)
    entry = integ._GRAPH_CACHE[func]
    func.edge_index, func.edge_weight = tB
    with torch.no_grad():
        gnpde.odeint(func, x, t, method='dopri5', rtol=1e-4, atol=1e-5)
    torch.cuda.synchronize()
    func.edge_index, func.edge_weight = tA
    again = rk4(func, True)
    ref.edge_index, ref.edge_weight = tA
    want = rk4(ref, False)
    torch.cuda.synchronize()
    assert torch.equal(first, want) and torch.equal(again, want)
    assert integ._GRAPH_CACHE[func] is not entry  # A's graph was rebuilt: recaptured, not replayed


def test_attention_block_eval_replays_across_forwards():
    """the attention block hands a new attention_weights tensor
    to the RHS every forward; the CSR-order weights are refreshed in place, so
    the second eval forward replays the cached step graphs and still matches an
    eager solve bitwise."""
    import gnpde.integrator as integ
    N, E, C, h, att = 2000, 12000, 32, 2, 16
    ei, rng = _graph(N, E, 105)
    opt = dict(OPT, hidden_dim=C, heads=h, attention_dim=att, block='attention', attention_norm_idx=1,
               method='rk4', step_size=0.1, max_nfe=10 ** 7)
    blk = gnpde.AttODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).eval()
    lay = blk.multihead_att_layer
    with torch.no_grad():
        for lin in (lay.Q, lay.K):
            lin.weight.copy_(torch.randn_like(lin.weight) * 0.1)
            lin.bias.copy_(torch.randn_like(lin.bias) * 0.1)
    data = gnpde.GraphData()
    data.new_graph(T(ei), N)
    xs = [T(rng.standard_normal((1, N, C)).astype(np.float32)) for _ in range(2)]
    with torch.no_grad():
        blk(xs[0], data)
        entry = integ._GRAPH_CACHE[blk.odefunc]
        z = blk(xs[1], data)
        assert integ._GRAPH_CACHE[blk.odefunc] is entry
        eager = gnpde.odeint(blk.odefunc, xs[1], torch.tensor([0.0, 1.0], device=DEV), method='rk4',
                             options={'step_size': 0.1, 'gnpde_graph': False})[1]
    torch.cuda.synchronize()
    assert torch.equal(z, eager)
    eo, wo = _prep_oracle(ei, N)
    attn = O.transformer_attention(xs[1].cpu().numpy(), eo, lay.Q.weight.detach().cpu().numpy(),
                                   lay.Q.bias.detach().cpu().numpy(), lay.K.weight.detach().cpu().numpy(),
                                   lay.K.bias.detach().cpu().numpy(), h, 1)
    f = lambda t, y: O.laplacian_rhs(eo, y, None, 0.0, 0.0, block='attention', attention_weights=attn)  # noqa
    assert rel(z, O.odeint_fixed(f, xs[1].cpu().numpy(), 0.0, 1.0, 'rk4', 0.1)) <= RTOL


def test_add_source_new_x0_each_forward_replays_with_new_x0():
    """set_x0 clones x0 every forward (src/base_classes.py:53-55): the stable x0
    buffer is refreshed in place, the cached graphs replay, and the result
    follows the new x0."""
    import gnpde.integrator as integ
    N, E, C = 2000, 12000, 16
    ei, rng = _graph(N, E, 106)
    opt = dict(OPT, hidden_dim=C, method='rk4', step_size=0.125, add_source=True, max_nfe=10 ** 7)
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).eval()
    with torch.no_grad():
        blk.odefunc.beta_train.fill_(0.5)
    data = gnpde.GraphData()
    data.new_graph(T(ei), N)
    x = T(rng.standard_normal((1, N, C)).astype(np.float32))
    with torch.no_grad():
        blk.set_x0(x)
        blk(x, data)
        entry = integ._GRAPH_CACHE[blk.odefunc]
        x0b = torch.randn_like(x)
        blk.set_x0(x0b)
        z = blk(x, data)
    assert integ._GRAPH_CACHE[blk.odefunc] is entry
    eo, wo = _prep_oracle(ei, N)
    xn, x0n = x.cpu().numpy(), x0b.cpu().numpy()
    f = lambda t, y: O.laplacian_rhs(eo, y, x0n, 0.0, 0.5, edge_weight=wo, add_source=True)  # noqa: E731
    assert rel(z, O.odeint_fixed(f, xn, 0.0, 1.0, 'rk4', 0.125)) <= RTOL


@pytest.mark.parametrize("fn,kw", [("get_rw_adj", dict(norm_dim=1)), ("get_rw_adj", dict(norm_dim=0)),
                                   ("gcn_norm_fill_val", {})])
@pytest.mark.parametrize("weighted", [None, "frac", "int", "bigint"])
def test_graph_normalisation_kernels_bit_exact_vs_host(fn, kw, weighted):
    """csrc/prep.hip (self loops + rw / gcn weights) equals the host restatement
    in gnpde.utils bit for bit: same edge order, the node's last existing loop
    weight, degrees added in COO order (= torch's CPU scatter_add_); and the
    fp64 oracle within fp32 rounding.  Batched, duplicated edges, repeated
    loops on one node, an isolated node, hub rows and columns longer than one
    wavefront (degree_long_kernel: the parallel sum for integral weights below
    2^24 — unit and small integer weights — the in-order sum for fractional ones
    and for integers whose sum reaches 2^24, where the order changes the bits)."""
    from gnpde import utils as gu
    rng = np.random.default_rng(107)
    B, N, E = 2, 500, 4000
    ei = rng.integers(0, N - 1, size=(B, 2, E))  # node N-1 isolated
    loop = ei[:, 0] == ei[:, 1]
    ei[:, 1][loop] = (ei[:, 1][loop] + 1) % (N - 1)  # no random loops: equal non-loop counts per batch element
    ei[:, 0, :30] = 4
    ei[:, 1, :30] = 4  # 30 loops on node 4 with different weights: the last one wins
    ei[:, :, 100:200] = ei[:, :, 200:300]  # duplicates
    ei[:, 0, 300:1300] = 7  # a hub row and a hub column (1000 edges)
    ei[:, 1, 1300:2300] = 9
    ei[:, 1, 300:1300][ei[:, 1, 300:1300] == 7] = 8
    ei[:, 0, 1300:2300][ei[:, 0, 1300:2300] == 9] = 8
    w = {None: None,
         "frac": lambda: rng.uniform(0.1, 2.0, size=(B, E)),
         "int": lambda: rng.integers(1, 5, size=(B, E)),
         "bigint": lambda: rng.integers(1, 2 ** 20, size=(B, E))}[weighted]
    w = None if w is None else w().astype(np.float32)
    # an integral loop fill keeps integral rows integral (the parallel path)
    args = dict(fill_value=1.5 if weighted == "frac" else 2.0, num_nodes=N, **kw)
    ge, gw = getattr(gu, fn)(T(ei), edge_weight=None if w is None else T(w), **args)
    he, hw = getattr(gu, fn)(torch.from_numpy(ei), edge_weight=None if w is None else torch.from_numpy(w), **args)
    assert torch.equal(ge.cpu(), he)
    assert torch.equal(gw.cpu(), hw), float((gw.cpu() - hw).abs().max())
    ge2, gw2 = getattr(gu, fn)(T(ei), edge_weight=None if w is None else T(w), **args)
    assert torch.equal(gw2, gw)
    oe, ow = getattr(O, fn)(ei, edge_weight=w, **args)
    assert np.array_equal(ge.cpu().numpy(), np.stack(oe, 0))
    ow = np.stack(ow, 0)
    assert np.abs(gw.double().cpu().numpy() - ow).max() <= 1e-6 * np.abs(ow).max()


def test_k1_launches_on_two_streams_share_a_plan_safely():
    """the hub arrival tickets live in the plan, so launches on one
    plan must not overlap; ops orders a launch on another stream behind the
    plan's previous stream.  Alternating streams, results stay bit-identical to
    a single-stream run."""
    from gnpde import ops
    N, E, C = 4000, 60000, 128
    ei, rng = _graph(N, E, 108)
    ei[0, 0, :20000] = rng.integers(0, 12, 20000)  # many hub rows
    g = ops.GraphCSR(T(ei), N)
    assert g.csr.plan.n_heavy >= 10
    w = g.gather_weights(T(rng.uniform(0.1, 1, size=(1, E)).astype(np.float32)))
    xs = [torch.randn(N, C, device=DEV) for _ in range(6)]
    alpha = torch.tensor(0.3, device=DEV)
    want = [ops.spmm_rhs(g, w, x, alpha=alpha) for x in xs]
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for rep in range(4):
        for i, x in enumerate(xs):
            with torch.cuda.stream(streams[i % 2]):
                got.append((i, ops.spmm_rhs(g, w, x, alpha=alpha)))
    torch.cuda.synchronize()
    for i, f in got:
        assert torch.equal(f, want[i])
    assert int(g.csr.plan.heavy.view(-1, 4)[:g.csr.plan.n_heavy, 3].abs().sum()) == 0  # tickets back to 0


def test_reference_statistics_on_two_streams_share_a_plan_safely():
    """the statistics of the reference-score attention share
    one SegPlan between launches.  Its hub destination groups run as chunks with
    arrival tickets in the plan (round 4; round 3 ran them as 1024-thread
    workgroups without tickets), so launches on one plan are ordered across
    streams (ops._TicketOrder): the attention RHS (norm_idx 1, a destination hub)
    alternating between two streams stays bit-identical to a single-stream run,
    and every ticket is back at 0."""
    from gnpde import ops
    N, E, C, H, att = 4000, 60000, 64, 2, 32
    ei, rng = _graph(N, E, 109)
    ei[0, 1, :9000] = 7  # destination hub: 18 statistics chunks
    g = ops.GraphCSR(T(ei), N)
    Wq, Wk = [T((rng.standard_normal((att, C)) * 0.1).astype(np.float32)) for _ in range(2)]
    bq, bk = [T((rng.standard_normal(att) * 0.1).astype(np.float32)) for _ in range(2)]
    xs = [torch.randn(N, C, device=DEV).view(1, N, C) for _ in range(4)]
    alpha = torch.tensor(0.3, device=DEV)

    def rhs(x):
        ns = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'reference')
        return ops.attn_rhs(g, ns, None, None, 1, x, alpha=alpha)

    want = [rhs(x) for x in xs]
    torch.cuda.synchronize()
    sp = g.csc.seg_plan(ops._lib.fn("gnpde_seg_block_edges")(ops._lib.SCORE_REFERENCE, H, att // H), True)
    assert sp.n_hub >= 2 and sp.n_heavy >= 1
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    got = []
    for rep in range(3):
        for i, x in enumerate(xs):
            with torch.cuda.stream(streams[i % 2]):
                got.append((i, rhs(x)))
    torch.cuda.synchronize()
    for i, f in got:
        assert torch.equal(f, want[i])
    assert int(sp.heavy.view(-1, 4)[:sp.n_heavy, 3].abs().sum()) == 0  # tickets back to 0


def test_rows_copy_entry_pass():
    """gnpde_rows_copy (the solve entry): dst = src[order], dst_copy = src, one read."""
    from gnpde import ops
    for dt, C in ((torch.float32, 128), (torch.float32, 12), (torch.bfloat16, 168)):
        src = torch.randn(3, 1001, C, device=DEV).to(dt)
        order = torch.randperm(3 * 1001, device=DEV)
        dst, cpy = torch.empty_like(src), torch.empty_like(src)
        ops.rows_copy(src, dst, order=order, dst_copy=cpy)
        assert torch.equal(dst.view(-1, C), src.view(-1, C)[order])
        assert torch.equal(cpy, src)
        dst2 = torch.empty_like(src)
        ops.rows_copy(src, dst2)
        assert torch.equal(dst2, src)
