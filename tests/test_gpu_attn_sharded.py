"""GPU: the transformer attention RHS sharded (gnpde.dist, SURVEY.md §8(e),
VERDICT r3 item 3) on the G-arxiv graph (N = 169,343, E' = 1.2M, C = 128, heads 2,
attention_dim 32 — configs[3]'s attention shape), every rank's share run in ONE
process through the HIP path (the multi-GPU runs are the driver's):

* column stripes: the key-sum and node-score shares of the stripes (fork
  scaled_dot) or their q | k projection shares (per-edge scaled_dot), summed as the
  all-reduce sums them, equal the unsharded scores (fp64: 1e-12; the fp32
  projection: 1e-6), and the stripes aggregated with them equal the unsharded
  RHS within 1e-6;
* row partition: each rank's key-sum share over its rows, its rows' node scores
  (or q | k), all-gathered, then its rows aggregated over a local plan: equal to
  the unsharded RHS within 1e-6 (bit-equal rows where the scores are);
* the sharded classes themselves in two processes on one GPU, their collectives
  staged through gloo: the same RHS as one process."""
import multiprocessing
import os
import random

import numpy as np
import pytest
import torch

from gnpde import dist as gd
from gnpde import ops, synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"
N, E, C, H, ATT = 169_343, 1_200_000, 128, 2, 32


def rel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


@pytest.fixture(scope="module")
def arxiv():
    ei, _ = synthetic.rw_graph(N, E, seed=0, device=DEV)
    g = ops.GraphCSR(ei, N)
    x = synthetic.features(1, N, C, seed=1, device=DEV)
    gen = torch.Generator(device=DEV)
    gen.manual_seed(2)
    Wq, Wk = [torch.randn(ATT, C, generator=gen, device=DEV) * 0.1 for _ in range(2)]
    bq, bk = [torch.randn(ATT, generator=gen, device=DEV) * 0.1 for _ in range(2)]
    yield ei, g, x, Wq, bq, Wk, bk
    torch.cuda.empty_cache()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_column_stripe_shares_reference(arxiv, world):
    ei, g, x, Wq, bq, Wk, bk = arxiv
    a = torch.tensor(0.3, device=DEV)
    ns_full = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'reference')
    f_full = ops.attn_rhs(g, ns_full, None, None, 1, x, alpha=a)
    cols = gd.col_blocks(C, world)
    S = sum(ops.ref_keysum(g, x[..., c0:c1].contiguous(), Wk[:, c0:c1].contiguous(),
                           bk if p == 0 else torch.zeros_like(bk)) for p, (c0, c1) in enumerate(cols))
    cs = sum(ops.ref_scores_from_keysum(g, x[..., c0:c1].contiguous(), S, Wq[:, c0:c1].contiguous(),
                                        bq if p == 0 else torch.zeros_like(bq), H) for p, (c0, c1) in enumerate(cols))
    assert rel(cs, ns_full.cs) <= 1e-12
    ns = ops.NodeScores(ops._lib.SCORE_REFERENCE, H, ATT // H, cs=cs)
    f = torch.cat([ops.attn_rhs(g, ns, None, None, 1, x[..., c0:c1].contiguous(), alpha=a) for c0, c1 in cols], -1)
    assert rel(f, f_full) <= 1e-6


@pytest.mark.parametrize("world,norm_idx", [(2, 0), (4, 1), (8, 0)])
def test_column_stripe_shares_per_edge(arxiv, world, norm_idx):
    ei, g, x, Wq, bq, Wk, bk = arxiv
    a = torch.tensor(0.3, device=DEV)
    W, b = torch.cat([Wq, Wk], 0), torch.cat([bq, bk], 0)
    ns_full = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'per_edge', wcat=(W, b))
    f_full = ops.attn_rhs(g, ns_full, None, None, norm_idx, x, alpha=a)
    cols = gd.col_blocks(C, world)
    qk = sum(ops.linear(x[..., c0:c1].contiguous(), W[:, c0:c1].contiguous(),
                        b if p == 0 else torch.zeros_like(b))[0] for p, (c0, c1) in enumerate(cols))
    ref = torch.cat([ns_full.q, ns_full.k], 1)
    assert rel(qk, ref) <= 1e-6
    ns = gd._qk_scores(qk, H, ATT)
    f = torch.cat([ops.attn_rhs(g, ns, None, None, norm_idx, x[..., c0:c1].contiguous(), alpha=a)
                   for c0, c1 in cols], -1)
    assert rel(f, f_full) <= 1e-6


@pytest.mark.parametrize("world,mode,norm_idx", [(2, 'reference', 1), (8, 'reference', 1), (4, 'per_edge', 0),
                                                 (2, 'per_edge', 1), (4, 'reference', 0)])
def test_row_partition_shares(arxiv, world, mode, norm_idx):
    """Every rank's rows through ops.spmm_rhs_rows with the scores assembled as the
    row-partitioned class assembles them (key-sum shares over its rows all-reduced,
    node scores / q | k of its rows all-gathered)."""
    ei, g, x, Wq, bq, Wk, bk = arxiv
    a = torch.tensor(0.3, device=DEV)
    xr = x.view(N, C)
    W, b = torch.cat([Wq, Wk], 0), torch.cat([bq, bk], 0)
    if mode == 'reference' and norm_idx == 0:
        ns_full = ops.uniform_scores(H)
        m, rl = ops.softmax_stats(g, ns_full, 0)
        w_uni = ops.attn_weights(g, ns_full, m, rl, 0)
        f_full = ops.spmm_rhs(g, w_uni, xr, alpha=a)
    elif mode == 'reference':
        ns_full = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'reference')
        f_full = ops.attn_rhs(g, ns_full, None, None, 1, x, alpha=a).view(N, C)
    else:
        ns_full = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'per_edge', wcat=(W, b))
        f_full = ops.attn_rhs(g, ns_full, None, None, norm_idx, x, alpha=a).view(N, C)
    blocks = gd.balanced_row_blocks(g.csr.rowptr.cpu().numpy(), world)
    if mode == 'reference' and norm_idx == 1:
        views = [gd._RowView(g, r0, r1) for r0, r1 in blocks]
        S = sum(ops.ref_keysum(v, xr[r0:r1], Wk, bk) for v, (r0, r1) in zip(views, blocks))
        cs = torch.cat([ops.ref_scores_from_keysum(v, xr[r0:r1], S, Wq, bq, H) for v, (r0, r1) in zip(views, blocks)])
        assert rel(cs, ns_full.cs) <= 1e-12
        ns = ops.NodeScores(ops._lib.SCORE_REFERENCE, H, ATT // H, cs=cs)
        _, _, mr = ops.softmax_stats(g, ns, 1, packed=True)
        wts, nsd, mrd = ops.RefDstWeights(cs, None, None, H, mr=mr), None, None
    elif mode == 'reference':
        wts, nsd, mrd = w_uni, None, None
    else:
        qk = torch.cat([ops.linear(xr[r0:r1], W, b)[0] for r0, r1 in blocks])
        nsd = gd._qk_scores(qk, H, ATT)
        mrd = ops.softmax_stats(g, nsd, 1, packed=True)[2] if norm_idx == 1 else None
        wts = None
    for r0, r1 in blocks:
        plan = gd._local_plan(g.csr, r0, r1, g.chunk)
        yl = xr[r0:r1].contiguous()
        loc = ops.spmm_rhs_rows(g, plan, wts, xr, yl, r0, alpha=a, ns=nsd, mr=mrd)
        assert rel(loc, f_full[r0:r1]) <= 1e-6, (world, r0)


@pytest.mark.parametrize("world,mode", [(2, 'reference'), (8, 'reference'), (4, 'per_edge'), (8, 'per_edge')])
def test_partitioned_destination_statistics(arxiv, world, mode):
    """the destination statistics (norm_idx 1) formed per block of
    destination rows (gnpde.dist: each rank one block, then all-gathered) — K2 over a
    row-range plan — equal the statistics of the whole CSC: the max bit for bit, the
    reciprocal sums within 1e-6 (a group's segmented sum runs in a lane order that
    depends on where the item packing put it, and a block boundary moves the packing:
    1-ulp differences on 2-4 of 169k rows measured, tools/dbg_stats.py)."""
    ei, g, x, Wq, bq, Wk, bk = arxiv
    kw = dict(wcat=(torch.cat([Wq, Wk], 0), torch.cat([bq, bk], 0))) if mode == 'per_edge' else {}
    ns = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', mode, **kw)
    _, _, mr = ops.softmax_stats(g, ns, 1, packed=True)
    blocks, nb = gd._dst_blocks(ei, N, world, g)
    assert blocks[0][0] == 0 and blocks[-1][1] == N and max(b - a for a, b in blocks) == nb
    got = torch.full_like(mr, float('nan'))
    for r0, r1 in blocks:
        part = gd._hip_stats_rows(g, ns, r0, r1)
        assert part is not None and len(part) == 1
        got[r0:r1] = part[0][r0:r1]
    nz = torch.diff(g.csc.rowptr) > 0
    assert torch.equal(got[nz, :H], mr[nz, :H])  # the max (stored fp32-exact)
    assert torch.allclose(got[nz, H:2 * H], mr[nz, H:2 * H], rtol=1e-6, atol=0)


@pytest.mark.parametrize("world,mode,norm_idx", [(2, 'reference', 1), (8, 'reference', 1), (4, 'per_edge', 1),
                                                 (8, 'per_edge', 0)])
def test_edge_sharded_weights_shares(arxiv, world, mode, norm_idx):
    """The edge-sharded weights of ColumnShardedTransformer: each rank's block of CSR
    positions (whole CSR rows, balanced by nnz) weighted edge-parallel
    (gnpde_attn_weights_f32 over [e0, e1)) from the statistics — the gathered
    destination ones (norm_idx 1) or its own rows' source ones from a row-range K2
    (norm_idx 0) — equals that block of the whole-graph weights bit for bit (norm_idx
    1) / within 1e-6 (norm_idx 0: the row-range K2's lane order); the stripes
    aggregated with the gathered weights equal the unsharded RHS within 1e-6."""
    ei, g, x, Wq, bq, Wk, bk = arxiv
    a = torch.tensor(0.3, device=DEV)
    kw = dict(wcat=(torch.cat([Wq, Wk], 0), torch.cat([bq, bk], 0))) if mode == 'per_edge' else {}
    ns = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', mode, **kw)
    f_full = ops.attn_rhs(g, ns, None, None, norm_idx, x, alpha=a)
    m, rl = ops.softmax_stats(g, ns, norm_idx, seg=False)
    w_full = ops.attn_weights(g, ns, m, rl, norm_idx, seg=False)
    blocks, rows = gd._HipAttentionLocal(g).edge_blocks(world)
    assert blocks[0][0] == 0 and blocks[-1][1] == g.nnz
    parts = []
    for (e0, e1), (r0, r1) in zip(blocks, rows):
        if norm_idx == 0:
            ms, rls = gd._HipAttentionLocal(g).src_stats(ns, r0, r1)
            wp = ops.attn_weights(g, ns, ms, rls, 0, edges=(e0, e1))
            assert torch.allclose(wp, w_full[e0:e1], rtol=1e-6, atol=0)
        else:
            wp = ops.attn_weights(g, ns, m, rl, 1, edges=(e0, e1))
            assert torch.equal(wp, w_full[e0:e1])
        parts.append(wp)
    w = torch.cat(parts)
    f = torch.cat([ops.spmm_rhs(g, w, x[..., c0:c1].contiguous(), alpha=a) for c0, c1 in gd.col_blocks(C, world)], -1)
    assert rel(f, f_full) <= 1e-6


def _two_rank_worker(rank, world, port, cls, mode, norm_idx, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "graph-neural-pde_amd"))
    import torch.distributed as dist
    from gnpde import dist as gdd, ops as o, synthetic as syn

    class StagedComm(object):
        """The class's collectives through gloo on host copies (two ranks share one GPU here)."""

        def all_reduce(self, t):
            h = t.cpu()
            dist.all_reduce(h)
            t.copy_(h)

        def all_gather_into_tensor(self, out, t):
            h = torch.empty(out.shape, dtype=out.dtype)
            dist.all_gather_into_tensor(h, t.cpu().contiguous())
            out.copy_(h)

    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        n, e, c = 20000, 200000, 64
        ei, _ = syn.rw_graph(n, e, seed=3, device="cuda")
        x = syn.features(1, n, c, seed=4, device="cuda")
        gen = torch.Generator(device="cuda")
        gen.manual_seed(5)
        Wq, Wk = [torch.randn(ATT, c, generator=gen, device="cuda") * 0.1 for _ in range(2)]
        bq, bk = [torch.randn(ATT, generator=gen, device="cuda") * 0.1 for _ in range(2)]
        a = torch.tensor(0.4, device="cuda")
        g = o.GraphCSR(ei, n)
        if mode == 'reference' and norm_idx == 0:
            ns = o.uniform_scores(H)
            m, rl = o.softmax_stats(g, ns, 0)
            want = o.spmm_rhs(g, o.attn_weights(g, ns, m, rl, 0), x, alpha=a)
        else:
            kw = dict(wcat=(torch.cat([Wq, Wk]), torch.cat([bq, bk]))) if mode == 'per_edge' else {}
            ns = o.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', mode, **kw)
            want = o.attn_rhs(g, ns, None, None, norm_idx, x, alpha=a)
        if cls == 'cols':
            sh = gdd.ColumnShardedTransformer(ei, n, c, Wq, bq, Wk, bk, H, norm_idx, a, score_mode=mode,
                                              comm=StagedComm())
            f = sh.gather(sh(None, sh.split(x)))
        else:
            sh = gdd.RowShardedTransformer(ei, n, c, Wq, bq, Wk, bk, H, norm_idx, a, score_mode=mode,
                                           comm=StagedComm())
            f = sh.gather(sh(None, sh.scatter(x)))
        torch.cuda.synchronize()
        q.put((rank, rel(f.view(want.shape), want)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cls,mode,norm_idx", [("cols", "reference", 1), ("cols", "per_edge", 0), ("cols", "per_edge", 1),
                                               ("rows", "reference", 1), ("rows", "per_edge", 1),
                                               ("rows", "reference", 0)])
def test_sharded_classes_two_ranks_one_gpu(cls, mode, norm_idx):
    import torch.multiprocessing as mp
    ctx = multiprocessing.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    mp.start_processes(_two_rank_worker, args=(2, port, cls, mode, norm_idx, q), nprocs=2, join=True,
                       start_method="spawn")
    res = sorted(q.get(timeout=120) for _ in range(2))
    for rank, err in res:
        assert err <= 1e-6, (rank, err)


@pytest.mark.parametrize("add_source", [False, True])
def test_row_sharded_laplacian_world_one_in_degree_numbering(tmp_path, add_source):
    """The row partition in the graph's in-degree numbering at a
    world of one (gloo, in-process): the integrator's state blocks are the gathered
    buffers themselves (in-place all-gather), the solve equals the unsharded one.
    With the source term the full x0 in the caller's numbering is
    scattered into the block by the class (x0=); a block of the wrong shape is
    rejected."""
    import torch.distributed as dist
    import gnpde
    init = not dist.is_initialized()
    if init:
        dist.init_process_group("gloo", init_method="file://%s" % (tmp_path / "pg"), rank=0, world_size=1)
    try:
        n, e, c = 40000, 300000, 64
        ei, w = synthetic.rw_graph(n, e, seed=12, device=DEV)
        x = synthetic.features(1, n, c, seed=13, device=DEV)
        x0 = synthetic.features(1, n, c, seed=14, device=DEV)
        a, b = torch.tensor(0.3, device=DEV), torch.tensor(-0.4, device=DEV)
        opt = {'block': 'constant', 'function': 'laplacian', 'add_source': add_source, 'no_alpha_sigmoid': False,
               'max_nfe': 10 ** 9, 'multi_modal': False, 'hidden_dim': c}
        func = gnpde.LaplacianODEFunc(c, c, opt, DEV).to(DEV)
        func.edge_index, func.edge_weight = ei, w
        if add_source:
            func.x0 = x0
        with torch.no_grad():
            func.alpha_train.fill_(0.3)
            func.beta_train.fill_(-0.4)
            t = torch.tensor([0.0, 1.0], device=DEV)
            want = gnpde.odeint(func, x, t, method='rk4', options={'step_size': 0.25})[1]
            kw = dict(beta=b, add_source=True, x0=x0) if add_source else {}
            sh = gd.RowShardedLaplacian(ei, w, n, a, **kw)
            assert sh.lay is not None  # the in-degree numbering
            y = gnpde.odeint(sh, sh.scatter(x), t, method='rk4', options={'step_size': 0.25})[1]
            got = sh.unpad(sh.gather(y)).view(want.shape)
            if add_source:
                with pytest.raises(ValueError):
                    gd.RowShardedLaplacian(ei, w, n, a, beta=b, add_source=True, x0_local=x0.view(n, c)[:100])
        assert len(sh._blocks_out) >= 2  # the solve's states were gathered in place
        assert rel(got, want) <= 1e-6
    finally:
        if init:
            dist.destroy_process_group()


@pytest.mark.parametrize("cls", ["rows", "cols"])
def test_sharded_laplacian_dopri5_krylov_world_one(tmp_path, cls):
    """Adaptive solves of the sharded Laplacians with their global error norm, at a world
    of one (gloo, in-process): the column stripes run the fused loop with the Krylov step
    (integrator._KrylovPlan; linear=True drops the source term); the row partition runs
    the restated torch loop (RowShardedLaplacian.fused_adaptive is False: its per-RHS
    all-gather sits between the wide stages) — which path ran is asserted.
    Both: the same step count as the unsharded solve and its values within 1e-6, with a
    source term."""
    import torch.distributed as dist
    import gnpde
    from gnpde import integrator as gi
    init = not dist.is_initialized()
    if init:
        dist.init_process_group("gloo", init_method="file://%s" % (tmp_path / "pg"), rank=0, world_size=1)
    try:
        n, e, c = 40000, 300000, 64
        ei, w = synthetic.rw_graph(n, e, seed=15, device=DEV)
        x = synthetic.features(1, n, c, seed=16, device=DEV)
        x0 = synthetic.features(1, n, c, seed=17, device=DEV)
        a, b = torch.tensor(0.3, device=DEV), torch.tensor(-0.4, device=DEV)
        opt = {'block': 'constant', 'function': 'laplacian', 'add_source': True, 'no_alpha_sigmoid': False,
               'max_nfe': 10 ** 9, 'multi_modal': False, 'hidden_dim': c}
        func = gnpde.LaplacianODEFunc(c, c, opt, DEV).to(DEV)
        func.edge_index, func.edge_weight = ei, w
        func.x0 = x0
        t = torch.tensor([0.0, 1.0], device=DEV)
        kw = dict(method='dopri5', rtol=1e-4, atol=1e-5)
        with torch.no_grad():
            func.alpha_train.fill_(0.3)
            func.beta_train.fill_(-0.4)
            want = gnpde.odeint(func, x, t, **kw)[1]
            n_want = gi.odeint.last_n_steps
            if cls == "rows":
                sh = gd.RowShardedLaplacian(ei, w, n, a, beta=b, add_source=True, x0=x0)
                y0 = sh.scatter(x)
            else:
                sh = gd.ColumnShardedLaplacian(ei, w, n, c, a, beta=b, add_source=True, x0_local=x0)
                y0 = sh.split(x)
            assert sh.affine
            y = gnpde.odeint(sh, y0, t, options=dict(norm=sh.global_rms_norm), **kw)[1]
            got = sh.unpad(sh.gather(y)).view(want.shape) if cls == "rows" else y.view(want.shape)
            path = gi.odeint.last_path
        assert path == ('restated' if cls == "rows" else 'fused_krylov'), path
        assert gi.odeint.last_n_steps == n_want
        assert rel(got, want) <= 1e-6
    finally:
        if init:
            dist.destroy_process_group()


def test_empty_row_range_statistics_and_edge_block(arxiv):
    """A rank whose block is empty (balanced_row_blocks gives equal cuts when one hub row
    holds more than 1/world of the nnz): the row-range statistics return full-size
    arrays without a launch, and the weights of an empty edge range are empty."""
    ei, g, x, Wq, bq, Wk, bk = arxiv
    ns = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'reference')
    m, rl = ops.softmax_stats(g, ns, 1, packed=False, rows=(7, 7))
    assert m.shape == (N, H) and rl.shape == (N, H)
    _, _, mr = ops.softmax_stats(g, ns, 1, packed=True, rows=(7, 7))
    assert mr.shape[0] == N
    w = ops.attn_weights(g, ns, m, rl, 1, edges=(100, 100))
    assert w.numel() == 0
