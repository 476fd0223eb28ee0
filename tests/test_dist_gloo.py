"""Multi-process (world_size 2, gloo, CPU) tests of the sharded RHS layouts in
gnpde.dist: the row-partitioned all-gather design (north star literal) and the
column-stripe design, driven by gnpde.odeint, against a single-process
integration of the same ODE.  The RHS arithmetic is injected as a CPU function
(the HIP kernels need a GPU); what is tested is the partitioning, the
collectives and the integrator coupling (incl. dopri5's global error norm)."""
import multiprocessing
import random

import numpy as np
import pytest
import torch.multiprocessing as mp

import dist_workers as W
from gnpde import dist as gd


def _run(fn, *args, world=2):
    ctx = multiprocessing.get_context("spawn")
    q = ctx.Queue()
    port = random.randint(20000, 40000)
    mp.start_processes(fn, args=(world, port) + args + (q,), nprocs=world, join=True, start_method="spawn")
    return sorted(q.get(timeout=60) for _ in range(world))


def test_row_blocks_and_col_blocks():
    blocks, nb = gd.row_blocks(10, 3)
    assert nb == 4 and blocks == [(0, 4), (4, 8), (8, 10)]
    blocks, nb = gd.row_blocks(2, 4)
    assert blocks == [(0, 1), (1, 2), (2, 2), (2, 2)]
    assert gd.col_blocks(128, 8) == [(16 * p, 16 * p + 16) for p in range(8)]
    assert gd.col_blocks(162, 8)[-1][1] == 162
    cb = gd.col_blocks(10, 3)
    assert cb[0][0] == 0 and cb[-1][1] == 10 and all(b > a for a, b in cb)


def test_balanced_row_blocks():
    """nnz-balanced contiguous row blocks: a power-law row pointer
    whose first rows hold most edges gets short first blocks."""
    import numpy as np
    deg = np.array([500, 300, 100] + [2] * 997)
    rp = np.concatenate([[0], np.cumsum(deg)])
    b = gd.balanced_row_blocks(rp, 4)
    assert b[0][0] == 0 and b[-1][1] == 1000 and all(b[i][1] == b[i + 1][0] for i in range(3))
    work = [rp[r1] - rp[r0] for r0, r1 in b]
    assert b[0] == (0, 2) and max(work) == 800  # rows are not split: the 500 + 300 head is the nearest cut
    # row_weight: each row also costs row_weight edges
    bw = gd.balanced_row_blocks(rp, 4, row_weight=10.0)
    cost = [rp[r1] - rp[r0] + 10 * (r1 - r0) for r0, r1 in bw]
    assert max(cost) - min(cost) <= 520
    # more ranks than rows: empty blocks at the end, still a cover
    assert gd.balanced_row_blocks(np.array([0, 3, 6]), 4)[-1] == (2, 2)
    # host_rowptr over a batch (block-diagonal rows)
    import torch
    ei = torch.tensor([[[0, 0, 2], [1, 2, 0]], [[1, 1, 1], [0, 0, 2]]])
    assert gd.host_rowptr(ei, 3).tolist() == [0, 2, 2, 3, 3, 6, 6]


def test_shard_batch():
    import torch
    ei = torch.zeros(5, 2, 3, dtype=torch.int64)
    x = torch.arange(5.0).view(5, 1, 1)
    parts = [gd.shard_batch(ei, x, r, 2) for r in range(2)]
    assert parts[0][2] == (0, 3) and parts[1][2] == (3, 5)
    assert torch.equal(torch.cat([p[1] for p in parts]), x)


@pytest.mark.parametrize("method", ["euler", "rk4"])
def test_row_sharded_integration_matches_single_process(method):
    res = _run(W.rows_worker, method)
    ei = W.problem()[0]
    want_blocks = [list(b) for b in gd.balanced_row_blocks(gd.host_rowptr(ei, 61), 2)]
    for rank, err, nfe, blocks in res:
        assert err < 1e-12
        assert nfe == (4 if method == "euler" else 16)
        assert blocks == want_blocks


@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_column_sharded_integration_matches_single_process(method):
    res = _run(W.cols_worker, method)
    for rank, err, steps, want_steps in res:
        assert err < 1e-9
        assert steps == want_steps  # same accept/reject sequence: the error norm is global


@pytest.mark.parametrize("method", ["euler", "midpoint", "rk4"])
def test_row_sharded_fused_stage_path(method):
    """The row partition's rhs_stage (all-gather + stage outputs in the epilogue)
    through the integrator's fused fixed-grid solve, on gloo with the arithmetic
    injected: every RHS call is a stage call and the result matches the
    single-process integration."""
    res = _run(W.rows_stage_worker, method)
    n = {"euler": 4, "midpoint": 8, "rk4": 16}[method]
    for rank, err, nfe, calls in res:
        assert err < 1e-12
        assert nfe == calls == n


@pytest.mark.parametrize("score_mode,norm_idx", [("reference", 1), ("reference", 0), ("per_edge", 0),
                                                 ("per_edge", 1)])
@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_column_sharded_transformer_matches_single_process(score_mode, norm_idx, method):
    """the transformer RHS in column stripes — the
    key-sum and node-score shares (fork scaled_dot) or the q | k projection shares
    (per-edge) all-reduced, the stripes aggregated — equals the oracle RHS of the
    whole state; integrated (rk4 through the fused stages, dopri5 through the
    global error norm) it matches the single-process integration."""
    res = _run(W.attn_cols_worker, score_mode, norm_idx, method, False)
    for rank, err_f, err_y, nfe, nbytes, dnb, ew in res:
        assert err_f < 1e-12
        assert err_y < 1e-9
        assert not ew  # a CPU local: the fused aggregation unless asked
        # norm_idx 1: each rank forms the statistics of a block of dnb destination rows, and
        # the blocks (max and sum-exp, [dnb, heads] fp64 each on this host path) are all-gathered
        stats = 2 * 2 * dnb * 2 * 8 if norm_idx == 1 else 0
        assert (dnb > 0) == (norm_idx == 1 and not (score_mode == "reference" and norm_idx == 0))
        if score_mode == "reference" and norm_idx == 0:
            assert nbytes == 0  # uniform 1/outdeg weights: no collective at all
        elif score_mode == "reference":
            assert nbytes == (8 + 41 * 2) * 8 + stats  # S [1, att] + cs [N, heads], fp64
        else:
            assert nbytes == 41 * 16 * 4 + stats  # q | k [N, 2 att], fp32


@pytest.mark.parametrize("score_mode,norm_idx", [("reference", 1), ("per_edge", 1), ("per_edge", 0)])
@pytest.mark.parametrize("method", ["rk4", "dopri5"])
def test_column_sharded_transformer_edge_weights(score_mode, norm_idx, method):
    """Edge-sharded weights: each rank forms the head-mean weights of one block of
    edges — from the gathered destination statistics (norm_idx 1) or its own source
    groups' (norm_idx 0, no statistics exchanged) — the blocks are all-gathered and
    every rank aggregates its columns with them: equals the oracle RHS of the whole
    state and the single-process integration; the payload adds the padded E x 4 bytes."""
    res = _run(W.attn_cols_worker, score_mode, norm_idx, method, True)
    for rank, err_f, err_y, nfe, nbytes, dnb, ew in res:
        assert ew
        assert err_f < 1e-12
        assert err_y < 1e-9
        stats = 2 * 2 * dnb * 2 * 8 if norm_idx == 1 else 0
        base = (8 + 41 * 2) * 8 if score_mode == "reference" else 41 * 16 * 4
        assert nbytes == base + stats + 2 * 150 * 4  # two ranks, 300 edges: blocks of 150


@pytest.mark.parametrize("score_mode,norm_idx,method,world,hub", [
    ("reference", 1, "rk4", 2, False), ("per_edge", 1, "rk4", 2, False), ("reference", 0, "rk4", 2, False),
    ("per_edge", 0, "dopri5", 2, False), ("reference", 1, "dopri5", 3, True), ("per_edge", 1, "rk4", 3, True)])
def test_row_sharded_transformer_matches_single_process(score_mode, norm_idx, method, world, hub):
    """VERDICT r4 item 4 / ADVICE r4: the transformer RHS row-partitioned (state
    all-gathered, key-sum shares all-reduced, node scores or q | k all-gathered, the
    rank's rows aggregated) equals the oracle RHS of the whole state and integrates
    to the single-process solution; with a hub row taking most of the nnz one rank's
    block is empty and the job still completes (that rank joins every collective)."""
    res = _run(W.attn_rows_worker, score_mode, norm_idx, method, hub, world=world)
    assert len(res) == world
    if hub:
        assert min(r[1] for r in res) == 0  # an empty row block
    nfe = {r[4] for r in res}
    assert len(nfe) == 1  # every rank took the same steps
    for rank, n, err_f, err_y, _ in res:
        assert err_f < 1e-12
        assert err_y < 1e-9
