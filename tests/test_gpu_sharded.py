"""GPU: the multi-GPU layouts of gnpde.dist on the configs[4] graph (G-rmat:
N = 2,000,000, E = 20,000,000, C = 256), every rank's part run in ONE process
through the HIP path (the 8-GPU runs are the driver's).

* Row partition (north-star literal design, nnz-balanced blocks, padded
  all-gather layout): each rank's rows are BIT-EQUAL to the unsharded K1 —
  same CSR, same hub chunking, same lane geometry, so the same sums in the
  same order.
* Column stripes: each stripe is the K1 of a narrower row, whose lane
  geometry (edges side by side per row) differs from the full-width one, so
  the fp32 sums are associated differently: equal to the unsharded K1 within
  1e-6 relative, bit-reproducible run to run.
* Full-size properties: rw normalisation is column-stochastic, so the column
  sums of A x equal those of x; linearity; and the oracle (fp64) on a sample of
  rows that includes the largest hubs.
"""
import numpy as np
import pytest
import torch

from gnpde import dist as gd
from gnpde import ops, synthetic
from test_gpu_parity import DEV, RTOL

pytestmark = pytest.mark.gpu

N, E, C = 2_000_000, 20_000_000, 256


@pytest.fixture(scope="module")
def grmat():
    ei, w = synthetic.rw_graph(N, E, seed=0, device=DEV)
    g = ops.GraphCSR(ei, N)
    wc = g.gather_weights(w)
    x = synthetic.features(1, N, C, seed=1, device=DEV).view(N, C)
    alpha = torch.tensor(0.3, device=DEV)
    full = ops.spmm_rhs(g, wc, x, alpha=alpha)
    torch.cuda.synchronize()
    g.coo = (ei, w)  # the COO the CSR was built from (test_grmat_csr_matches_coo_restatement)
    yield g, wc, x, alpha, full
    del g, wc, x, full
    torch.cuda.empty_cache()


def test_grmat_csr_matches_coo_restatement(grmat):
    """at configs[4] size the CSR itself (rowptr, col, perm) and the
    CSR-order weights equal a restatement from the COO edge list with torch ops (a
    stable sort by source: in-row order = COO order), so the sampled oracle check
    below is anchored on the edge list, not on the product's own structure."""
    g, wc, x, alpha, full = grmat
    ei, w = g.coo
    src, dst = ei[0, 0].long(), ei[0, 1].long()
    order = torch.argsort(src, stable=True)
    assert torch.equal(g.csr.perm.long(), order)
    assert torch.equal(g.csr.col.long(), dst[order])
    rp = torch.zeros(N + 1, dtype=torch.int64, device=DEV)
    rp[1:] = torch.cumsum(torch.bincount(src, minlength=N), 0)
    assert torch.equal(g.csr.rowptr.long(), rp)
    assert torch.equal(wc.view(-1), w.view(-1)[order])


@pytest.mark.parametrize("world", [2, 8])
def test_row_partition_bit_equal_to_unsharded(grmat, world):
    g, wc, x, alpha, full = grmat
    rp = g.csr.rowptr.cpu().numpy()
    parts = [gd.RowPartition(g, world, r) for r in range(world)]
    blocks = parts[0].blocks
    assert blocks[0][0] == 0 and blocks[-1][1] == N
    # balanced by nnz + ROW_WEIGHT x rows (each row also moves its own row and output) up to one row
    rw = gd.ROW_WEIGHT
    work = [int(rp[b] - rp[a]) + rw * (b - a) for a, b in blocks]
    assert max(work) <= 1.05 * (E + rw * N) / world + int(np.diff(rp).max()) + rw
    y_full = parts[0].pad_state(x)
    assert torch.equal(parts[0].unpad_state(y_full), x)
    for p in parts:
        loc = p.rhs(g, wc, y_full, p.local_block(x), alpha=alpha)
        assert torch.equal(loc[:p.r1 - p.r0], full[p.r0:p.r1]), (world, p.rank)
        # fused stage through the shifted pointers: out = y_local + 0.25 f
        yl = p.local_block(x)
        out = torch.empty_like(yl)
        p.rhs(g, wc, y_full, yl, alpha=alpha, stage=ops.Stage(outs=[(out, yl, 1.0, 0.25, [])]))
        assert torch.allclose(out[:p.r1 - p.r0], x[p.r0:p.r1] + 0.25 * full[p.r0:p.r1], atol=1e-6)
    torch.cuda.synchronize()


@pytest.mark.parametrize("world", [2, 8])
def test_column_stripes_match_unsharded(grmat, world):
    g, wc, x, alpha, full = grmat
    cols = gd.col_blocks(C, world)
    scale = float(full.abs().max())
    for c0, c1 in cols:
        xs = x[:, c0:c1].contiguous()
        fs = ops.spmm_rhs(g, wc, xs, alpha=alpha)
        assert float((fs - full[:, c0:c1]).abs().max()) <= 1e-6 * scale, (world, c0)
        assert torch.equal(fs, ops.spmm_rhs(g, wc, xs, alpha=alpha))  # deterministic (no float atomics)


def test_grmat_properties_and_sampled_oracle(grmat):
    g, wc, x, alpha, full = grmat
    ax = ops.spmm_rhs(g, wc, x, rhs=False)
    # column-stochastic A (rw, norm_dim=1): sum_i (A x)_i == sum_j x_j per column
    lhs, rhs = ax.double().sum(0), x.double().sum(0)
    assert float((lhs - rhs).abs().max()) <= 1e-6 * float(x.double().abs().sum(0).max())
    # linearity: A (a x + b y) = a A x + b A y
    y = torch.randn_like(x)
    lin = ops.spmm_rhs(g, wc, 0.5 * x - 2.0 * y, rhs=False)
    want = 0.5 * ax - 2.0 * ops.spmm_rhs(g, wc, y, rhs=False)
    assert float((lin - want).abs().max()) <= 1e-5 * float(want.abs().max())
    del y, lin, want
    # fp64 oracle on sampled rows: the 16 largest hubs + 4000 random rows
    rp = g.csr.rowptr.cpu().numpy().astype(np.int64)
    deg = np.diff(rp)
    rng = np.random.default_rng(5)
    rows = np.unique(np.concatenate([np.argsort(deg)[-16:], rng.integers(0, N, 4000)]))
    idx = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in rows])
    it = torch.from_numpy(idx).to(DEV)
    col = g.csr.col[it].long()
    cw = wc[it].double().cpu().numpy()
    xc = x[col].double().cpu().numpy()
    xr = x[torch.from_numpy(rows).to(DEV)].double().cpu().numpy()
    seg = np.repeat(np.arange(len(rows)), deg[rows])
    want = np.zeros((len(rows), C))
    np.add.at(want, seg, cw[:, None] * xc)
    a = 1.0 / (1.0 + np.exp(-0.3))
    want = a * (want - xr)
    got = full[torch.from_numpy(rows).to(DEV)].double().cpu().numpy()
    assert np.abs(got - want).max() <= RTOL * np.abs(want).max()
    assert deg[rows].max() > 1000  # the sample holds real hubs (split, combined in-launch)
