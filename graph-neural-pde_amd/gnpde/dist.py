"""Multi-GPU execution of the ODE RHS: one process per GPU, torch.distributed
with the RCCL backend ("nccl" on ROCm) over xGMI.

The reference has no multi-GPU hot path (only nn.DataParallel over the batch
axis, src/ray_tune.py:58-59).  Three ways to shard it are provided:

* ``shard_batch`` — independent objects: each rank integrates its slice of the
  batch axis B (the reference's own parallel axis).  No data-path collective;
  this is what ``bench.py --gpus N`` measures (weak scaling).
* ``RowShardedLaplacian`` — the north star's literal design: a 1-D partition of
  the graph rows (equal row blocks of the block-diagonal CSR); each RHS
  evaluation computes its rows of f and the next evaluation needs every row of
  the state, so the state is all-gathered (RCCL all_gather_into_tensor, half
  the volume of the all-reduce the north star names) before each RHS.  Volume
  per RHS = R*C*4 bytes in total.
* ``ColumnShardedLaplacian`` — feature-column stripes: rank p owns columns
  [c0, c1) of every node and a replicated CSR.  A*x is column-separable, so a
  fixed-grid integration needs no communication at all; dopri5 needs one
  all-reduce of the squared error norm per step (``global_rms_norm``); the
  columns are all-gathered once at the end.

``local_rhs`` lets tests substitute a CPU computation so the communication
pattern is exercised with the gloo backend; the default is the HIP path.
"""
import math

import torch
import torch.distributed as dist

from . import ops


def row_blocks(R, world):
    """Equal row blocks [(r0, r1)] of ceil(R/world) rows (last one shorter)."""
    nb = int(math.ceil(R / world))
    return [(min(R, p * nb), min(R, (p + 1) * nb)) for p in range(world)], nb


def col_blocks(C, world, align=4):
    """Contiguous column stripes, as equal as possible, multiples of ``align``
    where C allows (16-byte rows for the vectorised gathers)."""
    unit = align if C % align == 0 and C // align >= world else 1
    units = C // unit
    base, extra = divmod(units, world)
    out, c = [], 0
    for p in range(world):
        n = (base + (1 if p < extra else 0)) * unit
        out.append((c, c + n))
        c += n
    return out


def shard_batch(edge_index, x, rank, world):
    """Batch-axis shard (independent graphs) for replica parallelism."""
    B = edge_index.shape[0]
    per = int(math.ceil(B / world))
    b0, b1 = min(B, rank * per), min(B, (rank + 1) * per)
    return edge_index[b0:b1], x[b0:b1], (b0, b1)


class RowShardedLaplacian(object):
    """Row-partitioned Laplacian RHS with an all-gather of the state per RHS.

    State per rank: y_local [nb, C] (its row block, zero padded).  Calling the
    object with (t, y_local) all-gathers the blocks into y_full [world*nb, C]
    (global row order, padding at the end), aggregates the local rows of A and
    returns f_local [nb, C]; it drops into gnpde.odeint unchanged."""

    graph_capturable = False  # an RCCL all-gather per RHS: the integrator runs it eagerly

    def __init__(self, edge_index, edge_weight, num_nodes, alpha, beta=None, x0_local=None, add_source=False,
                 alpha_sigmoid=True, group=None, local_rhs=None, chunk=ops.DEFAULT_CHUNK):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        B, _, E = edge_index.shape
        self.N = int(num_nodes)
        self.R = B * self.N
        self.blocks, self.nb = row_blocks(self.R, self.world)
        self.r0, self.r1 = self.blocks[self.rank]
        self.alpha, self.beta = alpha, beta
        self.x0_local = x0_local
        self.add_source, self.alpha_sigmoid = add_source, alpha_sigmoid
        self.nfe = 0
        self.local_rhs = local_rhs
        if local_rhs is None:
            self.g = ops.GraphCSR(edge_index, self.N, chunk=chunk)
            self.w = self.g.gather_weights(edge_weight)
            self.plan = _local_plan(self.g.csr, self.r0, self.r1, chunk)

    def gather(self, y_local):
        """All-gather of the row blocks (RCCL over xGMI on ROCm)."""
        y_local = y_local.contiguous()
        out = torch.empty((self.world * self.nb,) + tuple(y_local.shape[1:]), dtype=y_local.dtype,
                          device=y_local.device)
        dist.all_gather_into_tensor(out, y_local, group=self.group)
        return out

    def __call__(self, t, y_local):
        self.nfe += 1
        y_full = self.gather(y_local)
        if self.local_rhs is not None:
            return self.local_rhs(t, y_full, self.r0, self.r1, y_local)
        return _rows_rhs(self, y_full, y_local, stage=None)

    def rhs_stage(self, t, y_local, stage):
        self.nfe += 1
        if self.local_rhs is not None:
            raise NotImplementedError
        y_full = self.gather(y_local)
        _rows_rhs(self, y_full, y_local, stage=stage)

    def scatter(self, y):
        """Full state [R, C] -> this rank's zero-padded block [nb, C]."""
        out = torch.zeros((self.nb,) + tuple(y.shape[1:]), dtype=y.dtype, device=y.device)
        out[:self.r1 - self.r0] = y[self.r0:self.r1]
        return out

    def unpad(self, y_full):
        return y_full[:self.R]


def _local_plan(csr, r0, r1, chunk):
    """Plan over rows [r0, r1) of a global CSR.  Items keep global edge offsets
    and get global row ids (row + r0), so the epilogue reads its own row from
    the gathered full state; outputs are addressed through pointers shifted by
    -r0 rows (ops.spmm_rhs_rows)."""
    if r1 <= r0:
        return None
    rowptr = csr.rowptr[r0:r1 + 1].contiguous()
    plan = ops.build_plan(rowptr, r1 - r0, int(csr.nnz), chunk)
    if plan.n_items:
        plan.items.view(-1, 4)[:plan.n_items, 0] += r0
    if plan.n_heavy:
        plan.heavy.view(-1, 4)[:plan.n_heavy, 0] += r0
    return plan


def _rows_rhs(sh, y_full, y_local, stage):
    """K1 over the local rows: gathers from y_full (global row order), the
    epilogue's own rows come from y_local (local row order)."""
    if sh.plan is None:
        return torch.zeros_like(y_local)
    return ops.spmm_rhs_rows(sh.g, sh.plan, sh.w, y_full, y_local, sh.r0, x0=sh.x0_local, alpha=sh.alpha,
                             beta=sh.beta, alpha_sigmoid=sh.alpha_sigmoid, add_source=sh.add_source, stage=stage)


class ColumnShardedLaplacian(object):
    """Column-striped Laplacian RHS: no communication per RHS."""

    def __init__(self, edge_index, edge_weight, num_nodes, C, alpha, beta=None, x0_local=None, add_source=False,
                 alpha_sigmoid=True, group=None, local_rhs=None, chunk=ops.DEFAULT_CHUNK):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.C = int(C)
        self.cols = col_blocks(self.C, self.world)
        self.c0, self.c1 = self.cols[self.rank]
        self.N = int(num_nodes)
        self.alpha, self.beta = alpha, beta
        self.x0_local = x0_local
        self.add_source, self.alpha_sigmoid = add_source, alpha_sigmoid
        self.nfe = 0
        self.local_rhs = local_rhs
        if local_rhs is None:
            self.g = ops.GraphCSR(edge_index, self.N, chunk=chunk)
            self.w = self.g.gather_weights(edge_weight)

    def split(self, x):
        """[B,N,C] -> this rank's contiguous column stripe [B,N,c1-c0]."""
        return x[..., self.c0:self.c1].contiguous()

    def __call__(self, t, x_local):
        self.nfe += 1
        if self.local_rhs is not None:
            return self.local_rhs(t, x_local)
        return ops.spmm_rhs(self.g, self.w, x_local, x0=self.x0_local, alpha=self.alpha, beta=self.beta,
                            alpha_sigmoid=self.alpha_sigmoid, add_source=self.add_source)

    def rhs_stage(self, t, x_local, stage):
        self.nfe += 1
        if self.local_rhs is not None:
            raise NotImplementedError
        ops.spmm_rhs(self.g, self.w, x_local, x0=self.x0_local, alpha=self.alpha, beta=self.beta,
                     alpha_sigmoid=self.alpha_sigmoid, add_source=self.add_source, stage=stage)

    def global_rms_norm(self, t):
        """RMS over the full state (all stripes): one all-reduce of 2 doubles."""
        v = torch.stack([t.double().pow(2).sum(), torch.tensor(float(t.numel()), dtype=torch.float64,
                                                                device=t.device)])
        dist.all_reduce(v, group=self.group)
        return (v[0] / v[1]).sqrt().to(t.dtype)

    def gather(self, x_local):
        """All stripes -> full [B,N,C] (once, at the end of an integration)."""
        widths = [c1 - c0 for c0, c1 in self.cols]
        wmax = max(widths)
        shp = tuple(x_local.shape[:-1])
        pad = torch.zeros(shp + (wmax,), dtype=x_local.dtype, device=x_local.device)
        pad[..., :x_local.shape[-1]] = x_local
        pad = pad.reshape((-1, wmax))
        out = torch.empty((self.world * pad.shape[0], wmax), dtype=x_local.dtype, device=x_local.device)
        dist.all_gather_into_tensor(out, pad, group=self.group)
        out = out.view((self.world,) + shp + (wmax,))
        return torch.cat([out[p][..., :widths[p]] for p in range(self.world)], dim=-1)
