"""Multi-GPU execution of the ODE RHS: one process per GPU, torch.distributed
with the RCCL backend ("nccl" on ROCm) over xGMI.

The reference has no multi-GPU hot path (only nn.DataParallel over the batch
axis, src/ray_tune.py:58-59).  Three ways to shard it are provided:

* ``ColumnShardedLaplacian`` — feature-column stripes of ONE graph: rank p
  owns columns [c0, c1) of every node and a replicated CSR.  A*x is
  column-separable, so a fixed-grid integration needs no communication at
  all; dopri5 needs one all-reduce of the squared error norm per step
  (``global_rms_norm``); the columns are all-gathered once at the end.  This is
  what ``bench.py --gpus N`` measures (strong scaling: one shared graph).
* ``RowShardedLaplacian`` — the north star's literal design: a 1-D partition of
  the graph rows into contiguous blocks balanced by nnz (``RowPartition``);
  each RHS evaluation computes its rows of f and the next evaluation needs
  every row of the state, so the state is all-gathered (RCCL
  all_gather_into_tensor, half the volume of the all-reduce the north star
  names) before each RHS.  Volume per RHS = world*nbmax*C*4 bytes.
  ``bench.py --gpus N`` reports it beside the column layout.
* ``shard_batch`` — independent objects: each rank integrates its slice of the
  batch axis B (the reference's own parallel axis); no data-path collective
  (``bench.py --mode replicas``, weak scaling).

``local_rhs`` / ``local_stage`` let tests substitute a CPU computation so the
communication pattern — including the fused-stage path the integrator runs
(``rhs_stage``) — is exercised with the gloo backend; the default is the HIP path.
"""
import math

import torch
import torch.distributed as dist

from . import ops


def row_blocks(R, world):
    """Equal row blocks [(r0, r1)] of ceil(R/world) rows (last one shorter)."""
    nb = int(math.ceil(R / world))
    return [(min(R, p * nb), min(R, (p + 1) * nb)) for p in range(world)], nb


def host_rowptr(edge_index, num_nodes):
    """Row pointer [B*N+1] (numpy int64) of the block-diagonal aggregation CSR of
    edge_index [B,2,E] (rows = sources), computed on the host."""
    import numpy as np
    ei = edge_index.detach().cpu().numpy() if isinstance(edge_index, torch.Tensor) else np.asarray(edge_index)
    B = ei.shape[0]
    rows = (ei[:, 0, :] + np.arange(B)[:, None] * int(num_nodes)).reshape(-1)
    rp = np.zeros(B * int(num_nodes) + 1, np.int64)
    rp[1:] = np.cumsum(np.bincount(rows, minlength=B * int(num_nodes)))
    return rp


def balanced_row_blocks(rowptr, world, row_weight=0.0):
    """Contiguous row blocks balanced by work, not by row count (SURVEY §8(e):
    "1-D partition ... balanced by nnz").  Block p ends at the row where the
    cumulative cost nnz(0..r) + row_weight * r is nearest to (p+1)/world of
    the total (rows are never split).  row_weight = 0: pure nnz balance (RMAT hub rows have low ids, so
    equal row counts hand rank 0 most of the edges); a positive weight also
    charges each row's share of the per-RHS state exchange.  ``rowptr``:
    host int array [R+1].  Returns [(r0, r1)] covering [0, R)."""
    import numpy as np
    rp = np.asarray(rowptr, dtype=np.int64)
    R = rp.shape[0] - 1
    cost = rp.astype(np.float64) + float(row_weight) * np.arange(R + 1, dtype=np.float64)
    total = cost[-1]
    cuts = [0]
    for p in range(1, world):
        target = total * p / world
        r = int(np.searchsorted(cost, target, side='left'))
        if 0 < r <= R and target - cost[r - 1] < cost[r] - target:
            r -= 1  # the nearer cut
        cuts.append(min(max(r, cuts[-1]), R))
    cuts.append(R)
    return [(cuts[p], cuts[p + 1]) for p in range(world)]


class RowPartition(object):
    """One rank's share of a row-partitioned CSR, process-group free (so one
    process can build and run every rank's part: tests/test_gpu_sharded.py).

    The gathered state is laid out in padded blocks: rank p's rows [r0_p, r1_p)
    sit at positions p*nbmax + (r - r0_p) of a [world*nbmax, C] buffer, which is
    what ``all_gather_into_tensor`` of equal [nbmax, C] blocks produces.  The
    column ids of the CSR are relabelled into those positions once per graph
    (``col``); the local plan's item rows are positions too, and the outputs are
    addressed through pointers shifted back by rank*nbmax rows."""

    def __init__(self, g, world, rank, row_weight=0.0, chunk=ops.DEFAULT_CHUNK, blocks=None):
        self.world, self.rank = int(world), int(rank)
        rowptr = g.csr.rowptr
        self.blocks = blocks if blocks is not None else balanced_row_blocks(rowptr.cpu().numpy(), world, row_weight)
        self.nbmax = max(max(r1 - r0 for r0, r1 in self.blocks), 1)
        self.r0, self.r1 = self.blocks[self.rank]
        self.pos0 = self.rank * self.nbmax           # position of this rank's first row
        dev = rowptr.device
        starts = torch.tensor([b[0] for b in self.blocks], dtype=torch.int64, device=dev)
        col = g.csr.col[:max(g.nnz, 1)].long()
        if g.nnz:
            blk = torch.searchsorted(starts, col, right=True) - 1
            col = col - starts[blk] + blk * self.nbmax
        self.col = col.to(torch.int32).contiguous()
        self.plan = _local_plan(g.csr, self.r0, self.r1, chunk, self.pos0)

    def pad_state(self, y):
        """Full state [R, C] (global row order) -> the padded [world*nbmax, C] layout."""
        out = torch.zeros((self.world * self.nbmax,) + tuple(y.shape[1:]), dtype=y.dtype, device=y.device)
        for p, (a, b) in enumerate(self.blocks):
            out[p * self.nbmax:p * self.nbmax + (b - a)] = y[a:b]
        return out

    def local_block(self, y):
        """Full state [R, C] -> this rank's zero-padded [nbmax, C] block."""
        out = torch.zeros((self.nbmax,) + tuple(y.shape[1:]), dtype=y.dtype, device=y.device)
        out[:self.r1 - self.r0] = y[self.r0:self.r1]
        return out

    def unpad_state(self, y_full):
        """Padded [world*nbmax, C] -> full [R, C] in global row order."""
        return torch.cat([y_full[p * self.nbmax:p * self.nbmax + (b - a)] for p, (a, b) in enumerate(self.blocks)], 0)

    def rhs(self, g, w, y_full, y_local, x0=None, alpha=None, beta=None, alpha_sigmoid=True, add_source=False,
            stage=None):
        """K1 over this rank's rows: gathers from the padded full state, the
        epilogue's own rows from y_local (x0 and outputs local too)."""
        if self.plan is None:
            return None if stage is not None else torch.zeros_like(y_local)
        return ops.spmm_rhs_rows(g, self.plan, w, y_full, y_local, self.pos0, x0=x0, alpha=alpha, beta=beta,
                                 alpha_sigmoid=alpha_sigmoid, add_source=add_source, stage=stage, col=self.col)


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

    Rows are split into contiguous blocks balanced by nnz (balanced_row_blocks;
    ``row_weight`` > 0 also weighs the rows themselves).  State per rank:
    y_local [nbmax, C] (its row block, zero padded to the largest block).
    Calling the object with (t, y_local) all-gathers the blocks into the padded
    [world*nbmax, C] layout of RowPartition, aggregates the local rows of A and
    returns f_local [nbmax, C]; it drops into gnpde.odeint unchanged."""

    graph_capturable = False  # an RCCL all-gather per RHS: the integrator runs it eagerly

    def __init__(self, edge_index, edge_weight, num_nodes, alpha, beta=None, x0_local=None, add_source=False,
                 alpha_sigmoid=True, group=None, local_rhs=None, chunk=ops.DEFAULT_CHUNK, row_weight=0.0,
                 local_stage=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        B, _, E = edge_index.shape
        self.N = int(num_nodes)
        self.R = B * self.N
        self.alpha, self.beta = alpha, beta
        self.x0_local = x0_local
        self.add_source, self.alpha_sigmoid = add_source, alpha_sigmoid
        self.nfe = 0
        self.local_rhs = local_rhs
        # local_stage(t, y_full, r0, r1, y_local, stage): an injected (test) RHS that also
        # writes the fused stage outputs; host_stages lets the integrator's fused path run it
        self.local_stage = local_stage
        self.host_stages = local_stage is not None
        if local_rhs is None and local_stage is None:
            self.g = ops.GraphCSR(edge_index, self.N, chunk=chunk)
            self.w = self.g.gather_weights(edge_weight)
            self.part = RowPartition(self.g, self.world, self.rank, row_weight=row_weight, chunk=chunk)
            self.blocks, self.nb = self.part.blocks, self.part.nbmax
        else:  # injected arithmetic (tests): the same nnz-balanced blocks from a host CSR row pointer
            self.part = None
            self.blocks = balanced_row_blocks(host_rowptr(edge_index, self.N), self.world, row_weight)
            self.nb = max(max(r1 - r0 for r0, r1 in self.blocks), 1)
        self.r0, self.r1 = self.blocks[self.rank]

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
            return self.local_rhs(t, self.unpad(y_full), self.r0, self.r1, y_local)
        return self.part.rhs(self.g, self.w, y_full, y_local, x0=self.x0_local, alpha=self.alpha, beta=self.beta,
                             alpha_sigmoid=self.alpha_sigmoid, add_source=self.add_source)

    def rhs_stage(self, t, y_local, stage):
        """One RHS with the solver's stage combination in the epilogue (the path
        gnpde.integrator's fused fixed-grid solve takes): all-gather, then K1
        over this rank's rows writing the stage outputs."""
        self.nfe += 1
        y_full = self.gather(y_local)
        if self.local_stage is not None:
            self.local_stage(t, self.unpad(y_full), self.r0, self.r1, y_local, stage)
            return
        if self.local_rhs is not None:
            raise NotImplementedError("rhs_stage needs local_stage (or the HIP path)")
        self.part.rhs(self.g, self.w, y_full, y_local, x0=self.x0_local, alpha=self.alpha, beta=self.beta,
                      alpha_sigmoid=self.alpha_sigmoid, add_source=self.add_source, stage=stage)

    def scatter(self, y):
        """Full state [R, C] -> this rank's zero-padded block [nb, C]."""
        out = torch.zeros((self.nb,) + tuple(y.shape[1:]), dtype=y.dtype, device=y.device)
        out[:self.r1 - self.r0] = y[self.r0:self.r1]
        return out

    def unpad(self, y_full):
        """Gathered padded blocks [world*nb, C] -> full state [R, C] in row order."""
        return torch.cat([y_full[p * self.nb:p * self.nb + (b - a)] for p, (a, b) in enumerate(self.blocks)], 0)


def _local_plan(csr, r0, r1, chunk, pos0=None):
    """Plan over rows [r0, r1) of a global CSR.  Items keep global edge offsets
    and get row ids shifted to the rows' positions in the gathered state
    (pos0 + row - r0; pos0 defaults to r0, i.e. global ids), so the epilogue
    reads its own row from the gathered state; outputs are addressed through
    pointers shifted back by pos0 rows (ops.spmm_rhs_rows)."""
    if r1 <= r0:
        return None
    pos0 = r0 if pos0 is None else pos0
    rowptr = csr.rowptr[r0:r1 + 1].contiguous()
    plan = ops.build_plan(rowptr, r1 - r0, int(csr.nnz), chunk)
    if plan.n_items:
        plan.items.view(-1, 4)[:plan.n_items, 0] += pos0
    if plan.n_heavy:
        plan.heavy.view(-1, 4)[:plan.n_heavy, 0] += pos0
    return plan


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
        self._layout = None   # the NodeLayout a fixed-grid solve runs in (gnpde.integrator), else None
        self._lay_ops = None  # (layout, its CSR-order weights, its x0 stripe)
        if local_rhs is None:
            self.edge_weight = edge_weight
            self.g = ops.GraphCSR(edge_index, self.N, chunk=chunk)
            self.w = self.g.gather_weights(edge_weight)

    def node_layout(self, x_local):
        """The graph's locality numbering for a fixed-grid solve of the stripes
        (ops.NodeLayout), decided on the FULL state's size so that every rank of
        a job — and the unsharded run it is compared with — runs the same
        numbering.  Bit-identical results (the stripe's rows are permuted, each
        row keeps its edges and their order)."""
        if self._layout is not None or self.local_rhs is not None or x_local.dim() != 3:
            return None
        if not ops.layout_worthwhile(x_local.shape[0] * x_local.shape[1], self.C, x_local.element_size()):
            return None
        return self.g.node_layout

    def _operands(self):
        """(graph, CSR-order weights, x0 stripe) in the numbering of the running solve."""
        lay = self._layout
        if lay is None:
            return self.g, self.w, self.x0_local
        if self._lay_ops is None or self._lay_ops[0] is not lay:
            x0 = lay.to_internal(self.x0_local) if (self.add_source and self.x0_local is not None) else None
            self._lay_ops = (lay, lay.graph.gather_weights(self.edge_weight), x0)
        return lay.graph, self._lay_ops[1], self._lay_ops[2]

    def graph_capture_state(self, x):
        """What a captured fused step reads (gnpde.integrator._capture_state)."""
        g, w, x0 = self._operands()
        return (g, w) + ((x0,) if self.add_source else ())

    def capture_key_tensors(self):
        return tuple(t for t in (self.alpha, self.beta) if isinstance(t, torch.Tensor))

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
        g, w, x0 = self._operands()
        ops.spmm_rhs(g, w, x_local, x0=x0, alpha=self.alpha, beta=self.beta,
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
