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
import os

import torch
import torch.distributed as dist

from . import ops

# Step graphs that capture the RHS's collectives (RCCL through torch.distributed into
# the hipGraph: tools/rccl_capture_check.py replays all_reduce / all_gather_into_tensor
# correctly).  A sharded RHS on the nccl backend is captured at a world of one (its
# collectives then run in the graph) and, with GNPDE_CAPTURE_COLLECTIVES=1, at any
# world — opt-in there: the multi-rank capture has not run on this build's hardware.
CAPTURE_COLLECTIVES = os.environ.get('GNPDE_CAPTURE_COLLECTIVES', '0') == '1'


def _capturable(group, world, collectives=True):
    """Whether a sharded RHS's steps may be captured and replayed: no collective in the
    RHS at all, or RCCL collectives at a world of one (or GNPDE_CAPTURE_COLLECTIVES)."""
    if not collectives:
        return True
    if dist.get_backend(group) != 'nccl':
        return False
    return world == 1 or CAPTURE_COLLECTIVES


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


# The row partition's default row weight: besides its edges' gathers a row costs its own row read and
# its output write — about two gathered rows.  G-rmat (configs[4]) at 8 ranks, the slowest rank's rk4-step
# compute (tools/mgpu_implied_grmat.py, profiles/r06_mgpu_rows_row_weight.jsonl): row_weight 0 / 1 / 2 / 4 / 8
# -> 3.23 / 2.32 / 1.78 / 1.98 / 2.44 ms (pure nnz balance leaves the low-degree tail of the in-degree
# numbering, every row of which still moves 2 KB, on the last rank).
ROW_WEIGHT = 2.0


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

    def __init__(self, g, world, rank, row_weight=ROW_WEIGHT, chunk=None, blocks=None):
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
        self.plan = _local_plan(g.csr, self.r0, self.r1, g.chunk if chunk is None else chunk, self.pos0)

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
    returns f_local [nbmax, C]; it drops into gnpde.odeint unchanged.

    On a large graph (ops.LAYOUT_MIN_ROWS, ops.NODE_ORDER 'degree') the rows are
    those of the graph's in-degree numbering (ops.NodeLayout, as the unsharded and
    column-striped solves): scatter() / unpad() map from / to the caller's numbering.
    The source term takes the full x0 (``x0=``, the caller's numbering; scattered
    here) or ``x0_local`` = scatter(x0); a block of another shape is rejected."""

    autonomous = True  # the RHS does not read t (gnpde.base_classes.ODEFunc.autonomous)

    fused_adaptive = False    # the adaptive solvers' wide stages run in column stripes or unsharded

    @property
    def graph_capturable(self):
        """An all-gather per RHS (none at a world of one: the state blocks are the
        gathered buffers): captured at a world of one, or with GNPDE_CAPTURE_COLLECTIVES
        on RCCL; injected host arithmetic never."""
        if self.part is None:
            return False
        return self.world == 1 or _capturable(self.group, self.world)

    def graph_capture_state(self, y):
        """What a captured step reads besides its state buffers (integrator._capture_state)."""
        return (self.g, self.w, self.part.col, self.part.plan) + ((self.x0_local,) if self.add_source else ())

    def capture_key_tensors(self):
        return tuple(t for t in (self.alpha, self.beta) if isinstance(t, torch.Tensor))

    def __init__(self, edge_index, edge_weight, num_nodes, alpha, beta=None, x0_local=None, add_source=False,
                 alpha_sigmoid=True, group=None, local_rhs=None, chunk=None, row_weight=ROW_WEIGHT,
                 local_stage=None, node_order=None, x0=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        B, _, E = edge_index.shape
        self.N = int(num_nodes)
        self.R = B * self.N
        self.alpha, self.beta = alpha, beta
        self.add_source, self.alpha_sigmoid = add_source, alpha_sigmoid
        self.nfe = 0
        self.local_rhs = local_rhs
        # local_stage(t, y_full, r0, r1, y_local, stage): an injected (test) RHS that also
        # writes the fused stage outputs; host_stages lets the integrator's fused path run it
        self.local_stage = local_stage
        self.host_stages = local_stage is not None
        self.lay = None
        if local_rhs is None and local_stage is None:
            self.g = ops.GraphCSR(edge_index, self.N, chunk=chunk)
            order = ops.NODE_ORDER if node_order is None else node_order
            if order == "degree" and self.R >= ops.LAYOUT_MIN_ROWS:
                # the rows of the in-degree numbering: hot gathered rows together (G-rmat rk4
                # 232 -> 281 RHS/s unsharded); COO-order weights apply unchanged
                self.lay = self.g.node_layout
                self.g = self.lay.graph
            self.w = self.g.gather_weights(edge_weight)
            self.part = RowPartition(self.g, self.world, self.rank, row_weight=row_weight, chunk=chunk)
            self.blocks, self.nb = self.part.blocks, self.part.nbmax
        else:  # injected arithmetic (tests): the same nnz-balanced blocks from a host CSR row pointer
            self.part = None
            self.blocks = balanced_row_blocks(host_rowptr(edge_index, self.N), self.world, row_weight)
            self.nb = max(max(r1 - r0 for r0, r1 in self.blocks), 1)
        self.r0, self.r1 = self.blocks[self.rank]
        if x0 is not None:
            x0_local = self.scatter(x0)
        if add_source and x0_local is not None and tuple(x0_local.shape[:1]) != (self.nb,):
            raise ValueError("RowShardedLaplacian: x0_local must be this rank's padded block [%d, C] (scatter(x0), "
                             "in the graph's numbering), got %s; or pass the full x0 as x0=" %
                             (self.nb, tuple(x0_local.shape)))
        self.x0_local = x0_local
        # data_ptr of a state block handed out by alloc_state -> a weak reference to its
        # gathered buffer's storage (no strong reference, so buffers the
        # integrator drops are freed; expired entries are pruned at the next alloc_state)
        self._blocks_out = {}
        self._gbuf = None  # the gathered buffer of other states

    def alloc_state(self, like):
        """A state block [nb, C] that is rank p's row block of a gathered buffer
        [world*nb, C] (gnpde.integrator places its stage inputs here): the all-gather
        before each RHS then runs in place — no send copy, and at world 1 no copy at
        all."""
        from torch.multiprocessing.reductions import StorageWeakRef
        for k in [k for k, w in self._blocks_out.items() if w.expired()]:
            del self._blocks_out[k]
        full = torch.empty((self.world * self.nb,) + tuple(like.shape[1:]), dtype=like.dtype, device=like.device)
        blk = full[self.rank * self.nb:(self.rank + 1) * self.nb]
        self._blocks_out[blk.data_ptr()] = StorageWeakRef(full.untyped_storage())
        return blk

    def _gathered_base(self, y_local):
        """The gathered buffer y_local is the row block of (alloc_state), else None."""
        base = y_local._base
        if base is None or y_local.data_ptr() not in self._blocks_out:
            return None
        shape = (self.world * self.nb,) + tuple(y_local.shape[1:])
        if (tuple(base.shape) != shape or base.dtype != y_local.dtype or not base.is_contiguous() or
                y_local.data_ptr() != base.data_ptr() + self.rank * self.nb * y_local[0].numel() * base.element_size()):
            return None
        return base

    def gather(self, y_local):
        """All-gather of the row blocks (RCCL over xGMI on ROCm): in place when
        y_local is a block of one of this object's gathered buffers (alloc_state),
        else into a persistent buffer."""
        y_local = y_local.contiguous()
        full = self._gathered_base(y_local)
        if full is not None:
            if self.world > 1:
                dist.all_gather_into_tensor(full, y_local, group=self.group)
            return full
        shape = (self.world * self.nb,) + tuple(y_local.shape[1:])
        out = self._gbuf
        if out is None or tuple(out.shape) != shape or out.dtype != y_local.dtype or out.device != y_local.device:
            out = self._gbuf = torch.empty(shape, dtype=y_local.dtype, device=y_local.device)
        if self.world == 1:
            out.copy_(y_local)  # no collective at a world of one (whatever the backend)
        else:
            dist.all_gather_into_tensor(out, y_local, group=self.group)
        return out

    def __call__(self, t, y_local):
        self.nfe += 1
        y_full = self.gather(y_local)
        if self.local_rhs is not None:
            return self.local_rhs(t, self.unpad(y_full), self.r0, self.r1, y_local)
        return self.part.rhs(self.g, self.w, y_full, y_local, x0=self.x0_local, alpha=self.alpha, beta=self.beta,
                             alpha_sigmoid=self.alpha_sigmoid, add_source=self.add_source)

    @property
    def affine(self):
        """f = σ(α)(A − I) y [+ β x0] is affine in y — on the HIP path; an injected
        test RHS is taken as it is.  The fused adaptive loop that would use it (the
        affine first stage, the Krylov step) is not taken by the row partition
        (fused_adaptive = False: its adaptive solves run the restated loop with the
        global norm); the flag serves its fixed-grid stages and the column stripes."""
        return self.local_rhs is None and self.local_stage is None

    def rhs_stage(self, t, y_local, stage, linear=False):
        """One RHS with the solver's stage combination in the epilogue (the path
        gnpde.integrator's fused solves take): all-gather, then K1 over this rank's
        rows writing the stage outputs.  linear=True: the linear part alone (no
        source term; Stage.f_lin, the Krylov step)."""
        self.nfe += 1
        y_full = self.gather(y_local)
        if self.local_stage is not None:
            self.local_stage(t, self.unpad(y_full), self.r0, self.r1, y_local, stage)
            return
        if self.local_rhs is not None:
            raise NotImplementedError("rhs_stage needs local_stage (or the HIP path)")
        src = self.add_source and not linear
        self.part.rhs(self.g, self.w, y_full, y_local, x0=self.x0_local if src else None, alpha=self.alpha,
                      beta=self.beta, alpha_sigmoid=self.alpha_sigmoid, add_source=src, stage=stage)

    def global_rms_norm(self, t):
        """RMS over the whole state (all row blocks, the padding rows excluded): the
        error norm an adaptive solve of the row partition must pass
        (options=dict(norm=sh.global_rms_norm)) so every rank takes the same steps;
        one all-reduce of 2 doubles."""
        n = self.r1 - self.r0
        own = t.reshape(-1, t.shape[-1])[:n]
        v = torch.stack([own.double().pow(2).sum(), torch.tensor(float(own.numel()), dtype=torch.float64,
                                                                  device=t.device)])
        dist.all_reduce(v, group=self.group)
        return (v[0] / v[1]).sqrt().to(t.dtype)

    def scatter(self, y):
        """Full state [R, C] (the caller's numbering) -> this rank's zero-padded block [nb, C]."""
        if self.lay is not None:
            y = self.lay.to_internal(y.reshape(-1, y.shape[-1]))
        out = torch.zeros((self.nb,) + tuple(y.shape[1:]), dtype=y.dtype, device=y.device)
        out[:self.r1 - self.r0] = y[self.r0:self.r1]
        return out

    def unpad(self, y_full):
        """Gathered padded blocks [world*nb, C] -> full state [R, C] in the caller's numbering."""
        y = torch.cat([y_full[p * self.nb:p * self.nb + (b - a)] for p, (a, b) in enumerate(self.blocks)], 0)
        return self.lay.to_user(y) if self.lay is not None else y


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

    autonomous = True  # the RHS does not read t (gnpde.base_classes.ODEFunc.autonomous)

    def __init__(self, edge_index, edge_weight, num_nodes, C, alpha, beta=None, x0_local=None, add_source=False,
                 alpha_sigmoid=True, group=None, local_rhs=None, chunk=None):
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

    @property
    def affine(self):
        """f is affine in the stripe (gnpde.integrator's affine first stage and Krylov
        step) on the HIP path."""
        return self.local_rhs is None

    def rhs_stage(self, t, x_local, stage, linear=False):
        """One RHS with the stage combination in the epilogue; linear=True: the linear
        part alone (no source term)."""
        self.nfe += 1
        if self.local_rhs is not None:
            raise NotImplementedError
        g, w, x0 = self._operands()
        src = self.add_source and not linear
        ops.spmm_rhs(g, w, x_local, x0=x0 if src else None, alpha=self.alpha, beta=self.beta,
                     alpha_sigmoid=self.alpha_sigmoid, add_source=src, stage=stage)

    def global_rms_norm(self, t):
        """RMS over the full state (all stripes): one all-reduce of 2 doubles."""
        v = torch.stack([t.double().pow(2).sum(), torch.tensor(float(t.numel()), dtype=torch.float64,
                                                                device=t.device)])
        dist.all_reduce(v, group=self.group)
        return (v[0] / v[1]).sqrt().to(t.dtype)

    def reduce_error_sq(self, pair):
        """dopri5's squared error sum and element count over all stripes (in place;
        the fused adaptive step, gnpde.integrator._RKAdaptiveFused)."""
        dist.all_reduce(pair, group=self.group)

    def gather(self, x_local):
        """All stripes -> full [B,N,C] (once, at the end of an integration)."""
        return _gather_cols(x_local, self.cols, self.world, self.group)


# --------------------------------------------------------------------------- transformer attention RHS
class _Comm(object):
    """The collectives of the sharded transformer RHS: torch.distributed on the
    job's group (RCCL over xGMI for device tensors).  Tests substitute an object
    with the same two methods (e.g. staging device tensors through gloo)."""

    def __init__(self, group=None):
        self.group = group

    def all_reduce(self, t):
        dist.all_reduce(t, group=self.group)

    def all_gather_into_tensor(self, out, t):
        dist.all_gather_into_tensor(out, t, group=self.group)


class _HipAttentionLocal(object):
    """A rank's arithmetic of the sharded transformer RHS on the HIP path (tests
    inject a CPU object with the same methods to run the collectives under gloo)."""

    def __init__(self, g):
        self.g = g
        self._uni = None

    def keysum(self, x, Wk, bk):
        return ops.ref_keysum(self.g, x, Wk, bk)

    def node_scores(self, x, S, Wq, bq, heads):
        return ops.ref_scores_from_keysum(self.g, x, S, Wq, bq, heads)

    def project(self, x, W, b):
        return ops.linear(x, W, b)[0]

    def uniform_weights(self, heads):
        if self._uni is None:
            ns = ops.uniform_scores(heads)
            m, rl = ops.softmax_stats(self.g, ns, 0)
            self._uni = ops.attn_weights(self.g, ns, m, rl, 0)
        return self._uni

    def stats_rows(self, ns, r0, r1, packed=None):
        """The destination statistics (norm_idx 1) of groups [r0, r1) only: a list of
        full-size tensors with those rows written (packed records for two-head
        reference and per-edge scores, m and rl otherwise or with packed=False), or
        None outside K2."""
        return _hip_stats_rows(self.g, ns, r0, r1, packed)

    def aggregate(self, ns, norm_idx, x, stage=None, stats=None, **kw):
        if ns is None:  # uniform weights (fork scaled_dot, norm_idx 0): graph-only
            return ops.spmm_rhs(self.g, self.uniform_weights(kw.pop('heads')), x, stage=stage, **kw)
        kw.pop('heads', None)
        m, rl, mr = _stats_args(stats)
        return ops.attn_rhs(self.g, ns, m, rl, norm_idx, x, stage=stage, mr=mr, **kw)

    def n_edges(self):
        return self.g.nnz

    def edge_blocks(self, world):
        """Blocks of CSR positions, one per rank, aligned to CSR rows and balanced by
        nnz: under source-grouped softmax (norm_idx 0) a block holds whole groups.
        Returns ([(e0, e1)], [(r0, r1)])."""
        rp = self.g.csr.rowptr.cpu().numpy()
        rows = balanced_row_blocks(rp, world)
        return [(int(rp[a]), int(rp[b])) for a, b in rows], rows

    def src_stats(self, ns, r0, r1):
        """The source-grouped statistics (norm_idx 0) of rows [r0, r1): [m, rl] full-size
        with those rows written (K2 over a row-range plan), or None outside K2."""
        r = ops.softmax_stats(self.g, ns, 0, packed=False, rows=(r0, r1))
        return None if r is NotImplemented else [r[0], r[1]]

    def edge_weights(self, ns, norm_idx, stats, e0, e1):
        """The head-mean weights of CSR positions [e0, e1) from the gathered m, rl."""
        return ops.attn_weights(self.g, ns, stats[0], stats[1], norm_idx, edges=(e0, e1))

    def weighted(self, w, x, stage=None, **kw):
        """K1 over this rank's columns with the gathered [nnz] weights."""
        kw.pop('heads', None)
        return ops.spmm_rhs(self.g, w, x, stage=stage, **kw)


def _hip_stats_rows(g, ns, r0, r1, packed=None):
    if packed is None:
        packed = ns.heads == 2 or ns.mode != ops._lib.SCORE_REFERENCE
    r = ops.softmax_stats(g, ns, 1, packed=packed, rows=(r0, r1))
    if r is NotImplemented:
        return None
    return [r[2]] if packed else [r[0], r[1]]


def _stats_args(stats):
    """(m, rl, mr) for ops.attn_rhs from a gathered statistics list (None: compute them)."""
    if stats is None:
        return None, None, None
    return (None, None, stats[0]) if len(stats) == 1 else (stats[0], stats[1], None)


def _gather_row_blocks(comm, v, blocks, rank, world, nb):
    """Rows [r0, r1) of this rank's full-size [R, k] tensor v, exchanged so every rank
    holds all of them: padded [nb, k] blocks all-gathered, then unpadded."""
    r0, r1 = blocks[rank]
    if world == 1:
        return v
    blk = torch.zeros((nb,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
    blk[:r1 - r0] = v[r0:r1]
    pad = torch.empty((world * nb,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
    comm.all_gather_into_tensor(pad, blk)
    return torch.cat([pad[p * nb:p * nb + (b - a)] for p, (a, b) in enumerate(blocks)], 0)


def _gather_edge_blocks(comm, w, blocks, world):
    """This rank's weights of CSR positions [e0, e1), exchanged so every rank holds all
    nnz of them: padded blocks all-gathered, then unpadded (one copy of E floats)."""
    if world == 1:
        return w
    nb = max(max(b - a for a, b in blocks), 1)
    blk = torch.zeros(nb, dtype=w.dtype, device=w.device)
    blk[:w.numel()] = w
    pad = torch.empty(world * nb, dtype=w.dtype, device=w.device)
    comm.all_gather_into_tensor(pad, blk)
    return torch.cat([pad[p * nb:p * nb + (b - a)] for p, (a, b) in enumerate(blocks)], 0)


def _dst_blocks(edge_index, N, world, g=None):
    """Destination-row blocks balanced by in-degree (the CSC's nnz): each rank forms the
    softmax statistics of one block (norm_idx 1)."""
    rp = g.csc.rowptr.cpu().numpy() if g is not None else host_rowptr(edge_index.flip(1) if isinstance(
        edge_index, torch.Tensor) else edge_index[:, ::-1], N)
    blocks = balanced_row_blocks(rp, world)
    return blocks, max(max(b - a for a, b in blocks), 1)


def _qk_scores(qk, heads, att):
    """NodeScores of the per-edge scaled_dot over a [R, 2 att] q | k buffer (rows of
    ld 2 att: q and k are column views of it)."""
    ns = ops.NodeScores(ops._lib.SCORE_DOT, heads, att // heads, q=qk[:, :att], k=qk[:, att:])
    ns.ldqk = qk.shape[1]
    return ns


class ColumnShardedTransformer(object):
    """Column-striped transformer attention RHS (ODEFuncTransformerAtt,
    src/function_transformer_attention.py:44-59, 218-267):
    rank p holds columns [c0, c1) of every node and the replicated CSR / CSC.
    The scores read all C columns, but both score forms are LINEAR in the
    columns, so each rank forms its stripe's share and one all-reduce completes
    it; the aggregation is then column-local:

    * fork scaled_dot (score_mode 'reference'): the key sum S [B, att] (fp64, the
      stripe's columns of Wk) all-reduced, then the node scores cs [R, heads]
      (fp64, the stripe's columns of Wq) all-reduced — 2 R heads 8 bytes per RHS;
      under source-grouped softmax (norm_idx 0) the weights are 1/outdeg: no
      communication at all;
    * per-edge scaled_dot: the projection q | k [R, 2 att] (fp32, the stripe's
      columns of [Wq; Wk]) all-reduced — R 2 att 4 bytes per RHS.

    The biases enter on rank 0 only.  Under destination-grouped softmax (norm_idx
    1) each rank forms the statistics of one block of destination rows and the
    blocks are all-gathered; with ``edge_weights`` (default at world > 1) each
    rank also forms the head-mean weights of one block of edges, all-gathered
    (E x 4 bytes), and aggregates its own columns with the plain-weight K1;
    otherwise it aggregates with the fused kernels.  Drops into gnpde.odeint: __call__ /
    rhs_stage (fixed-grid fused stages, the adaptive solvers' wide stages),
    global_rms_norm / reduce_error_sq (dopri5's error norm over all stripes)."""

    autonomous = True  # the RHS does not read t (gnpde.base_classes.ODEFunc.autonomous)

    @property
    def graph_capturable(self):
        """Collectives per RHS (the uniform weights have none): captured on RCCL at a
        world of one, or at any world with GNPDE_CAPTURE_COLLECTIVES=1."""
        if not isinstance(self.local, _HipAttentionLocal):
            return False
        return _capturable(self.group, self.world, collectives=not self.uniform)

    def graph_capture_state(self, y):
        """The derived objects a captured step reads (integrator._capture_state)."""
        return (self.local.g, self.Wq, self.Wk, self.bq, self.bk, self.Wcat, self.bcat) + \
            ((self.x0_local,) if self.add_source else ())

    def capture_key_tensors(self):
        return tuple(t for t in (self.alpha, self.beta) if isinstance(t, torch.Tensor))

    def __init__(self, edge_index, num_nodes, C, Wq, bq, Wk, bk, heads, norm_idx, alpha, score_mode='reference',
                 beta=None, x0_local=None, add_source=False, alpha_sigmoid=True, group=None, local=None,
                 chunk=None, comm=None, partition_stats=True, edge_weights=None):
        self.group = group
        self.comm = comm if comm is not None else _Comm(group)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.C = int(C)
        self.cols = col_blocks(self.C, self.world)
        self.c0, self.c1 = self.cols[self.rank]
        self.N = int(num_nodes)
        self.heads, self.norm_idx = int(heads), int(norm_idx)
        self.score_mode = score_mode
        self.att = int(Wq.shape[0])
        self.alpha, self.beta = alpha, beta
        self.x0_local = x0_local
        self.add_source, self.alpha_sigmoid = add_source, alpha_sigmoid
        self.nfe = 0
        first = self.rank == 0
        sl = slice(self.c0, self.c1)
        self.Wq, self.Wk = Wq[:, sl].contiguous(), Wk[:, sl].contiguous()
        self.bq = bq.clone() if first else torch.zeros_like(bq)
        self.bk = bk.clone() if first else torch.zeros_like(bk)
        self.Wcat = torch.cat([self.Wq, self.Wk], 0).contiguous()
        self.bcat = torch.cat([self.bq, self.bk], 0).contiguous()
        self.uniform = score_mode == 'reference' and self.norm_idx == 0
        g = ops.GraphCSR(edge_index, self.N, chunk=chunk) if local is None else None
        self.local = local if local is not None else _HipAttentionLocal(g)
        # destination-grouped softmax (norm_idx 1): each rank forms the statistics of one block
        # of destination rows and the blocks are all-gathered, instead of
        # every rank forming all of them
        self.partition_stats = bool(partition_stats) and self.norm_idx == 1 and not self.uniform
        if self.partition_stats:
            self.dblocks, self.dnb = _dst_blocks(edge_index, self.N, self.world, g)
        # edge-sharded weights (norm_idx 1, the statistics partitioned): each rank forms the
        # head-mean weights of one block of CSR positions from the gathered statistics, the
        # blocks are all-gathered (E x 4 bytes) and every rank aggregates its columns with the
        # plain-weight K1 — the per-edge work (scores, exponentials, the statistics' loads)
        # divided by the world instead of repeated in every rank's fused K1.  Default: on for
        # world > 1 on the HIP path (at one rank the fused K1 is faster).
        # Under source-grouped softmax (norm_idx 0, per-edge scores) the blocks are whole CSR
        # rows: a rank forms its rows' statistics and their weights, and only the weights are
        # exchanged.
        if edge_weights is None:
            edge_weights = self.world > 1 and isinstance(self.local, _HipAttentionLocal)
        self.edge_weights = bool(edge_weights) and not self.uniform and (self.partition_stats or self.norm_idx == 0)
        if self.edge_weights:
            self.eblocks, self.erows = self.local.edge_blocks(self.world)
        self.bytes_per_rhs = 0  # collective payload of the last RHS (bench.py)

    def split(self, x):
        """[B,N,C] -> this rank's contiguous column stripe."""
        return x[..., self.c0:self.c1].contiguous()

    def _kw(self):
        return dict(x0=self.x0_local, alpha=self.alpha, beta=self.beta, rhs=True, alpha_sigmoid=self.alpha_sigmoid,
                    add_source=self.add_source, heads=self.heads)

    def scores(self, x_local):
        """The full node-level operands of the scores (None for uniform weights)."""
        if self.uniform:
            self.bytes_per_rhs = 0
            return None
        if self.score_mode == 'reference':
            S = self.local.keysum(x_local, self.Wk, self.bk)
            self.comm.all_reduce(S)
            cs = self.local.node_scores(x_local, S, self.Wq, self.bq, self.heads)
            self.comm.all_reduce(cs)
            self.bytes_per_rhs = S.numel() * 8 + cs.numel() * 8
            return ops.NodeScores(ops._lib.SCORE_REFERENCE, self.heads, self.att // self.heads, cs=cs)
        qk = self.local.project(x_local, self.Wcat, self.bcat)
        self.comm.all_reduce(qk)
        self.bytes_per_rhs = qk.numel() * 4
        return _qk_scores(qk, self.heads, self.att)

    def stats(self, ns):
        """This rank's block of the destination statistics, all-gathered (None: the
        aggregation forms them all itself)."""
        if not self.partition_stats:
            return None
        d0, d1 = self.dblocks[self.rank]
        st = self.local.stats_rows(ns, d0, d1, packed=False) if getattr(self, 'edge_weights', False) else \
            self.local.stats_rows(ns, d0, d1)
        if st is None:
            return None
        st = [_gather_row_blocks(self.comm, v, self.dblocks, self.rank, self.world, self.dnb) for v in st]
        if self.world > 1:
            self.bytes_per_rhs += sum(self.world * self.dnb * v[0].numel() * v.element_size() for v in st)
        return st

    def weights(self, ns, stats):
        """This rank's block of the [nnz] weights from the gathered statistics, all-gathered."""
        e0, e1 = self.eblocks[self.rank]
        w = self.local.edge_weights(ns, self.norm_idx, stats, e0, e1)
        w = _gather_edge_blocks(self.comm, w, self.eblocks, self.world)
        if self.world > 1:
            self.bytes_per_rhs += self.world * max(max(b - a for a, b in self.eblocks), 1) * 4
        return w

    def _aggregate(self, x_local, stage):
        ns = self.scores(x_local)
        if self.edge_weights and self.norm_idx == 0:
            st = self.local.src_stats(ns, *self.erows[self.rank])  # this rank's groups: no exchange
            if st is not None:
                return self.local.weighted(self.weights(ns, st), x_local, stage=stage, **self._kw())
            stats = None
        else:
            stats = self.stats(ns)
        if self.edge_weights and stats is not None:
            return self.local.weighted(self.weights(ns, stats), x_local, stage=stage, **self._kw())
        return self.local.aggregate(ns, self.norm_idx, x_local, stage=stage, stats=stats, **self._kw())

    def __call__(self, t, x_local):
        self.nfe += 1
        return self._aggregate(x_local, None)

    def rhs_stage(self, t, x_local, stage):
        self.nfe += 1
        self._aggregate(x_local, stage)

    def global_rms_norm(self, t):
        v = torch.stack([t.double().pow(2).sum(), torch.tensor(float(t.numel()), dtype=torch.float64,
                                                                device=t.device)])
        self.comm.all_reduce(v)
        return (v[0] / v[1]).sqrt().to(t.dtype)

    def reduce_error_sq(self, pair):
        """dopri5's squared error sum and element count over all stripes (in place)."""
        self.comm.all_reduce(pair)

    def gather(self, x_local):
        """All stripes -> full [B,N,C] (once, at the end of an integration)."""
        return _gather_cols(x_local, self.cols, self.world, self.group)


def _gather_cols(x_local, cols, world, group):
    widths = [c1 - c0 for c0, c1 in cols]
    wmax = max(widths)
    shp = tuple(x_local.shape[:-1])
    pad = torch.zeros(shp + (wmax,), dtype=x_local.dtype, device=x_local.device)
    pad[..., :x_local.shape[-1]] = x_local
    pad = pad.reshape((-1, wmax))
    out = torch.empty((world * pad.shape[0], wmax), dtype=x_local.dtype, device=x_local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    out = out.view((world,) + shp + (wmax,))
    return torch.cat([out[p][..., :widths[p]] for p in range(world)], dim=-1)


class _RowView(object):
    """The B = 1 row range [r0, r1) of a GraphCSR as the node-score kernels see a
    graph (B, N, R, indeg): the key sum and node scores of one rank's rows."""

    def __init__(self, g, r0, r1):
        self.B, self.N, self.R = 1, r1 - r0, r1 - r0
        self.indeg = g.indeg[r0:r1]
        self._owner = g


class _HipRowAttentionLocal(object):
    """A rank's arithmetic of RowShardedTransformer on the HIP path: the shares of
    its own rows [r0, r1) (key sum, node scores, q | k projection), the softmax
    statistics over the whole (replicated) CSC, and K1 over its rows' local plan.
    An empty row block (a hub row can take a whole rank's share of the nnz) has
    zero shares and no aggregation, but its rank still joins every collective
    (ADVICE r4).  Tests inject a CPU object with the same methods."""

    def __init__(self, g, r0, r1, chunk):
        self.g, self.r0, self.r1 = g, r0, r1
        self.n = r1 - r0
        self.plan = _local_plan(g.csr, r0, r1, g.chunk if chunk is None else chunk)  # item rows = global row ids
        self.view = _RowView(g, r0, r1)
        self._uni = None

    def keysum(self, own, Wk, bk):
        if self.n == 0:
            return torch.zeros((1, Wk.shape[0]), dtype=torch.float64, device=Wk.device)
        return ops.ref_keysum(self.view, own, Wk, bk)

    def node_scores(self, own, S, Wq, bq, heads):
        if self.n == 0:
            return torch.zeros((0, heads), dtype=torch.float64, device=Wq.device)
        return ops.ref_scores_from_keysum(self.view, own, S, Wq, bq, heads)

    def project(self, own, W, b):
        if self.n == 0:
            return torch.zeros((0, W.shape[0]), dtype=torch.float32, device=W.device)
        return ops.linear(own, W, b)[0]

    def stats_rows(self, ns, r0, r1):
        return _hip_stats_rows(self.g, ns, r0, r1)

    def aggregate(self, ns, norm_idx, x_full, y_local, stage=None, heads=None, stats=None, **kw):
        g = self.g
        if self.plan is None:  # no rows: nothing to write (the block is padding)
            return None if stage is not None else torch.zeros_like(y_local)
        kw['stage'] = stage
        m0, rl0, mr0 = _stats_args(stats)
        if ns is None:  # fork scaled_dot under source-grouped softmax: 1/outdeg weights, graph-only
            if self._uni is None:
                un = ops.uniform_scores(heads)
                m, rl = ops.softmax_stats(g, un, 0)
                self._uni = ops.attn_weights(g, un, m, rl, 0)
            return ops.spmm_rhs_rows(g, self.plan, self._uni, x_full, y_local, self.r0, **kw)
        if ns.mode == ops._lib.SCORE_REFERENCE:  # destination-grouped (norm_idx 1)
            if mr0 is not None:
                w = ops.RefDstWeights(ns.cs, None, None, 2, mr=mr0)
            elif m0 is not None:
                w = ops.RefDstWeights(ns.cs, m0, rl0, heads)
            elif heads == 2:
                _, _, mr = ops.softmax_stats(g, ns, 1, packed=True)
                w = ops.RefDstWeights(ns.cs, None, None, 2, mr=mr)
            else:
                m, rl = ops.softmax_stats(g, ns, 1)
                w = ops.RefDstWeights(ns.cs, m, rl, heads)
            return ops.spmm_rhs_rows(g, self.plan, w, x_full, y_local, self.r0, **kw)
        if ops._lib.fn("gnpde_attn_dot_supported")(ns.heads, ns.dk, x_full.shape[-1]):
            mr = None
            if norm_idx == 1:
                mr = mr0 if mr0 is not None else ops.softmax_stats(g, ns, 1, packed=True)[2]
            return ops.spmm_rhs_rows(g, self.plan, None, x_full, y_local, self.r0, ns=ns, mr=mr, **kw)
        # shapes outside the fused per-edge kernel: the head-mean weights in
        # CSR order (K2), then the plain K1 over this rank's rows
        m, rl = ops.softmax_stats(g, ns, norm_idx)
        w = ops.attn_weights(g, ns, m, rl, norm_idx)
        return ops.spmm_rhs_rows(g, self.plan, w, x_full, y_local, self.r0, **kw)


class RowShardedTransformer(object):
    """Row-partitioned transformer attention RHS (the north star's literal 1-D
    partition): contiguous row blocks balanced by nnz
    (balanced_row_blocks), rank p owns rows [r0, r1) — its rows' state, scores
    and RHS.  Per RHS:

    * the state is all-gathered (RCCL all_gather_into_tensor of the padded blocks,
      unpadded into global row order): the aggregation gathers any row;
    * fork scaled_dot: each rank's share of the key sum S over its own rows (fp64)
      is all-reduced, its rows' node scores cs are all-gathered; per-edge
      scaled_dot: each rank projects its own rows and q | k [n, 2 att] is
      all-gathered (4x less than the state at att = C/4);
    * the destination-grouped softmax statistics (norm_idx 1) are formed by every
      rank over the whole CSC (score-sized, replicated);
    * the rank's rows are aggregated by the fused kernels over a local plan
      (ops.spmm_rhs_rows), written through pointers shifted to its block.

    Every rank takes part in every collective of an RHS, also a rank whose row
    block is empty (zero shares).  ``local`` replaces the HIP arithmetic
    (_HipRowAttentionLocal; tests inject a host restatement and run the
    collectives under gloo).  B = 1 (one graph; batches shard as replicas,
    shard_batch)."""

    autonomous = True  # the RHS does not read t (gnpde.base_classes.ODEFunc.autonomous)

    fused_adaptive = False    # the adaptive solvers' wide stages run in column stripes or unsharded

    @property
    def graph_capturable(self):
        """The state all-gather and the score collectives per RHS: captured on RCCL at a
        world of one, or at any world with GNPDE_CAPTURE_COLLECTIVES=1."""
        if not isinstance(self.local, _HipRowAttentionLocal):
            return False
        return _capturable(self.group, self.world)

    def graph_capture_state(self, y):
        lc = self.local
        return (lc.g, lc.plan, self.Wq, self.Wk, self.bq, self.bk, self.Wcat, self.bcat) + \
            ((self.x0_local,) if self.add_source else ())

    capture_key_tensors = ColumnShardedTransformer.capture_key_tensors

    def __init__(self, edge_index, num_nodes, C, Wq, bq, Wk, bk, heads, norm_idx, alpha, score_mode='reference',
                 beta=None, x0_local=None, add_source=False, alpha_sigmoid=True, group=None,
                 chunk=None, row_weight=ROW_WEIGHT, comm=None, local=None, partition_stats=True):
        if edge_index.shape[0] != 1:
            raise NotImplementedError("RowShardedTransformer: one graph (B = 1); shard batches with shard_batch")
        if int(norm_idx) not in (0, 1) or score_mode not in ('reference', 'per_edge'):
            raise ValueError("RowShardedTransformer: norm_idx 0 | 1 and score_mode 'reference' | 'per_edge'")
        if int(Wq.shape[0]) % int(heads):
            raise ValueError("attention_dim %d not divisible by heads %d" % (int(Wq.shape[0]), int(heads)))
        self.group = group
        self.comm = comm if comm is not None else _Comm(group)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.N = self.R = int(num_nodes)
        self.C = int(C)
        self.heads, self.norm_idx, self.score_mode = int(heads), int(norm_idx), score_mode
        self.att = int(Wq.shape[0])
        self.Wq, self.bq, self.Wk, self.bk = Wq.contiguous(), bq.contiguous(), Wk.contiguous(), bk.contiguous()
        self.Wcat = torch.cat([self.Wq, self.Wk], 0).contiguous()
        self.bcat = torch.cat([self.bq, self.bk], 0).contiguous()
        self.alpha, self.beta = alpha, beta
        self.x0_local = x0_local
        self.add_source, self.alpha_sigmoid = add_source, alpha_sigmoid
        self.nfe = 0
        if local is None:
            g = ops.GraphCSR(edge_index, self.N, chunk=chunk)
            self.blocks = balanced_row_blocks(g.csr.rowptr.cpu().numpy(), self.world, row_weight)
        else:
            g = None
            self.blocks = balanced_row_blocks(host_rowptr(edge_index, self.N), self.world, row_weight)
        self.nb = max(max(r1 - r0 for r0, r1 in self.blocks), 1)
        self.r0, self.r1 = self.blocks[self.rank]
        self.local = local if local is not None else _HipRowAttentionLocal(g, self.r0, self.r1, chunk)
        self.uniform = score_mode == 'reference' and self.norm_idx == 0
        # destination statistics (norm_idx 1) formed per block of destination rows and
        # all-gathered (ColumnShardedTransformer.stats)
        self.partition_stats = bool(partition_stats) and self.norm_idx == 1 and not self.uniform
        if self.partition_stats:
            self.dblocks, self.dnb = _dst_blocks(edge_index, self.N, self.world, g)
        self.bytes_per_rhs = 0

    def global_rms_norm(self, t):
        """RMS over the whole state (all row blocks, the padding rows excluded): the
        error norm an adaptive solve of the row partition must pass
        (options=dict(norm=sh.global_rms_norm)) so every rank takes the same steps;
        one all-reduce of 2 doubles."""
        n = self.r1 - self.r0
        own = t.reshape(-1, t.shape[-1])[:n]
        v = torch.stack([own.double().pow(2).sum(), torch.tensor(float(own.numel()), dtype=torch.float64,
                                                                  device=t.device)])
        self.comm.all_reduce(v)
        return (v[0] / v[1]).sqrt().to(t.dtype)

    def scatter(self, y):
        """Full state [1, N, C] or [N, C] -> this rank's zero-padded block [nb, C]."""
        y = y.reshape(-1, y.shape[-1])
        out = torch.zeros((self.nb, y.shape[-1]), dtype=y.dtype, device=y.device)
        out[:self.r1 - self.r0] = y[self.r0:self.r1]
        return out

    def _gather_rows(self, v_local):
        """Padded blocks [nb, K] of every rank -> [R, K] in global row order (a view of
        the gathered buffer when there is no padding to drop: a world of one)."""
        v_local = v_local.contiguous()
        pad = torch.empty((self.world * self.nb,) + tuple(v_local.shape[1:]), dtype=v_local.dtype,
                          device=v_local.device)
        self.comm.all_gather_into_tensor(pad, v_local)
        if all(b - a == self.nb for a, b in self.blocks):
            return pad
        return torch.cat([pad[p * self.nb:p * self.nb + (b - a)] for p, (a, b) in enumerate(self.blocks)], 0)

    def gather(self, y_local):
        """All blocks -> the full state [N, C] (global row order)."""
        return self._gather_rows(y_local)

    def _blockify(self, v_own):
        if v_own.shape[0] == self.nb and v_own.is_contiguous():
            return v_own  # a full block: sent as it is
        out = torch.zeros((self.nb,) + tuple(v_own.shape[1:]), dtype=v_own.dtype, device=v_own.device)
        out[:v_own.shape[0]] = v_own
        return out

    def scores(self, own):
        """The full node-level score operands from this rank's rows (collectives:
        every rank, whatever its block holds); None for the uniform weights."""
        if self.uniform:
            return None, 0
        if self.score_mode == 'reference':
            S = self.local.keysum(own, self.Wk, self.bk)
            self.comm.all_reduce(S)
            cs = self._gather_rows(self._blockify(self.local.node_scores(own, S, self.Wq, self.bq, self.heads)))
            ns = ops.NodeScores(ops._lib.SCORE_REFERENCE, self.heads, self.att // self.heads, cs=cs)
            return ns, S.numel() * 8 + cs.numel() * 8
        qk = self._gather_rows(self._blockify(self.local.project(own, self.Wcat, self.bcat)))  # [N, 2 att]
        return _qk_scores(qk, self.heads, self.att), qk.numel() * qk.element_size()

    stats = ColumnShardedTransformer.stats

    def _rhs(self, y_local, stage):
        self.nfe += 1
        x_full = self._gather_rows(y_local)                     # [N, C]
        ns, nbytes = self.scores(x_full[self.r0:self.r1])
        self.bytes_per_rhs = x_full.numel() * x_full.element_size() + nbytes
        st = self.stats(ns) if ns is not None else None
        return self.local.aggregate(ns, self.norm_idx, x_full, y_local, stage=stage, heads=self.heads, stats=st,
                                    x0=self.x0_local, alpha=self.alpha, beta=self.beta,
                                    alpha_sigmoid=self.alpha_sigmoid, add_source=self.add_source)

    def __call__(self, t, y_local):
        return self._rhs(y_local, None)

    def rhs_stage(self, t, y_local, stage):
        self._rhs(y_local, stage)
