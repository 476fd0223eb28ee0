"""Tensor-level wrappers over the C ABI (include/gnpde.h).

Everything here runs on the GPU through libgnpde.so; there is no CPU path.
Tensors must live on a ROCm device; every launch goes onto torch's current
stream, so the calls compose with torch ops and are hipGraph-capturable (the
graph build / plan functions are once-per-graph and synchronous).

Layout: node features [B,N,C] fp32 row-major, viewed as
[R=B*N, C]; graphs are block-diagonal over the batch as an int32 CSR
(rowptr[R+1], col[nnz] global node ids, perm[nnz] CSR pos -> COO edge id).
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib

# hub-splitting threshold (edges per K1 work item).  With the longest-first item
# order below, full-bench A/B on G-arxiv: 128 -> 8,048-8,200, 256 -> 8,485-8,496,
# 384 -> 8,434-8,450 RHS/s (in row order 128 was best: 121 against 128 us per RHS)
DEFAULT_CHUNK = int(os.environ.get("GNPDE_CHUNK", 256))
# Small graphs (fewer rows than SMALL_GRAPH_ROWS, configs[1]'s Cora-sized graph) are
# latency-bound: the launch is one round of short work items and its time is the
# longest item's chain of dependent loads, so their rows split at SMALL_CHUNK edges
# (the Cora-sized transformer's K1: 38 us at 256-edge items, 16 at 32; its dopri5
# step 0.358 ms at 32, 0.348 at 16, 0.428 at 64: gpurun_out/r05m, r05p).
# GNPDE_CHUNK set in the environment applies to every graph.
SMALL_GRAPH_ROWS = 50000
SMALL_CHUNK = int(os.environ.get("GNPDE_SMALL_CHUNK", 16))


SEG_LONG_SPLIT = os.environ.get("GNPDE_SEG_LONG_SPLIT", "1") != "0"  # small graphs: one-pass long items


def auto_chunk(R, chunk=None):
    """The hub-row split of a graph of R rows: ``chunk`` if given, else the
    environment's GNPDE_CHUNK, else SMALL_CHUNK below SMALL_GRAPH_ROWS rows and
    DEFAULT_CHUNK above."""
    if chunk is not None:
        return int(chunk)
    if "GNPDE_CHUNK" in os.environ:
        return DEFAULT_CHUNK
    return SMALL_CHUNK if R < SMALL_GRAPH_ROWS else DEFAULT_CHUNK
STATS_CHUNK = 64     # items of the softmax-statistics kernel (8 lanes per item)
# K1 work items ordered by power-of-two length class, longest first, row order inside a class
# ("classes", the default since round 2: tools/stripe_sweep2.sh, profiles/r02c_plan_order_sweep.jsonl —
# rk4 step G-arxiv C = 128 / 16: 0.429 / 0.121 ms against 0.435 / 0.128 with a plain longest-first
# sort ("lpt", round 1: 8,130-8,205 against 7,917-7,932 RHS/s in row order), G-rmat at 32 columns
# 2.59 against 2.63 ms).
# GNPDE_PLAN_ORDER=rows keeps the builder's row order; =classes sorts by power-of-two length class
# only (row order inside a class); =hubs puts the hub chunks first.  Results do not depend on it.
PLAN_ORDER = os.environ.get("GNPDE_PLAN_ORDER", "classes")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_gpu(t, name, dtype=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError("%s must be a torch.Tensor" % name)
    if not t.is_cuda:
        raise RuntimeError("gnpde: %s must be a ROCm device tensor (the native path has no CPU fallback); got %s"
                           % (name, t.device))
    if dtype is not None and t.dtype != dtype:
        raise TypeError("gnpde: %s must be %s, got %s" % (name, dtype, t.dtype))


def _rows(x, name, dtype=torch.float32):
    """[B,N,C] or [R,C] -> contiguous [R,C] view (fp32 unless stated)."""
    _require_gpu(x, name, dtype)
    x = x.contiguous()
    return x.reshape(-1, x.shape[-1])


STATE_DTYPES = (torch.float32, torch.bfloat16)  # K1 storage types (fp32 math either way)


# --------------------------------------------------------------------------- graph
class _TicketOrder(object):
    """Launch ordering of a plan whose kernels keep arrival tickets in it (K1's
    hub rows, the statistics kernel's long groups: heavy[].w, include/gnpde.h):
    two launches on one plan must never overlap.  A launch on a different stream
    than the plan's previous one first waits for everything already queued on
    that stream (an event; free for the usual single-stream use).  During graph
    capture the capture itself orders the launches."""
    last_stream = None
    n_heavy = 0

    def order_launch(self, dev):
        if self.n_heavy == 0:
            return
        s = torch.cuda.current_stream(dev)
        last = self.last_stream
        if last is not None and last != s and not torch.cuda.is_current_stream_capturing():
            ev = torch.cuda.Event()
            ev.record(last)
            s.wait_event(ev)
        self.last_stream = s


class Plan(_TicketOrder):
    """Wavefront work items over a grouped CSR (gnpde_plan_build)."""

    def __init__(self, items, heavy, n_items, n_heavy, n_slots, chunk):
        self.items, self.heavy = items, heavy
        self.n_items, self.n_heavy, self.n_slots = n_items, n_heavy, n_slots
        self.chunk = chunk
        self.last_stream = None


class GroupedCSR(object):
    """Edges grouped by one endpoint: key_row 0 -> aggregation CSR (by source),
    key_row 1 -> CSC (by destination)."""

    def __init__(self, rowptr, col, perm, R, nnz, key_row, plan):
        self.rowptr, self.col, self.perm = rowptr, col, perm
        self.R, self.nnz, self.key_row, self.plan = R, nnz, key_row, plan
        self._rowidx = None
        self._stats_plan = None
        self._seg_plans = {}

    @property
    def rowidx(self):
        """Row of every CSR position (edge-parallel kernels)."""
        if self._rowidx is None:
            ri = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=self.rowptr.device)
            _lib.call("gnpde_csr_rowidx", _ptr(self.rowptr), self.R, self.nnz, _ptr(ri), _stream(ri.device))
            self._rowidx = ri
        return self._rowidx

    def seg_plan(self, eb, long_items=False, long_max=None):
        """Edge-block plan of the segmented-softmax kernel (K2) for blocks of at
        most ``eb`` edges (SegPlan), built once per grouped CSR and block size.
        long_items=True (reference-score statistics): groups longer than eb
        as long items of at most ``long_max`` edges (default seg_long_max())
        instead of eb-edge chunks + a fixup launch."""
        key = (eb, bool(long_items), long_max)
        if key not in self._seg_plans:
            self._seg_plans[key] = build_seg_plan(self.rowptr, eb, long_items, long_max)
        return self._seg_plans[key]

    def seg_plan_rows(self, r0, r1, eb, long_items=False, long_max=None):
        """seg_plan over the groups [r0, r1) only (their group ids the CSR's): the
        statistics of one rank's block of destination rows (softmax_stats(rows=))."""
        key = ('rows', int(r0), int(r1), eb, bool(long_items), long_max)
        if key not in self._seg_plans:
            self._seg_plans[key] = build_seg_plan(self.rowptr[int(r0):int(r1) + 1], eb, long_items, long_max,
                                                  group_offset=r0)
        return self._seg_plans[key]

    @property
    def stats_plan(self):
        """Plan with small chunks for the 8-lanes-per-group statistics kernel."""
        if self._stats_plan is None:
            self._stats_plan = build_plan(self.rowptr, self.R, self.nnz, STATS_CHUNK)
        return self._stats_plan


def validate_edge_index(edge_index, num_nodes):
    _require_gpu(edge_index, "edge_index", torch.int64)
    if edge_index.dim() != 3 or edge_index.shape[1] != 2:
        raise ValueError("edge_index must be [B,2,E], got %s" % (tuple(edge_index.shape),))
    if edge_index.numel():
        lo, hi = int(edge_index.min()), int(edge_index.max())  # once per graph
        if lo < 0 or hi >= num_nodes:
            raise IndexError("edge_index values must be in [0, %d), got [%d, %d]" % (num_nodes, lo, hi))


def build_plan(rowptr, R, nnz, chunk=DEFAULT_CHUNK):
    dev = rowptr.device
    cap_items = R + 2 * (nnz // chunk) + 2
    cap_heavy = nnz // chunk + 2
    items = torch.empty(cap_items * 4, dtype=torch.int32, device=dev)
    heavy = torch.empty(cap_heavy * 4, dtype=torch.int32, device=dev)
    ws_bytes = _lib.fn("gnpde_plan_workspace_bytes")(R)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    n_it, n_hv, n_sl = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.call("gnpde_plan_build", _ptr(rowptr), R, chunk, _ptr(items), cap_items, _ptr(heavy), cap_heavy,
              ctypes.byref(n_it), ctypes.byref(n_hv), ctypes.byref(n_sl), _ptr(ws), ws_bytes, _stream(dev))
    if PLAN_ORDER != "rows" and n_it.value > 1:
        it = items[:n_it.value * 4].view(-1, 4)
        ln = (it[:, 2] - it[:, 1]).long()
        if PLAN_ORDER == "classes":
            # length classes (powers of two) longest first, row order inside a class: the
            # wavefronts dispatched last are short, and neighbouring items touch neighbouring rows
            key = -torch.floor(torch.log2(ln.clamp(min=1).double())).long()
        elif PLAN_ORDER == "hubs":
            key = (it[:, 3] < 0).long()  # hub chunks first, then every row in row order
        else:
            key = -ln  # longest items first (stable): the wavefronts dispatched last are the short ones
        order = torch.argsort(key, stable=True)
        it.copy_(it[order])
    return Plan(items, heavy, n_it.value, n_hv.value, n_sl.value, chunk)


class SegPlan(_TicketOrder):
    """Work items of gnpde_seg_softmax_f32 (include/gnpde.h): ``items`` int4
    {e_begin, e_end, -1, first_group} — consecutive whole groups packed greedily
    up to ``eb`` edges — and ``chunk_items`` {e_begin, e_end, slot, group}
    covering groups of more than eb edges in eb-edge chunks, ``heavy`` {group,
    first_slot, n_chunks, 0} per long group."""

    def __init__(self, eb, items, n_items, chunk_items, n_chunk, heavy, n_heavy, n_hub=0, n_long=0):
        self.eb = eb
        self.items, self.n_items = items, n_items
        # reference statistics: hub chunk items, then long items (one wavefront
        # each) at the front of ``items``
        self.n_hub, self.n_long = n_hub, n_long
        self.chunk_items, self.n_chunk = chunk_items, n_chunk
        self.heavy, self.n_heavy = heavy, n_heavy
        self.n_slots = n_chunk
        self.last_stream = None


def seg_long_max():
    """Edges of a long statistics item (gnpde_seg_long_edges, csrc/attention.hip kSegLongMax)."""
    return int(_lib.fn("gnpde_seg_long_edges")())


def build_seg_plan(rowptr, eb, long_items=False, long_max=None, group_offset=0):
    """gnpde_seg_plan_build on a host copy of rowptr (once per graph and block size).
    long_items=True (the reference statistics over the CSC): every group longer
    than eb becomes LONG item {e_begin, e_end, -2, group} (one wavefront) when it
    has at most seg_long_max() edges, else seg_long_max()-edge HUB CHUNK items
    {e_begin, e_end, slot, hub} with a hub table entry {group, first_slot,
    n_chunks, 0} (``heavy``: arrival tickets, the last chunk merges); hub chunks
    first (longest hubs first), then long items longest first, then the packed
    short items.  ``rowptr`` may be a row range [r0, r1] of a grouped CSR (edge
    positions stay absolute): ``group_offset`` = r0 then turns the plan's group ids
    into the CSR's (the statistics of one rank's destination rows, gnpde.dist)."""
    rp = np.ascontiguousarray(rowptr.cpu().numpy().astype(np.int32))
    R = rp.shape[0] - 1
    nnz = int(rp[-1])
    cap_i, cap_c, cap_h = max(R, 1), nnz // eb + R + 1, nnz // eb + 2
    items = np.zeros((cap_i, 4), np.int32)
    chunks = np.zeros((cap_c, 4), np.int32)
    heavy = np.zeros((cap_h, 4), np.int32)
    ni, nc, nh = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
    _lib.call("gnpde_seg_plan_build", rp.ctypes.data, R, eb, items.ctypes.data, cap_i, chunks.ctypes.data, cap_c,
              heavy.ctypes.data, cap_h, ctypes.byref(ni), ctypes.byref(nc), ctypes.byref(nh))
    dev = rowptr.device

    def dev32(a, n):
        return torch.from_numpy(np.ascontiguousarray(a[:max(n, 1)]).reshape(-1)).to(dev)

    go = int(group_offset)
    items[:ni.value, 3] += go  # first group of a short item
    if long_items:
        long_max = seg_long_max() if long_max is None else int(long_max)
        rows = heavy[:nh.value, 0].astype(np.int64)
        s0, s1 = rp[rows].astype(np.int64), rp[rows + 1].astype(np.int64)
        order = np.argsort(-(s1 - s0), kind="stable")
        hub_chunks, hubs = [], []
        for i in order:
            if s1[i] - s0[i] <= long_max:
                continue
            first = len(hub_chunks)
            for c0 in range(int(s0[i]), int(s1[i]), long_max):
                hub_chunks.append((c0, min(c0 + long_max, int(s1[i])), len(hub_chunks), len(hubs)))
            hubs.append((int(rows[i]) + go, first, len(hub_chunks) - first, 0))
        longs = [(int(s0[i]), int(s1[i]), -2, int(rows[i]) + go) for i in order if s1[i] - s0[i] <= long_max]
        front = np.asarray(hub_chunks + longs, np.int32).reshape(-1, 4)
        all_items = np.concatenate([front, items[:ni.value]], 0)
        table = np.asarray(hubs, np.int32).reshape(-1, 4)
        plan = SegPlan(eb, dev32(all_items, all_items.shape[0]), all_items.shape[0],
                       dev32(np.zeros((1, 4), np.int32), 0), 0, dev32(table, len(hubs)), len(hubs),
                       n_hub=len(hub_chunks), n_long=len(longs))
        plan.n_slots = len(hub_chunks)
        return plan

    chunks[:nc.value, 3] += go
    heavy[:nh.value, 0] += go
    # items and chunk items back to back in one buffer: K2 then covers both in one launch
    both = dev32(np.concatenate([items[:ni.value], chunks[:max(nc.value, 1)]], 0), ni.value + max(nc.value, 1))
    it_view = both[:max(ni.value, 1) * 4] if ni.value else dev32(items, 0)
    ch_view = both[ni.value * 4:]
    return SegPlan(eb, it_view, ni.value, ch_view, nc.value, dev32(heavy, nh.value), nh.value)


def build_grouped(edge_index, num_nodes, key_row, chunk=DEFAULT_CHUNK, plan=True):
    """COO [B,2,E] -> block-diagonal CSR grouped by edge_index[:, key_row] (+ plan)."""
    B, _, E = edge_index.shape
    N = int(num_nodes)
    R, nnz = B * N, B * E
    dev = edge_index.device
    ei = edge_index.contiguous()
    rowptr = torch.empty(R + 1, dtype=torch.int32, device=dev)
    col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    perm = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
    ws_bytes = _lib.fn("gnpde_csr_workspace_bytes")(B, E, N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    _lib.call("gnpde_csr_build", _ptr(ei), B, E, N, key_row, _ptr(rowptr), _ptr(col), _ptr(perm), _ptr(ws), ws_bytes,
              _stream(dev))
    plan = build_plan(rowptr, R, nnz, chunk) if plan else None
    return GroupedCSR(rowptr, col, perm, R, nnz, key_row, plan)


# --------------------------------------------------------------------------- graph normalisation
def add_self_loops(edge_index, edge_weight, fill_value, num_nodes):
    """gnpde_add_self_loops: non-loop edges in COO order, then one loop per node
    with its last existing loop's weight or fill_value (intended semantics of
    src/utils.py:16-42).  -> (edge_index [B,2,K+N] int64, weights [B,K+N] fp32)."""
    validate_edge_index(edge_index, num_nodes)  # the kernels index per-node arrays with these ids
    B, _, E = edge_index.shape
    N = int(num_nodes)
    ei = edge_index.contiguous()
    dev = ei.device
    w = None
    if edge_weight is not None:
        _require_gpu(edge_weight, "edge_weight", torch.float32)
        w = edge_weight.contiguous()
        if tuple(w.shape) != (B, E):
            raise ValueError("edge_weight shape %s != [%d,%d]" % (tuple(w.shape), B, E))
    ws_bytes = _lib.fn("gnpde_self_loops_workspace_bytes")(B, E, N)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    counts = (ctypes.c_int64 * B)()
    _lib.call("gnpde_self_loops_count", _ptr(ei), B, E, counts, _ptr(ws), ws_bytes, _stream(dev))
    ks = sorted(set(int(c) for c in counts))
    if len(ks) != 1:
        raise ValueError("batched edge lists have different lengths after self-loop insertion %s; the [B,2,E] "
                         "format needs equal counts per batch element" % sorted(k + N for k in ks))
    K = ks[0]
    ei_out = torch.empty(B, 2, K + N, dtype=torch.int64, device=dev)
    w_out = torch.empty(B, K + N, dtype=torch.float32, device=dev)
    _lib.call("gnpde_add_self_loops", _ptr(ei), _ptr(w), B, E, N, float(fill_value), K, _ptr(ei_out), _ptr(w_out),
              _ptr(ws), ws_bytes, _stream(dev))
    return ei_out, w_out


def norm_weights(edge_index, edge_weight, num_nodes, mode):
    """gnpde_norm_weights_f32: rw (norm_dim 0 / 1) or symmetric gcn weights, degrees
    summed in COO order over a grouped CSR (src/utils.py:177-194, :215-233)."""
    validate_edge_index(edge_index, num_nodes)  # the kernels index per-node arrays with these ids
    B, _, E = edge_index.shape
    N = int(num_nodes)
    ei = edge_index.contiguous()
    w = None
    if edge_weight is not None:
        _require_gpu(edge_weight, "edge_weight", torch.float32)
        w = edge_weight.contiguous()
    key_row = 0 if mode == _lib.NORM_RW_ROW else 1
    grouped = build_grouped(ei, N, key_row, plan=False)
    fac = torch.empty(B * N, dtype=torch.float32, device=ei.device)
    out = torch.empty(B, E, dtype=torch.float32, device=ei.device)
    _lib.call("gnpde_norm_weights_f32", _ptr(ei), _ptr(w), B, E, N, _ptr(grouped.rowptr), _ptr(grouped.perm), int(mode),
              _ptr(fac), _ptr(out), _stream(ei.device))
    return out


class GraphCSR(object):
    """All per-graph device structures the RHS needs, built once and reused by
    every RHS evaluation (the reference rebuilds a dense [B,N,N] per call)."""

    def __init__(self, edge_index, num_nodes, chunk=None, validate=True):
        if validate:
            validate_edge_index(edge_index, num_nodes)
        self.edge_index = edge_index
        self.B, _, self.E = edge_index.shape
        self.N = int(num_nodes)
        self.R = self.B * self.N
        self.nnz = self.B * self.E
        self.chunk = chunk = auto_chunk(self.R, chunk)
        self.csr = build_grouped(edge_index, self.N, 0, chunk)
        self._csc = None
        self._indeg = None

    @property
    def csc(self):
        if self._csc is None:
            self._csc = build_grouped(self.edge_index, self.N, 1, self.chunk)
        return self._csc

    @property
    def indeg(self):
        """In-degree per row: the CSC's row lengths (the reference scores' key sum is
        the only reader and runs with the CSC's statistics; a per-edge atomic count
        contends on the hub columns: 0.3-1.9 ms per graph)."""
        if self._indeg is None:
            rp = self.csc.rowptr
            self._indeg = (rp[1:] - rp[:-1]).to(torch.int32).contiguous()
        return self._indeg

    def gather_weights(self, w, transpose=False, out=None):
        """COO-order weights [B,E] or attention [B,E,h] -> CSR-order [nnz] (head mean);
        transpose=True gives CSC order.  ``out``: an existing [nnz] fp32 buffer to fill."""
        _require_gpu(w, "edge weights", torch.float32)
        w = w.contiguous()
        if w.dim() == 2:
            H = 1
        elif w.dim() == 3:
            H = w.shape[2]
        else:
            raise ValueError("weights must be [B,E] or [B,E,h]")
        if w.shape[0] != self.B or w.shape[1] != self.E:
            raise ValueError("weights shape %s does not match edge_index [%d,2,%d]" % (tuple(w.shape), self.B,
                                                                                        self.E))
        if out is None:
            out = torch.empty(max(self.nnz, 1), dtype=torch.float32, device=w.device)
        elif out.dtype != torch.float32 or out.numel() != max(self.nnz, 1) or not out.is_contiguous() or \
                out.device != w.device:
            raise ValueError("gather_weights: out must be a contiguous fp32 [%d] buffer on %s" % (max(self.nnz, 1),
                                                                                              w.device))
        perm = self.csc.perm if transpose else self.csr.perm
        _lib.call("gnpde_gather_weights_f32", _ptr(w), self.nnz, H, _ptr(perm), _ptr(out),
                  _stream(w.device))
        return out

    @property
    def node_layout(self):
        """The graph's locality numbering (NodeLayout), built once."""
        if getattr(self, '_layout', None) is None:
            self._layout = NodeLayout(self)
        return self._layout


# --------------------------------------------------------------------------- state layout
# The fixed-grid integrator keeps the state of a large graph in a locality
# numbering of its nodes for the whole solve (gnpde.integrator.odeint_fixed):
# permuted once on entry, back once on exit.  "degree": nodes by in-degree,
# descending (stable), per batch element — the rows the aggregation gathers most
# sit together at the front of the state.  G-arxiv rk4 step (tools/reorder_bench.py,
# profiles/r02b_reorder.jsonl): 420 -> 370 us; the same numbering applied to the
# item ORDER only (rows of x where they were) gains nothing, so it is where the
# gathered rows live, not when they are gathered.  "none" disables.
NODE_ORDER = os.environ.get("GNPDE_NODE_ORDER", "degree")
LAYOUT_MIN_ROWS = 32768          # below this the state sits in L2 / the Infinity Cache anyway
# and the two permutations would cost more than they save (GNPDE_LAYOUT_MIN_MB overrides)
LAYOUT_MIN_BYTES = int(float(os.environ.get("GNPDE_LAYOUT_MIN_MB", 16)) * (1 << 20))


class NodeLayout(object):
    """In-degree numbering of a GraphCSR's nodes and the same graph relabelled.

    ``order[k]`` = user row held at internal row k, ``new_id[i]`` = internal row
    of user row i (global rows, batch elements kept in their own row ranges).
    ``graph`` is the GraphCSR of ``new_id[edge_index]``: the COO edge order is
    unchanged (so COO-order weights apply as they are) and each row keeps its
    edges in COO order, so every output row is summed over the same edges in the
    same order — results are bit-identical to the user numbering."""

    def __init__(self, g):
        B, N, R = g.B, g.N, g.R
        dev = g.edge_index.device
        deg = g.indeg.view(B, N).long()
        local_order = torch.argsort(-deg, dim=1, stable=True)  # old local id at each new position
        base = (torch.arange(B, device=dev, dtype=torch.int64) * N).view(B, 1)
        self.order = (local_order + base).reshape(R)
        self.order32 = self.order.to(torch.int32)  # the stage epilogue's out_rows (last step of a solve)
        self.new_id = torch.empty_like(self.order)
        self.new_id[self.order] = torch.arange(R, device=dev, dtype=torch.int64)
        local_new = self.new_id.view(B, N) - base
        ei = g.edge_index
        eip = torch.gather(local_new, 1, ei.reshape(B, -1)).view(ei.shape)
        self.graph = GraphCSR(eip, N, chunk=g.chunk, validate=False)
        self.R = R

    def to_internal(self, y):
        """[B,N,C] (or [R,C]) in user order -> the same in internal order (new tensor)."""
        C = y.shape[-1]
        return y.reshape(-1, C).index_select(0, self.order).view(y.shape)

    def to_user(self, y):
        """[..., B, N, C] in internal order -> user order (new tensor)."""
        C = y.shape[-1]
        return y.reshape(-1, self.R, C).index_select(1, self.new_id).view(y.shape)


def layout_worthwhile(R, C, elem_size):
    return NODE_ORDER == "degree" and R >= LAYOUT_MIN_ROWS and R * C * elem_size >= LAYOUT_MIN_BYTES


# --------------------------------------------------------------------------- block weight producers
def mix_weights(att, edge_weight=None, gamma=None):
    """COO-order [B,E] weights from attention [B,E,h] (or [B,E]):
    mean_h(att) [* (1 - sigmoid(gamma)) + edge_weight * sigmoid(gamma)]
    (MixedODEblock.get_mixed_attention, src/block_mixed.py:29-33; gamma=None:
    the plain head mean of src/block_transformer_hard_attention.py:42,60)."""
    _require_gpu(att, "attention", torch.float32)
    att = att.contiguous()
    if att.dim() == 2:
        H = 1
    elif att.dim() == 3:
        H = att.shape[2]
    else:
        raise ValueError("attention must be [B,E] or [B,E,h]")
    B, E = att.shape[0], att.shape[1]
    if (gamma is None) != (edge_weight is None):
        raise ValueError("mix_weights: gamma and edge_weight go together")
    if edge_weight is not None:
        _require_gpu(edge_weight, "edge_weight", torch.float32)
        edge_weight = edge_weight.contiguous()
        if tuple(edge_weight.shape) != (B, E):
            raise ValueError("edge_weight shape %s != [%d,%d]" % (tuple(edge_weight.shape), B, E))
        gamma = _scalar(gamma, "gamma", att.device)
    out = torch.empty(B, E, dtype=torch.float32, device=att.device)
    _lib.call("gnpde_mix_weights_f32", _ptr(att), H, _ptr(edge_weight), _ptr(gamma), B * E, _ptr(out),
              _stream(att.device))
    return out


def group_normalize(grouped, w):
    """w[e] / (sum of w over e's group + 1e-16) in COO order, groups = rows of
    ``grouped`` (HardAttODEblock.renormalise_attention,
    src/block_transformer_hard_attention.py:32-35)."""
    _require_gpu(w, "weights", torch.float32)
    w = w.contiguous()
    if w.numel() != grouped.nnz:
        raise ValueError("group_normalize: %d weights for %d edges" % (w.numel(), grouped.nnz))
    out = torch.empty_like(w)
    nbytes = _lib.fn("gnpde_group_normalize_workspace_bytes")(grouped.nnz)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=w.device)
    _lib.call("gnpde_group_normalize_f32", _ptr(grouped.rowptr), _ptr(grouped.perm), grouped.R, grouped.nnz,
              _ptr(w), _ptr(out), _ptr(ws), nbytes, _stream(w.device))
    return out


def quantile(v, q):
    """torch.quantile(v, q) (linear interpolation) as a device scalar [1]."""
    _require_gpu(v, "values", torch.float32)
    v = v.contiguous().reshape(-1)
    n = v.numel()
    if n == 0:
        raise ValueError("quantile of an empty tensor")
    ws_bytes = _lib.fn("gnpde_quantile_workspace_bytes")(n)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=v.device)
    out = torch.empty(1, dtype=torch.float32, device=v.device)
    _lib.call("gnpde_quantile_f32", _ptr(v), n, float(q), _ptr(out), _ptr(ws), ws_bytes, _stream(v.device))
    return out


def threshold_mask(v, thr):
    """(v with every entry <= *thr set to 0, device int64 count of the kept ones):
    the hard-attention sampling as weights over the full graph (gnpde_threshold_mask_f32)."""
    _require_gpu(v, "values", torch.float32)
    _require_gpu(thr, "threshold", torch.float32)
    v = v.contiguous()
    out = torch.empty_like(v)
    count = torch.empty(1, dtype=torch.int64, device=v.device)
    _lib.call("gnpde_threshold_mask_f32", _ptr(v), v.numel(), _ptr(thr), _ptr(out), _ptr(count), _stream(v.device))
    return out, count


# --------------------------------------------------------------------------- epilogue helpers
def _flags(rhs, alpha_sigmoid, add_source):
    f = 0
    if rhs:
        f |= _lib.EPI_RHS
        if alpha_sigmoid:
            f |= _lib.ALPHA_SIGMOID
        if add_source:
            f |= _lib.ADD_SOURCE
    return f


def _scalar(t, name, dev):
    if t is None:
        return None
    if not isinstance(t, torch.Tensor):
        t = torch.tensor(float(t), dtype=torch.float32, device=dev)
    _require_gpu(t, name)
    if t.dtype != torch.float32:
        t = t.float()
    return t.reshape(1).contiguous()


class Stage(object):
    """Fused Runge-Kutta stage outputs of one RHS evaluation (gnpde_stage_epilogue_t):
    ``f_out`` receives f (optional); each entry of ``outs`` is
    (out, base, cb, cf, [(k_j, c_j), ...]) meaning out = cb*base + cf*f + sum_j c_j*k_j.
    ``base`` may be None, the RHS input x, or ``out`` itself (in place).  No
    output may alias the RHS input.  The k operands of all outputs (and of the
    error term) are collected into the stage's shared operand table, each
    distinct tensor once (read once per row by the kernel).

    ``err`` (the adaptive solvers' embedded-pair error rows): (rows, (base, cb,
    cf, [(k_j, c_j)...]), y0, y1_out, atol, rtol) -> rows[r] = sum_c (e / tol)^2
    in fp64 with e the combination, tol = atol + rtol * max(|y0|, |y1|), y1 = the
    RHS input (y1_out = -1) or output ``y1_out``.

    ``dense`` (ABI 8, the plain-weight K1 only): the step's dense output folded into
    the launch — (slot, rows, t, dt, tab, table): ``slot`` a device int64 holding the
    output array's address, ``rows`` its int32 row map or None, ``t`` device fp64
    {step start, output time}, ``dt`` the device fp64 step size, ``tab`` device fp32
    scratch of STAGE_MAX_K + 3 (the launch's coefficients), ``table`` the
    basis coefficients: {'base': [5], 'f': [5], k tensor: [5]} over w = (cy0 + cy1 +
    cym, h cy1, h cym, cf0, cf1) of torchdiffeq's interpolant (include/gnpde.h).
    The launch that applies them has a ``slot``; an earlier launch of the step forms
    ``tab``: slot None and ``table`` the applying stage's ``dense_matrix()``.
    ``scale_rows`` (ABI 8, with ``err``): fp64 [R], rows[r] = sum_c (y0 / tol)^2."""

    def __init__(self, f_out=None, outs=(), out_rows=None, dot=None, err=None, scale=None, f_lin=0.0,
                 unscaled=(), dense=None, scale_rows=None):
        self.f_out = f_out
        # indices of the outputs whose cf / c_j do NOT take ``scale`` (ABI 6 unscaled_outs)
        self.unscaled = tuple(unscaled)
        # nonzero: the RHS value becomes x + scale*f_lin*f (the affine stage derivative, ABI 5)
        self.f_lin = float(f_lin)
        # a device fp32 0-d tensor multiplying every cf and c_j (not cb): the adaptive step size
        self.scale = scale
        self.outs = list(outs)
        self.out_rows = out_rows  # int32 [R] or None: row r's ``outs`` stores go to row out_rows[r]
        # (y, rows, coef, accumulate) or None: rows[r] (+)= coef * <f[r], y[r]> in fp64 (fp32 state)
        self.dot = dot
        self.err = err
        self.dense = dense
        self.scale_rows = scale_rows

    def _operands(self):
        """The distinct k tensors of every combination, in first-use order."""
        ks, seen = [], set()
        combos = [o[4] for o in self.outs] + ([self.err[1][3]] if self.err is not None else [])
        if self.dense is not None:
            if isinstance(self.dense[5], dict):
                combos.append([(k, 0.0) for k in self.dense[5] if isinstance(k, torch.Tensor)])
        for terms in combos:
            for k, _ in terms:
                if k.data_ptr() not in seen:
                    seen.add(k.data_ptr())
                    ks.append(k)
        return ks

    @property
    def wide(self):
        """True when the stage needs the adaptive solvers' wide epilogue (error rows,
        or more operands than the fixed-grid epilogues prefetch)."""
        return self.err is not None or len(self._operands()) > _lib.STAGE_PRE_K

    def tensors(self):
        ts = [self.f_out] if self.f_out is not None else []
        if self.dot is not None:
            ts.append(self.dot[0])
        for out, base, _cb, _cf, _ks in self.outs:
            ts.append(out)
            if base is not None:
                ts.append(base)
        if self.err is not None:
            if self.err[1][0] is not None:
                ts.append(self.err[1][0])
            ts.append(self.err[2])
        ts.extend(self._operands())
        return ts

    def struct(self, x_input, shift=0, like=None):
        """ctypes struct; every pointer is moved back by ``shift`` bytes (row-block
        buffers addressed with global row ids, dist.RowShardedLaplacian).
        ``x_input`` = the RHS input (None for a stage applied without one: ``like``
        then gives the row shape)."""
        ref = x_input if x_input is not None else like
        if len(self.outs) > _lib.STAGE_MAX_OUT:
            raise ValueError("at most %d stage outputs" % _lib.STAGE_MAX_OUT)
        ks = self._operands()
        if len(ks) > _lib.STAGE_MAX_K:
            raise ValueError("at most %d distinct k operands per stage" % _lib.STAGE_MAX_K)
        slot = {k.data_ptr(): j for j, k in enumerate(ks)}
        st = _lib.StageEpilogue()
        st.f_out = self.f_out.data_ptr() - shift if self.f_out is not None else None
        st.n_out = len(self.outs)
        st.nk = len(ks)
        for j, k in enumerate(ks):
            st.k[j] = k.data_ptr() - shift
        if self.out_rows is not None:
            if shift:
                raise ValueError("out_rows cannot be combined with shifted row-block buffers")
            _require_gpu(self.out_rows, "out_rows", torch.int32)
            if self.out_rows.numel() * ref.shape[-1] != ref.numel():
                raise ValueError("out_rows must hold one row index per RHS row")
            st.out_rows = self.out_rows.data_ptr()
        if self.dot is not None:
            y, rows, coef, accumulate = self.dot
            _require_gpu(rows, "dot rows", torch.float64)
            if rows.numel() * ref.shape[-1] != ref.numel() or shift:
                raise ValueError("dot rows must hold one fp64 per RHS row")
            st.dot_with, st.dot_rows = y.data_ptr(), rows.data_ptr()
            st.dot_coef, st.dot_accumulate = float(coef), int(bool(accumulate))

        def fill(o, out, base, cb, cf, terms):
            o.out = out.data_ptr() - shift if out is not None else None
            o.base = base.data_ptr() - shift if base is not None else None
            o.cb = float(cb)
            o.cf = float(cf)
            for k, c in terms:
                o.c[slot[k.data_ptr()]] += float(c)

        for i, (out, base, cb, cf, terms) in enumerate(self.outs):
            if x_input is not None and out.data_ptr() == x_input.data_ptr():
                raise ValueError("a stage output may not alias the RHS input")
            fill(st.o[i], out, base, cb, cf, terms)
        if self.err is not None:
            rows, (base, cb, cf, terms), y0, y1_out, atol, rtol = self.err
            _require_gpu(rows, "error rows", torch.float64)
            if rows.numel() * ref.shape[-1] != ref.numel() or shift:
                raise ValueError("error rows must hold one fp64 per RHS row")
            st.err_rows = rows.data_ptr()
            fill(st.err, None, base, cb, cf, terms)
            st.err_y0 = y0.data_ptr()
            st.err_y1 = int(y1_out)
            st.atol, st.rtol = float(atol), float(rtol)
        if self.scale is not None:
            _require_gpu(self.scale, "coefficient scale", torch.float32)
            st.coef_scale = self.scale.data_ptr()
        st.f_lin = self.f_lin
        st.unscaled_outs = sum(1 << i for i in self.unscaled)
        if self.scale_rows is not None:
            _require_gpu(self.scale_rows, "scale rows", torch.float64)
            if self.err is None or self.dot is not None or self.scale_rows.numel() * ref.shape[-1] != ref.numel():
                raise ValueError("scale rows: one fp64 per RHS row, with err and without dot")
            st.scale_rows = self.scale_rows.data_ptr()
        if self.dense is not None:
            dslot, drows, dtt, ddt, dtab, table = self.dense
            _require_gpu(dtab, "dense coefficient scratch", torch.float32)
            if dtab.numel() < _lib.DENSE_SLOTS + 1:
                raise ValueError("dense: coefficient scratch of %d floats" % (_lib.DENSE_SLOTS + 1))
            st.dense_tab = dtab.data_ptr()
            if shift:
                raise ValueError("dense: unshifted buffers only")
            if dslot is not None:  # the launch that applies the coefficients
                _require_gpu(dslot, "dense slot", torch.int64)
                if not self.outs:
                    raise ValueError("dense: needs output 0 (its base is y0)")
                st.dense_out = dslot.data_ptr()
                if drows is not None:
                    _require_gpu(drows, "dense rows", torch.int32)
                    if drows.numel() * ref.shape[-1] != ref.numel():
                        raise ValueError("dense rows must hold one row index per RHS row")
                    st.dense_rows = drows.data_ptr()
            if dtt is not None:  # the times: the launch that forms the coefficients
                _require_gpu(dtt, "dense times", torch.float64)
                _require_gpu(ddt, "dense step", torch.float64)
                if dtt.numel() < 2:
                    raise ValueError("dense: two times")
                st.dense_t, st.dense_dt = dtt.data_ptr(), ddt.data_ptr()
            mat = table if not isinstance(table, dict) else self._dense_matrix(table, slot)
            for m in range(_lib.DENSE_BASIS):
                for q in range(_lib.DENSE_SLOTS):
                    st.dense_m[m][q] = float(mat[m][q])
        return st

    @staticmethod
    def _dense_matrix(table, slot):
        mat = [[0.0] * _lib.DENSE_SLOTS for _ in range(_lib.DENSE_BASIS)]
        for key, w in table.items():
            if isinstance(key, str):
                q = {'base': 0, 'f': _lib.DENSE_SLOTS - 1}[key]
            else:
                q = 1 + slot[key.data_ptr()]
            if len(w) != _lib.DENSE_BASIS:
                raise ValueError("dense: %d basis coefficients per operand" % _lib.DENSE_BASIS)
            for m, v in enumerate(w):
                mat[m][q] += float(v)
        return mat

    def dense_matrix(self):
        """The basis-coefficient matrix [DENSE_BASIS][DENSE_SLOTS] of this stage's dense
        table over its own operand slots (what the launch forming the coefficients carries)."""
        ks = self._operands()
        return self._dense_matrix(self.dense[5], {k.data_ptr(): j for j, k in enumerate(ks)})


def stage_apply(stage, f, x, like):
    """The stage epilogue as a pass of its own (gnpde_stage_apply_f32 / _bf16):
    ``f`` the RHS value (None: a plain combination), ``x`` the RHS input (None
    unless a base or the error tolerance reads it), ``like`` any row array of the
    stage (fixes the row count, width and storage type)."""
    dt = like.dtype
    if dt not in STATE_DTYPES:
        raise TypeError("stage_apply: state dtype %s" % dt)
    lr = _rows(like, "stage rows", dt)
    R, C = lr.shape
    for t in stage.tensors() + [v for v in (f, x) if v is not None]:
        _require_gpu(t, "stage tensor", dt)
        if not t.is_contiguous() or t.numel() != lr.numel():
            raise ValueError("stage tensors must be contiguous and shaped alike")
    st = stage.struct(x, like=lr)
    name = "gnpde_stage_apply_bf16" if dt == torch.bfloat16 else "gnpde_stage_apply_f32"
    _lib.call(name, R, C, C, _ptr(f), _ptr(x), ctypes.byref(st), _stream(lr.device))


def spmm_rhs(g, w_csr, x, x0=None, alpha=None, beta=None, rhs=True, alpha_sigmoid=True, add_source=False,
             out=None, transpose=False, stage=None):
    """K1: f = a*(A x - x) [+ b*x0] (or A x with rhs=False).  x [B,N,C] fp32, or
    bf16 storage (gnpde_spmm_rhs_bf16: x, x0, f and stage tensors bf16, sums in
    fp32).

    transpose=True aggregates over the CSC instead (A^T x; ``w_csr`` must then
    be in CSC order) — the backward of the RHS with respect to x.
    stage: a ``Stage`` -> the fused Runge-Kutta outputs are written instead of f
    (returns None).  The adaptive solvers' wide stages (Stage.wide) are fused
    with plain weights; with weights computed on the fly (RefDstWeights) f is
    formed first and the stage applied in a second pass (stage_apply)."""
    if stage is not None and stage.wide and isinstance(w_csr, RefDstWeights):
        f = spmm_rhs(g, w_csr, x, x0=x0, alpha=alpha, beta=beta, rhs=rhs, alpha_sigmoid=alpha_sigmoid,
                     add_source=add_source, transpose=transpose)
        stage_apply(stage, f, x, x)
        return None
    shape = x.shape
    dt = x.dtype if isinstance(x, torch.Tensor) and x.dtype in STATE_DTYPES else torch.float32
    xr = _rows(x, "x", dt)
    C = xr.shape[1]
    if xr.shape[0] != g.R:
        raise ValueError("x has %d rows, graph has %d" % (xr.shape[0], g.R))
    dev = xr.device
    a = _scalar(alpha, "alpha", dev) if rhs else None
    if rhs and a is None:
        raise ValueError("spmm_rhs: alpha required")
    b = _scalar(beta, "beta", dev) if add_source else None
    x0r = _rows(x0, "x0", dt) if add_source else None
    st = None
    if stage is not None:
        for t in stage.tensors():
            _require_gpu(t, "stage tensor", dt)
            if not t.is_contiguous() or t.numel() != xr.numel():
                raise ValueError("stage tensors must be contiguous and shaped like x")
        st = ctypes.byref(stage.struct(xr))
    elif out is None:
        out = torch.empty_like(xr)
    grouped = g.csc if transpose else g.csr
    plan = grouped.plan
    partials = _partials(plan, C, dev)
    plan.order_launch(dev)
    epi = (C, _ptr(xr), C, _ptr(x0r), C, _ptr(a), _ptr(b), _flags(rhs, alpha_sigmoid, add_source), _ptr(out), C,
           _ptr(partials), plan.n_slots, st, _stream(dev))
    items, col = plan.items, grouped.col
    if isinstance(w_csr, CompactWeights):  # the sampled graph: the plan's items over the retained edges
        if w_csr.grouped is not grouped or w_csr.transpose != bool(transpose):
            raise ValueError("spmm_rhs: compacted weights of another grouped CSR")
        items, col, w_csr = w_csr.items, w_csr.col, w_csr.w
    if dt == torch.bfloat16:
        if isinstance(w_csr, RefDstWeights):
            raise ValueError("bf16 storage takes precomputed weights (attn_rhs(..., fuse=False))")
        _lib.call("gnpde_spmm_rhs_bf16", _ptr(items), plan.n_items, _ptr(plan.heavy), plan.n_heavy,
                  _ptr(col), _ptr(w_csr), *epi)
    elif isinstance(w_csr, RefDstWeights):
        if transpose:
            raise ValueError("on-the-fly attention weights aggregate over the CSR only")
        _lib.call("gnpde_attn_ref_rhs_f32", _ptr(plan.items), plan.n_items, _ptr(plan.heavy), plan.n_heavy,
                  _ptr(grouped.col), _ptr(w_csr.cs), _ptr(w_csr.m), _ptr(w_csr.rl), _ptr(w_csr.mr), w_csr.heads,
                  *epi)
    else:
        _lib.call("gnpde_spmm_rhs_f32", _ptr(items), plan.n_items, _ptr(plan.heavy), plan.n_heavy,
                  _ptr(col), _ptr(w_csr), *epi)
    return None if stage is not None else out.view(shape)


class CompactWeights(object):
    """Grouped-order weights with zeros (the sampled graph of HardAttODEblock training,
    src/block_transformer_hard_attention.py:52-56) compacted inside the plan's items
    (gnpde_compact_items_f32): ``items`` / ``col`` / ``w`` replace the grouped CSR's
    for K1, which then gathers the retained edges only, in the full plan's order and
    hub chunks (the masked full graph's sums: dropped edges added exact zeros).
    ``full`` is the uncompacted grouped-order weights.  Refreshed in place
    (compact_weights(..., out=)), so captured step graphs keep replaying."""

    def __init__(self, grouped, transpose, full, col, w, items):
        self.grouped, self.transpose = grouped, transpose
        self.full, self.col, self.w, self.items = full, col, w, items


def compact_weights(grouped, w_full, transpose, out=None):
    """CompactWeights of grouped-order weights ``w_full`` [nnz] over ``grouped`` (a
    GroupedCSR: the CSR, or the CSC with transpose=True); ``out``: an earlier
    CompactWeights of the same grouped CSR refreshed in place."""
    plan = grouped.plan
    dev = w_full.device
    _require_gpu(w_full, "w_full", torch.float32)
    if out is None:
        out = CompactWeights(grouped, transpose, w_full, torch.empty_like(grouped.col),
                             torch.empty(max(grouped.nnz, 1), dtype=torch.float32, device=dev),
                             torch.empty_like(plan.items))
    elif out.grouped is not grouped or out.transpose != transpose:
        raise ValueError("compact_weights: out belongs to another grouped CSR")
    out.full = w_full
    _lib.call("gnpde_compact_items_f32", _ptr(plan.items), plan.n_items, _ptr(grouped.col), _ptr(w_full),
              _ptr(out.col), _ptr(out.w), _ptr(out.items), _stream(dev))
    return out


# byte offsets of the hub partial stores are 32-bit (buffer addressing, csrc/common.hpp kBufRecords)
_PARTIALS_MAX_BYTES = 0xffffff00


def _partials(plan, C, dev):
    """fp32 scratch of the hub chunk partial sums: n_slots * C floats."""
    if not plan.n_slots:
        return None
    if plan.n_slots * C * 4 >= _PARTIALS_MAX_BYTES:
        raise ValueError("gnpde: %d hub partial slots x %d columns exceed the 4 GiB of 32-bit buffer offsets the "
                         "in-launch hub combine addresses; use a larger chunk (opt['gnpde_chunk'])" % (plan.n_slots, C))
    return torch.empty(plan.n_slots * C, dtype=torch.float32, device=dev)


class RefDstWeights(object):
    """Weights K1 computes on the fly (gnpde_attn_ref_rhs_f32): the fork's
    scaled_dot under destination-grouped softmax, head-mean per edge from the
    node scores cs [R,h] and the CSC statistics m [R,h], rl [R,h] or their
    packed records mr [R, stats_record_floats(h)] fp32 (two heads)."""

    def __init__(self, cs, m, rl, heads, mr=None):
        self.cs, self.m, self.rl, self.heads, self.mr = cs, m, rl, int(heads), mr


def spmm_rhs_rows(g, plan, w_csr, x_src, x_rows, row0, x0=None, alpha=None, beta=None, alpha_sigmoid=True,
                  add_source=False, stage=None, out=None, col=None, ns=None, mr=None):
    """K1 over a row block: ``plan`` covers rows [row0, row0 + n) by their
    positions in ``x_src`` (the gathered state); gathers read ``x_src`` through
    ``col`` (default: the CSR's global ids; dist.RowPartition passes ids
    relabelled into its padded layout); the block's own state ``x_rows`` [n, C],
    ``x0`` and the outputs are local buffers addressed through pointers shifted
    back by row0 rows (never dereferenced outside the block).  The epilogue's
    x_r comes from x_src[row], which holds the same values.

    Weights: ``w_csr`` in CSR order (plain), a RefDstWeights (the fork's scaled_dot
    under destination-grouped softmax, formed in the gather loop:
    gnpde_attn_ref_rhs_f32), or ``ns`` = per-edge scaled_dot NodeScores over the
    whole state (q, k rows at the positions of x_src; ``mr``: destination
    statistics records for norm_idx 1, None for source-grouped softmax: the fused
    gnpde_attn_dot_rhs_f32)."""
    if isinstance(w_csr, CompactWeights):
        raise ValueError("spmm_rhs_rows: compacted (sampled-graph) weights take the whole-graph K1 (spmm_rhs)")
    xs = _rows(x_src, "x_src")
    xl = _rows(x_rows, "x_rows")
    C = xs.shape[1]
    dev = xs.device
    shift = int(row0) * C * 4
    sp = lambda t: ctypes.c_void_p(t.data_ptr() - shift) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    a = _scalar(alpha, "alpha", dev)
    b = _scalar(beta, "beta", dev) if add_source else None
    x0r = _rows(x0, "x0") if add_source else None
    st = None
    if stage is not None:
        for t in stage.tensors():
            _require_gpu(t, "stage tensor", torch.float32)
        if stage.wide:
            raise ValueError("spmm_rhs_rows: the adaptive solvers' wide stages run unsharded or in column stripes")
        st = ctypes.byref(stage.struct(xs, shift))
    elif out is None:
        out = torch.empty_like(xl)
    cp = _ptr(g.csr.col if col is None else col)
    epi = (C, _ptr(xs), C, sp(x0r), C, _ptr(a), _ptr(b), _flags(True, alpha_sigmoid, add_source),
           sp(out) if out is not None else ctypes.c_void_p(0), C)
    plan.order_launch(dev)
    if ns is not None:
        H, dk = ns.heads, ns.dk
        if not _lib.fn("gnpde_attn_dot_supported")(H, dk, C):
            raise ValueError("spmm_rhs_rows: per-edge scores of heads=%d dk=%d C=%d outside the fused kernel" %
                             (H, dk, C))
        nws = int(_lib.fn("gnpde_attn_dot_workspace_floats")(H, C, plan.n_slots))
        ws = torch.empty(max(nws, 4), dtype=torch.float32, device=dev)
        _lib.call("gnpde_attn_dot_rhs_f32", _ptr(plan.items), plan.n_items, _ptr(plan.heavy), plan.n_heavy, cp,
                  _ptr(ns.q), _ptr(ns.k), ns.ldqk, H, dk, _ptr(mr), *epi, _ptr(ws), plan.n_slots, st, _stream(dev))
    elif isinstance(w_csr, RefDstWeights):
        partials = _partials(plan, C, dev)
        _lib.call("gnpde_attn_ref_rhs_f32", _ptr(plan.items), plan.n_items, _ptr(plan.heavy), plan.n_heavy, cp,
                  _ptr(w_csr.cs), _ptr(w_csr.m), _ptr(w_csr.rl), _ptr(w_csr.mr), w_csr.heads, *epi, _ptr(partials),
                  plan.n_slots, st, _stream(dev))
    else:
        partials = _partials(plan, C, dev)
        _lib.call("gnpde_spmm_rhs_f32", _ptr(plan.items), plan.n_items, _ptr(plan.heavy), plan.n_heavy, cp,
                  _ptr(w_csr), *epi, _ptr(partials), plan.n_slots, st, _stream(dev))
    return None if stage is not None else out.view(x_rows.shape)


# --------------------------------------------------------------------------- attention
SCORE_MODES = {
    ('scaled_dot', 'reference'): _lib.SCORE_REFERENCE,
    ('scaled_dot', 'per_edge'): _lib.SCORE_DOT,
    ('exp_kernel', 'reference'): _lib.SCORE_EXP_KERNEL,
    ('exp_kernel', 'per_edge'): _lib.SCORE_EXP_KERNEL,
    ('cosine_sim', 'reference'): _lib.SCORE_COSINE,
    ('cosine_sim', 'per_edge'): _lib.SCORE_COSINE,
    ('pearson', 'reference'): _lib.SCORE_PEARSON,
    ('pearson', 'per_edge'): _lib.SCORE_PEARSON,
}


def linear(x, W, bias=None, split=None):
    """MFMA projection: x [R,K] @ W[Nout,K]^T + bias -> (out[:, :split], out[:, split:]).
    x fp32, or bf16 storage (gnpde_linear_bf16: widened exactly on load, so the same
    values and bits as the projection of x.float()); outputs fp32."""
    xdt = x.dtype if isinstance(x, torch.Tensor) and x.dtype in STATE_DTYPES else torch.float32
    xr = _rows(x, "x", xdt)
    _require_gpu(W, "W", torch.float32)
    W = W.contiguous()
    Nout, K = W.shape
    if xr.shape[1] != K:
        raise ValueError("linear: x has %d columns, W expects %d" % (xr.shape[1], K))
    if bias is not None:
        _require_gpu(bias, "bias", torch.float32)
        bias = bias.contiguous()
    split = Nout if split is None else int(split)
    R = xr.shape[0]
    out_a = torch.empty(R, split, dtype=torch.float32, device=xr.device)
    out_b = torch.empty(R, Nout - split, dtype=torch.float32, device=xr.device) if split < Nout else None
    name = "gnpde_linear_bf16" if xdt == torch.bfloat16 else "gnpde_linear_f32"
    _lib.call(name, _ptr(xr), R, K, K, _ptr(W), _ptr(bias), Nout, split, _ptr(out_a), max(split, 1),
              _ptr(out_b), max(Nout - split, 1), _stream(xr.device))
    return out_a, out_b


def linear_wgrad(gy, x):
    """gW = gy^T x [M, K] on the fp32 matrix cores (gnpde_linear_wgrad_f32): the
    weight gradient of the Q / K projections (the backward of nn.Linear,
    function_transformer_attention.py:224-225), rows reduced in a fixed order."""
    gyr = _rows(gy, "gy")
    xr = _rows(x, "x")
    if gyr.shape[0] != xr.shape[0]:
        raise ValueError("linear_wgrad: gy has %d rows, x has %d" % (gyr.shape[0], xr.shape[0]))
    R, M = gyr.shape
    K = xr.shape[1]
    out = torch.empty(M, K, dtype=torch.float32, device=xr.device)
    nb = _lib.fn("gnpde_linear_wgrad_workspace_bytes")(R, M, K)
    ws = torch.empty(nb, dtype=torch.uint8, device=xr.device)
    _lib.call("gnpde_linear_wgrad_f32", _ptr(gyr), R, M, M, _ptr(xr), K, K, _ptr(out), K, _ptr(ws), nb,
              _stream(xr.device))
    return out


class NodeScores(object):
    """Per-RHS node-level operands of the attention scores."""

    def __init__(self, mode, heads, dk, cs=None, q=None, k=None, p0=1.0, p1=1.0):
        self.mode, self.heads, self.dk = mode, heads, dk
        self.cs, self.q, self.k = cs, q, k
        self.p0, self.p1 = float(p0), float(p1)
        self.ldqk = q.shape[1] if q is not None else 1


def _keysum_workspace(g, dev, nbytes):
    """Scratch of gnpde_ref_scores_f32 (tile partials, U and v), held by the graph
    (freed with it) per stream and size, so that captured step graphs
    keep reading the buffer they were captured with and two streams never share one."""
    d = g.__dict__.setdefault('_keysum_ws', {})
    key = (torch.cuda.current_stream(dev).cuda_stream, int(nbytes))
    ws = d.get(key)
    if ws is None:
        ws = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
        d[key] = ws
    return ws


def node_scores(g, x, Wq, bq, Wk, bk, heads, attention_type='scaled_dot', score_mode='reference',
                output_var=1.0, lengthscale=1.0, wcat=None):
    """Q/K-side work of SpGraphTransAttentionLayer.forward (function_transformer_attention.py:224-259)."""
    mode = SCORE_MODES[(attention_type, score_mode)]
    # the per-edge modes project a bf16 state directly (gnpde_linear_bf16); the reference
    # mode's key sum and node scores read fp32
    bf = isinstance(x, torch.Tensor) and x.dtype == torch.bfloat16 and mode != _lib.SCORE_REFERENCE
    xr = _rows(x, "x", torch.bfloat16 if bf else torch.float32)
    att = Wq.shape[0]
    if att % heads:
        raise ValueError("attention_dim %d not divisible by heads %d" % (att, heads))
    dk = att // heads
    if mode == _lib.SCORE_REFERENCE:
        B, N, C = g.B, g.N, xr.shape[1]
        cs = torch.empty(g.R, heads, dtype=torch.float64, device=xr.device)
        ws_bytes = _lib.fn("gnpde_keysum_workspace_bytes")(B, N, C, att)
        ws = _keysum_workspace(g, xr.device, ws_bytes)
        for name, t in (("Wq", Wq), ("bq", bq), ("Wk", Wk), ("bk", bk)):
            _require_gpu(t, name, torch.float32)
        _lib.call("gnpde_ref_scores_f32", _ptr(xr), B, N, C, C, _ptr(g.indeg), _ptr(Wq.contiguous()),
                  _ptr(bq.contiguous()), _ptr(Wk.contiguous()), _ptr(bk.contiguous()), att, heads, _ptr(cs), _ptr(ws),
                  ws_bytes, _stream(xr.device))
        return NodeScores(mode, heads, dk, cs=cs)
    if wcat is not None:
        W, b = wcat
    else:
        W = torch.cat([Wq, Wk], 0)
        b = torch.cat([bq, bk], 0) if bq is not None else None
    q, k = linear(xr, W, b, split=att)
    return NodeScores(mode, heads, dk, q=q, k=k, p0=output_var, p1=lengthscale)


def ref_keysum(g, x, Wk, bk):
    """The fork's global key sum S [B, att] fp64 of a (column stripe of the) state:
    S_b = Wk xbar_b + (sum indeg) bk with xbar_b = sum_n indeg(n) x_n
    (gnpde_ref_keysum_f32; function_transformer_attention.py:249's
    sum over e' of k_dst(e')).  Linear in x's columns: the shares of the stripes of
    a state sum to the key sum of the whole (bk on one stripe only)."""
    xr = _rows(x, "x")
    C = xr.shape[1]
    att = Wk.shape[0]
    for name, t in (("Wk", Wk), ("bk", bk)):
        _require_gpu(t, name, torch.float32)
    S = torch.empty(g.B, att, dtype=torch.float64, device=xr.device)
    nb = _lib.fn("gnpde_keysum_workspace_bytes")(g.B, g.N, C, att)
    ws = _keysum_workspace(g, xr.device, nb)
    _lib.call("gnpde_ref_keysum_f32", _ptr(xr), g.B, g.N, C, C, _ptr(g.indeg), _ptr(Wk.contiguous()),
              _ptr(bk.contiguous()), att, _ptr(S), _ptr(ws), nb, _stream(xr.device))
    return S


def ref_scores_from_keysum(g, x, S, Wq, bq, heads):
    """Node scores cs [R, heads] fp64 = q . S / sqrt(dk) of a (column stripe of the)
    state from a given key sum S (gnpde_ref_scores_from_keysum_f32): the stripe's
    share of cs (bq on one stripe only)."""
    xr = _rows(x, "x")
    C = xr.shape[1]
    att = Wq.shape[0]
    _require_gpu(S, "S", torch.float64)
    for name, t in (("Wq", Wq), ("bq", bq)):
        _require_gpu(t, name, torch.float32)
    cs = torch.empty(g.R, heads, dtype=torch.float64, device=xr.device)
    nb = _lib.fn("gnpde_keysum_workspace_bytes")(g.B, g.N, C, att)
    ws = _keysum_workspace(g, xr.device, nb)
    _lib.call("gnpde_ref_scores_from_keysum_f32", _ptr(xr), g.B, g.N, C, C, _ptr(S.contiguous()),
              _ptr(Wq.contiguous()), _ptr(bq.contiguous()), att, heads, _ptr(cs), _ptr(ws), nb, _stream(xr.device))
    return cs


def uniform_scores(heads):
    """Source-grouped softmax of the fork's scaled_dot: every score of a source
    row is q_i . S / sqrt(dk), identical within the group, so softmax gives
    exp(0)/(outdeg + 1e-16) whatever x, Q and K are.  The
    weights depend on the graph only and are computed once per graph."""
    return NodeScores(_lib.SCORE_UNIFORM, heads, 1)


def stats_record_floats(heads):
    """Floats per packed statistics record (include/gnpde.h GNPDE_STATS_RECORD_FLOATS)."""
    return (2 * heads + 3) & ~3


def _seg_call(g, ns, norm_idx, out_kind, packed=False, rows=None):
    """K2 (gnpde_seg_softmax_f32) over the grouped CSR of the softmax groups:
    out_kind 0 -> head-mean weights in aggregation-CSR order (norm_idx 0 only);
    1 -> (m, rl), or with packed=True (None, None, mr): the packed statistics
    records only.  NotImplemented when the shape is outside the kernel."""
    if ns.mode == _lib.SCORE_UNIFORM or (ns.mode == _lib.SCORE_REFERENCE and out_kind == 0):
        return NotImplemented
    eb = _lib.fn("gnpde_seg_block_edges")(ns.mode, ns.heads, ns.dk)
    if eb <= 0:
        return NotImplemented
    if ns.q is not None and (ns.ldqk % 4 or ns.q.data_ptr() % 16 or ns.k.data_ptr() % 16):
        return NotImplemented
    grouped = g.csr if norm_idx == 0 else g.csc
    long_items = ns.mode == _lib.SCORE_REFERENCE and out_kind == 1 and norm_idx == 1
    # a small graph's statistics launch is one round of items: every long item one pass
    # (its hub groups in one-pass chunks), so no wavefront walks a group alone
    long_max = int(_lib.fn("gnpde_seg_long_pass_edges")(ns.heads)) if (long_items and g.R < SMALL_GRAPH_ROWS and
                                                                        SEG_LONG_SPLIT) else None
    if rows is not None:  # the groups of rows [r0, r1) only (outputs: full-size, those rows written)
        if out_kind != 1:
            return NotImplemented
        if rows[1] <= rows[0]:  # an empty block (a rank with no groups): nothing to form
            dev, H = grouped.col.device, ns.heads
            if packed:
                return None, None, torch.zeros(g.R, stats_record_floats(H), dtype=torch.float32, device=dev)
            return (torch.zeros(g.R, H, dtype=torch.float64, device=dev),
                    torch.zeros(g.R, H, dtype=torch.float32, device=dev))
        plan = grouped.seg_plan_rows(rows[0], rows[1], eb, long_items=long_items, long_max=long_max)
    else:
        plan = grouped.seg_plan(eb, long_items=long_items, long_max=long_max)
    dev = grouped.col.device
    H = ns.heads
    packed = packed and out_kind == 1
    need_stats = not packed and (out_kind == 1 or plan.n_chunk > 0)
    m = torch.empty(g.R, H, dtype=torch.float64, device=dev) if need_stats else None
    rl = torch.empty(g.R, H, dtype=torch.float32, device=dev) if need_stats else None
    mr = torch.empty(g.R, stats_record_floats(H), dtype=torch.float32, device=dev) if packed else None
    partials = torch.empty(plan.n_slots * 2 * H, dtype=torch.float64, device=dev) if plan.n_slots else None
    w = torch.empty(max(g.nnz, 1), dtype=torch.float32, device=dev) if out_kind == 0 else None
    plan.order_launch(dev)  # chunked plans' statistics fixups read partials written by this launch
    rc = _lib.call_rc("gnpde_seg_softmax_f32", _ptr(plan.items), plan.n_items, plan.n_hub, plan.n_long,
                      _ptr(plan.chunk_items), plan.n_chunk,
                      _ptr(plan.heavy), plan.n_heavy, _ptr(grouped.rowptr), _ptr(grouped.rowidx), _ptr(grouped.col),
                      int(norm_idx == 1), out_kind, ns.mode, H, ns.dk, _ptr(ns.cs), _ptr(ns.q), _ptr(ns.k), ns.ldqk,
                      ns.p0, ns.p1, _ptr(w), _ptr(m), _ptr(rl), _ptr(mr), _ptr(partials), _stream(dev))
    if rc == _lib.EUNSUPPORTED:
        return NotImplemented
    _lib.check(rc, "gnpde_seg_softmax_f32")
    if out_kind == 0:
        return w
    return (None, None, mr) if packed else (m, rl)


def softmax_stats(g, ns, norm_idx, seg=True, packed=False, rows=None):
    """m [R,h] fp64, rl [R,h]: per-group max and 1/(sum-exp + 1e-16)
    (utils.softmax, src/utils.py:116-127).  seg=True: the edge-block kernel K2;
    shapes outside it (and seg=False) use the per-group kernels
    (gnpde_softmax_stats_f32).  packed=True returns (None, None, mr): the same
    statistics as packed records [R, stats_record_floats(h)] fp32 only (the form
    the fused-weight K1 reads in one cache line per edge).  rows=(r0, r1): only
    the groups [r0, r1) are formed (K2; full-size outputs with those rows written,
    the same values as the full launch) — NotImplemented outside K2's shapes."""
    if rows is not None:
        return _seg_call(g, ns, norm_idx, 1, packed=packed, rows=rows) if seg else NotImplemented
    if seg:
        r = _seg_call(g, ns, norm_idx, 1, packed=packed)
        if r is not NotImplemented:
            return r
    grouped = g.csr if norm_idx == 0 else g.csc
    plan = grouped.stats_plan
    dev = grouped.col.device
    H = ns.heads
    m = None if packed else torch.empty(g.R, H, dtype=torch.float64, device=dev)
    rl = None if packed else torch.empty(g.R, H, dtype=torch.float32, device=dev)
    mr = torch.empty(g.R, stats_record_floats(H), dtype=torch.float32, device=dev) if packed else None
    partials = torch.empty(plan.n_slots * 2 * H, dtype=torch.float64, device=dev) if plan.n_slots else None
    _lib.call("gnpde_softmax_stats_f32", _ptr(plan.items), plan.n_items, _ptr(plan.heavy), plan.n_heavy,
              _ptr(grouped.col), int(norm_idx == 1), ns.mode, H, ns.dk, _ptr(ns.cs), _ptr(ns.q), _ptr(ns.k), ns.ldqk,
              ns.p0, ns.p1, _ptr(m), _ptr(rl), _ptr(mr), _ptr(partials), _stream(dev))
    return (None, None, mr) if packed else (m, rl)


def attn_weights(g, ns, m, rl, norm_idx, seg=True, edges=None):
    """Head-mean softmax weights in aggregation-CSR order [nnz].  norm_idx 0:
    K2 computes them straight from the scores (m, rl unused, may be None);
    norm_idx 1 (and shapes outside K2): edge-parallel from the group
    statistics (gnpde_attn_weights_f32).  edges=(e0, e1): only the CSR
    positions [e0, e1), edge-parallel from the given m, rl ([e1 - e0] weights,
    the same values as the full pass: gnpde.dist's edge-sharded weights)."""
    dev = g.csr.col.device
    if edges is not None:
        e0, e1 = (int(v) for v in edges)
        if m is None or rl is None or not 0 <= e0 <= e1 <= g.nnz:
            raise ValueError("attn_weights: edges needs the statistics m, rl and 0 <= e0 <= e1 <= nnz")
        w = torch.empty(max(e1 - e0, 1), dtype=torch.float32, device=dev)
        if e1 > e0:
            _lib.call("gnpde_attn_weights_f32", _ptr(g.csr.rowidx[e0:e1]), _ptr(g.csr.col[e0:e1]), e1 - e0,
                      int(norm_idx), ns.mode, ns.heads, ns.dk, _ptr(ns.cs), _ptr(ns.q), _ptr(ns.k), ns.ldqk, ns.p0,
                      ns.p1, _ptr(m), _ptr(rl), _ptr(w), _stream(dev))
        return w[:e1 - e0]
    if seg and norm_idx == 0:
        w = _seg_call(g, ns, 0, 0)
        if w is not NotImplemented:
            return w
    if m is None:
        m, rl = softmax_stats(g, ns, norm_idx, seg=seg)
    w = torch.empty(max(g.nnz, 1), dtype=torch.float32, device=dev)
    _lib.call("gnpde_attn_weights_f32", _ptr(g.csr.rowidx), _ptr(g.csr.col), g.nnz, int(norm_idx), ns.mode, ns.heads,
              ns.dk, _ptr(ns.cs), _ptr(ns.q), _ptr(ns.k), ns.ldqk, ns.p0, ns.p1, _ptr(m), _ptr(rl), _ptr(w),
              _stream(dev))
    return w


# Small graphs (SMALL_GRAPH_ROWS): the fork's scaled_dot weights under destination-grouped
# softmax as a separate edge-parallel pass (gnpde_attn_weights_f32, every edge at once)
# instead of in K1's gather loop, whose chain per edge (the destination's statistics, one
# exp per head) is the launch's critical path there.  "wide": for the adaptive solvers'
# wide stages only (then K1 fuses the stage: no stage pass); "all"; "none".
SMALL_PRECOMPUTE = os.environ.get("GNPDE_SMALL_PRECOMPUTE", "wide")


# Any graph: the adaptive solvers' wide stages take the weights pass too, so the plain-weight
# K1 fuses the stage (STG 4) instead of forming f and applying the stage in a second pass
# over f and its operands (gnpde_stage_apply_f32) — GNPDE_WIDE_PRECOMPUTE=0: the pass.
WIDE_PRECOMPUTE = os.environ.get("GNPDE_WIDE_PRECOMPUTE", "1") != "0"


def _small_precompute(g, stage):
    if WIDE_PRECOMPUTE and stage is not None and stage.wide:
        return True
    if g.R >= SMALL_GRAPH_ROWS or SMALL_PRECOMPUTE == "none":
        return False
    return SMALL_PRECOMPUTE == "all" or (stage is not None and stage.wide)


def attn_rhs(g, ns, m, rl, norm_idx, x, x0=None, alpha=None, beta=None, rhs=True, alpha_sigmoid=True,
             add_source=False, out=None, stage=None, seg=True, fuse=True, mr=None):
    """K2 + K1: f = a*(A_att x - x) [+ b x0], A_att = head-mean softmax weights
    (m, rl: destination statistics for norm_idx 1, or None to compute them;
    mr: the same statistics as packed records, softmax_stats(packed=True)).
    Reference scores under norm_idx 1 (fuse=True): the weights are computed
    inside K1 from (cs, m, rl) or (cs, mr) — same bits as the separate weights
    pass.  Two heads with no statistics given: the packed records.  Per-edge
    scaled_dot (fuse=True, shapes of gnpde_attn_dot_supported): one fused pass
    (attn_dot_rhs) for either grouping."""
    if fuse and norm_idx == 1 and ns.mode == _lib.SCORE_REFERENCE and x.dtype == torch.float32 and \
            not _small_precompute(g, stage):
        if m is None and mr is None:
            if ns.heads == 2:
                _, _, mr = softmax_stats(g, ns, 1, seg=seg, packed=True)
            else:
                m, rl = softmax_stats(g, ns, 1, seg=seg)
        w = RefDstWeights(ns.cs, m, rl, ns.heads, mr=mr)
        return spmm_rhs(g, w, x, x0=x0, alpha=alpha, beta=beta, rhs=rhs, alpha_sigmoid=alpha_sigmoid,
                        add_source=add_source, out=out, stage=stage)
    if fuse and ns.mode == _lib.SCORE_DOT and (x.dtype == torch.float32 or (x.dtype == torch.bfloat16 and
                                                                              norm_idx == 0)) and \
            _lib.fn("gnpde_attn_dot_supported")(ns.heads, ns.dk, x.shape[-1]):
        if norm_idx == 1 and mr is None:
            _, _, mr = softmax_stats(g, ns, 1, seg=seg, packed=True)
        r = attn_dot_rhs(g, ns, x, x0=x0, alpha=alpha, beta=beta, rhs=rhs, alpha_sigmoid=alpha_sigmoid,
                         add_source=add_source, out=out, stage=stage, mr=mr if norm_idx == 1 else None)
        if r is not NotImplemented:
            return r
    w = attn_weights(g, ns, m, rl, norm_idx, seg=seg)
    return spmm_rhs(g, w, x, x0=x0, alpha=alpha, beta=beta, rhs=rhs, alpha_sigmoid=alpha_sigmoid,
                    add_source=add_source, out=out, stage=stage)


def attn_dot_rhs(g, ns, x, x0=None, alpha=None, beta=None, rhs=True, alpha_sigmoid=True, add_source=False,
                 out=None, stage=None, mr=None):
    """The per-edge scaled_dot RHS in one aggregation pass (gnpde_attn_dot_rhs_f32,
    csrc/flash.hip): under source-grouped softmax (norm_idx 0; mr None) the pass
    forms each row's softmax statistics itself; under destination-grouped softmax
    (norm_idx 1) ``mr`` holds the destinations' packed statistics records
    (softmax_stats(..., packed=True)) and the pass weights every scored edge with
    them.  No [nnz] weights.  NotImplemented for shapes outside the fused kernel
    (gnpde_attn_dot_supported)."""
    dt = x.dtype if isinstance(x, torch.Tensor) and x.dtype in STATE_DTYPES else torch.float32
    bf = dt == torch.bfloat16
    xr = _rows(x, "x", dt)
    C = xr.shape[1]
    H, dk = ns.heads, ns.dk
    if not _lib.fn("gnpde_attn_dot_supported")(H, dk, C):
        return NotImplemented
    if stage is not None and (stage.wide or len(stage.outs) > 1 or stage.dot is not None):
        return NotImplemented  # fused here: single-output fixed-grid stages (the caller takes K2 + K1)
    if bf and mr is not None:
        return NotImplemented  # a bf16 state: source-grouped softmax only (K2 + the bf16 K1 otherwise)
    row_align = 8 if bf else 16
    if ns.ldqk % 4 or ns.q.data_ptr() % 16 or ns.k.data_ptr() % 16 or xr.data_ptr() % row_align:
        return NotImplemented
    if xr.shape[0] != g.R:
        raise ValueError("x has %d rows, graph has %d" % (xr.shape[0], g.R))
    dev = xr.device
    a = _scalar(alpha, "alpha", dev) if rhs else None
    if rhs and a is None:
        raise ValueError("attn_dot_rhs: alpha required")
    b = _scalar(beta, "beta", dev) if add_source else None
    x0r = _rows(x0, "x0", dt) if add_source else None
    if x0r is not None and x0r.data_ptr() % row_align:
        return NotImplemented
    st = None
    if stage is not None:
        for t in stage.tensors():
            _require_gpu(t, "stage tensor", dt)
            if not t.is_contiguous() or t.numel() != xr.numel():
                raise ValueError("stage tensors must be contiguous and shaped like x")
        st = ctypes.byref(stage.struct(xr))
    elif out is None:
        out = torch.empty_like(xr)
    plan = g.csr.plan
    nws = int(_lib.fn("gnpde_attn_dot_workspace_floats")(H, C, plan.n_slots))
    ws = None
    if nws:
        if nws * 4 >= _PARTIALS_MAX_BYTES:
            return NotImplemented
        ws = torch.empty(nws, dtype=torch.float32, device=dev)
    plan.order_launch(dev)
    rc = _lib.call_rc("gnpde_attn_dot_rhs_bf16" if bf else "gnpde_attn_dot_rhs_f32", _ptr(plan.items), plan.n_items,
                      _ptr(plan.heavy), plan.n_heavy,
                      _ptr(g.csr.col), _ptr(ns.q), _ptr(ns.k), ns.ldqk, H, dk, _ptr(mr), C, _ptr(xr), C,
                      _ptr(x0r), C, _ptr(a), _ptr(b), _flags(rhs, alpha_sigmoid, add_source), _ptr(out), C, _ptr(ws),
                      plan.n_slots, st, _stream(dev))
    if rc == _lib.EUNSUPPORTED:
        return NotImplemented
    _lib.check(rc, "gnpde_attn_dot_rhs_f32")
    return None if stage is not None else out.view(x.shape)


def edge_attention(g, ns, m, rl, norm_idx):
    """attention [B,E,h] in COO order (SpGraphTransAttentionLayer.forward's first output)."""
    dev = g.csr.col.device
    att = torch.empty(g.B, g.E, ns.heads, dtype=torch.float32, device=dev)
    _lib.call("gnpde_edge_attention_f32", _ptr(g.csr.rowidx), _ptr(g.csr.col), _ptr(g.csr.perm), g.nnz, int(norm_idx),
              ns.mode, ns.heads, ns.dk, _ptr(ns.cs), _ptr(ns.q), _ptr(ns.k), ns.ldqk, ns.p0, ns.p1, _ptr(m), _ptr(rl),
              _ptr(att), _stream(dev))
    return att


# --------------------------------------------------------------------------- backward passes
def sddmm(g, gf, x, heads=1, alpha=None, alpha_sigmoid=False):
    """d <gf, a (A(w) x)> / d w in COO order: [B,E] (heads=1) or [B,E,heads]
    (w = the head mean of an [B,E,heads] attention): a <gf[src], x[dst]> / heads."""
    gfr = _rows(gf, "gf")
    xr = _rows(x, "x")
    C = xr.shape[1]
    dev = xr.device
    a = _scalar(alpha, "alpha", dev)
    shape = (g.B, g.E) if heads == 1 else (g.B, g.E, heads)
    out = torch.empty(shape, dtype=torch.float32, device=dev)
    _lib.call("gnpde_sddmm_f32", _ptr(g.csr.rowidx), _ptr(g.csr.col), _ptr(g.csr.perm), g.nnz, C, _ptr(gfr), C,
              _ptr(xr), C, _ptr(a), int(alpha_sigmoid), int(heads), _ptr(out), _stream(dev))
    return out


def softmax_backward(grouped, att, g_att):
    """Edge-softmax backward over the groups of ``grouped`` (COO [B,E,H] in and out)."""
    _require_gpu(att, "attention", torch.float32)
    _require_gpu(g_att, "attention grad", torch.float32)
    att, g_att = att.contiguous(), g_att.contiguous()
    H = att.shape[-1]
    gs = torch.empty_like(att)
    _lib.call("gnpde_softmax_backward_f32", _ptr(grouped.rowptr), _ptr(grouped.perm), grouped.R, grouped.nnz, H,
              _ptr(att), _ptr(g_att), _ptr(gs), _stream(att.device))
    return gs


def segment_sum(grouped, vals):
    """[R,H] fp64 sums of COO per-edge values [B,E,H] over the rows of ``grouped``."""
    _require_gpu(vals, "values", torch.float32)
    vals = vals.contiguous()
    H = vals.shape[-1]
    out = torch.empty(grouped.R, H, dtype=torch.float64, device=vals.device)
    _lib.call("gnpde_segment_sum_f64", _ptr(grouped.rowptr), _ptr(grouped.perm), grouped.R, grouped.nnz, H,
              _ptr(vals), _ptr(out), _stream(vals.device))
    return out


def dot(a, b, out=None):
    """<a, b> of two fp32 device tensors of the same size, accumulated in fp64
    (gnpde_dot_f64, fixed order): 0-d float64 tensor on the device (``out``: a
    one-element fp64 device tensor, e.g. a slot of a record, written in place)."""
    _require_gpu(a, "a", torch.float32)
    _require_gpu(b, "b", torch.float32)
    if a.numel() != b.numel():
        raise ValueError("dot: sizes differ (%d, %d)" % (a.numel(), b.numel()))
    a, b = a.contiguous(), b.contiguous()
    if out is None:
        out = torch.empty((), dtype=torch.float64, device=a.device)
    else:
        _require_gpu(out, "dot out", torch.float64)
        if out.numel() != 1:
            raise ValueError("dot: out must hold one fp64")
    nbytes = _lib.fn("gnpde_dot_workspace_bytes")()
    ws = torch.empty(nbytes, dtype=torch.uint8, device=a.device)
    _lib.call("gnpde_dot_f64", a.numel(), _ptr(a), _ptr(b), _ptr(out), _ptr(ws), nbytes, _stream(a.device))
    return out


def sum_f64(v, out=None, accumulate=False):
    """sum of an fp64 device vector (gnpde_sum_f64, fixed order) into a 0-d fp64
    tensor (added to ``out`` with accumulate=True)."""
    _require_gpu(v, "v", torch.float64)
    v = v.contiguous()
    if out is None:
        out = torch.zeros((), dtype=torch.float64, device=v.device)
    nbytes = _lib.fn("gnpde_dot_workspace_bytes")()
    ws = torch.empty(nbytes, dtype=torch.uint8, device=v.device)
    _lib.call("gnpde_sum_f64", v.numel(), _ptr(v), _ptr(out), int(bool(accumulate)), _ptr(ws), nbytes,
              _stream(v.device))
    return out


def scaled_sq_sums(y0, f0, f1, atol, rtol, out):
    """The squared sums of the initial-step selection for one component of a mixed
    norm (gnpde_scaled_sq_sums_f32): f1 None -> out[0] = sum (y0/sc)^2, out[1] =
    sum (f0/sc)^2; else out[0] = sum ((f1 - f0)/sc)^2; sc = atol + |y0| rtol.
    out: fp64 device [2] (a view is fine)."""
    for t in (y0, f0) + ((f1,) if f1 is not None else ()):
        _require_gpu(t, "scaled_sq_sums operand", torch.float32)
        if not t.is_contiguous() or t.numel() != y0.numel():
            raise ValueError("scaled_sq_sums: operands must be contiguous and shaped alike")
    _require_gpu(out, "scaled_sq_sums out", torch.float64)
    if out.numel() < 2 or not out.is_contiguous():
        raise ValueError("scaled_sq_sums: out needs 2 contiguous doubles")
    nbytes = _lib.fn("gnpde_initial_step_workspace_bytes")()
    ws = torch.empty(nbytes, dtype=torch.uint8, device=y0.device)
    _lib.call("gnpde_scaled_sq_sums_f32", y0.numel(), _ptr(y0), _ptr(f0), _ptr(f1), float(atol), float(rtol),
              _ptr(out), _ptr(ws), nbytes, _stream(y0.device))


def segment_sums(v, out):
    """out[s] = sum of row s of the fp64 device matrix v [nseg, len] (gnpde_segment_sums_f64,
    fixed order per segment): several epilogue row channels reduced in one pass."""
    _require_gpu(v, "segment_sums v", torch.float64)
    _require_gpu(out, "segment_sums out", torch.float64)
    if v.dim() != 2 or not v.is_contiguous():
        raise ValueError("segment_sums: v must be a contiguous [nseg, len] matrix")
    if out.numel() < v.shape[0] or not out.is_contiguous():
        raise ValueError("segment_sums: out needs nseg contiguous doubles")
    nbytes = _lib.fn("gnpde_segment_sums_workspace_bytes")(v.shape[0])
    ws = torch.empty(max(nbytes, 8), dtype=torch.uint8, device=v.device)
    _lib.call("gnpde_segment_sums_f64", v.shape[0], v.shape[1], _ptr(v), _ptr(out), _ptr(ws), nbytes,
              _stream(v.device))


def initial_step(y0, f0, f1, atol, rtol, order, h, hf=None, ws=None):
    """torchdiffeq's _select_initial_step on the device (gnpde_initial_step_*):
    phase 0 (f1 None) writes h[0] = h0, h[1] = d1 and hf = float(h0); phase 1
    (f1 = f(y0 + h0 f0)) writes h[2] = the first step.  h: fp64 [3], hf: fp32 0-d."""
    dt = y0.dtype
    if dt not in STATE_DTYPES:
        raise TypeError("initial_step: state dtype %s" % dt)
    for t in (y0, f0) + ((f1,) if f1 is not None else ()):
        _require_gpu(t, "initial_step state", dt)
        if not t.is_contiguous() or t.numel() != y0.numel():
            raise ValueError("initial_step: y0, f0, f1 must be contiguous and shaped alike")
    _require_gpu(h, "h", torch.float64)
    if h.numel() < 3 or (f1 is None and hf is None):
        raise ValueError("initial_step: h needs 3 doubles; phase 0 needs hf")
    if hf is not None:
        _require_gpu(hf, "hf", torch.float32)
    nbytes = _lib.fn("gnpde_initial_step_workspace_bytes")()
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=y0.device)
    name = "gnpde_initial_step_bf16" if dt == torch.bfloat16 else "gnpde_initial_step_f32"
    _lib.call(name, y0.numel(), _ptr(y0), _ptr(f0), _ptr(f1), float(atol), float(rtol), float(order), _ptr(h),
              _ptr(hf), _ptr(ws), nbytes, _stream(y0.device))


def initial_step_lin(y0, v, atol, rtol, order, h, hf=None, ws=None):
    """Phase 1 of the device initial step from v = L f0 (gnpde_initial_step_lin_*):
    d2 = rms(v / scale); writes h[2] (and hf).  h: fp64 [3] after phase 0."""
    dt = y0.dtype
    if dt not in STATE_DTYPES:
        raise TypeError("initial_step_lin: state dtype %s" % dt)
    for t in (y0, v):
        _require_gpu(t, "initial_step state", dt)
        if not t.is_contiguous() or t.numel() != y0.numel():
            raise ValueError("initial_step_lin: y0 and v must be contiguous and shaped alike")
    _require_gpu(h, "h", torch.float64)
    if hf is not None:
        _require_gpu(hf, "hf", torch.float32)
    nbytes = _lib.fn("gnpde_initial_step_workspace_bytes")()
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=y0.device)
    name = "gnpde_initial_step_lin_f32" if dt == torch.float32 else "gnpde_initial_step_lin_bf16"
    _lib.call(name, y0.numel(), _ptr(y0), _ptr(v), float(atol), float(rtol), float(order), _ptr(h), _ptr(hf),
              _ptr(ws), ws.numel(), _stream(y0.device))


def initial_step_rows(rows_a, rows_b, n, order, h, hf, ws=None):
    """gnpde_initial_step_rows: the initial-step rules from the squared-sum rows of the f0
    launch (phase 0: rows_a its err_rows, rows_b its scale_rows) or of the launch over L f0
    (phase 1: rows_b None).  h: fp64 [3], hf: fp32 0-d (device)."""
    _require_gpu(rows_a, "rows", torch.float64)
    if rows_b is not None:
        _require_gpu(rows_b, "rows", torch.float64)
    _require_gpu(h, "h", torch.float64)
    if hf is not None:
        _require_gpu(hf, "hf", torch.float32)
    nbytes = _lib.fn("gnpde_initial_step_workspace_bytes")()
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=rows_a.device)
    _lib.call("gnpde_initial_step_rows", rows_a.numel(), _ptr(rows_a), _ptr(rows_b), float(n), float(order), _ptr(h),
              _ptr(hf), _ptr(ws), ws.numel(), _stream(rows_a.device))


def adaptive_control(err_rows, n, order, safety, ifactor, dfactor, dt, scale, rec, ws=None, t=None):
    """The step's error-row sum and torchdiffeq's step-size controller on the device
    (gnpde_adaptive_control): rec = {error ratio, dt, next dt, squared error sum};
    dt (fp64 0-d) and scale (fp32 0-d) advance to the next step's size; ``t`` (fp64,
    optional: its first element) advances by the step when it is accepted (the step
    start a folded dense output reads, Stage.dense).  ``ws``: a reusable workspace
    (gnpde_dot_workspace_bytes() bytes)."""
    _require_gpu(err_rows, "err_rows", torch.float64)
    _require_gpu(dt, "dt", torch.float64)
    _require_gpu(scale, "scale", torch.float32)
    _require_gpu(rec, "rec", torch.float64)
    if rec.numel() < 4:
        raise ValueError("adaptive_control: rec needs 4 doubles")
    if t is not None:
        _require_gpu(t, "t", torch.float64)
    nbytes = _lib.fn("gnpde_dot_workspace_bytes")()
    if ws is None:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=err_rows.device)
    _lib.call("gnpde_adaptive_control", err_rows.numel(), _ptr(err_rows), float(n), float(order), float(safety),
              float(ifactor), float(dfactor), _ptr(dt), _ptr(scale), _ptr(rec), _ptr(t), _ptr(ws), ws.numel(),
              _stream(err_rows.device))


def wcolsum(x, B, N, w):
    """y [B,H,C+1] fp64: y[b,h,:C] = sum_n w[b*N+n,h] x[b,n,:], y[b,h,C] = sum_n w[b*N+n,h]."""
    xr = _rows(x, "x")
    _require_gpu(w, "weights", torch.float64)
    w = w.contiguous()
    H = w.shape[-1]
    C = xr.shape[1]
    ws_bytes = _lib.fn("gnpde_wcolsum_workspace_bytes")(B, N, C, H)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=xr.device)
    y = torch.empty(B, H, C + 1, dtype=torch.float64, device=xr.device)
    _lib.call("gnpde_wcolsum_f64", _ptr(xr), B, N, C, C, _ptr(w), H, _ptr(y), _ptr(ws), ws_bytes,
              _stream(xr.device))
    return y


def score_input_grad(gcs, U, deg, gxbar, B, N, C, out=None):
    """gx [R,C] fp32 = gcs U_b^T + deg * gxbar_b  (reference-mode node-score backward)."""
    H = gcs.shape[-1]
    dev = gcs.device
    gx = torch.empty(B * N, C, dtype=torch.float32, device=dev) if out is None else out
    _lib.call("gnpde_score_input_grad_f32", _ptr(gcs.contiguous()), _ptr(U.contiguous()), _ptr(deg),
              _ptr(gxbar.contiguous()), B, N, C, H, _ptr(gx), C, int(out is not None), _stream(dev))
    return gx


def score_grad(grouped, side, ns, gs, with_params=False):
    """gnpde_score_grad_f32: dL/d(q) (side 0, over the aggregation CSR) or dL/d(k)
    (side 1, over the CSC) [R, att] from gs = dL/ds [B,E,H] (COO) for the per-edge
    score modes; with_params (exp_kernel): also the per-edge terms of
    dL/d(output_var), dL/d(lengthscale) summed in fp64 -> (out, g_p0, g_p1)."""
    _require_gpu(gs, "score grad", torch.float32)
    gs = gs.contiguous()
    att = ns.heads * ns.dk
    dev = gs.device
    out = torch.empty(grouped.R, att, dtype=torch.float32, device=dev)
    gp = torch.empty(max(grouped.nnz, 1), 2 * ns.heads, dtype=torch.float32, device=dev) if with_params else None
    _lib.call("gnpde_score_grad_f32", _ptr(grouped.rowptr), _ptr(grouped.col), _ptr(grouped.perm), grouped.R,
              grouped.nnz, int(side), ns.mode, ns.heads, ns.dk, _ptr(ns.q), _ptr(ns.k), ns.ldqk, ns.p0, ns.p1, _ptr(gs),
              _ptr(out), att, _ptr(gp), _stream(dev))
    if not with_params:
        return out
    if grouped.nnz == 0:
        z = torch.zeros((), dtype=torch.float64, device=dev)
        return out, z, z
    gpd = gp[:grouped.nnz].double()
    return out, gpd[:, :ns.heads].sum(), gpd[:, ns.heads:].sum()


def gather_head(grouped, w, h, scale=1.0):
    """scale * w[:, :, h] (COO [B,E,H]) in ``grouped`` order [nnz]."""
    _require_gpu(w, "values", torch.float32)
    w = w.contiguous()
    H = w.shape[-1]
    out = torch.empty(max(grouped.nnz, 1), dtype=torch.float32, device=w.device)
    _lib.call("gnpde_gather_head_f32", _ptr(w), grouped.nnz, H, int(h), _ptr(grouped.perm), float(scale), _ptr(out),
              _stream(w.device))
    return out


# --------------------------------------------------------------------------- solver glue
def rows_copy(src, dst, order=None, dst_copy=None):
    """gnpde_rows_copy: dst[k] = src[order[k]] (rows = the leading dims flattened,
    order int64 or None = identity) and, when given, dst_copy[order[k]] = the same
    row (a plain copy of src) from the same read."""
    _require_gpu(src, "src")
    src = src.contiguous()
    C = src.shape[-1]
    rows = src.numel() // max(C, 1)
    for t, nm in ((dst, "dst"), (dst_copy, "dst_copy")):
        if t is not None:
            _require_gpu(t, nm, src.dtype)
            if not t.is_contiguous() or t.numel() != src.numel():
                raise ValueError("rows_copy: %s must be contiguous and sized like src" % nm)
    if order is not None:
        _require_gpu(order, "order", torch.int64)
        if order.numel() != rows:
            raise ValueError("rows_copy: %d order entries for %d rows" % (order.numel(), rows))
    _lib.call("gnpde_rows_copy", _ptr(src), rows, C * src.element_size(), _ptr(order), _ptr(dst), _ptr(dst_copy),
              _stream(src.device))
    return dst


def rk_combine(y0, ks, coefs, scale, out=None):
    """out = y0 + scale * sum_j coefs[j] * ks[j]  (one fused pass; y0=None means 0)."""
    ref = y0 if y0 is not None else ks[0]
    _require_gpu(ref, "y0", torch.float32)
    if y0 is not None:
        y0 = y0.contiguous()
    if out is None:
        out = torch.empty_like(ref, memory_format=torch.contiguous_format)
    nk = len(ks)
    kp = (ctypes.c_void_p * max(nk, 1))()
    cf = (ctypes.c_double * max(nk, 1))()
    keep = []
    for j, (k, c) in enumerate(zip(ks, coefs)):
        _require_gpu(k, "k%d" % j, torch.float32)
        k = k.contiguous()
        keep.append(k)
        kp[j] = k.data_ptr()
        cf[j] = float(c)
    _lib.call("gnpde_rk_combine_f32", ref.numel(), _ptr(y0), nk, kp, cf, float(scale), _ptr(out),
              _stream(ref.device))
    return out
