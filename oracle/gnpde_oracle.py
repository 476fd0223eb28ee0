"""CPU oracle for the GRAND/BLEND ODE right-hand side — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The shipped path (``graph-neural-pde_amd/gnpde``) never imports it and has
no CPU fallback.

It restates, in float64 numpy, the arithmetic of the reference hot path
(alimt1992/graph-neural-pde @ 2025-01-17).  Every function cites the reference
lines it follows.  Parity is PINNED: ``tests/test_oracle_golden.py`` checks
every function below against the golden vectors in ``tests/golden/`` that
``tests/golden/gen_golden.py`` produced by running the reference modules
themselves (float64), plus the reference tests' known answers
(test/test_utils.py:62-79, test/test_function_laplacian_diffusion.py:56-86,
test/test_transformer_attention.py:98-106).  Exceptions, documented in
DESIGN.md §Parity: the graph-normalisation helpers (the fork's versions crash
on batched input, SURVEY §0.5 — pinned by the KATs only), the ``per_edge``
score mode (upstream GRAND semantics, not in the fork: parity unpinned) and the
integrators (torchdiffeq is absent; no reference test checks integrated values:
parity unpinned).

Layout conventions (same as the reference): ``edge_index [B,2,E]`` int64 with
row 0 = source / aggregating node and row 1 = destination / gathered node;
node features ``x [B,N,C]``; per-edge weights ``[B,E]`` or ``[B,E,h]``.
"""
import numpy as np

try:  # scipy is only a speed-up for the aggregation at large sizes
    import scipy.sparse as _sp
except Exception:  # pragma: no cover
    _sp = None


def _as64(a):
    return np.asarray(a, dtype=np.float64)


def _sigmoid(a):
    return 1.0 / (1.0 + np.exp(-a))


# --------------------------------------------------------------------------- aggregation
def aggregate(edge_index, w, x):
    """``ax[b,i,:] = sum_{e: edge[b,0,e]=i} w[b,e] * x[b, edge[b,1,e], :]``.

    Restates the sparse-COO -> to_dense -> matmul of
    src/function_laplacian_diffusion.py:39-58 (and
    src/function_transformer_attention.py:34-41); duplicates are summed, as
    ``to_dense`` sums coalesced duplicates.
    """
    edge_index = np.asarray(edge_index)
    w = _as64(w)
    x = _as64(x)
    B, N, C = x.shape
    out = np.zeros((B, N, C))
    for b in range(B):
        src, dst = edge_index[b, 0], edge_index[b, 1]
        if _sp is not None:
            A = _sp.coo_matrix((w[b], (src, dst)), shape=(N, N)).tocsr()
            out[b] = A @ x[b]
        else:
            np.add.at(out[b], src, w[b][:, None] * x[b][dst])
    return out


def alpha_value(alpha_train, no_alpha_sigmoid):
    """src/function_laplacian_diffusion.py:69-72 / src/function_transformer_attention.py:52-55."""
    a = float(alpha_train)
    return a if no_alpha_sigmoid else float(_sigmoid(a))


def rhs_epilogue(ax, x, x0, alpha_train, beta_train, add_source, no_alpha_sigmoid):
    """``f = alpha*(ax - x) [+ beta_train * x0]`` — function_laplacian_diffusion.py:69-77."""
    f = alpha_value(alpha_train, no_alpha_sigmoid) * (ax - _as64(x))
    if add_source:
        f = f + float(beta_train) * _as64(x0)
    return f


def laplacian_weights(block, edge_weight=None, attention_weights=None):
    """Weight source by ``opt['block']`` — function_laplacian_diffusion.py:45-57."""
    if block == 'attention':
        return _as64(attention_weights).mean(axis=2)
    if block in ('mixed', 'hard_attention'):
        return _as64(attention_weights)
    return _as64(edge_weight)


def laplacian_rhs(edge_index, x, x0, alpha_train, beta_train, block='constant', edge_weight=None,
                  attention_weights=None, add_source=False, no_alpha_sigmoid=False):
    """LaplacianODEFunc.forward — src/function_laplacian_diffusion.py:60-77."""
    w = laplacian_weights(block, edge_weight, attention_weights)
    ax = aggregate(edge_index, w, x)
    return rhs_epilogue(ax, x, x0, alpha_train, beta_train, add_source, no_alpha_sigmoid)


# --------------------------------------------------------------------------- block weight producers
def mixed_attention(attention, edge_weight, gamma):
    """MixedODEblock.get_mixed_attention — src/block_mixed.py:29-33:
    ``attention.mean(dim=2) * (1 - sigmoid(gamma)) + edge_weight * sigmoid(gamma)``."""
    g = float(_sigmoid(float(gamma)))
    return _as64(attention).mean(axis=2) * (1.0 - g) + _as64(edge_weight) * g


def quantile_f32(v, q):
    """torch.quantile(v, q) with linear interpolation, restated in float32 as
    ATen computes it (sort; rank = q*(n-1) in the input dtype; lerp with ATen's
    two-sided formula) — the threshold of src/block_transformer_hard_attention.py:52."""
    s = np.sort(np.asarray(v, dtype=np.float32).reshape(-1))
    n = s.size
    rank = np.float32(q) * np.float32(n - 1)
    lo = int(np.floor(rank))
    hi = int(np.ceil(rank))
    w = np.float32(rank - np.float32(lo))
    a, b = s[lo], s[hi]
    if abs(w) < 0.5:
        return np.float32(a + w * (b - a))
    return np.float32(b - (b - a) * (np.float32(1) - w))


def group_normalize(w, index, num_nodes):
    """HardAttODEblock.renormalise_attention (upstream single-graph semantics) —
    src/block_transformer_hard_attention.py:32-35: ``w / (scatter_sum(w, index)[index] + 1e-16)``."""
    w = _as64(w)
    sums = np.zeros(num_nodes)
    np.add.at(sums, np.asarray(index), w)
    return w / (sums[np.asarray(index)] + 1e-16)


def hard_attention_sample(edge_index, attention, att_samp_pct, norm_idx, num_nodes):
    """Training-mode attention sampling of HardAttODEblock.forward —
    src/block_transformer_hard_attention.py:42-57 (B = 1, use_flux off):
    keep edges whose head-mean attention exceeds the (1 - att_samp_pct)
    quantile; renormalise the kept weights per group of row ``norm_idx``.
    Returns (edge_index [1,2,E'], weights [1,E'])."""
    mean_att = np.asarray(attention, dtype=np.float32)
    if mean_att.ndim == 3:
        mean_att = (mean_att.sum(axis=2, dtype=np.float32) / np.float32(mean_att.shape[2])).astype(np.float32)
    thr = quantile_f32(mean_att, 1 - att_samp_pct)
    mask = mean_att[0] > thr
    ei = np.asarray(edge_index)[:, :, mask]
    w = group_normalize(mean_att[0, mask], ei[0, norm_idx], num_nodes)
    return ei, w[None, :]


# --------------------------------------------------------------------------- edge softmax
def edge_softmax(src, index, num_nodes=None):
    """utils.softmax — src/utils.py:116-127.

    ``out = exp(s - max_g s) / (sum_g exp(s - max_g s) + 1e-16)`` with groups
    ``g = index[b, e]`` per batch element, broadcast over the head axis.
    """
    src = _as64(src)
    index = np.asarray(index)
    B, E, H = src.shape
    if num_nodes is None:
        num_nodes = int(index.max()) + 1 if index.size else 0
    out = np.empty_like(src)
    for b in range(B):
        mx = np.full((num_nodes, H), -np.inf)
        np.maximum.at(mx, index[b], src[b])
        ex = np.exp(src[b] - mx[index[b]])
        sm = np.zeros((num_nodes, H))
        np.add.at(sm, index[b], ex)
        out[b] = ex / (sm[index[b]] + 1e-16)
    return out


def squareplus(src, index, num_nodes=None):
    """utils.squareplus — src/utils.py:129-140 (intended call with num_nodes).

    Per batch element: ``out = (s' + sqrt(s'^2 + 4))/2`` with ``s' = s - max(s)``
    (max over all edges and heads of that element), normalised per group.
    """
    src = _as64(src)
    index = np.asarray(index)
    B, E, H = src.shape
    if num_nodes is None:
        num_nodes = int(index.max()) + 1
    out = np.empty_like(src)
    for b in range(B):
        s = src[b] - src[b].max()
        s = (s + np.sqrt(s * s + 4.0)) / 2.0
        sm = np.zeros((num_nodes, H))
        np.add.at(sm, index[b], s)
        out[b] = s / (sm[index[b]] + 1e-16)
    return out


# --------------------------------------------------------------------------- attention scores
def project(x, W, b):
    """nn.Linear(x) = x W^T + b — function_transformer_attention.py:224-226."""
    return _as64(x) @ _as64(W).T + _as64(b)


def split_heads(q, heads):
    """view(B,N,h,d_k).transpose(2,3) -> [B,N,d_k,h] — function_transformer_attention.py:230-238."""
    B, N, A = q.shape
    return q.reshape(B, N, heads, A // heads).transpose(0, 1, 3, 2)


def attention_scores(x, edge_index, Wq, bq, Wk, bk, heads, attention_type='scaled_dot', score_mode='reference',
                     output_var=1.0, lengthscale=1.0):
    """``prods [B,E,h]`` — function_transformer_attention.py:218-259 (standard, non-beltrami branch).

    score_mode='reference' restates the fork's scaled_dot (:249) exactly:
    ``sum(matmul(src[B,h,E,dk], dst_k[B,h,dk,E] / sqrt(dk)), dim=3)``, which
    equals ``q_src(e),h . (sum_e' k_dst(e'),h) / sqrt(dk)`` — one global key-sum
    per (batch, head), computed here in O(E*d).  score_mode='per_edge' is the
    upstream-GRAND ``q_src . k_dst / sqrt(dk)`` (not in the fork: unpinned).
    exp_kernel (:246-247), cosine_sim (:250-252, torch>=1.12 CosineSimilarity:
    each operand divided by max(norm, eps)), pearson (:253-259) are per-edge.
    """
    edge_index = np.asarray(edge_index)
    q = split_heads(project(x, Wq, bq), heads)  # [B,N,dk,h]
    k = split_heads(project(x, Wk, bk), heads)
    B = q.shape[0]
    dk = q.shape[2]
    out = []
    for b in range(B):
        src = q[b][edge_index[b, 0]]  # [E,dk,h]
        dst = k[b][edge_index[b, 1]]
        if attention_type == 'scaled_dot':
            if score_mode == 'reference':
                ksum = dst.sum(axis=0)  # [dk,h]
                p = (src * ksum[None]).sum(axis=1) / np.sqrt(dk)
            else:
                p = (src * dst).sum(axis=1) / np.sqrt(dk)
        elif attention_type == 'exp_kernel':
            p = output_var ** 2 * np.exp(-((src - dst) ** 2).sum(axis=1) / (2 * lengthscale ** 2))
        elif attention_type in ('cosine_sim', 'pearson'):
            if attention_type == 'pearson':
                src = src - src.mean(axis=1, keepdims=True)
                dst = dst - dst.mean(axis=1, keepdims=True)
            eps = 1e-5
            ns = np.maximum(np.sqrt((src ** 2).sum(axis=1, keepdims=True)), eps)
            nd = np.maximum(np.sqrt((dst ** 2).sum(axis=1, keepdims=True)), eps)
            p = ((src / ns) * (dst / nd)).sum(axis=1)
        else:
            raise ValueError(attention_type)
        out.append(p)
    return np.stack(out, 0)


def transformer_attention(x, edge_index, Wq, bq, Wk, bk, heads, norm_idx, attention_type='scaled_dot',
                          score_mode='reference', square_plus=False, output_var=1.0, lengthscale=1.0):
    """SpGraphTransAttentionLayer.forward -> attention [B,E,h] — function_transformer_attention.py:159-267."""
    prods = attention_scores(x, edge_index, Wq, bq, Wk, bk, heads, attention_type, score_mode, output_var,
                             lengthscale)
    index = np.asarray(edge_index)[:, norm_idx, :]
    if square_plus:
        return squareplus(prods, index)
    return edge_softmax(prods, index)


def transformer_rhs(edge_index, x, x0, Wq, bq, Wk, bk, heads, norm_idx, alpha_train, beta_train,
                    attention_type='scaled_dot', score_mode='reference', add_source=False, no_alpha_sigmoid=False,
                    square_plus=False, output_var=1.0, lengthscale=1.0):
    """ODEFuncTransformerAtt.forward — function_transformer_attention.py:44-59 with
    multiply_attention (mix_features=False, :33-41): head-mean weights x aggregation."""
    att = transformer_attention(x, edge_index, Wq, bq, Wk, bk, heads, norm_idx, attention_type, score_mode,
                                square_plus, output_var, lengthscale)
    ax = aggregate(edge_index, att.mean(axis=2), x)
    return rhs_epilogue(ax, x, x0, alpha_train, beta_train, add_source, no_alpha_sigmoid)


def transformer_rhs_f32(edge_index, x, Wq, bq, Wk, bk, heads, norm_idx, alpha_train, score_mode='per_edge'):
    """The transformer RHS in FLOAT32 arithmetic, in the reference's operation
    order — the precision the reference itself runs in (the torch fp32 CPU path):
    nn.Linear Q/K (function_transformer_attention.py:224-225, x W^T + b in fp32),
    the gathers (:240-244), ``(src * dst_k).sum(dk) / sqrt(dk)`` per edge and head
    (upstream GRAND's scaled_dot; the fork's global key sum with
    score_mode='reference', :249), utils.softmax in fp32 (src/utils.py:116-127:
    group max, exp(s - max), group sum, / (sum + 1e-16)), the head mean (:34) and
    the aggregation + epilogue (:33-41, :52-59), every array float32.

    Not a parity target: the yardstick of how far an fp32 evaluation of the
    reference's own formula sits from the float64 restatement above on the same
    inputs.  At score ranges in the hundreds the fp32 score alone carries a
    relative error of ~1e-5 in the output (tests/test_gpu_flash.py)."""
    f32 = np.float32
    edge_index = np.asarray(edge_index)
    x = np.asarray(x, f32)
    B, N, C = x.shape
    q = x @ np.asarray(Wq, f32).T + np.asarray(bq, f32)
    k = x @ np.asarray(Wk, f32).T + np.asarray(bk, f32)
    A = q.shape[-1]
    dk = A // heads
    inv = f32(1.0 / np.sqrt(dk))
    a = f32(alpha_value(alpha_train, False))
    out = np.empty_like(x)
    for b in range(B):
        src, dst = edge_index[b, 0], edge_index[b, 1]
        qs = q[b][src].reshape(-1, heads, dk)
        kd = k[b][dst].reshape(-1, heads, dk)
        if score_mode == 'reference':
            s = (qs * kd.sum(axis=0, dtype=f32)[None]).sum(axis=2, dtype=f32) * inv
        else:
            s = (qs * kd).sum(axis=2, dtype=f32) * inv
        g = edge_index[b, norm_idx]
        mx = np.full((N, heads), -np.inf, f32)
        np.maximum.at(mx, g, s)
        ex = np.exp(s - mx[g]).astype(f32)
        sm = np.zeros((N, heads), f32)
        np.add.at(sm, g, ex)
        att = ex / (sm[g] + f32(1e-16))
        w = att.mean(axis=1, dtype=f32)
        ax = np.zeros((N, C), f32)
        np.add.at(ax, src, w[:, None] * x[b][dst])
        out[b] = a * (ax - x[b])
    return out


# --------------------------------------------------------------------------- graph preparation
def add_remaining_self_loops(edge_index, edge_weight, fill_value, num_nodes):
    """Intended semantics of src/utils.py:16-42 (the fork's batched rewrite
    corrupts the edge set): upstream GRAND / PyG
    ``add_remaining_self_loops`` applied per batch element — non-loop edges are
    kept in order, then one loop per node whose weight is the node's existing
    loop weight (last one wins) or ``fill_value``.  Returns lists per batch
    element (counts may differ)."""
    edge_index = np.asarray(edge_index)
    B, _, E = edge_index.shape
    if edge_weight is None:
        edge_weight = np.ones((B, E))
    out_e, out_w = [], []
    for b in range(B):
        row, col = edge_index[b]
        w = _as64(edge_weight[b])
        mask = row != col
        loop_w = np.full(num_nodes, float(fill_value))
        inv = ~mask
        loop_w[row[inv]] = w[inv]
        ei = np.concatenate([edge_index[b][:, mask], np.stack([np.arange(num_nodes)] * 2)], axis=1)
        out_e.append(ei)
        out_w.append(np.concatenate([w[mask], loop_w]))
    return out_e, out_w


def get_rw_adj(edge_index, edge_weight=None, norm_dim=1, fill_value=0.0, num_nodes=None):
    """Intended semantics of src/utils.py:215-233 pinned by test/test_utils.py:62-79:
    dense result == sklearn ``normalize(A + s*I, 'l1', axis = 0 if norm_dim==1 else 1)``."""
    edge_index = np.asarray(edge_index)
    B, _, E = edge_index.shape
    if num_nodes is None:
        num_nodes = int(edge_index.max()) + 1
    if edge_weight is None:
        edge_weight = np.ones((B, E))
    if fill_value != 0:
        eis, ws = add_remaining_self_loops(edge_index, edge_weight, fill_value, num_nodes)
    else:
        eis = [edge_index[b] for b in range(B)]
        ws = [_as64(edge_weight[b]) for b in range(B)]
    out_w = []
    for ei, w in zip(eis, ws):
        idx = ei[0] if norm_dim == 0 else ei[1]
        deg = np.zeros(num_nodes)
        np.add.at(deg, idx, w)
        with np.errstate(divide='ignore'):
            inv = 1.0 / deg
        out_w.append(inv[idx] * w)
    return eis, out_w


def gcn_norm_fill_val(edge_index, edge_weight=None, fill_value=0.0, num_nodes=None):
    """Intended semantics of src/utils.py:177-194 (test/test_function_laplacian_diffusion.py:73-85,
    test/test_ICML_gnn.py): ``D^-1/2 (A + s*I) D^-1/2`` with deg over the column index, inf -> 0."""
    edge_index = np.asarray(edge_index)
    B, _, E = edge_index.shape
    if num_nodes is None:
        num_nodes = int(edge_index.max()) + 1
    if edge_weight is None:
        edge_weight = np.ones((B, E))
    if int(fill_value) != 0:
        eis, ws = add_remaining_self_loops(edge_index, edge_weight, fill_value, num_nodes)
    else:
        eis = [edge_index[b] for b in range(B)]
        ws = [_as64(edge_weight[b]) for b in range(B)]
    out_w = []
    for ei, w in zip(eis, ws):
        deg = np.zeros(num_nodes)
        np.add.at(deg, ei[1], w)
        with np.errstate(divide='ignore'):
            dis = deg ** -0.5
        dis[np.isinf(dis)] = 0.0
        out_w.append(dis[ei[0]] * w * dis[ei[1]])
    return eis, out_w


def to_dense(edge_index_b, w_b, num_nodes):
    """Dense [N,N] of one batch element (duplicates summed) — utils.to_dense_adj :102-113."""
    A = np.zeros((num_nodes, num_nodes))
    np.add.at(A, (edge_index_b[0], edge_index_b[1]), w_b)
    return A


# --------------------------------------------------------------------------- integrators
def fixed_grid(t0, t1, step_size):
    """torchdiffeq FixedGridODESolver grid (0.2.x ``_grid_constructor_from_step_size``):
    ``niters = ceil((t1-t0)/h + 1)``, ``t = arange(niters)*h + t0``, last point := t1.
    Computed in float32, the dtype the reference's ``t.type_as(x)`` gives
    (src/block_constant.py:23)."""
    t0 = np.float32(t0)
    t1 = np.float32(t1)
    h = np.float32(step_size)
    niters = int(np.ceil(np.float32((t1 - t0) / h) + np.float32(1)))
    grid = np.arange(niters, dtype=np.float32) * h + t0
    grid[-1] = t1
    return grid


def odeint_fixed(func, y0, t0, t1, method, step_size):
    """euler / rk4 (torchdiffeq ``rk4_alt_step_func``, 3/8 rule) over the fixed grid;
    parity unpinned."""
    y = _as64(y0)
    grid = fixed_grid(t0, t1, step_size)
    for ta, tb in zip(grid[:-1], grid[1:]):
        dt = float(tb) - float(ta)
        if method == 'euler':
            y = y + dt * func(float(ta), y)
        elif method == 'rk4':
            k1 = func(float(ta), y)
            k2 = func(float(ta) + dt / 3.0, y + dt * k1 / 3.0)
            k3 = func(float(ta) + dt * 2.0 / 3.0, y + dt * (k2 - k1 / 3.0))
            k4 = func(float(tb), y + dt * (k1 - k2 + k3))
            y = y + (k1 + 3.0 * (k2 + k3) + k4) * dt * 0.125
        else:
            raise ValueError(method)
    return y


# Embedded explicit RK pairs of torchdiffeq 0.2.x (dopri5.py, bosh3.py, fehlberg2.py,
# adaptive_heun.py): (order, A rows, b of the propagated solution, b - b_hat, dense-output mid).
_DPS = (5, [[1 / 5], [3 / 40, 9 / 40], [44 / 45, -56 / 15, 32 / 9],
            [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
            [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
            [35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84]],
        [35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84, 0],
        [35 / 384 - 1951 / 21600, 0, 500 / 1113 - 22642 / 50085, 125 / 192 - 451 / 720,
         -2187 / 6784 + 12231 / 42400, 11 / 84 - 649 / 6300, -1 / 60],
        [v / 2 for v in (6025192743 / 30085553152, 0, 51252292925 / 65400821598, -2691868925 / 45128329728,
                         187940372067 / 1594534317056, -1776094331 / 19743644256, 11237099 / 235043384)])
ADAPTIVE_TABLEAUS = {
    'dopri5': _DPS,
    'bosh3': (3, [[1 / 2], [0, 3 / 4], [2 / 9, 1 / 3, 4 / 9]], [2 / 9, 1 / 3, 4 / 9, 0],
              [2 / 9 - 7 / 24, 1 / 3 - 1 / 4, 4 / 9 - 1 / 3, -1 / 8], [0, 1 / 2, 0, 0]),
    'fehlberg2': (2, [[1 / 2], [1 / 256, 255 / 256]], [1 / 512, 255 / 256, 1 / 512],
                  [-1 / 512, 0, 1 / 512], [0, 1 / 2, 0]),
    'adaptive_heun': (2, [[1.0]], [1 / 2, 1 / 2], [1 / 2, -1 / 2], [1 / 2, 0]),
}


def odeint_adaptive(func, y0, ts, method, rtol, atol, first_step=None):
    """torchdiffeq 0.2.x ``RKAdaptiveStepsizeODESolver`` in float64 numpy: initial
    step from ``_select_initial_step`` (Hairer's d0/d1/d2 rule), RMS error ratio
    over ``atol + rtol*max(|y0|,|y1|)``, step factor ``min(10, max(0.9 r^(-1/order),
    0.2 if rejected else 1))``, the next step's f0 = the last stage (as torchdiffeq,
    also for the non-FSAL pairs) and the quartic ``_interp_fit`` dense output at
    every requested time.  ``first_step`` replaces the initial-step rule (torchdiffeq's
    options['first_step']).  Returns (solution [len(ts), ...], n_steps).  Parity
    unpinned (torchdiffeq absent): checked against exact flows."""
    order, A, b, e, mid = ADAPTIVE_TABLEAUS[method]
    fsal = b[-1] == 0 and list(b[:-1]) == list(A[-1])
    rms = lambda v: float(np.sqrt(np.mean(np.square(v))))  # noqa: E731
    y = _as64(y0)
    ts = [float(v) for v in ts]
    f = func(ts[0], y)
    sc = atol + np.abs(y) * rtol
    d0, d1 = rms(y / sc), rms(f / sc)
    h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    f_probe = func(ts[0] + h0, y + h0 * f)
    d2 = rms((f_probe - f) / sc) / h0
    h1 = max(1e-6, h0 * 1e-3) if (d1 <= 1e-15 and d2 <= 1e-15) else (0.01 / max(d1, d2)) ** (1.0 / order)
    h = min(100 * h0, h1) if first_step is None else float(first_step)
    t = ts[0]
    out = [y]
    seg = None  # (t_a, t_b, y_a, y_b, f_a, f_b, y_mid) of the last accepted step
    n = 0
    for target in ts[1:]:
        while target > t:
            ks = [f]
            for row in A:
                ks.append(func(t + h * sum(row), y + h * sum(c * k for c, k in zip(row, ks))))
            y_new = y + h * sum(c * k for c, k in zip(A[-1], ks)) if fsal else \
                y + h * sum(c * k for c, k in zip(b, ks))
            err = h * sum(c * k for c, k in zip(e, ks))
            ratio = rms(err / (atol + rtol * np.maximum(np.abs(y), np.abs(y_new))))
            if ratio <= 1:
                seg = (t, t + h, y, y_new, ks[0], ks[-1], y + h * sum(c * k for c, k in zip(mid, ks)), h)
                t, y, f = t + h, y_new, ks[-1]
            if ratio == 0:
                h = h * 10.0
            else:
                h = h * min(10.0, max(0.9 * ratio ** (-1.0 / order), 0.2 if ratio >= 1 else 1.0))
            n += 1
        if seg is None or target == t:
            out.append(y)
        else:
            ta, tb, ya, yb, fa, fb, ym, hs = seg
            p4 = 2 * hs * (fb - fa) - 8 * (yb + ya) + 16 * ym
            p3 = hs * (5 * fa - 3 * fb) + 18 * ya + 14 * yb - 32 * ym
            p2 = hs * (fb - 4 * fa) - 11 * ya - 5 * yb + 16 * ym
            x = (target - ta) / (tb - ta)
            out.append(ya + x * (hs * fa) + x ** 2 * p2 + x ** 3 * p3 + x ** 4 * p4)
    return np.stack(out, 0), n


# --------------------------------------------------------------------------- prepared CSR (timed CPU baseline)
class LaplacianCSR(object):
    """The Laplacian RHS with the COO -> CSR conversion done once (scipy), so the
    CPU baseline times the steady-state RHS the way the GPU path is timed.
    Same arithmetic as ``laplacian_rhs`` (function_laplacian_diffusion.py:39-77);
    float32 storage and arithmetic, like the reference's fp32 runs."""

    def __init__(self, edge_index, w, num_nodes, dtype=np.float32):
        edge_index = np.asarray(edge_index)
        self.B = edge_index.shape[0]
        self.N = int(num_nodes)
        self.A = [_sp.coo_matrix((np.asarray(w[b], dtype), (edge_index[b, 0], edge_index[b, 1])),
                                 shape=(self.N, self.N)).tocsr() for b in range(self.B)]
        self.dtype = dtype

    def rhs(self, x, alpha, x0=None, beta=0.0, add_source=False, no_alpha_sigmoid=False):
        a = self.dtype(alpha_value(alpha, no_alpha_sigmoid))
        out = np.empty_like(x)
        for b in range(self.B):
            out[b] = a * (self.A[b] @ x[b] - x[b])
            if add_source:
                out[b] += self.dtype(beta) * x0[b]
        return out


# --------------------------------------------------------------------------- C restatement (timed baseline)
class COracle(object):
    """ctypes view of oracle/build/liboracle.so (oracle/c/rhs_oracle.c): the
    Laplacian RHS in fp32 over a CSR built once, OpenMP over rows."""

    def __init__(self, path=None):
        import ctypes
        import os
        path = path or os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "liboracle.so")
        self.lib = ctypes.CDLL(path)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        self.lib.gnpde_oracle_csr.argtypes = [vp, i64, i64, i64, vp, vp, vp, vp]
        self.lib.gnpde_oracle_laplacian_rhs.argtypes = [vp, vp, vp, i64, i64, vp, vp, ctypes.c_float,
                                                        ctypes.c_float, ctypes.c_int, ctypes.c_int, vp,
                                                        ctypes.c_int]
        self.ct = ctypes

    def csr(self, edge_index, w, num_nodes):
        ei = np.ascontiguousarray(edge_index, dtype=np.int64)
        B, _, E = ei.shape
        R = B * int(num_nodes)
        rowptr = np.empty(R + 1, np.int64)
        col = np.empty(max(B * E, 1), np.int32)
        wc = np.empty(max(B * E, 1), np.float32)
        wf = np.ascontiguousarray(w, dtype=np.float32).reshape(-1)
        p = lambda a: a.ctypes.data_as(self.ct.c_void_p)  # noqa: E731
        rc = self.lib.gnpde_oracle_csr(p(ei), B, E, int(num_nodes), p(wf), p(rowptr), p(col), p(wc))
        if rc != 0:
            raise ValueError("gnpde_oracle_csr failed (%d)" % rc)
        return rowptr, col, wc

    def laplacian_rhs(self, csr, x, alpha_train, x0=None, beta_train=0.0, no_alpha_sigmoid=False, add_source=False,
                      nthreads=0):
        rowptr, col, wc = csr
        x = np.ascontiguousarray(x, dtype=np.float32)
        C = x.shape[-1]
        R = x.size // C
        f = np.empty_like(x)
        x0a = np.ascontiguousarray(x0, dtype=np.float32) if add_source else x
        p = lambda a: a.ctypes.data_as(self.ct.c_void_p)  # noqa: E731
        self.lib.gnpde_oracle_laplacian_rhs(p(rowptr), p(col), p(wc), R, C, p(x), p(x0a), float(alpha_train),
                                            float(beta_train), int(no_alpha_sigmoid), int(add_source), p(f),
                                            int(nthreads))
        return f
