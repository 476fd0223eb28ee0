"""Bundled ODE integrator with torchdiffeq's calling convention.

The reference integrates with ``torchdiffeq.odeint`` (src/block_constant.py:46-51,
src/block_transformer_attention.py:40-52); torchdiffeq (README.md:29 pins 0.2.1,
requirements.txt:20 0.1.1) is not installed in this image, so the solver loop
is restated here from its published algorithm (torchdiffeq 0.2.x):

* fixed grid (``euler``, ``midpoint``, ``rk4``): ``FixedGridODESolver`` with
  ``_grid_constructor_from_step_size`` (niters = ceil((t1-t0)/h + 1), the last
  grid point snapped to t1) and linear interpolation onto the requested times;
  rk4 is ``rk4_alt_step_func`` (the 3/8 rule);
* ``dopri5``, ``bosh3``, ``fehlberg2``, ``adaptive_heun``:
  ``RKAdaptiveStepsizeODESolver`` with the solver's embedded tableau,
  ``_select_initial_step``, the RMS error norm, the safety 0.9 / ifactor 10 /
  dfactor 0.2 controller and 4th-order dense output (``_interp_fit`` with the
  solver's mid-point coefficients) at the requested times.  adaptive_heun is the
  reference's default ``adjoint_method`` (src/run_GNN.py:334).

Stage combinations ``y0 + dt * sum_j b_j k_j`` are single fused HIP passes
(gnpde_rk_combine_f32).  The RHS calls are whatever ``func`` is (the gnpde
ODEFuncs run entirely in HIP).  Parity of integrated values is UNPINNED: the
reference's tests only check shapes.
"""
import itertools
import math
import os
import weakref

import numpy as np
import torch

from . import _lib, ops
from ._cache import _tensor_key
from .utils import MaxNFEException

# Dormand-Prince-Shampine (torchdiffeq dopri5.py)
_DP_ALPHA = [1 / 5, 3 / 10, 4 / 5, 8 / 9, 1., 1.]
_DP_BETA = [
    [1 / 5],
    [3 / 40, 9 / 40],
    [44 / 45, -56 / 15, 32 / 9],
    [19372 / 6561, -25360 / 2187, 64448 / 6561, -212 / 729],
    [9017 / 3168, -355 / 33, 46732 / 5247, 49 / 176, -5103 / 18656],
    [35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84],
]
_DP_C_SOL = [35 / 384, 0, 500 / 1113, 125 / 192, -2187 / 6784, 11 / 84, 0]
_DP_C_ERROR = [
    35 / 384 - 1951 / 21600,
    0,
    500 / 1113 - 22642 / 50085,
    125 / 192 - 451 / 720,
    -2187 / 6784 - -12231 / 42400,
    11 / 84 - 649 / 6300,
    -1. / 60.,
]
_DP_C_MID = [
    6025192743 / 30085553152 / 2, 0, 51252292925 / 65400821598 / 2, -2691868925 / 45128329728 / 2,
    187940372067 / 1594534317056 / 2, -1776094331 / 19743644256 / 2, 11237099 / 235043384 / 2,
]

# Bogacki-Shampine 3(2) (torchdiffeq bosh3.py)
_BS_ALPHA = [1 / 2, 3 / 4, 1.]
_BS_BETA = [[1 / 2], [0., 3 / 4], [2 / 9, 1 / 3, 4 / 9]]
_BS_C_SOL = [2 / 9, 1 / 3, 4 / 9, 0.]
_BS_C_ERROR = [2 / 9 - 7 / 24, 1 / 3 - 1 / 4, 4 / 9 - 1 / 3, -1 / 8]
_BS_C_MID = [0., 0.5, 0., 0.]

# Heun-Euler 2(1) (torchdiffeq adaptive_heun.py; the reference's default adjoint_method,
# src/run_GNN.py:334, src/best_params.py)
_AH_ALPHA = [1.]
_AH_BETA = [[1.]]
_AH_C_SOL = [0.5, 0.5]
_AH_C_ERROR = [0.5, -0.5]
_AH_C_MID = [0.5, 0.]

# Runge-Kutta-Fehlberg 2(1) (torchdiffeq fehlberg2.py)
_FE_ALPHA = [1 / 2, 1.]
_FE_BETA = [[1 / 2], [1 / 256, 255 / 256]]
_FE_C_SOL = [1 / 512, 255 / 256, 1 / 512]
_FE_C_ERROR = [-1 / 512, 0., 1 / 512]
_FE_C_MID = [0., 0.5, 0.]

# name -> (order, alpha, beta, c_sol, c_error, c_mid)
_TABLEAUS = {
    'dopri5': (5, _DP_ALPHA, _DP_BETA, _DP_C_SOL, _DP_C_ERROR, _DP_C_MID),
    'bosh3': (3, _BS_ALPHA, _BS_BETA, _BS_C_SOL, _BS_C_ERROR, _BS_C_MID),
    'fehlberg2': (2, _FE_ALPHA, _FE_BETA, _FE_C_SOL, _FE_C_ERROR, _FE_C_MID),
    'adaptive_heun': (2, _AH_ALPHA, _AH_BETA, _AH_C_SOL, _AH_C_ERROR, _AH_C_MID),
}

FIXED_METHODS = ('euler', 'midpoint', 'rk4')
ADAPTIVE_METHODS = ('dopri5', 'bosh3', 'fehlberg2', 'adaptive_heun')


class _CombineFn(torch.autograd.Function):
    """The fused HIP stage combination under autograd: forward one streaming pass
    (gnpde_rk_combine_f32) instead of a clone plus a multiply and an add per
    term; backward d/dy0 = g, d/dk_j = scale * c_j * g."""

    @staticmethod
    def forward(ctx, y0, scale, coefs, *ks):
        ctx.scale, ctx.coefs, ctx.has_y0 = scale, coefs, y0 is not None
        return ops.rk_combine(y0, list(ks), list(coefs), scale).view(ks[0].shape)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        gk = [g * float(ctx.scale * c) for c in ctx.coefs]
        return (g if ctx.has_y0 else None, None, None) + tuple(gk)


class _Combine(object):
    """y0 + scale * sum_j c_j k_j on the device (fused HIP pass).  When autograd
    has to see the combination (grad enabled and an operand requires grad) it
    runs through _CombineFn so gradients flow through the solver (torch ops for
    CPU tensors: the host-logic tests' injected RHS)."""

    def __call__(self, y0, ks, coefs, scale):
        if torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in [y0] + list(ks)):
            if ks[0].is_cuda and ks[0].dtype == torch.float32:
                return _CombineFn.apply(y0, float(scale), tuple(float(c) for c in coefs), *ks)
            return _torch_combine(y0, ks, coefs, scale)
        if ks[0].dtype == torch.bfloat16:
            # bf16 state outside the fused paths: the stage pass (gnpde_stage_apply_bf16: fp32
            # arithmetic, one rounding to bf16 per output) — VERDICT r3 weak 7
            nz = [(k, c) for k, c in zip(ks, coefs) if c != 0]  # the tableaus' zero entries (dopri5 b2)
            ops_ok = ks[0].is_cuda and 0 < len(nz) <= _lib.STAGE_MAX_K and all(
                k.is_contiguous() and k.shape == ks[0].shape for k in ks) and (
                y0 is None or (y0.is_contiguous() and y0.shape == ks[0].shape and y0.dtype == ks[0].dtype))
            if ops_ok:
                out = torch.empty_like(ks[0])
                ops.stage_apply(ops.Stage(outs=[(out, y0, 1.0, 0.0, [(k, float(scale * c)) for k, c in nz])]),
                                None, None, out)
                return out
            acc = _torch_combine(None if y0 is None else y0.float(), [k.float() for k in ks], coefs, scale)
            return acc.to(torch.bfloat16)
        return ops.rk_combine(y0, ks, coefs, scale).view(ks[0].shape)


def _torch_combine(y0, ks, coefs, scale):
    """Host-logic testing aid only (tests inject it for CPU oracle funcs)."""
    acc = torch.zeros_like(ks[0]) if y0 is None else y0.clone()
    for k, c in zip(ks, coefs):
        acc = acc + (scale * c) * k
    return acc


def _rms_norm(t):
    return t.abs().pow(2).mean().sqrt()


def fixed_grid(t, step_size):
    """torchdiffeq ``_grid_constructor_from_step_size`` (dtype of t)."""
    start_time, end_time = t[0], t[-1]
    niters = torch.ceil((end_time - start_time) / step_size + 1).item()
    t_infer = torch.arange(0, niters, dtype=t.dtype, device=t.device) * step_size + start_time
    t_infer[-1] = t[-1]
    return t_infer


def _linear_interp(t0, t1, y0, y1, t):
    if t == t0:
        return y0
    if t == t1:
        return y1
    slope = (t - t0) / (t1 - t0)
    return y0 + slope * (y1 - y0)


def _fixed_step(method, func, t0, dt, t1, y0, combine):
    """Returns y1 = y0 + dy (one grid step)."""
    if method == 'euler':
        f0 = func(t0, y0)
        return combine(y0, [f0], [1.0], dt)
    if method == 'midpoint':
        f0 = func(t0, y0)
        y_mid = combine(y0, [f0], [0.5], dt)
        f_mid = func(t0 + 0.5 * dt, y_mid)
        return combine(y0, [f_mid], [1.0], dt)
    if method == 'rk4':  # rk4_alt_step_func (3/8 rule)
        k1 = func(t0, y0)
        k2 = func(t0 + dt / 3.0, combine(y0, [k1], [1.0 / 3.0], dt))
        k3 = func(t0 + dt * 2.0 / 3.0, combine(y0, [k1, k2], [-1.0 / 3.0, 1.0], dt))
        k4 = func(t1, combine(y0, [k1, k2, k3], [1.0, -1.0, 1.0], dt))
        return combine(y0, [k1, k2, k3, k4], [0.125, 0.375, 0.375, 0.125], dt)
    raise ValueError(method)


def _fusable(func, y0, combine):
    """The RHS can emit the stage combinations itself (gnpde ODEFuncs, no autograd).
    A host-side RHS object with ``host_stages`` (tests/dist_workers.py: the gloo
    tests of gnpde.dist) takes the same path on CPU tensors."""
    if not (isinstance(combine, _Combine) and hasattr(func, 'rhs_stage')) or torch.is_grad_enabled():
        return False
    return y0.dtype in ops.STATE_DTYPES if y0.is_cuda else bool(getattr(func, 'host_stages', False))


RHS_PER_STEP = {'euler': 1, 'midpoint': 2, 'rk4': 4}


def _fused_step(method, func, t0, dt, t1, y0, ws, out=None, out_rows=None):
    """One grid step with the stage combinations fused into the RHS epilogues
    (gnpde_stage_epilogue_t): same arithmetic as _fixed_step, ~7 fewer passes
    over the state per rk4 step and no separate combine launches.  ``out``:
    the buffer that receives y1 (default: a new tensor); ``out_rows`` (int32
    [R]): y1's row r is stored at row out_rows[r] of ``out`` (the last step of
    a solve run in a node renumbering writes the caller's numbering)."""
    y0 = y0.contiguous()
    if method == 'euler':
        y1 = torch.empty_like(y0) if out is None else out
        func.rhs_stage(t0, y0, ops.Stage(outs=[(y1, y0, 1.0, dt, [])], out_rows=out_rows))
        return y1
    if method == 'midpoint':
        ym = ws.get('a', y0)
        y1 = torch.empty_like(y0) if out is None else out
        func.rhs_stage(t0, y0, ops.Stage(outs=[(ym, y0, 1.0, 0.5 * dt, [])]))
        func.rhs_stage(t0 + 0.5 * dt, ym, ops.Stage(outs=[(y1, y0, 1.0, dt, [])], out_rows=out_rows))
        return y1
    if method == 'rk4':
        # rk4_alt_step_func (3/8 rule).  With x2 = y + dt k1/3 the stage inputs
        # and the result are affine in rows the epilogue already holds (its own
        # input row comes for free), so no k_i is ever stored:
        #   x3 = y + dt (k2 - k1/3)      = 2 y  - x2 + dt k2
        #   x4 = y + dt (k1 - k2 + k3)   = 2 x2 - x3 + dt k3
        #   y1 = y + dt/8 (k1 + 3k2 + 3k3 + k4) = (6 x3 + 3 x4 - y + dt k4) / 8
        # 8 state passes per step besides the gathers (one write per stage,
        # reads of y, x2, y + x3), where storing k's and an accumulator takes 15.
        x2, x3, x4 = ws.get('a', y0), ws.get('b', y0), ws.get('c', y0)
        y1 = torch.empty_like(y0) if out is None else out
        func.rhs_stage(t0, y0, ops.Stage(outs=[(x2, y0, 1.0, dt / 3.0, [])]))
        func.rhs_stage(t0 + dt / 3.0, x2, ops.Stage(outs=[(x3, x2, -1.0, dt, [(y0, 2.0)])]))
        func.rhs_stage(t0 + dt * 2.0 / 3.0, x3, ops.Stage(outs=[(x4, x3, -1.0, dt, [(x2, 2.0)])]))
        func.rhs_stage(t1, x4, ops.Stage(outs=[(y1, x4, 0.375, dt * 0.125, [(x3, 0.75), (y0, -0.125)])],
                                         out_rows=out_rows))
        return y1
    raise ValueError(method)


class _Workspace(dict):
    """Stage-input buffers of the fused steps.  A RHS object may place the state
    itself (``alloc_state(like)``: dist.RowShardedLaplacian hands out row blocks of
    its gathered buffers, so the all-gather before each RHS is in place)."""

    def __init__(self, alloc=None):
        dict.__init__(self)
        self.alloc = alloc

    def get(self, name, like):
        t = dict.get(self, name)
        if t is None or t.shape != like.shape or t.device != like.device:
            t = _new_state(like, self.alloc)
            self[name] = t
        return t


def _new_state(like, alloc=None):
    return alloc(like) if alloc is not None else torch.empty_like(like, memory_format=torch.contiguous_format)


# Graph replay of fixed-grid steps (hipGraph through torch.cuda.CUDAGraph): a run
# of k equal steps is replayed as the binary decomposition of k into captured
# blocks of 2^i steps (at most GRAPH_BLOCK each), so a solve costs a handful of
# graph launches whatever its length (each launch leaves the GPU idle ~18 us
# between replays: profiles/r03a trace).  Capture itself costs host time, so a
# solve shorter than GRAPH_MIN_STEPS runs eagerly.
GRAPH_MIN_STEPS = 6
# Largest block graph, in steps (a power of two; GNPDE_GRAPH_BLOCK overrides).
GRAPH_BLOCK = int(os.environ.get('GNPDE_GRAPH_BLOCK', '64'))
# Set to a list to receive (start_event, end_event, n_rhs) per graph replay
# (bench.py's per-launch roofline timing); None in normal use.
replay_events = None


def _pow2_blocks(k, cap):
    """k as a sum of powers of two <= cap, largest first (odd sizes last)."""
    out = []
    b = 1
    while b * 2 <= max(cap, 1):
        b *= 2
    while k > 0:
        while b > k:
            b //= 2
        out.append(b)
        k -= b
    return out


class _StatePool(object):
    """The two ping-pong state buffers and the stage-input workspace of a
    module's fused fixed-grid solves of one state shape (kept across calls, so
    the captured graphs that read them stay valid and a solve needs no
    allocation)."""

    def __init__(self, like, alloc=None):
        self.bufs = [_new_state(like, alloc) for _ in range(2)]
        self.ws = _Workspace(alloc)


_POOLS = weakref.WeakKeyDictionary()  # module -> {(shape, dtype, device): _StatePool}


def _state_pool(func, y):
    # keyed by stream too: two concurrent solves of one module on two streams
    # must not share ping-pong buffers or stage workspaces
    sid = torch.cuda.current_stream(y.device).cuda_stream if y.is_cuda else None
    key = (tuple(y.shape), y.dtype, str(y.device), sid)
    d = _POOLS.get(func)
    if d is None:
        d = {}
        _POOLS[func] = d
    pool = d.get(key)
    if pool is None:
        if len(d) >= 4:
            d.clear()
        pool = _StatePool(y, getattr(func, 'alloc_state', None))
        d[key] = pool
    return pool


class _StepGraphs(object):
    """Captured blocks of fixed-dt grid steps over a _StatePool: graph (s, p)
    runs s steps starting from bufs[p] (ping-ponging, so it ends in bufs[p ^ (s & 1)]);
    captured on first use.  The launches are those of the eager fused step (same
    kernels, same arguments, same bits).  ``warm`` is False until one eager step
    of this entry has run: every per-graph structure (CSR, plans, cached weights,
    scratch) is built by an eager call before anything is captured, so nothing
    synchronises inside a capture."""

    def __init__(self, method, func, dt, pool):
        self.method, self.dt, self.pool = method, dt, pool
        self.n_rhs = RHS_PER_STEP[method]
        self.graphs = {}
        self.mempool = None
        self.warm = False

    def graph(self, func, s, p):
        g = self.graphs.get((s, p))
        if g is None:
            nfe = getattr(func, 'nfe', None)
            bufs, ws = self.pool.bufs, self.pool.ws
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.mempool):
                for k in range(s):
                    i = p ^ (k & 1)
                    _fused_step(self.method, func, 0.0, self.dt, self.dt, bufs[i], ws, out=bufs[1 - i])
            if self.mempool is None:
                self.mempool = g.pool()
            if nfe is not None:
                func.nfe = nfe  # capture records launches, it evaluates nothing
            self.graphs[(s, p)] = g
        return g

    def replay(self, func, s, p):
        """Replay s steps from bufs[p]; counts the RHS evaluations like the eager
        calls; returns the parity the state ends in."""
        g = self.graph(func, s, p)
        if hasattr(func, 'nfe'):
            func.nfe += s * self.n_rhs
        if replay_events is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            g.replay()
            ev1.record()
            replay_events.append((ev0, ev1, s * self.n_rhs))
        else:
            g.replay()
        return p ^ (s & 1)


# Captured step graphs kept per RHS module between odeint calls (one entry per
# module, replaced when its key changes), so repeated solves — every forward
# of a GRAND model in eval — replay without re-capturing.  A weak key: the
# entry goes with the module.
_GRAPH_CACHE = weakref.WeakKeyDictionary()


def _capture_state(func, y):
    """The derived device objects a captured step reads (device CSR and plans,
    CSR-order weights, the stable x0 buffer, cached projection weights ...),
    refreshed in place from the module's current tensors by
    ``func.graph_capture_state(y)``; None when the module offers no such hook
    (its graphs are then captured per call and never cached)."""
    fn = getattr(func, 'graph_capture_state', None)
    return None if fn is None else tuple(fn(y))


def _graph_cache_key(func, method, y, state):
    """Everything a captured step reads besides its own buffers: the module's
    parameters and buffers (identity + version: in-place updates recapture,
    host-read scalars such as exp_kernel's lengthscale are baked into the
    launches), its options, the state's shape and layout, and the IDENTITY of
    every derived object in ``state``.  The cache entry holds ``state``
    itself, so the buffers a replay reads stay alive however the module
    rebuilds its own caches (a solve on another graph replaces func._graph;
    the replayed step then finds a different object and recaptures instead of
    reading freed memory).  Source tensors (edge_index, edge_weight,
    attention_weights, x0) are NOT in the key: what the launches read is the
    derived buffers, refreshed in place when only the values change."""
    if state is None:
        return None
    if hasattr(func, 'parameters'):
        tens = [_tensor_key(t) for t in itertools.chain(func.parameters(), func.buffers())]
    else:  # a plain RHS object (gnpde.dist shards): the scalars it reads by pointer
        tens = [_tensor_key(t) for t in getattr(func, 'capture_key_tensors', lambda: ())()]
    opt = getattr(func, 'opt', None)
    okey = _opt_key(opt) if isinstance(opt, dict) else None
    return (method, tuple(y.shape), tuple(y.stride()), y.dtype, str(y.device), okey, tuple(tens),
            tuple(id(o) for o in state))


_OPT_KEYS = {}  # id(opt dict) -> (its items when keyed, key string)


def _opt_key(opt):
    """The options part of a graph cache key: the sorted repr of the dict, recomputed only
    when its items changed (an in-place edit of the module's opt changes them)."""
    items = tuple(opt.items())
    hit = _OPT_KEYS.get(id(opt))
    try:
        if hit is not None and hit[0] == items:
            return hit[1]
    except (TypeError, ValueError):  # values without a plain equality (arrays): no cache
        return repr(sorted(opt.items(), key=lambda kv: str(kv[0])))
    key = repr(sorted(opt.items(), key=lambda kv: str(kv[0])))
    if len(_OPT_KEYS) > 256:
        _OPT_KEYS.clear()
    _OPT_KEYS[id(opt)] = (items, key)
    return key


def _replayable(func):
    """Steps of ``func`` may be captured and replayed as hipGraphs: no collective per RHS
    (graph_capturable) and f(t, x) independent of t (autonomous) — a replay passes the
    stage times recorded at capture."""
    return getattr(func, 'graph_capturable', True) and getattr(func, 'autonomous', False)


def _nfe_headroom(func, n):
    """True when n more RHS calls cannot trip the MaxNFEException guard (the
    eager path raises at the exact call, as the reference does)."""
    opt = getattr(func, 'opt', None)
    if not hasattr(func, 'nfe') or not isinstance(opt, dict) or 'max_nfe' not in opt:
        return True
    return func.nfe + n - 1 <= opt['max_nfe']


# Experiment knob: byte multiple bf16 rows are padded to (default 16).  Whole
# 128-byte lines for BLEND's bf16 rows (162 -> 192 columns instead of 168) measured
# 0.391 against 0.315 ms per rk4 step: the wider row leaves the three-rows-per-
# wavefront geometry (tools/pad_ab.sh).
PAD_ALIGN_BF16 = int(os.environ.get('GNPDE_PAD_ALIGN_BF16', '16'))


def _padded_width(func, y0):
    """Feature width the fused path pads the state to, or None.  Rows whose byte
    length is not a multiple of 16 (C = 162 in fp32 or bf16, BLEND) cannot take
    16-byte vector gathers; a RHS whose arithmetic is column-independent
    (func.supports_feature_padding) integrates a zero-padded copy instead — the
    padding columns stay exactly 0 (A 0 - 0 = 0) — and the result is cut back."""
    per16 = 16 // y0.element_size()
    C = y0.shape[-1]
    if C % per16 == 0 or y0.dim() != 3:
        return None
    ok = getattr(func, 'supports_feature_padding', None)
    if ok is None or not ok():
        return None
    align = max(16, PAD_ALIGN_BF16 if y0.element_size() == 2 else 16) // y0.element_size()
    return (C + align - 1) // align * align


# --------------------------------------------------------------------------- training path
# Fixed-grid solves of the (linear) Laplacian RHS under autograd: the discrete
# adjoint of the whole solve as ONE autograd node.  GNPDE_FUSED_BACKWARD=0 falls
# back to autograd through every RHS and stage combination.
FUSED_BACKWARD = os.environ.get('GNPDE_FUSED_BACKWARD', '1') != '0'


def _fused_backward_ok(func, y0, combine, grid_h, t_h):
    if not (FUSED_BACKWARD and torch.is_grad_enabled() and isinstance(combine, _Combine) and y0.is_cuda and
            y0.dtype == torch.float32 and y0.dim() == 3):
        return False
    fn = getattr(func, 'fixed_grid_backward_ok', None)
    if fn is None or not fn():
        return False
    params = [y0, func.alpha_train, func.beta_train]
    if not any(p.requires_grad for p in params):
        return False
    gs = set(grid_h)
    return all(v in gs for v in t_h)  # every output time is a grid point (no interpolation)


class _LaplacianFixedGridFn(torch.autograd.Function):
    """The discrete adjoint of a fixed-grid solve (euler, midpoint, rk4 3/8) of
    f(x) = a (A x - x) [+ b x0], a = sigma(alpha_train) (or alpha_train),
    b = beta_train: exactly the gradient of the stepped computation, like
    backprop through every RHS call, but formed with the fused kernels.

    Forward: the fused steps (stage combinations in the K1 epilogues), the state
    at every step start and the stage inputs kept (3 states per rk4 step).
    Backward, step by step from the last, for rk4
        gk4 = dt/8 g              u4 = (A^T - I) gk4
        gk3 = 3dt/8 g + dt a u4   u3 = (A^T - I) gk3
        gk2 = 3dt/8 g - dt a u4 + dt a u3                       ...
        gk1 = dt/8 g + dt a u4 - dt/3 a u3 + dt/3 a u2
        g  <- g + a (u4 + u3 + u2 + u1)
    (formed as gk2 = gk3 + dt a u3 - 2 dt a u4, gk1 = gk2/3 + dt a (u2 + 4 u4 - 2 u3)/3
    and a running sum that carries g, so that each launch reads as few rows as it can)
        d alpha += a'(alpha) sum_i <u_i, x_i>,  d beta += sum_i <gk_i, x0>
    (K1 over the CSC for (A^T - I), each gk line and the running sum formed in
    the epilogue of the launch before it (gnpde_stage_epilogue_t), and the
    d alpha terms <u_i, x_i> added per row in fp64 by the same epilogues
    (dot_rows), summed once at the end): four transpose launches per rk4 step
    instead of autograd's ~40 elementwise kernels and a second K1 per RHS for
    d alpha."""

    @staticmethod
    def forward(ctx, y0, alpha_train, beta_train, func, method, steps, t_h):
        # everything the backward reads is taken NOW: a second forward with
        # another graph, x0 or alpha before this backward must not change its gradient.
        # The solve and its adjoint run in the graph's in-degree numbering when the module
        # offers one (as the no-grad solves, ops.NodeLayout); the solution and the input
        # gradient are in the caller's numbering.
        lay = _node_layout(func, y0)
        y0d = y0.detach().contiguous()
        sol = torch.empty((len(t_h),) + tuple(y0.shape), dtype=y0.dtype, device=y0.device)
        if lay is not None:  # sol[0] = y0 and the solve's copy in one pass
            y = torch.empty_like(y0d)
            _entry_copy(y0d, y, sol[0], lay.order)
            func._layout = lay
        else:
            sol[0].copy_(y0d)
            y = y0d
        sig = not func.opt.get('no_alpha_sigmoid', False)
        try:
            gr = func.graph_for(y0)
            starts, stage_inputs = [], []
            j = 1
            for n_step, (ta, tb) in enumerate(steps):
                starts.append(y)
                ws = _Workspace()  # a fresh one per step: its stage inputs are kept for the backward
                if n_step == len(steps) - 1 and j == len(t_h) - 1 and t_h[j] == tb:
                    # the last step writes the result in the caller's numbering (no exit pass;
                    # the backward never reads the last step's output)
                    _fused_step(method, func, ta, tb - ta, tb, y, ws, out=sol[j],
                                out_rows=lay.order32 if lay is not None else None)
                    stage_inputs.append([ws[k] for k in ('a', 'b', 'c') if k in ws])
                    j += 1
                    break
                y = _fused_step(method, func, ta, tb - ta, tb, y, ws)
                stage_inputs.append([ws[k] for k in ('a', 'b', 'c') if k in ws])
                while j < len(t_h) and tb >= t_h[j]:
                    _to_user(y, sol[j], lay)
                    j += 1
            # The backward's own copies, taken after the forward launches are queued (the GPU
            # starts on the solve while the host does this; still before this call returns):
            # alpha (rk4's adjoint scales its a-dependent coefficients by a on the device, the
            # stage epilogue's coef_scale; the other methods' combinations need a on the host,
            # copied behind an event so the backward does not drain the queue to read it), and a
            # private CSC-order copy of the weights (grad mode is off inside a
            # Function's forward, so the module's cached buffer counts as no_grad-made and a
            # later no_grad call with new weights would refresh it in place under this node's
            # pending backward).
            ctx.alpha = func.alpha_train.detach().clone()
            ctx.a_dev = torch.sigmoid(ctx.alpha) if sig else ctx.alpha
            ctx.a_scale = ctx.a_dev.reshape(()).float().contiguous()
            ctx.a_host = _host_scalar(ctx.a_dev) if method != 'rk4' else None
            w, tag = func._weights_tensor()
            src = w.detach().float() if w.dtype != torch.float32 else w.detach()
            ctx.w_csc = gr.gather_weights(src, transpose=True)
            ctx.gr = gr
            ctx.sig = sig
            ctx.add_source = bool(func.opt.get('add_source', False))
            ctx.x0 = func.stable_x0(y0).clone() if ctx.add_source else None
        finally:
            func._layout = None
        ctx.func, ctx.method, ctx.steps, ctx.t_h, ctx.lay = func, method, steps, t_h, lay
        ctx.starts, ctx.stage_inputs = starts, stage_inputs
        return sol

    @staticmethod
    def backward(ctx, g_sol):
        func, method, steps, t_h = ctx.func, ctx.method, ctx.steps, ctx.t_h
        g_sol = g_sol.contiguous()
        lay = ctx.lay
        with torch.no_grad():
            gr, w_csc = ctx.gr, ctx.w_csc
            one = _device_one(g_sol.device)
            sig = ctx.sig
            a_dev = ctx.a_dev
            a = ctx.a_host() if ctx.a_host is not None else None  # euler / midpoint combinations
            asc = ctx.a_scale  # rk4: coef_scale of every adjoint launch (cb unscaled, cf and c_j times a)
            add_source = ctx.add_source
            x0 = ctx.x0

            def u_of(v):  # (A^T - I) v
                return ops.spmm_rhs(gr, w_csc, v, alpha=one, rhs=True, alpha_sigmoid=False, transpose=True)

            comb = ops.rk_combine
            # the output-time gradients join the running gradient at their grid points
            out_at = {}
            j = 1
            for n, (ta, tb) in enumerate(steps):
                while j < len(t_h) and tb >= t_h[j]:
                    out_at.setdefault(n, []).append(j)
                    j += 1
            s0 = ctx.starts[0]
            g = None  # the running gradient (None: still zero)
            nfe = getattr(func, 'nfe', None)
            # d alpha, d beta and (rk4) the alpha gradient's per-row terms <u_i, x_i>, which
            # accumulate in the transpose launches' epilogues (gnpde_stage_epilogue_t dot_rows)
            # and are summed once at the end: one zero-filled fp64 buffer for the three
            n_drow = s0.numel() // s0.shape[-1] if method == 'rk4' else 0
            acc64 = torch.zeros(2 + n_drow, dtype=torch.float64, device=s0.device)
            ga, gb = acc64[0], acc64[1]
            drow = acc64[2:] if method == 'rk4' else None
            # rk4 in a renumbered solve: the first step's last launch stores the input gradient
            # straight into the caller's numbering (its out_rows), as the forward's last step
            # stores the solution — no exit pass
            user_rows = lay.order32 if (lay is not None and method == 'rk4' and not out_at.get(-1)) else None
            def g_at(jj):  # an output time's gradient in the solve's numbering (one gnpde_rows_copy pass)
                if lay is None:
                    return g_sol[jj]
                return _to_internal(g_sol[jj], lay)

            for n in range(len(steps) - 1, -1, -1):
                for jj in out_at.get(n, []):
                    g = g_at(jj) if g is None else g + g_at(jj)
                if g is None:
                    g = torch.zeros_like(s0)
                ta, tb = steps[n]
                dt = tb - ta
                y = ctx.starts[n]
                if method == 'rk4':
                    # the adjoint stage combinations ride in the transpose launches' epilogues
                    # (v = (A^T - I) g, so u4 = dt/8 v by linearity)
                    x2, x3, x4 = ctx.stage_inputs[n]
                    e = lambda: torch.empty_like(g)  # noqa: E731
                    v, gk3, u3, gk2, gk1, acc, g_new = (e() for _ in range(7))
                    c8 = dt / 8.0
                    T = dict(alpha=one, rhs=True, alpha_sigmoid=False, transpose=True)
                    # d alpha += a'(alpha) (dt/8 <v, x4> + <u3, x3> + <u2, x2> + <u1, y>): the epilogue of
                    # each launch adds its row terms; u2 and u1 are used only inside their own launch
                    # Each gk line is written against the launch's own input where it can (that row is
                    # in registers already): gk2 = gk3 + ad u3 - 2 ad c8 v, gk1 = gk2/3 + ad/3 u2 +
                    # 4/3 ad c8 v - 2/3 ad u3, and the running sum carries g (acc = g + a(c8 v + u3 + u2)),
                    # so g is read by the third launch only: 20 state passes per step, not 23
                    # (coefficients written without a: the epilogue multiplies cf and every c_j by *asc)
                    ops.spmm_rhs(gr, w_csc, g, stage=ops.Stage(f_out=v, outs=[(gk3, g, 3 * c8, dt * c8, [])],
                                                               dot=(x4, drow, c8, True), scale=asc), **T)
                    ops.spmm_rhs(gr, w_csc, gk3, stage=ops.Stage(f_out=u3, outs=[(gk2, gk3, 1.0, dt,
                                                                                  [(v, -2.0 * dt * c8)])],
                                                                 dot=(x3, drow, 1.0, True), scale=asc), **T)
                    ops.spmm_rhs(gr, w_csc, gk2, stage=ops.Stage(outs=[
                        (gk1, gk2, 1.0 / 3.0, dt / 3.0, [(v, 4.0 * dt * c8 / 3.0), (u3, -2.0 * dt / 3.0)]),
                        (acc, g, 1.0, 1.0, [(v, c8), (u3, 1.0)])], dot=(x2, drow, 1.0, True), scale=asc), **T)
                    last = n == 0 and user_rows is not None
                    ops.spmm_rhs(gr, w_csc, gk1, stage=ops.Stage(outs=[(g_new, acc, 1.0, 1.0, [])],
                                                                 out_rows=user_rows if last else None,
                                                                 dot=(y, drow, 1.0, True), scale=asc), **T)
                    if add_source:
                        gb = gb + c8 * ops.dot(g, x0) + ops.dot(gk3, x0) + ops.dot(gk2, x0) + ops.dot(gk1, x0)
                    g = g_new
                    if last:
                        lay = None  # g is in the caller's numbering now
                    continue
                if method == 'euler':
                    gk = [comb(None, [g], [dt], 1.0)]
                    xs = [y]
                    us = [u_of(gk[0])]
                else:  # midpoint
                    ym = ctx.stage_inputs[n][0]
                    gk2 = comb(None, [g], [dt], 1.0)
                    u2 = u_of(gk2)
                    gk1 = comb(None, [u2], [0.5 * dt * a], 1.0)
                    u1 = u_of(gk1)
                    gk, xs, us = [gk2, gk1], [ym, y], [u2, u1]
                for u, xv in zip(us, xs):
                    ga = ga + ops.dot(u, xv)
                if add_source:
                    for gkv in gk:
                        gb = gb + ops.dot(gkv, x0)
                g = comb(g, us, [a] * len(us), 1.0).view(g.shape)
            if nfe is not None:
                func.nfe = nfe  # the recomputed stages are not new RHS evaluations
            if drow is not None:
                ga = ops.sum_f64(drow, out=ga, accumulate=True)
            if g is None:
                g = torch.zeros_like(s0)
            for jj in out_at.get(-1, []):
                g = g + g_at(jj)
            if lay is not None:
                gu = torch.empty_like(g)
                _to_user(g, gu, lay)
                g = gu
            g = g + g_sol[0] if g._base is g_sol else g.add_(g_sol[0])  # (never g_sol itself in place)
            if sig:
                ga = ga * (a_dev * (1 - a_dev)).double()
        gy = g if ctx.needs_input_grad[0] else None
        galpha = ga.to(func.alpha_train.dtype).reshape(func.alpha_train.shape) if ctx.needs_input_grad[1] else None
        # without add_source beta_train is not on the path: no gradient, as autograd through
        # the reference's RHS leaves it (src/function_laplacian_diffusion.py:74-77)
        gbeta = gb.to(func.beta_train.dtype).reshape(func.beta_train.shape) \
            if ctx.needs_input_grad[2] and add_source else None
        return gy, galpha, gbeta, None, None, None, None


def _host_scalar(v):
    """A device scalar's value for the host later: an asynchronous copy into pinned
    memory behind an event; the returned callable waits for that event only (not
    for the work queued after it) and returns the float."""
    if not v.is_cuda:
        val = float(v)
        return lambda: val
    h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
    h.copy_(v, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()

    def get():
        ev.synchronize()
        return float(h)
    return get


_ONES = {}


def _device_one(device):
    """A read-only fp32 1.0 on `device` (the adjoint launches' alpha operand), made once
    per device rather than filled per backward."""
    one = _ONES.get(device)
    if one is None:
        one = torch.ones((), dtype=torch.float32, device=device)
        if not torch.cuda.is_current_stream_capturing():  # a captured fill runs only on replay
            _ONES[device] = one
    return one


def _node_layout(func, y0):
    """The locality numbering (ops.NodeLayout) the fused path keeps the state in, or None."""
    fn = getattr(func, 'node_layout', None)
    return fn(y0) if fn is not None else None


# Host copies of time grids.  A solve needs t on the host (the loop is there); a
# device t costs a device->host copy, i.e. a wait for everything queued before it.
# The values of a device t are kept per tensor object (and version), so a model
# that integrates over the same ``self.t`` every forward (ODEblock) reads it once.
_T_HOST = {}
_GRIDS = {}


def _host_times(t):
    if not t.is_cuda:
        return [float(v) for v in t.tolist()]
    hit = _T_HOST.get(id(t))
    if hit is not None and hit[0]() is t and hit[1] == t._version and hit[2] == t.data_ptr():
        return hit[3]
    vals = [float(v) for v in t.tolist()]
    if len(_T_HOST) >= 64:
        _T_HOST.clear()
    _T_HOST[id(t)] = (weakref.ref(t), t._version, t.data_ptr(), vals)
    return vals


def _host_grid(t_h, dtype, step_size):
    """torchdiffeq's grid for the host times t_h (built with CPU torch ops in t's
    dtype: IEEE on the host as on the device, the same values), cached."""
    if step_size is None:
        return list(t_h)
    key = (tuple(t_h), dtype, float(step_size))
    g = _GRIDS.get(key)
    if g is None:
        g = [float(v) for v in fixed_grid(torch.tensor(t_h, dtype=dtype), step_size).tolist()]
        if len(_GRIDS) >= 256:
            _GRIDS.clear()
        _GRIDS[key] = g
    return g


def odeint_fixed(func, y0, t, method, step_size=None, combine=None, graph=None):
    combine = combine or _Combine()
    t_h = _host_times(t)
    grid_h = _host_grid(t_h, t.dtype, step_size)
    if not (grid_h[0] == t_h[0] and grid_h[-1] == t_h[-1]):
        raise AssertionError("time grid does not cover t")
    steps = list(zip(grid_h[:-1], grid_h[1:]))
    if _fusable(func, y0, combine):
        cp = _padded_width(func, y0)
        if cp is not None:
            C = y0.shape[-1]
            yp = torch.zeros(*y0.shape[:-1], cp, dtype=y0.dtype, device=y0.device)
            yp[..., :C] = y0
            out = _solve_fused(func, yp, t_h, steps, method, graph)
            return out[..., :C].contiguous()
        return _solve_fused(func, y0, t_h, steps, method, graph)
    if _fused_backward_ok(func, y0, combine, grid_h, t_h) and _nfe_headroom(func, len(steps) * RHS_PER_STEP[method]):
        return _LaplacianFixedGridFn.apply(y0, func.alpha_train, func.beta_train, func, method, steps, t_h)
    solution = [y0]
    j = 1
    yc = y0
    for ta, tb in steps:
        y1 = _fixed_step(method, func, ta, tb - ta, tb, yc, combine)
        while j < len(t_h) and tb >= t_h[j]:
            solution.append(_linear_interp(ta, tb, yc, y1, t_h[j]))
            j += 1
        yc = y1
    while j < len(t_h):  # a degenerate grid (t0 == t1): the state itself
        solution.append(yc)
        j += 1
    return torch.stack(solution, 0)


def _entry_copy(y0, buf, sol0, order):
    """buf = y0 in the solve's numbering (order: internal row k holds user row
    order[k]), sol0 = y0: one pass (gnpde_rows_copy) when rows are 16-byte
    multiples, torch copies otherwise."""
    if y0.is_cuda and (y0.shape[-1] * y0.element_size()) % 16 == 0 and y0.is_contiguous():
        ops.rows_copy(y0, buf, order=order, dst_copy=sol0)
        return
    sol0.copy_(y0)
    if order is None:
        buf.copy_(y0)
    else:
        C = y0.shape[-1]
        torch.index_select(y0.reshape(-1, C), 0, order, out=buf.view(-1, C))


def _to_internal(src, lay):
    """src (caller's numbering) gathered into the solve's numbering: a fresh tensor."""
    if src.is_cuda and (src.shape[-1] * src.element_size()) % 16 == 0 and src.is_contiguous():
        dst = torch.empty_like(src)
        ops.rows_copy(src, dst, order=lay.order)
        return dst
    return lay.to_internal(src)


def _to_user(src, dst, lay):
    """dst = src in the caller's numbering (a fresh solution slice)."""
    if lay is None:
        dst.copy_(src)
    elif src.is_cuda and (src.shape[-1] * src.element_size()) % 16 == 0:
        ops.rows_copy(src, dst, order=lay.new_id)
    else:
        C = src.shape[-1]
        torch.index_select(src.reshape(-1, C), 0, lay.new_id, out=dst.view(-1, C))


def _solve_fused(func, y0, t_h, steps, method, graph):
    """A fixed-grid solve whose RHS emits the stage combinations itself (gnpde
    ODEFuncs, no autograd), in the graph's node numbering when the module offers
    one (ops.NodeLayout: bit-identical results).

    The solution tensor is allocated once; the entry pass writes its t0 slice
    and the working state (renumbered) in one read of y0; runs of equal steps
    replay captured block graphs over two ping-pong buffers; when the last
    requested time is the last grid point, the last step's epilogue writes the
    result straight into the solution in the caller's numbering (out_rows), so
    there is no exit pass.  Other output times are copied out (or linearly
    interpolated, as torchdiffeq) when their step has run."""
    lay = _node_layout(func, y0)
    n = len(steps)
    if graph is None:
        # a RHS with a collective inside (dist.RowShardedLaplacian) opts out of capture
        graph = n >= GRAPH_MIN_STEPS and _replayable(func)
    sol = torch.empty((len(t_h),) + tuple(y0.shape), dtype=y0.dtype, device=y0.device)
    pool = _state_pool(func, y0)
    bufs, ws = pool.bufs, pool.ws
    _entry_copy(y0.contiguous(), bufs[0], sol[0], lay.order if lay is not None else None)
    if lay is not None:
        func._layout = lay
    try:
        sg = None
        if graph and n >= 2:
            # the first step's dt; the captured graphs replay only runs of exactly this dt
            state = _capture_state(func, bufs[0])
            key = _graph_cache_key(func, method, bufs[0], state)
            dt0 = steps[0][1] - steps[0][0]
            hit = _GRAPH_CACHE.get(func) if key is not None else None
            if hit is not None and hit[0] == key and hit[1].dt == dt0 and hit[1].pool is pool:
                sg = hit[1]
            else:
                sg = _StepGraphs(method, func, dt0, pool)
                if key is not None:
                    _GRAPH_CACHE[func] = (key, sg, state)
        p = 0      # the state is in bufs[p]
        i = 0      # next step to run
        j = 1      # next output time
        while j < len(t_h):
            if i >= n:  # a degenerate grid (t0 == t1): the state itself
                _to_user(bufs[p], sol[j], lay)
                j += 1
                continue
            m = i
            while m < n - 1 and steps[m][1] < t_h[j]:
                m += 1
            p = _advance(func, method, steps, i, m, p, pool, sg)
            ta, tb = steps[m]
            if m == n - 1 and j == len(t_h) - 1 and t_h[j] == tb:
                # the last step writes the result in the caller's numbering
                _fused_step(method, func, ta, tb - ta, tb, bufs[p], ws, out=sol[j],
                            out_rows=lay.order32 if lay is not None else None)
                j += 1
                break
            p = _advance(func, method, steps, m, m + 1, p, pool, sg)
            ya, yb = bufs[1 - p], bufs[p]
            while j < len(t_h) and tb >= t_h[j]:
                if t_h[j] == tb:
                    _to_user(yb, sol[j], lay)
                else:
                    _to_user(_linear_interp(ta, tb, ya, yb, t_h[j]), sol[j], lay)
                j += 1
            i = m + 1
    finally:
        func._layout = None
    return sol


def _advance(func, method, steps, i, m, p, pool, sg):
    """Run steps i .. m-1 from bufs[p]; returns the parity the state ends in.
    Steps of the captured dt go through block graphs (binary decomposition),
    others — and every step while the module is not warm or too close to its
    max_nfe — run eagerly (a MaxNFEException is then raised at the exact call)."""
    bufs, ws = pool.bufs, pool.ws
    first = sg is not None and not sg.warm and i == 0 and p == 0
    while i < m:
        ta, tb = steps[i]
        dt = tb - ta
        if first and i == 1 and sg.warm:
            # the first solve of a new entry ran step 0 eagerly; the next solves will replay
            # steps 0 .. m-1 from bufs[0]: capture that decomposition now too (capture only
            # records launches), so a later solve of the same length captures nothing
            k = 1
            while k < m and steps[k][1] - steps[k][0] == sg.dt:
                k += 1
            q = 0
            for s in _pow2_blocks(k, GRAPH_BLOCK):
                sg.graph(func, s, q)
                q ^= s & 1
        if sg is not None and sg.warm and dt == sg.dt:
            k = 1
            while i + k < m and steps[i + k][1] - steps[i + k][0] == dt:
                k += 1
            if _nfe_headroom(func, k * sg.n_rhs):
                for s in _pow2_blocks(k, GRAPH_BLOCK):
                    p = sg.replay(func, s, p)
                i += k
                continue
        _fused_step(method, func, ta, dt, tb, bufs[p], ws, out=bufs[1 - p])
        if sg is not None and dt == sg.dt:
            sg.warm = True
        p = 1 - p
        i += 1
    return p


class _RKAdaptive(object):
    """torchdiffeq RKAdaptiveStepsizeODESolver (0.2.x rk_common.py) restated for an
    explicit embedded tableau (dopri5, bosh3, fehlberg2, adaptive_heun)."""

    def __init__(self, func, y0, rtol, atol, combine, method='dopri5', first_step=None, safety=0.9, ifactor=10.0,
                 dfactor=0.2, max_num_steps=2 ** 31 - 1, norm=_rms_norm):
        (self.order, self.alpha, self.beta, self.c_sol, self.c_error, self.c_mid) = _TABLEAUS[method]
        # FSAL tableaus (dopri5, bosh3): c_sol == beta[-1] and c_sol[-1] == 0, so y1 is the last stage input
        self.fsal = self.c_sol[-1] == 0 and list(self.c_sol[:-1]) == list(self.beta[-1])
        dtype = torch.promote_types(torch.float64, y0.dtype)
        dev = y0.device
        self.func, self.y0, self.combine, self.norm = func, y0, combine, norm
        self.dtype = dtype
        # the controller's scalars as given; their device tensors (the torch restatement's
        # arithmetic) are made on first use, so the fused solver (host floats) moves none
        self._scalars = {'rtol': rtol, 'atol': atol, 'safety': safety, 'ifactor': ifactor, 'dfactor': dfactor,
                         'first_step': first_step}
        self._tensors = {}
        self._dev = dev
        self.max_num_steps = max_num_steps
        self.n_steps = 0

    def _scalar_tensor(self, name):
        v = self._tensors.get(name)
        if v is None:
            raw = self._scalars[name]
            v = None if raw is None else torch.as_tensor(raw, dtype=self.dtype, device=self._dev)
            self._tensors[name] = v
        return v

    rtol = property(lambda self: self._scalar_tensor('rtol'))
    atol = property(lambda self: self._scalar_tensor('atol'))
    safety = property(lambda self: self._scalar_tensor('safety'))
    ifactor = property(lambda self: self._scalar_tensor('ifactor'))
    dfactor = property(lambda self: self._scalar_tensor('dfactor'))
    first_step = property(lambda self: self._scalar_tensor('first_step'))

    def _select_initial_step(self, t0, f0):
        y0, rtol, atol, norm, func = self.y0, self.rtol, self.atol, self.norm, self.func
        dtype, dev = y0.dtype, y0.device
        t_dtype = t0.dtype
        scale = atol + torch.abs(y0) * rtol
        d0 = norm(y0 / scale).abs()
        d1 = norm(f0 / scale).abs()
        if d0 < 1e-5 or d1 < 1e-5:
            h0 = torch.tensor(1e-6, dtype=dtype, device=dev)
        else:
            h0 = 0.01 * d0 / d1
        h0 = h0.abs()
        y1 = y0 + h0 * f0
        f1 = func(t0.to(dtype) + h0, y1)
        d2 = torch.abs(norm((f1 - f0) / scale) / h0)
        if d1 <= 1e-15 and d2 <= 1e-15:
            h1 = torch.max(torch.tensor(1e-6, dtype=dtype, device=dev), h0 * 1e-3)
        else:
            h1 = (0.01 / max(d1, d2)) ** (1. / float(self.order))
        h1 = h1.abs()
        return torch.min(100 * h0, h1).to(t_dtype)

    def _optimal_step_size(self, last_step, error_ratio):
        if error_ratio == 0:
            return last_step * self.ifactor
        dfactor = self.dfactor
        if error_ratio < 1:
            dfactor = torch.ones((), dtype=last_step.dtype, device=last_step.device)
        error_ratio = error_ratio.type_as(last_step)
        exponent = torch.tensor(self.order, dtype=last_step.dtype, device=last_step.device).reciprocal()
        factor = torch.min(self.ifactor, torch.max(self.safety / error_ratio ** exponent, dfactor))
        return last_step * factor

    def _step(self, y0, f0, t0, dt):
        dtf = float(dt.detach()) if isinstance(dt, torch.Tensor) else float(dt)
        t0f = float(t0.detach()) if isinstance(t0, torch.Tensor) else float(t0)
        k = [f0]
        yi = y0
        for i, (a_i, beta_i) in enumerate(zip(self.alpha, self.beta)):
            ti = t0f + dtf if a_i == 1. else t0f + a_i * dtf
            yi = self.combine(y0, k, beta_i, dtf)
            k.append(self.func(ti, yi))
        # non-FSAL tableaus (adaptive_heun, fehlberg2): y1 from c_sol, while the next
        # step's f0 is still the last stage k[-1], exactly as torchdiffeq does
        y1 = yi if self.fsal else self.combine(y0, k, self.c_sol, dtf)
        f1 = k[-1]
        y1_error = self.combine(None, k, self.c_error, dtf)
        return y1, f1, y1_error, k

    def _interp(self, y0, y1, k, dt, t0, t1, t):
        dtf = float(dt.detach()) if isinstance(dt, torch.Tensor) else float(dt)
        y_mid = self.combine(y0, k, self.c_mid, dtf)
        f0, f1 = k[0], k[-1]
        a = 2 * dtf * (f1 - f0) - 8 * (y1 + y0) + 16 * y_mid
        b = dtf * (5 * f0 - 3 * f1) + 18 * y0 + 14 * y1 - 32 * y_mid
        c = dtf * (f1 - 4 * f0) - 11 * y0 - 5 * y1 + 16 * y_mid
        d = dtf * f0
        e = y0
        x = (t - t0) / (t1 - t0)
        x = float(x.detach()) if isinstance(x, torch.Tensor) else float(x)
        total = e + x * d
        xp = x
        for coeff in (c, b, a):
            xp = xp * x
            total = total + xp * coeff
        return total

    def integrate(self, t):
        t = t.to(self.dtype)
        solution = [self.y0]
        t0 = t[0]
        f0 = self.func(t0, self.y0)
        dt = self._select_initial_step(t0, f0) if self.first_step is None else self.first_step
        y, f = self.y0, f0
        t_prev, t_cur = t0, t0
        last = None  # (y_prev, y_cur, k, dt) of the last accepted step
        for i in range(1, len(t)):
            next_t = t[i]
            while next_t > t_cur:
                if not bool(t_cur + dt > t_cur):
                    raise AssertionError('underflow in dt {}'.format(float(dt)))
                if self.n_steps >= self.max_num_steps:
                    raise AssertionError('max_num_steps exceeded ({}>={})'.format(self.n_steps, self.max_num_steps))
                y1, f1, y1_err, k = self._step(y, f, t_cur, dt)
                error_tol = self.atol + self.rtol * torch.max(y.abs(), y1.abs())
                error_ratio = self.norm(y1_err / error_tol).abs()
                if error_ratio <= 1:
                    last = (y, y1, k, dt)
                    t_prev, t_cur = t_cur, t_cur + dt
                    y, f = y1, f1
                dt = self._optimal_step_size(dt, error_ratio)
                self.n_steps += 1
            if last is None or next_t == t_cur:
                solution.append(y)
            else:
                y_prev, y_cur, k, dts = last
                solution.append(self._interp(y_prev, y_cur, k, dts, t_prev, t_cur, next_t))
        return torch.stack(solution, 0)


# --------------------------------------------------------------------------- fused adaptive steps
# An embedded Runge-Kutta step of torchdiffeq's adaptive solver (dopri5 — the method
# of every src/best_params.py entry — bosh3, fehlberg2, adaptive_heun) with every
# stage combination and the error estimate in the RHS epilogues (gnpde_stage_
# epilogue_t, the wide epilogue): launch i evaluates k_{i+1} = f(X_i) and writes the
# next stage input X_{i+1} from the rows it holds; the last launch forms the rows of
# the squared error norm.  One host read per step (the norm); no separate
# combination passes besides the step's first stage input.  The plan below derives
# every launch's operands from the tableau, choosing per combination the form that
# reads fewest state arrays:
#   from the launch's own input:  X_{i+1} = X_i + dt sum_j (b_{i+1,j} - b_{i,j}) k_j + dt b_{i+1,i+1} f
#   from the step start:          X_{i+1} = y0  + dt sum_j b_{i+1,j} k_j + dt b_{i+1,i+1} f
# (same values up to rounding: a combination of the k's scaled by dt, never a
# difference of states, so the error estimate keeps its precision).

def _nz(c):
    return c != 0.0


class _AdaptivePlan(object):
    """Per-launch operands of one step of an embedded tableau.

    Symbols: 'Y' the step start y0, 'X' the launch's own input, 'E' the error
    partial, 'K<j>' stage derivative j (K0 = f0 from the previous step).  Each
    combination is (base symbol or None, [(K<j>, coefficient / dt)...], f
    coefficient / dt); dt multiplies every k and f coefficient at run time."""

    def __init__(self, method):
        order, alpha, beta, c_sol, c_err, c_mid = _TABLEAUS[method]
        self.method, self.order, self.alpha, self.beta = method, order, alpha, beta
        self.c_sol, self.c_err, self.c_mid = c_sol, c_err, c_mid
        ns = len(alpha)
        self.ns = ns
        self.fsal = c_sol[-1] == 0 and list(c_sol[:-1]) == list(beta[-1])
        self.launches = []
        reads = []  # K indices each launch reads
        for i in range(ns):
            L = {'next': None, 'y1': None, 'epart': None, 'err': None}
            rd = set()
            if i < ns - 1:
                d = [(j, beta[i + 1][j] - beta[i][j]) for j in range(i + 1)]
                d = [(j, c) for j, c in d if _nz(c)]
                yv = [(j, beta[i + 1][j]) for j in range(i + 1) if _nz(beta[i + 1][j])]
                if len(d) <= len(yv) + 1:
                    L['next'] = ('X', [('K%d' % j, c) for j, c in d], beta[i + 1][i + 1])
                    rd |= {j for j, _ in d}
                else:
                    L['next'] = ('Y', [('K%d' % j, c) for j, c in yv], beta[i + 1][i + 1])
                    rd |= {j for j, _ in yv}
            else:
                if not self.fsal:
                    yv = [(j, c_sol[j]) for j in range(ns) if _nz(c_sol[j])]
                    L['y1'] = ('Y', [('K%d' % j, c) for j, c in yv], c_sol[ns])
                    rd |= {j for j, _ in yv}
            reads.append(rd)
            self.launches.append(L)
        # the error combination e = dt sum_j c_err[j] k_j (k_ns = the last launch's f): all in
        # the last launch, or its first ns terms precomputed by the launch before (a second
        # output 'E') when that launch already reads most of their operands
        last = ns - 1
        ev = [(j, c_err[j]) for j in range(ns) if _nz(c_err[j])]
        direct = {j for j, _ in ev if j < ns} - reads[last]
        pre_ok = ns >= 2
        if pre_ok:
            held = reads[last - 1] | {last}  # launch ns-2 reads its operands and holds k_{ns-1} = its own f
            pre_cost = 2 + len({j for j, _ in ev} - held)
            pre_ok = pre_cost < len(direct) + (0 if last in reads[last] else 0)
        if pre_ok:
            self.launches[last - 1]['epart'] = (None, [('K%d' % j, c) for j, c in ev if j < last], c_err[last])
            self.launches[last]['err'] = ('E', [], c_err[ns])
            reads[last - 1] |= {j for j, _ in ev if j < last}
        else:
            self.launches[last]['err'] = (None, [('K%d' % j, c) for j, c in ev], c_err[ns])
            reads[last] |= {j for j, _ in ev}
        self.reads = reads
        # k_j stored when a later launch reads it (k_ns: always, the next step's f0)
        self.store = set()
        for i in range(ns):
            for j in reads[i]:
                if j >= 1:
                    self.store.add(j)
        self.store.add(ns)
        # dense output (a step that may cross an output time): every k with a c_mid term
        self.store_mid = {j for j in range(1, ns + 1) if _nz(c_mid[j])} - self.store

    def state_passes(self):
        """Full-state reads / writes per step beyond each launch's own gathers,
        input row and one output (the bench's overhead check)."""
        r = 2  # the step's first stage input: y0 and k0
        w = 1
        for i, L in enumerate(self.launches):
            outs = [c for c in (L['next'], L['y1'], L['epart']) if c is not None]
            r += len(self.reads[i]) + sum(1 for c in outs if c[0] in ('Y', 'E'))
            if L['err'] is not None:
                r += 1 + (1 if L['err'][0] == 'E' else 0)  # y0 for the tolerance, E
            stored = (i + 1) in self.store
            w += len(outs) + (1 if stored else 0) - 1
        return r, w


_PLANS = {}


def _adaptive_plan(method):
    p = _PLANS.get(method)
    if p is None:
        p = _PLANS[method] = _AdaptivePlan(method)
    return p


class _KrylovPlan(object):
    """The step of an FSAL tableau for an affine RHS f(y) = L y + s in the Krylov basis
    u_p = (dt L)^p f0 (u_0 = f0 = f(y0)).  Every stage derivative is a fixed
    combination of them: k_0 = u_0, k_{i+1} = f(y0 + dt sum_j beta[i][j] k_j)
    = k_0 + sum_j beta[i][j] (dt L) k_j, so k_i = sum_p B[i][p] u_p with
    B[i+1][p] = sum_j beta[i][j] B[j][p-1].  A step is ns launches of the linear part,
    u_{p+1} = dt L u_p, each reading only its own input (no stage operand); the last
    (over u_{ns-1}, with f_lin = 1: f' = u_{ns-1} + u_ns) forms
      y1  = y0 + dt sum_p G[p] u_p,                 G[p]   = sum_j c_sol[j] B[j][p]
      f1  = sum_p B[ns][p] u_p                      (the next step's f0: unscaled)
      e   = dt sum_p Eps[p] u_p,                    Eps[p] = sum_j c_err[j] B[j][p]
    with u_ns = f' - u_{ns-1} substituted.  Mathematically the tableau's step; Eps[p]
    vanishes exactly for p below the embedded order (the order conditions of the
    linear problem), which the fp64 sums leave at rounding level and the plan zeroes,
    so the error estimate carries no stage-combination cancellation noise.  Dense
    output: y_mid = y0 + dt (sum_p Mu[p] u_p + c_mid[ns] f1), Mu[p] = sum_{j<ns}
    c_mid[j] B[j][p], with y1 restated on the u_p (one pass over ns + 2 rows)."""

    def __init__(self, plan):
        ns, beta = plan.ns, plan.beta
        B = [[1.0]]
        for i in range(ns):
            B.append([1.0] + [sum(beta[i][j] * B[j][p - 1] for j in range(p - 1, i + 1))
                              for p in range(1, i + 2)])
        self.B = B

        def comb(c, upto):
            v = [sum(c[j] * B[j][p] for j in range(p, upto)) for p in range(ns + 1)]
            big = max(1.0, max(abs(x) for x in v))
            return [0.0 if abs(x) < 1e-12 * big else x for x in v]
        self.G = comb(plan.c_sol, ns + 1)
        self.Eps = comb(plan.c_err, ns + 1)
        self.Mu = comb(plan.c_mid, ns)
        self.Bn = list(B[ns])
        self.ns = ns

    def last_launch_terms(self):
        """(y1 terms, (f1 terms, f1 cf), (error terms, error cf)) of the last launch over
        u_{ns-1}, as [(p, coefficient)] with u_ns = f' - u_{ns-1} substituted."""
        ns = self.ns

        def sub(v):
            t = [(p, v[p]) for p in range(ns - 1) if v[p] != 0.0]
            c = v[ns - 1] - v[ns]
            if c != 0.0:
                t.append((ns - 1, c))
            return t, v[ns]
        y1 = [(p, self.G[p]) for p in range(ns) if self.G[p] != 0.0]
        return y1, sub(self.Bn), sub(self.Eps)

    def state_passes(self):
        """Full-state reads / writes per step beyond each launch's gathers, input row
        and one output: the last launch reads y0 (the y1 base and the tolerance) and
        u_0 .. u_{ns-2}, and writes a second output (f1)."""
        return self.ns, 1


KRYLOV_STEP = os.environ.get('GNPDE_KRYLOV_STEP', '1') != '0'
_KRYLOV_PLANS = {}


def _krylov_plan(plan):
    """The _KrylovPlan of a tableau plan, built once (its fp64 sums cost ~50 us of host
    time, which every solve paid before its first launch)."""
    k = _KRYLOV_PLANS.get(plan.method)
    if k is None:
        k = _KRYLOV_PLANS[plan.method] = _KrylovPlan(plan)
    return k
# The dense output of a one-output-time Krylov solve folded into its steps' last launch
# (ABI 8 Stage.dense; GNPDE_DENSE_FOLD=0: the separate pass of _interp_into)
DENSE_FOLD = os.environ.get('GNPDE_DENSE_FOLD', '1') != '0'
# The initial-step selection of an affine RHS from row sums the f0 and probe launches form
# (ABI 8 scale_rows, err_y1 = -2, gnpde_initial_step_rows; GNPDE_INIT_ROWS=0: the passes of
# gnpde_initial_step_f32 over y0, f0 and f1 = f(y0 + h0 f0), in torch's fp32 arithmetic).
# Off by default: the wide epilogue the two launches then take costs more than the passes
# it saves (G-arxiv: f0 launch 80 -> 124 us, probe 76 -> 109 us)
INIT_ROWS = os.environ.get('GNPDE_INIT_ROWS', '0') == '1'
# The initial-step probe of an affine Krylov solve as v = L f0 (gnpde_initial_step_lin_*: d2 =
# rms(v / scale)), run beside the phase-0 reduction on a second stream; v is the first step's
# u_1 / dt, so that step scales it in place instead of launching K1 (GNPDE_LIN_INIT=0: the probe
# f0 + h0 L f0 after phase 0 and a first step like the others)
LIN_INIT = os.environ.get('GNPDE_LIN_INIT', '1') != '0'
# The f0 launch and the lin_init initial step replayed as one captured graph once warm
# (GNPDE_PROLOGUE_GRAPH=1).  Off by default: measured no faster (G-arxiv 2.705 against 2.698 ms
# per solve) — once the first launch runs, the host stays ahead of the device anyway.
PROLOGUE_GRAPH = os.environ.get('GNPDE_PROLOGUE_GRAPH', '0') == '1'


def _fused_adaptive_ok(func, y0, combine, options):
    """The fused adaptive step applies: a gnpde RHS (rhs_stage) without autograd, a
    device state (or a host-stage test RHS on CPU), torchdiffeq's RMS norm (or a
    sharded RHS's global one, reduced through func.reduce_error_sq)."""
    if not (isinstance(combine, _Combine) and hasattr(func, 'rhs_stage')) or torch.is_grad_enabled():
        return False
    if not getattr(func, 'fused_adaptive', True) or os.environ.get('GNPDE_FUSED_ADAPTIVE', '1') == '0':
        return False
    norm = options.get('norm')
    if norm is not None and not (getattr(norm, '__self__', None) is func and hasattr(func, 'reduce_error_sq')):
        return False
    if y0.is_cuda:
        return y0.dtype in ops.STATE_DTYPES
    return bool(getattr(func, 'host_stages', False)) and hasattr(func, 'host_stage_apply')


# Backprop through adaptive solves of the Laplacian (gnpde.adaptive_backprop; GNPDE_ADAPTIVE_BACKPROP=0: the
# restated loop with autograd through every RHS and stage combination)
ADAPTIVE_BACKPROP = os.environ.get('GNPDE_ADAPTIVE_BACKPROP', '1') != '0'


def _adaptive_backprop_ok(func, y0, combine, options):
    """An adaptive solve under autograd of a gnpde LaplacianODEFunc on a device fp32
    state with torchdiffeq's RMS norm, the sigmoid alpha and something to differentiate."""
    if not (ADAPTIVE_BACKPROP and torch.is_grad_enabled() and isinstance(combine, _Combine)):
        return False
    if not (hasattr(func, '_weights_tensor') and hasattr(func, 'rhs_stage')) or 'norm' in options:
        return False
    if not (y0.is_cuda and y0.dtype == torch.float32 and y0.dim() == 3) or getattr(func, '_layout', None) is not None:
        return False
    if func.opt.get('no_alpha_sigmoid', False):
        return False
    w, _ = func._weights_tensor()
    return any(v.requires_grad for v in (y0, func.alpha_train, func.beta_train, w))


class _LaplacianAdaptiveFn(torch.autograd.Function):
    """An adaptive solve of f(y) = sigma(alpha)(A(w) y - y) [+ beta x0] with its discrete
    adjoint (gnpde.adaptive_backprop): gradients to y0, alpha_train, beta_train and the
    weights (the attention an AttODEblock hands the Laplacian)."""

    @staticmethod
    def forward(ctx, y0, alpha_train, beta_train, w, func, t_h, method, rtol, atol, first_step, max_num_steps):
        from .adaptive_backprop import AdaptiveBackprop
        with torch.no_grad():
            solver = AdaptiveBackprop(func, y0.detach(), t_h, method, rtol, atol, first_step, max_num_steps)
            sol = solver.forward()
        odeint.last_n_steps = solver.n_steps
        ctx.solver = solver
        ctx.shapes = (alpha_train.shape, alpha_train.dtype, beta_train.shape, beta_train.dtype)
        return sol

    @staticmethod
    def backward(ctx, g):
        with torch.no_grad():
            ybar, ga, gb, gw = ctx.solver.backward(g)
        ctx.solver = None
        ash, adt, bsh, bdt = ctx.shapes
        need = ctx.needs_input_grad
        gy = ybar.view(g.shape[1:]) if need[0] else None
        gal = ga.to(adt).reshape(ash) if need[1] else None
        gbe = None
        if need[2]:
            gbe = gb.to(bdt).reshape(bsh) if gb is not None else torch.zeros(bsh, dtype=bdt, device=g.device)
        gwo = gw if need[3] else None
        return (gy, gal, gbe, gwo) + (None,) * 7


class _HostRecord(object):
    """A pinned host copy of a step's device record that its step graph writes."""
    __slots__ = ('buf',)

    def __init__(self, buf):
        self.buf = buf


# The replayed step graph copies the controller's record to pinned memory itself
# (GNPDE_GRAPH_RECORD_COPY=0: a copy enqueued behind each replay)
GRAPH_RECORD_COPY = os.environ.get('GNPDE_GRAPH_RECORD_COPY', '1') != '0'


# Captured adaptive steps (hipGraph): one graph per (buffer binding, dense-output
# variant) replays a whole step — the stage-input pass, the RHS launches and the
# error reduction — whatever dt (the coefficients scale by a device scalar), so a
# step costs one graph launch and one host read.  GNPDE_ADAPTIVE_GRAPH=0 runs
# every step eagerly.
ADAPTIVE_GRAPH = os.environ.get('GNPDE_ADAPTIVE_GRAPH', '1') != '0'
AFFINE_STAGE = os.environ.get('GNPDE_AFFINE_STAGE', '1') != '0'
ADAPTIVE_SPEC = os.environ.get('GNPDE_ADAPTIVE_SPEC', '1') != '0'  # steps enqueued ahead (_integrate)
_ADAPTIVE_CACHE = weakref.WeakKeyDictionary()  # module -> (key, _AdaptiveState)


class _AdaptiveState(object):
    """Buffers and captured step graphs of one module's fused adaptive solves of one
    state shape and tolerance (kept across odeint calls, like _StatePool)."""

    def __init__(self, plan, y0, host):
        new = lambda: torch.empty_like(y0, memory_format=torch.contiguous_format)  # noqa: E731
        b = {'Y': new(), 'Y1': new(), 'K0': new()}
        for j in sorted(plan.store | plan.store_mid):
            b['K%d' % j] = new()
        xa, xb = new(), new()
        for i in range(plan.ns):
            b['X%d' % i] = b['Y1'] if (plan.fsal and i == plan.ns - 1) else (xa if i % 2 == 0 else xb)
        if any(L['epart'] is not None for L in plan.launches):
            b['E'] = new()
        self.bufs = b
        self.rows = torch.empty(y0.numel() // y0.shape[-1], dtype=torch.float64, device=y0.device)
        # the step size the stage coefficients are scaled by (device fp32 scalar; the host-stage
        # test RHS objects apply it in their own precision)
        self.scale = torch.zeros((), dtype=torch.float32 if not host else torch.float64, device=y0.device)
        # the device controller's step size (fp64) and its record {ratio, dt, next dt} (device solves)
        # h = {h0, d1, first step} of the device initial-step selection; dt is h[2] (a view), so
        # the first step's size and scale are in place when the selection ends
        self.h = None if host else torch.zeros(3, dtype=torch.float64, device=y0.device)
        self.dt = None if host else self.h[2]
        self.rec = None if host else torch.zeros(4, dtype=torch.float64, device=y0.device)
        self.ws = None if host else torch.empty(_lib.fn("gnpde_dot_workspace_bytes")(), dtype=torch.uint8,
                                                device=y0.device)
        self.rec_host, self.rec_slot = None, 0  # pinned copies of rec (_rec_reader)
        # the folded dense output (DENSE_FOLD): the device time {step start, output time} the controller
        # advances, the slot holding the output array's address, the output row map (a copy: the
        # captured launch reads this buffer whatever layout object the solve has)
        # one device record {t0, t_out, output address} (fp64 / fp64 / int64 views) set per solve by one
        # copy from a pinned host twin
        self.dsc = None if host else torch.zeros(3, dtype=torch.float64, device=y0.device)
        self.dsc_host = None if host else torch.zeros(3, dtype=torch.float64, pin_memory=True)
        self.dsc_np = None if host else self.dsc_host.numpy()  # (host writes through numpy: no torch ops)
        self.tdev = None if host else self.dsc[:2]
        self.dslot = None if host else self.dsc[2:].view(torch.int64)
        self.dtab = None if host else torch.zeros(_lib.DENSE_SLOTS + 1, dtype=torch.float32, device=y0.device)
        self.drows, self.drows_src = None, None
        # the initial-step selection from the f0 / probe launches' row sums (INIT_ROWS): a second
        # row array (the f0 launch's scale_rows) and the reduction's workspace
        self.rows2, self.iws = None, None
        self.side = None  # the second stream of the initial step (LIN_INIT)
        # the captured prologue of a lin_init solve (f0 and the initial-step launches) and the
        # workspaces of its two reductions (phase 0 runs beside the probe: two buffers)
        self.pro = None
        self.iws0 = self.iws1 = None
        self.canon = None  # the y / f0 buffer binding every solve starts from (_integrate)
        self.graphs = {}   # (id Y, id K0, mid, fold, renumbered) -> (graph, error-sum tensor)
        self.mempool = None
        self.warm = False


class _RKAdaptiveFused(_RKAdaptive):
    """_RKAdaptive with the step formed by the RHS epilogues (_AdaptivePlan): the same
    controller (torchdiffeq's, in host float64 arithmetic), the same accepted /
    rejected sequence, dense output from the stored stage derivatives.  Per step:
    one stage-input pass, len(alpha) RHS launches carrying the combinations and the
    error rows, one fixed-order fp64 reduction and one host read of it; the step
    replayed from a captured hipGraph once the module's structures are built."""

    def __init__(self, func, y0, rtol, atol, combine, method='dopri5', options=None, **kw):
        super(_RKAdaptiveFused, self).__init__(func, y0, rtol, atol, combine, method=method, **kw)
        self.options = dict(options or {})
        self.plan = _adaptive_plan(method)
        self.host = not y0.is_cuda
        self.rtol_f, self.atol_f = float(rtol), float(atol)
        # f(y) = L y + s (func.affine): the step's first stage derivative is k0 + dt b00 L k0 from
        # a launch over k0 (Stage.f_lin) — no X0 = y0 + dt b00 k0 pass.  Needs k0 = f(y0): the FSAL
        # pairs (dopri5, bosh3); torchdiffeq's non-FSAL pairs carry k0 = the last stage of the previous
        # step instead.  GNPDE_AFFINE_STAGE=0 disables it.
        self.affine = bool(getattr(func, 'affine', False)) and AFFINE_STAGE and self.plan.fsal
        # the affine step in the Krylov basis (_KrylovPlan): ns launches, no stage operands
        # before the last; its u_1 .. u_{ns-1} live in the K1 .. K{ns-1} buffers
        P = self.plan
        self.krylov = None
        if self.affine and KRYLOV_STEP and P.ns <= _lib.STAGE_MAX_K and \
                set(range(1, P.ns + 1)) <= (P.store | P.store_mid):
            self.krylov = _krylov_plan(P)
        sc = self._scalars
        self.safety_f, self.ifactor_f, self.dfactor_f = float(sc['safety']), float(sc['ifactor']), float(sc['dfactor'])
        self.fold = False  # this solve's dense output folded into the Krylov steps (_integrate)
        self.init_rows = False  # its initial step from the f0 / probe launches' row sums (_integrate)
        self.lin_init = False   # its probe v = L f0, reused as the first step's u_1 (_integrate)
        self._first = False     # the next step is the first attempt after a lin_init probe
        self.lay = None

    # ---- device primitives (host-stage RHS objects supply CPU versions: tests only)
    def _apply(self, stage, f, x, like):
        if self.host:
            self.func.host_stage_apply(stage, f, x, like)
        else:
            ops.stage_apply(stage, f, x, like)

    def _err_sum(self, rows):
        """The step's squared error sum (0-d fp64 tensor) and its element count."""
        v = rows.sum() if self.host else ops.sum_f64(rows)
        n = float(rows.numel() * self.C)
        red = getattr(self.func, 'reduce_error_sq', None)
        if red is not None and 'norm' in self.options:
            pair = torch.stack([v.reshape(()), torch.tensor(n, dtype=torch.float64, device=rows.device)])
            red(pair)
            return pair
        return v

    def _combo(self, spec, bufs, x):
        """(base tensor, cb, cf, [(k tensor, c)]) of a plan combination; the k and f
        coefficients are the tableau's, scaled by dt on the device (Stage.scale)."""
        base, terms, cfc = spec
        bt = {'Y': bufs['Y'], 'X': x, 'E': bufs.get('E'), None: None}[base]
        return bt, (1.0 if bt is not None else 0.0), cfc, [(bufs[k], c) for k, c in terms]

    def _launch(self, i, st, x, t, mid):
        P = self.plan
        bufs = st.bufs
        L = P.launches[i]
        lin = self.affine and i == 0
        if lin:
            # the affine first stage: the launch reads k0 and forms k1 = k0 + dt b00 L k0 (Stage.f_lin),
            # never X0 = y0 + dt b00 k0; its combinations on X0 are restated on y0 (X0 = y0 + dt b00 k0)
            x = bufs['K0']
        outs = []
        for key, dst in (('next', 'X%d' % (i + 1)), ('y1', 'Y1'), ('epart', 'E')):
            if L[key] is not None:
                spec = self._on_y0(L[key]) if lin else L[key]
                b, cb, cf, ks = self._combo(spec, bufs, x)
                outs.append((bufs[dst], b, cb, cf, ks))
        err = None
        if L['err'] is not None:
            spec = self._on_y0(L['err']) if lin else L['err']
            if lin and L['y1'] is None:
                raise RuntimeError("gnpde: an affine one-stage tableau needs its y1 output for the tolerance")
            b, cb, cf, ks = self._combo(spec, bufs, x)
            err = (st.rows, (b, cb, cf, ks), bufs['Y'], 0 if L['y1'] is not None else -1, self.atol_f, self.rtol_f)
        j = i + 1
        f_out = bufs['K%d' % j] if (j in P.store or (mid and j in P.store_mid)) else None
        if lin:
            self.func.rhs_stage(t, x, ops.Stage(f_out=f_out, outs=outs, err=err, scale=st.scale,
                                                f_lin=P.beta[0][0]), linear=True)
        else:
            self.func.rhs_stage(t, x, ops.Stage(f_out=f_out, outs=outs, err=err, scale=st.scale))

    def _on_y0(self, spec):
        """A launch-0 combination on base X0 restated on y0: X0 + dt(sum d_j k_j + cf f)
        = y0 + dt((b00 + d_0) k0 + ...) (X0 = y0 + dt b00 k0)."""
        base, terms, cf = spec
        if base != 'X':
            return spec
        b00 = self.plan.beta[0][0]
        d = dict(terms)
        d['K0'] = d.get('K0', 0.0) + b00
        return ('Y', [(k, c) for k, c in d.items() if c != 0.0], cf)

    def _step(self, st, t_cur, dt, mid, first=False):
        """Enqueue one step (stage-input pass, RHS launches, error reduction); returns
        the device error sum."""
        P = self.plan
        bufs = st.bufs
        if self.krylov is not None:
            self._krylov_launches(st, t_cur, first)
        else:
            if not self.affine:  # the first stage input X0 = y0 + dt b00 k0 (the affine mode never forms it)
                self._apply(ops.Stage(outs=[(bufs['X0'], bufs['Y'], 1.0, 0.0, [(bufs['K0'], P.beta[0][0])])],
                                      scale=st.scale), None, None, bufs['Y'])
            for i in range(P.ns):
                ti = t_cur + dt if P.alpha[i] == 1. else t_cur + P.alpha[i] * dt
                self._launch(i, st, bufs['X%d' % i], ti, mid)
        if self._dev_control():  # the error sum and the controller: two launches, no host work
            ops.adaptive_control(st.rows, st.rows.numel() * self.C, self.order, self.safety_f, self.ifactor_f,
                                 self.dfactor_f, st.dt, st.scale, st.rec, ws=st.ws, t=st.tdev)
            return st.rec
        return self._err_sum(st.rows)

    def _krylov_launches(self, st, t, first=False):
        """The launches of one affine step in the Krylov basis (_KrylovPlan): u_{p+1} =
        dt L u_p into K{p+1} for p < ns - 1, then the launch over u_{ns-1} that writes y1,
        f1 (K{ns}) and the error rows.  The RHS is autonomous: every launch at t."""
        K = self.krylov
        ns = K.ns
        bufs = st.bufs
        u = [bufs['K0']] + [bufs['K%d' % p] for p in range(1, ns)]
        y1t, (ft, fcf), (et, ecf) = K.last_launch_terms()
        outs = [(bufs['Y1'], bufs['Y'], 1.0, 0.0, [(u[p], c) for p, c in y1t]),
                (bufs['K%d' % ns], None, 0.0, fcf, [(u[p], c) for p, c in ft])]
        err = (st.rows, (None, 0.0, ecf, [(u[p], c) for p, c in et]), bufs['Y'], 0, self.atol_f, self.rtol_f)
        last = ops.Stage(outs=outs, err=err, scale=st.scale, f_lin=1.0, unscaled=(1,))
        # the first attempt after a lin_init probe: u_1 = dt v in place (v = L f0 in K1, the same
        # fp32 product the launch over u_0 would store), the K1 launches from u_1 on
        p0 = 1 if first else 0
        if first:
            if hasattr(self.func, 'nfe'):  # the reference evaluates it: the counter keeps torchdiffeq's NFE
                self.func.nfe += 1
            ops.stage_apply(ops.Stage(outs=[(u[1], None, 0.0, 0.0, [(u[1], 1.0)])], scale=st.scale), None, None,
                            u[1])
        form = None  # the folded dense output: the step's first launch forms its coefficients, the last applies them
        if self.fold and ns >= 2:
            last.dense = (st.dslot, st.drows if self.lay is not None else None, None, None, st.dtab,
                          self._dense_table(u, ft, fcf))
            form = (None, None, st.tdev, st.dt, st.dtab, last.dense_matrix())
        for p in range(p0, ns - 1):
            self.func.rhs_stage(t, u[p], ops.Stage(outs=[(u[p + 1], None, 0.0, 1.0, [])], scale=st.scale,
                                                   dense=form if p == p0 else None), linear=True)
        self.func.rhs_stage(t, u[ns - 1], last, linear=True)

    def _dense_table(self, u, ft, fcf):
        """The basis coefficients of the step's dense output over the last Krylov launch's
        operands (ABI 8 Stage.dense): with w = (cy0 + cy1 + cym, h cy1, h cym, cf0, cf1),
        out = w0 y0 + sum_p [w1 G[p] + w2 (Mu[p] + c_mid[ns] f1_p) + w3 [p = 0] + w4 f1_p] u_p
              + (w2 c_mid[ns] + w4) fcf f'
        where f1 = sum_p f1_p u_p + fcf f' is the next step's f0 (u_ns substituted) — the
        combination _interp_into forms from y0, the u_p and f1 in a pass of its own."""
        K, P = self.krylov, self.plan
        ns = K.ns
        cm = P.c_mid[ns]
        f1 = dict(ft)
        table = {'base': [1.0, 0.0, 0.0, 0.0, 0.0], 'f': [0.0, 0.0, cm * fcf, 0.0, fcf]}
        for p in range(ns):
            b = f1.get(p, 0.0)
            w = [0.0, K.G[p], K.Mu[p] + cm * b, 1.0 if p == 0 else 0.0, b]
            if any(v != 0.0 for v in w):
                table[u[p]] = w
        return table

    def _dev_control(self):
        """The step-size controller runs on the device (a device solve with the
        default RMS norm): the host reads {ratio, dt, next dt} once per step."""
        return not self.host and 'norm' not in self.options

    def _rotate(self, bufs, kn, d):
        """Advance (d = 1) or undo (d = -1) the binding of y0 / f0 after an accepted
        step: two buffers swap; with the third (steps ahead) the three rotate."""
        P = self.plan
        for a, b, c in (('Y', 'Y1', 'Ys'), ('K0', kn, 'Ks')):
            if c not in bufs:
                bufs[a], bufs[b] = bufs[b], bufs[a]
            elif d > 0:
                bufs[a], bufs[b], bufs[c] = bufs[b], bufs[c], bufs[a]
            else:
                bufs[a], bufs[b], bufs[c] = bufs[c], bufs[a], bufs[b]
        if P.fsal:
            bufs['X%d' % (P.ns - 1)] = bufs['Y1']

    def _rec_reader(self, st, rec, slot=None):
        """A device fp64 record (the step's {ratio, dt, next dt, e2}; h of the initial
        step, slot 2) copied to pinned host memory behind an event (slots 0 / 1
        alternate: a step ahead may be in flight): a callable that waits for that copy
        only and returns the values."""
        if isinstance(rec, _HostRecord):  # copied by the replayed step graph itself
            ev = torch.cuda.Event()
            ev.record()
            hb = rec.buf

            def read_graph():
                ev.synchronize()
                return hb.tolist()
            return read_graph
        if st.rec_host is None:
            st.rec_host = torch.empty((3, 4), dtype=torch.float64, pin_memory=True)
        if slot is None:
            slot = st.rec_slot
            st.rec_slot ^= 1
        h = st.rec_host[slot, :rec.numel()]
        h.copy_(rec, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()

        def read():
            ev.synchronize()
            return h.tolist()
        return read

    def _lin_init_launches(self, st, t0):
        """The lin_init initial step: phase 0 (y0, f0 -> h0, d1) on a second stream beside the
        probe v = L f0 (it needs no h0), then phase 1 from v; v lands in K1, the first step's
        u_1 buffer (_krylov_launches).  No host read (capturable: _prologue)."""
        bufs = st.bufs
        Y, K0, v = bufs['Y'], bufs['K0'], bufs['K1']
        h, hf = st.h, st.scale
        if st.iws0 is None:
            nb = _lib.fn("gnpde_initial_step_workspace_bytes")()
            st.iws0 = torch.empty(nb, dtype=torch.uint8, device=Y.device)
            st.iws1 = torch.empty(nb, dtype=torch.uint8, device=Y.device)
        main = torch.cuda.current_stream(Y.device)
        if st.side is None:
            st.side = torch.cuda.Stream(Y.device)
        st.side.wait_stream(main)
        with torch.cuda.stream(st.side):
            ops.initial_step(Y, K0, None, self.atol_f, self.rtol_f, self.order, h, hf, ws=st.iws0)
        self.func.rhs_stage(t0, K0, ops.Stage(f_out=v), linear=True)
        main.wait_stream(st.side)
        ops.initial_step_lin(Y, v, self.atol_f, self.rtol_f, self.order, h, hf, ws=st.iws1)

    def _prologue(self, st, graphs_ok, t0):
        """f0 into K0 and the lin_init initial step as ONE captured graph (PROLOGUE_GRAPH) once
        the module is warm.  Returns True when replayed (the caller reads h)."""
        if not (PROLOGUE_GRAPH and graphs_ok and st.warm and _nfe_headroom(self.func, 2)):
            return False
        bufs = st.bufs
        if st.pro is None:
            nfe = getattr(self.func, 'nfe', None)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=st.mempool):
                self.func.rhs_stage(t0, bufs['Y'], ops.Stage(f_out=bufs['K0']))
                self._lin_init_launches(st, t0)
            if st.mempool is None:
                st.mempool = g.pool()
            if nfe is not None:
                self.func.nfe = nfe  # capture records launches, it evaluates nothing
            st.pro = g
        st.pro.replay()
        if hasattr(self.func, 'nfe'):
            self.func.nfe += 2
        self._first = True
        return True

    def _initial_step_device(self, st, t0):
        """_select_initial_step on the device (gnpde_initial_step_*: the two fixed-order
        norm reductions and the scalar rules in HIP, the probe y0 + h0 f0 as one stage
        pass with h0 as its device coefficient scale, f1 by the RHS): one host read.
        The probe's RHS is evaluated at t0 (the RHS is autonomous: h0 stays on the
        device)."""
        bufs = st.bufs
        Y, K0 = bufs['Y'], bufs['K0']
        h, hf = st.h, st.scale  # h[2] is st.dt: the device controller starts from it
        if self.lin_init:
            self._lin_init_launches(st, t0)
            self._first = True
            return self._rec_reader(st, h, slot=2)
        if self.init_rows:
            # from the f0 launch's rows; then the rows of L f0 (the probe's linear part on f0, no
            # output): d2 = rms(L f0 / scale) = rms((f1 - f0) / scale) / h0 for f1 = f(y0 + h0 f0)
            n = float(st.rows.numel() * self.C)
            ops.initial_step_rows(st.rows, st.rows2, n, self.order, h, hf, ws=st.iws)
            self.func.rhs_stage(t0, K0, ops.Stage(err=(st.rows, (None, 0.0, 1.0, []), Y, -2, self.atol_f,
                                                       self.rtol_f)), linear=True)
            ops.initial_step_rows(st.rows, None, n, self.order, h, hf, ws=st.iws)
            return self._rec_reader(st, h, slot=2)
        ops.initial_step(Y, K0, None, self.atol_f, self.rtol_f, self.order, h, hf)
        probe, f1 = bufs['X0'], bufs['Y1']  # free until the first step
        if self.affine:  # f1 = f0 + h0 L f0 from a launch over f0 (no probe pass)
            self.func.rhs_stage(t0, K0, ops.Stage(f_out=f1, scale=hf, f_lin=1.0), linear=True)
        else:
            ops.stage_apply(ops.Stage(outs=[(probe, Y, 1.0, 0.0, [(K0, 1.0)])], scale=hf), None, None, Y)
            self.func.rhs_stage(t0, probe, ops.Stage(f_out=f1))
        ops.initial_step(Y, K0, f1, self.atol_f, self.rtol_f, self.order, h, hf)
        return self._rec_reader(st, h, slot=2)  # the first step's size: read when it is needed

    def _state(self, y0):
        """The module's cached buffers / graphs for this shape, tolerance and graph
        state (a new entry when any of them changed)."""
        P = self.plan
        if self.host or not ADAPTIVE_GRAPH or not _replayable(self.func) or \
                'norm' in self.options:  # a sharded RHS's global norm: a collective inside the step
            return _AdaptiveState(P, y0, self.host), False
        state = _capture_state(self.func, y0)
        key = _graph_cache_key(self.func, 'adaptive:' + P.method + (':krylov' if self.krylov is not None else ''), y0, state)
        if key is None:
            return _AdaptiveState(P, y0, self.host), False
        key = key + (self.atol_f, self.rtol_f, torch.cuda.current_stream(y0.device).cuda_stream,
                     'norm' in self.options)
        hit = _ADAPTIVE_CACHE.get(self.func)
        if hit is not None and hit[0] == key:
            return hit[1], True
        ast = _AdaptiveState(P, y0, self.host)
        _ADAPTIVE_CACHE[self.func] = (key, ast, state)
        return ast, True

    def _run_step(self, st, graphs_ok, t_cur, dt, mid):
        """One step: replayed from its graph when the binding's graph exists (captured
        on first use once the module is warm), eagerly otherwise.  The first attempt after
        a lin_init probe takes its own variant (u_1 from the probe)."""
        P = self.plan
        first, self._first = self._first, False
        if graphs_ok and st.warm and _nfe_headroom(self.func, P.ns):
            gk = (id(st.bufs['Y']), id(st.bufs['K0']), bool(mid), self.fold, self.lay is not None, GRAPH_RECORD_COPY,
                  first)
            ent = st.graphs.get(gk)
            if ent is None:
                nfe = getattr(self.func, 'nfe', None)
                g = torch.cuda.CUDAGraph()
                # the device controller's record copied to a pinned buffer of this graph by the graph
                # itself (GRAPH_RECORD_COPY): no separate copy behind the replay (the same graph is
                # replayed again only after its record was read: the bindings rotate through three)
                hb = torch.empty(4, dtype=torch.float64, pin_memory=True) \
                    if (GRAPH_RECORD_COPY and self._dev_control()) else None
                with torch.cuda.graph(g, pool=st.mempool):
                    err = self._step(st, t_cur, dt, mid, first)
                    if hb is not None:
                        hb.copy_(err, non_blocking=True)
                if st.mempool is None:
                    st.mempool = g.pool()
                if nfe is not None:
                    self.func.nfe = nfe  # capture records launches, it evaluates nothing
                ent = (g, err if hb is None else _HostRecord(hb))
                st.graphs[gk] = ent
            ent[0].replay()
            if hasattr(self.func, 'nfe'):
                self.func.nfe += P.ns
            return ent[1]
        err = self._step(st, t_cur, dt, mid, first)
        st.warm = True
        return err

    def integrate(self, t):
        """The adaptive loop.  A device solve of a module offering a locality numbering
        (ops.NodeLayout, as the fixed-grid path) runs in it: the entry pass writes
        sol[0] and the permuted state from one read of y0, every RHS launch gathers
        from the degree-ordered rows, and outputs return to the caller's numbering
        (the dense output's single pass stores there directly, out_rows).  Row
        values are bit-identical to the user numbering; the error norm's fixed-order
        sum runs over rows in the other order (fp64 rounding only)."""
        P = self.plan
        th = _host_times(t)  # cached per time tensor: no device read for an ODEblock's self.t
        y0 = self.y0.contiguous()
        self.C = y0.shape[-1]
        dev = y0.device
        sol = torch.empty((len(th),) + tuple(y0.shape), dtype=y0.dtype, device=dev)
        lay = None if self.host else _node_layout(self.func, y0)
        self.lay = lay
        if lay is not None:
            self.func._layout = lay
        try:
            return self._integrate(th, y0, sol, lay)
        finally:
            if lay is not None:
                self.func._layout = None

    def _integrate(self, th, y0, sol, lay):
        P = self.plan
        dev = y0.device
        st, graphs_ok = self._state(y0)
        bufs = st.bufs
        if st.canon is not None:
            # every solve starts from the same binding of the rotating y / f0 buffers, so it walks
            # the same sequence of bindings and replays the same step graphs (a solve starting
            # where the last one ended met bindings whose graphs were not captured yet)
            bufs.update(st.canon)
        # The dense output folded into the last launch of every step (DENSE_FOLD; ABI 8): a
        # solve to one output time in the Krylov basis under the device controller.  Each
        # step's launch writes the interpolant at th[1] straight into sol[1] (the caller's
        # numbering) when the step crosses it, by the device time the controller advances;
        # the accepted crossing step writes last (a rejected or discarded step either does
        # not cross or is followed by one that does), so no dense-output pass follows.
        self.fold = (DENSE_FOLD and not self.host and self.krylov is not None and self.krylov.ns >= 2 and
                     self._dev_control() and
                     len(th) == 2 and th[1] > th[0] and getattr(self.func, 'fold_dense', False))
        if not self.host:
            hv = st.dsc_np
            hv[0], hv[1] = th[0], th[-1]
            hv[2:].view(np.int64)[0] = sol[1].data_ptr() if self.fold else 0
            st.dsc.copy_(st.dsc_host, non_blocking=True)
        if self.fold:
            if lay is not None and st.drows_src is not lay.order32:
                if st.drows is None:
                    st.drows = torch.empty_like(lay.order32)
                st.drows.copy_(lay.order32)
                st.drows_src = lay.order32
        if self.host:
            sol[0].copy_(y0)
            bufs['Y'].copy_(y0)
        else:
            _entry_copy(y0, bufs['Y'], sol[0], lay.order if lay is not None else None)
        t0 = torch.tensor(th[0], dtype=torch.float64)
        dev_init = not self.host and getattr(self.func, 'autonomous', False) and 'norm' not in self.options
        # the initial-step selection's squared sums formed by the f0 and probe launches themselves
        # (an affine RHS: the probe is the linear part on f0), no passes over y0, f0, f1
        self.init_rows = (INIT_ROWS and dev_init and self.affine and self._scalars['first_step'] is None)
        self.lin_init = (LIN_INIT and not self.init_rows and dev_init and self.krylov is not None and
                         self.krylov.ns >= 3 and self._scalars['first_step'] is None)
        dt_read = None  # the device initial step's reader: the first step is enqueued before it is read
        if self.init_rows:
            if st.rows2 is None:
                st.rows2 = torch.empty_like(st.rows)
                st.iws = torch.empty(_lib.fn("gnpde_initial_step_workspace_bytes")(), dtype=torch.uint8,
                                     device=dev)
            # f0 into K0 with the rows sum (f0 / scale)^2 (err) and sum (y0 / scale)^2 (scale_rows),
            # scale = atol + rtol |y0| (err_y1 = -2)
            self.func.rhs_stage(t0, bufs['Y'], ops.Stage(
                f_out=bufs['K0'], err=(st.rows, (None, 0.0, 1.0, []), bufs['Y'], -2, self.atol_f, self.rtol_f),
                scale_rows=st.rows2))
        elif dev_init and self.lin_init and self._prologue(st, graphs_ok, t0):
            dt_read = self._rec_reader(st, st.h, slot=2)  # f0 and the initial step replayed
        elif dev_init:  # f0 straight into K0 (the RHS epilogue's f_out)
            self.func.rhs_stage(t0, bufs['Y'], ops.Stage(f_out=bufs['K0']))
        else:
            f0 = self.func(t0, bufs['Y'])
            bufs['K0'].copy_(f0)
        dt_on_device = False
        if self._scalars['first_step'] is None:
            if dev_init:
                if dt_read is None:
                    dt_read = self._initial_step_device(st, t0)
                dt = None
                dt_on_device = True  # st.dt and st.scale hold it already
            else:
                dt = float(self._select_initial_step(t0.to(dev) if not self.host else t0, bufs['K0']))
        else:
            dt = float(self._scalars['first_step'])
        t_cur = th[0]
        last = None  # (t_prev, dt) of the last accepted step
        self._dense = None
        order = float(P.order)
        safety, ifactor, dfactor = self.safety_f, self.ifactor_f, self.dfactor_f
        kn = 'K%d' % P.ns
        dev_ctl = self._dev_control()
        if dev_ctl and not dt_on_device:  # the device controller carries dt (and the scale) from step to step
            st.dt.fill_(dt)
            st.scale.fill_(dt)
        # Steps enqueued ahead (ADAPTIVE_SPEC): while the host waits for step n's record, step
        # n+1 already runs on the binding an acceptance gives, from the device controller's dt.
        # A third y / f0 buffer keeps step n's inputs intact, so a rejection only discards the
        # step ahead (its RHS evaluations are not counted) and restores dt on the device.
        # In this mode every step keeps its dense-output k's (one variant per binding, so a
        # solve replays three captured graphs): whether a step crosses an output time is
        # known only once its dt is read.
        spec_ok = dev_ctl and graphs_ok and ADAPTIVE_SPEC and P.fsal
        if spec_ok and 'Ys' not in bufs:
            bufs['Ys'], bufs['Ks'] = torch.empty_like(bufs['Y']), torch.empty_like(bufs['K0'])
        if st.canon is None or len(st.canon) < len(bufs):  # (no step has rotated them in this solve yet)
            st.canon = dict(bufs)
        pending = None  # the record reader of the step enqueued ahead: the current step
        pre_interp = None  # (output index, t0, dt) of a dense output enqueued ahead of its step's record
        if dt_read is not None:
            if spec_ok and th[-1] > th[0]:  # the first step runs while the host waits for its size
                pending = self._rec_reader(st, self._run_step(st, graphs_ok, t_cur, 0.0, True))
            dt = dt_read()[2]
        for i_out in range(1, len(th)):
            next_t = th[i_out]
            while next_t > t_cur:
                if not (t_cur + dt > t_cur):
                    raise AssertionError('underflow in dt {}'.format(dt))
                if self.n_steps >= self.max_num_steps:
                    raise AssertionError('max_num_steps exceeded ({}>={})'.format(self.n_steps, self.max_num_steps))
                mid = t_cur + dt >= next_t  # an accepted step would cross an output time: keep the dense-output k's
                if pending is not None:
                    read, pending = pending, None
                else:
                    if not dev_ctl:
                        st.scale.fill_(dt)
                    err = self._run_step(st, graphs_ok, t_cur, dt, mid or spec_ok)
                    read = self._rec_reader(st, err) if dev_ctl else None
                ahead = None
                # ahead only after a step whose k's the dense output does not need (the step ahead
                # overwrites them); it keeps its own (mid variant: its dt is not known yet)
                if spec_ok and st.warm and not mid and self.n_steps + 1 < self.max_num_steps and \
                        _nfe_headroom(self.func, 2 * P.ns):
                    self._rotate(bufs, kn, 1)
                    ahead = self._rec_reader(st, self._run_step(st, graphs_ok, t_cur + dt, dt, True))
                # the step crossing next_t (steps-ahead mode, its k's kept): its dense output is
                # enqueued before its record is read, so the pass follows the step on the device
                # without the host's round trip; used if the step is accepted (a rejected step's
                # successor writes the output again)
                if spec_ok and mid and ahead is None and t_cur + dt > next_t and not self.fold:
                    self._dense = dict(bufs, scale=dt)
                    self._interp_into(sol[i_out], (t_cur, dt), next_t, t_cur + dt, lay)
                    pre_interp = (i_out, t_cur, dt)
                dt_next = None
                if dev_ctl:
                    ratio, _dt, dt_next, _e2 = read()  # the one host read of the step
                elif err.dim() == 0:
                    ratio = math.sqrt(float(err) / (y0.numel()))  # the one host read of the step
                else:
                    e2, n = (float(v) for v in err.tolist())
                    ratio = math.sqrt(e2 / n) if n > 0 else 0.0
                if ratio <= 1:
                    t_prev, t_cur = t_cur, t_cur + dt
                    last = (t_prev, dt)
                    # a step that crossed an output time keeps its operands for the dense output (the
                    # references as they are now; the buffers are only rewritten by the next step)
                    self._dense = dict(bufs, scale=dt) if mid else None
                    if ahead is not None:
                        pending = ahead  # already on the accepted binding
                    else:
                        self._rotate(bufs, kn, 1)
                elif ahead is not None:  # rejected: discard the step ahead, step n again from its inputs
                    self._rotate(bufs, kn, -1)
                    st.dt.fill_(dt_next)
                    st.scale.fill_(dt_next)
                    st.tdev[0].fill_(t_cur)  # (the discarded step's controller may have advanced it)
                    if hasattr(self.func, 'nfe'):
                        self.func.nfe -= P.ns
                if dt_next is not None:
                    dt = dt_next
                elif ratio == 0:
                    dt = dt * ifactor
                else:
                    df = 1.0 if ratio < 1 else dfactor
                    dt = dt * min(ifactor, max(safety / ratio ** (1.0 / order), df))
                self.n_steps += 1
            if next_t == t_cur or last is None:
                if self.host:
                    sol[i_out].copy_(bufs['Y'])
                else:
                    _to_user(bufs['Y'], sol[i_out], lay)
            elif pre_interp != (i_out,) + tuple(last) and not self.fold:  # (not already enqueued / folded)
                self._interp_into(sol[i_out], last, next_t, t_cur, lay)
        return sol

    def _interp_into(self, out, last, t, t1, lay=None):
        """torchdiffeq's 4th-order dense output (_interp_fit / _interp_evaluate, with the
        tableau's mid-point coefficients) of the last accepted step at time t:
        y_mid = y0 + dt sum_j c_mid[j] k_j, then the polynomial, a combination of y0,
        y1, y_mid, f0 and f1 — folded into ONE stage pass over y0 (its base), f1 (its
        f input) and the other rows as operands (y_mid substituted), stored in the
        caller's numbering (out_rows); two passes when the operands exceed the
        stage's table."""
        P = self.plan
        t0, dt = last
        d = self._dense
        if d is None:
            raise RuntimeError("gnpde: dense output of a step whose stage derivatives were not kept")
        y_prev, y_cur = d['Y'], d['Y1']
        f0, f1 = d['K0'], d['K%d' % P.ns]
        x = (t - t0) / (t1 - t0)
        x2, x3, x4 = x * x, x * x * x, x * x * x * x
        cy0 = 1.0 - 11.0 * x2 + 18.0 * x3 - 8.0 * x4
        cy1 = -5.0 * x2 + 14.0 * x3 - 8.0 * x4
        cym = 16.0 * x2 - 32.0 * x3 + 16.0 * x4
        cf0 = dt * (x - 4.0 * x2 + 5.0 * x3 - 2.0 * x4)
        cf1 = dt * (x2 - 3.0 * x3 + 2.0 * x4)
        rows = None if (lay is None or self.host) else lay.order32
        K = self.krylov
        if K is not None:
            # y1 and y_mid restated on the u_p (K0 .. K{ns-1}): one pass over y0, the u_p and f1
            terms = []
            for p in range(P.ns):
                c = cy1 * dt * K.G[p] + cym * dt * K.Mu[p] + (cf0 if p == 0 else 0.0)
                if c != 0.0:
                    terms.append((d['K%d' % p], c))
            stage = ops.Stage(outs=[(out, y_prev, cy0 + cy1 + cym, cym * dt * P.c_mid[P.ns] + cf1, terms)],
                              out_rows=rows)
            if self.host:
                self.func.host_stage_apply(stage, f1, y_prev, y_prev)
            else:
                ops.stage_apply(stage, f1, y_prev, y_prev)
            return
        # one pass: out = (cy0 + cym) y0 + cy1 y1 + sum_j cym dt c_mid[j] k_j + cf0 f0 + cf1 f1
        coef = {}  # id -> [tensor, coefficient] of the operands besides y0 (base) and f1 (f input)
        order_ = []

        def add(tn, c):
            if c == 0.0:
                return
            if id(tn) not in coef:
                coef[id(tn)] = [tn, 0.0]
                order_.append(id(tn))
            coef[id(tn)][1] += c
        add(y_cur, cy1)
        for j in range(P.ns + 1):
            if _nz(P.c_mid[j]):
                add(d['K%d' % j] if j < P.ns else f1, cym * dt * P.c_mid[j])
        add(f0, cf0)
        cf_f1 = coef.pop(id(f1))[1] + cf1 if id(f1) in coef else cf1
        terms = [tuple(coef[k]) for k in order_ if k in coef]
        if len(terms) <= _lib.STAGE_MAX_K and (not self.host or hasattr(self.func, 'host_stage_apply')):
            stage = ops.Stage(outs=[(out, y_prev, cy0 + cym, cf_f1, terms)], out_rows=rows)
            if self.host:
                self.func.host_stage_apply(stage, f1, y_prev, y_prev)
            else:
                ops.stage_apply(stage, f1, y_prev, y_prev)
            return
        ymid = torch.empty_like(out)
        mterms = [(d['K%d' % j], dt * P.c_mid[j]) for j in range(P.ns + 1) if _nz(P.c_mid[j])]
        self._apply(ops.Stage(outs=[(ymid, y_prev, 1.0, 0.0, mterms)]), None, None, y_prev)
        self._apply(ops.Stage(outs=[(out, y_prev, cy0, 0.0, [(y_cur, cy1), (ymid, cym), (f0, cf0), (f1, cf1)])],
                              out_rows=rows), None, None, y_prev)


def adaptive_step_graph(func):
    """A captured fused adaptive step of ``func`` (the last solve's cache entry), or
    None: replaying it re-runs one whole step (its launches, the error reduction and
    the device controller) on the buffers it was captured with — the measurement hook
    of bench.py's dopri5 line and tools/pmc_run.py (not part of a solve)."""
    hit = _ADAPTIVE_CACHE.get(func)
    if hit is None or not hit[1].graphs:
        return None
    # a step like most of a solve's: not the first attempt after a lin_init probe (key[-1])
    ents = [e for k, e in hit[1].graphs.items() if not k[-1]] or list(hit[1].graphs.values())
    return ents[0][0]


def odeint(func, y0, t, rtol=1e-7, atol=1e-9, method=None, options=None, combine=None):
    """torchdiffeq.odeint(func, y0, t, rtol, atol, method, options) -> [len(t), *y0.shape]."""
    method = method or 'dopri5'
    options = dict(options or {})
    if combine is None:
        if not y0.is_cuda:
            raise RuntimeError("gnpde.odeint: y0 must be a ROCm device tensor (stage combinations run in HIP)")
        combine = _Combine()
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t)
    if t.dim() != 1 or len(t) < 2:
        raise ValueError("t must be a 1-D tensor with at least two time points")
    if method in FIXED_METHODS:
        return odeint_fixed(func, y0, t, method, options.get('step_size'), combine, graph=options.get('gnpde_graph'))
    if method in ADAPTIVE_METHODS:
        kw = dict(method=method, first_step=options.get('first_step'),
                  max_num_steps=options.get('max_num_steps', 2 ** 31 - 1), norm=options.get('norm', _rms_norm))
        if _fused_adaptive_ok(func, y0, combine, options):
            solver = _RKAdaptiveFused(func, y0, rtol, atol, combine, options=options, **kw)
            odeint.last_path = 'fused_krylov' if solver.krylov is not None else 'fused_stage'
        elif _adaptive_backprop_ok(func, y0, combine, options):
            # backprop through the adaptive solve of the Laplacian as one node (gnpde.adaptive_backprop)
            w, _ = func._weights_tensor()
            out = _LaplacianAdaptiveFn.apply(y0, func.alpha_train, func.beta_train, w, func, _host_times(t), method,
                                             rtol, atol, options.get('first_step'), kw['max_num_steps'])
            odeint.last_path = 'fused_backprop'
            odeint.last_dense_fold = False
            return out
        else:
            solver = _RKAdaptive(func, y0, rtol, atol, combine, **kw)
            odeint.last_path = 'restated'
        out = solver.integrate(t)
        odeint.last_n_steps = solver.n_steps
        odeint.last_dense_fold = bool(getattr(solver, 'fold', False))
        return out
    raise NotImplementedError("gnpde.odeint: method %r not supported (supported: %s)" %
                              (method, ', '.join(FIXED_METHODS + ADAPTIVE_METHODS)))


odeint.last_n_steps = 0
odeint.last_path = None  # the last adaptive solve's loop: 'fused_krylov', 'fused_stage' or 'restated'
odeint.last_dense_fold = False  # whether its dense output was folded into the steps (DENSE_FOLD)


# --------------------------------------------------------------------------- adjoint
def _mixed_norm_fn(sizes):
    """torchdiffeq's norm for tuple states (max over the components of their RMS
    norms), applied to the flattened augmented state [y | adj_y | adj_params...]."""
    bounds = []
    o = 0
    for n in sizes:
        bounds.append((o, o + n))
        o += n

    def norm(z):
        return torch.stack([_rms_norm(z[a:b]) for a, b in bounds if b > a]).max()
    return norm


def _laplacian_aug(func, params, y_shape, ny, ans):
    """The augmented RHS of _OdeintAdjoint for the Laplacian (src/function_laplacian_diffusion.py,
    f = sigma(alpha)(A y - y) [+ beta x0]) without autograd: per evaluation two K1 launches
    and at most one dot,
        dy/ds     = -f(y)                          K1 over the CSR, its epilogue storing -f
        da/ds     = L^T a                          K1 over the CSC (L = sigma(alpha)(A - I))
        dalpha/ds = (1 - sigma(alpha)) <L^T a, y>  fp64 row terms in that launch's epilogue
        dbeta/ds  = <a, x0>                        (add_source) one fp64 dot
    written into one output buffer in the packed layout [y | a | params]; the other
    parameters' components are 0.  For the adaptive adjoint methods (torchdiffeq's
    solver loop, the mixed norm); the fixed-grid rk4 adjoint runs _LaplacianAdjointFn.
    None when the RHS is not the HIP Laplacian on a device fp32 state."""
    fn = getattr(func, 'adjoint_direct_ok', None)
    if not (FUSED_ADJOINT and fn is not None and fn(params) and hasattr(func, 'rhs_stage')) or \
            func.opt.get('no_alpha_sigmoid', False) or not ans.is_cuda or ans.dtype != torch.float32 or \
            len(y_shape) != 3:
        return None
    own = {id(p) for p in func.parameters()}
    if not all(id(p) in own for p in params):
        return None
    y0 = ans[0]
    g = func.graph_for(y0)
    w, tag = func._weights_tensor()
    w_csr = func.csr_weights(g, w, tag)
    w_csc = g.gather_weights(w.detach().float() if w.dtype != torch.float32 else w.detach(), transpose=True)
    add_source = bool(func.opt.get('add_source', False))
    x0 = func.stable_x0(y0) if add_source else None
    alpha, beta = func.alpha_train.detach(), func.beta_train.detach()
    R = y0.numel() // y0.shape[-1]
    drow = torch.empty(R, dtype=torch.float64, device=y0.device)
    slots = {}
    o = 2 * ny
    for p in params:
        slots[id(p)] = (o, p.numel())
        o += p.numel()

    def aug(s, z):
        # one RHS evaluation per augmented one, as torchdiffeq's backward calls func (and its guard)
        if func.nfe > func.opt["max_nfe"]:
            raise MaxNFEException
        func.nfe += 1
        y = z[:ny].view(y_shape)
        a = z[ny:2 * ny].view(y_shape)
        out = torch.empty_like(z)
        ops.spmm_rhs(g, w_csr, y, x0=x0, alpha=alpha, beta=beta, rhs=True, alpha_sigmoid=True,
                     add_source=add_source, stage=ops.Stage(outs=[(out[:ny].view(y_shape), None, 0.0, -1.0, [])]))
        ops.spmm_rhs(g, w_csc, a, alpha=alpha, rhs=True, alpha_sigmoid=True, transpose=True,
                     stage=ops.Stage(outs=[(out[ny:2 * ny].view(y_shape), None, 0.0, 1.0, [])],
                                     dot=(y, drow, 1.0, False)))
        out[2 * ny:].zero_()
        if id(func.alpha_train) in slots:
            oa, _ = slots[id(func.alpha_train)]
            ga = ops.sum_f64(drow) * (1.0 - torch.sigmoid(alpha.double()))
            out[oa:oa + 1].copy_(ga.reshape(1))
        if add_source and id(func.beta_train) in slots:
            ob, _ = slots[id(func.beta_train)]
            out[ob:ob + 1].copy_(ops.dot(a, x0).reshape(1))
        return out
    return aug


FUSED_ADAPTIVE_ADJOINT = os.environ.get('GNPDE_FUSED_ADAPTIVE_ADJOINT', '1') != '0'


def _adaptive_adjoint_ok(func, ans, a_method, params, a_options):
    """The adaptive adjoint of a Laplacian RHS runs fused (gnpde.adjoint_adaptive): an
    adaptive adjoint method with torchdiffeq's default adjoint norm (no user 'norm'),
    a device fp32 state, weights that are not adjoint parameters, the sigmoid alpha,
    and adjoint parameters among the module's own."""
    if not (FUSED_ADJOINT and FUSED_ADAPTIVE_ADJOINT and a_method in ADAPTIVE_METHODS) or \
            'norm' in (a_options or {}):
        return False
    if not (ans.is_cuda and ans.dtype == torch.float32 and ans.dim() == 4):
        return False
    fn = getattr(func, 'adjoint_direct_ok', None)
    if fn is None or not fn(params) or func.opt.get('no_alpha_sigmoid', False) or not hasattr(func, 'rhs_stage'):
        return False
    own = {id(p) for p in func.parameters()}
    return all(id(p) in own for p in params)


class _OdeintAdjoint(torch.autograd.Function):
    """torchdiffeq.odeint_adjoint (0.2.x OdeintAdjointMethod) restated: the
    forward integrates without recording; the backward integrates the augmented
    system (y, a_y, a_theta) from t[-1] back to t[0] with
        dy/dt = f,  da_y/dt = -a_y^T df/dy,  da_theta/dt = -a_y^T df/dtheta
    (vector-Jacobian products through the RHS autograd: K1 over the CSC, the
    SDDMM and the attention backward), adding the output gradient at every
    requested time.  Time runs backwards by integrating in s = -t."""

    @staticmethod
    def forward(ctx, y0, t, cfg, *params):
        func, rtol, atol, method, options = cfg[:5]
        with torch.no_grad():
            ans = odeint(func, y0, t, rtol=rtol, atol=atol, method=method, options=options)
        ctx.cfg = cfg
        ctx.params = params  # the leaf parameters themselves: the VJPs are taken with respect to them
        ctx.save_for_backward(t, ans)
        return ans

    @staticmethod
    def backward(ctx, grad_y):
        func, _rtol, _atol, _method, _options, a_rtol, a_atol, a_method, a_options = ctx.cfg
        t, ans = ctx.saved_tensors
        params = ctx.params
        if _adaptive_adjoint_ok(func, ans, a_method, params, a_options):
            # the Laplacian's adaptive adjoint, fused (gnpde.adjoint_adaptive): the same loop with the
            # packed state's stage combinations, error rows and alpha integrand in the K1 epilogues
            from .adjoint_adaptive import AdaptiveAdjoint
            with torch.no_grad():
                solver = AdaptiveAdjoint(func, params, a_method, a_rtol, a_atol, a_options)
                gy, pg = solver.run(_host_times(t), ans, grad_y)
            _OdeintAdjoint.last_path = 'fused_adaptive'
            out = []
            for p in params:
                v = pg.get(id(p))
                out.append(torch.zeros_like(p) if v is None else
                           torch.full(p.shape, v, dtype=p.dtype, device=p.device))
            return (gy.view(grad_y.shape[1:]).to(grad_y.dtype), None, None) + tuple(out)
        y_shape = ans.shape[1:]
        ny = ans[0].numel()
        sizes = [ny, ny] + [p.numel() for p in params]

        def pack(y, ay, ap):
            return torch.cat([y.reshape(-1).float(), ay.reshape(-1).float()] + [a.reshape(-1).float() for a in ap])

        def aug_autograd(s, z):
            y = z[:ny].view(y_shape)
            ay = z[ny:2 * ny].view(y_shape)
            with torch.enable_grad():
                yv = y.detach().requires_grad_(True)
                f = func(-s, yv)
                grads = torch.autograd.grad(f, (yv,) + tuple(params), -ay, allow_unused=True)
            vjp_y = grads[0] if grads[0] is not None else torch.zeros_like(y)
            vjp_p = [torch.zeros_like(p) if g is None else g for g, p in zip(grads[1:], params)]
            return -pack(f.detach(), vjp_y, vjp_p)  # d/ds = -d/dt

        # the Laplacian's vector-Jacobian products by K1 launches (no autograd), else autograd's
        aug = _laplacian_aug(func, params, y_shape, ny, ans)
        _OdeintAdjoint.last_path = 'direct_aug' if aug is not None else 'autograd'
        aug = aug or aug_autograd
        opts = dict(a_options or {})
        if a_method in ADAPTIVE_METHODS and 'norm' not in opts:
            opts['norm'] = _mixed_norm_fn(sizes)
        ay = grad_y[-1]
        ap = [torch.zeros_like(p) for p in params]
        # weights the RHS closes over are constants of the backward (torchdiffeq: VJPs w.r.t. y and
        # adjoint_params only): the autograd VJPs see them detached
        const_w = hasattr(func, 'adjoint_const_weights') and func.adjoint_direct_ok(params)
        try:
            if const_w:
                func.adjoint_const_weights = True
            with torch.no_grad():
                for i in range(len(t) - 1, 0, -1):
                    z0 = pack(ans[i], ay, ap)
                    s = torch.stack([-t[i], -t[i - 1]])
                    z1 = odeint(aug, z0, s, rtol=a_rtol, atol=a_atol, method=a_method, options=opts)[1]
                    ay = z1[ny:2 * ny].view(y_shape).to(grad_y.dtype) + grad_y[i - 1]
                    o = 2 * ny
                    ap = []
                    for p in params:
                        ap.append(z1[o:o + p.numel()].view(p.shape).to(p.dtype))
                        o += p.numel()
        finally:
            if const_w:
                func.adjoint_const_weights = False
        return (ay, None, None) + tuple(ap)


_OdeintAdjoint.last_path = None  # which backward the last one ran: 'fused_adaptive', 'direct_aug' or 'autograd'


# Fused continuous adjoint of the Laplacian RHS (src/base_classes.py:45-49 with opt['adjoint'],
# src/block_constant.py:34-44: odeint_adjoint with adjoint_method / adjoint_step_size; the
# ogbn-arxiv and Photo best_params run adjoint_method 'rk4', src/best_params.py:6-7).
FUSED_ADJOINT = os.environ.get('GNPDE_FUSED_ADJOINT', '1') != '0'


class _AdjointRHS(object):
    """The adjoint component of the augmented system in s = -t, a' = L^T a with
    L = sigma(alpha)(A - I): K1 over the CSC with the RHS epilogue, whose dot term
    adds coef_i <o_i, y_i> (o_i = L^T a_i, y_i the y component's input at the same
    stage) per row in fp64 — the alpha gradient's integrand sigma'(alpha)<(A^T - I)a, y>
    up to the factor (1 - sigma(alpha)) applied once at the end."""

    def __init__(self, gr, w_csc, alpha, sig, drow):
        self.gr, self.w_csc, self.alpha, self.sig, self.drow = gr, w_csc, alpha, sig, drow
        self.ys, self.coefs, self.i = None, None, 0

    def begin_step(self, ys, coefs):
        self.ys, self.coefs, self.i = ys, coefs, 0

    def rhs_stage(self, t, x, stage):
        stage.dot = (self.ys[self.i], self.drow, self.coefs[self.i], True)
        self.i += 1
        ops.spmm_rhs(self.gr, self.w_csc, x, alpha=self.alpha, rhs=True, alpha_sigmoid=self.sig, transpose=True,
                     stage=stage)


def _fused_adjoint_ok(func, y0, adjoint_method, adjoint_params):
    """odeint_adjoint of a Laplacian RHS with a fixed-grid rk4 adjoint runs fused
    (_LaplacianAdjointFn): a device fp32 state, weights without their own gradient,
    the sigmoid alpha, and adjoint parameters among the module's own."""
    if not (FUSED_ADJOINT and adjoint_method == 'rk4' and y0.is_cuda and y0.dtype == torch.float32 and
            y0.dim() == 3):
        return False
    fn = getattr(func, 'adjoint_direct_ok', None)
    if fn is None or not fn(adjoint_params) or func.opt.get('no_alpha_sigmoid', False) or \
            not hasattr(func, 'rhs_stage'):
        return False
    own = {id(p) for p in func.parameters()}
    return all(id(p) in own for p in adjoint_params)


class _LaplacianAdjointFn(torch.autograd.Function):
    """torchdiffeq.odeint_adjoint (0.2.x OdeintAdjointMethod) of f(y) = sigma(alpha)(A y - y)
    [+ beta x0] with a fixed-grid rk4 adjoint, fused.  Forward: the no-grad solve
    (the fused adaptive step for dopri5).  Backward, per interval [t_{i-1}, t_i] from
    the last, the augmented system integrated over s = -t with torchdiffeq's grid
    (adjoint_options step_size) exactly as torchdiffeq does — y restarts from the
    forward solution at t_i and is integrated backwards too:
        dy/ds = -f(y)                      a fused rk4 step of f with dt = -h
        da/ds = L^T a                      a fused rk4 step over the CSC (_AdjointRHS)
        d alpha/ds = sigma'(alpha) <(A^T - I) a, y>   row terms in the CSC epilogues (dot_rows)
        d beta/ds  = <a, x0>               (add_source) fp64 dots of the stage inputs
    and a += grad_y[i-1] at each output time.  Eight K1 launches per rk4 step, the
    stage combinations in their epilogues, the state in the graph's in-degree
    numbering; the parameter gradients summed once at the end.  The RHS counter
    advances by one per augmented evaluation, as torchdiffeq's backward calls func."""

    @staticmethod
    def forward(ctx, y0, t, cfg, *params):
        func, rtol, atol, method, options = cfg[:5]
        with torch.no_grad():
            ans = odeint(func, y0, t, rtol=rtol, atol=atol, method=method, options=options)
        ctx.cfg = cfg
        ctx.params = params
        ctx.save_for_backward(t, ans)
        return ans

    @staticmethod
    def backward(ctx, grad_y):
        func = ctx.cfg[0]
        a_options = ctx.cfg[8] or {}
        t, ans = ctx.saved_tensors
        params = ctx.params
        t_h = _host_times(t)
        grad_y = grad_y.contiguous()
        with torch.no_grad():
            lay = _node_layout(func, ans[0])
            if lay is not None:
                func._layout = lay
            try:
                gr = func.graph_for(ans[0])
                w, tag = func._weights_tensor()
                w_csc = gr.gather_weights(w.detach().float() if w.dtype != torch.float32 else w.detach(),
                                          transpose=True)
                R = ans[0].numel() // ans[0].shape[-1]
                acc = torch.zeros(1 + R, dtype=torch.float64, device=ans.device)
                gb, drow = acc[0], acc[1:]
                add_source = bool(func.opt.get('add_source', False))
                x0 = func.stable_x0(ans[0]) if add_source else None
                arhs = _AdjointRHS(gr, w_csc, func.alpha_train.detach(), True, drow)
                step = a_options.get('step_size')

                def internal(v):
                    if lay is None:
                        return v.clone()
                    return _to_internal(v, lay)
                a = internal(grad_y[-1])
                ws_y, ws_a = _Workspace(), _Workspace()
                ybuf = [torch.empty_like(a), torch.empty_like(a)]
                abuf = [torch.empty_like(a), torch.empty_like(a)]
                for i in range(len(t_h) - 1, 0, -1):
                    y = internal(ans[i])
                    # torchdiffeq's grid of the flipped interval, in t's dtype (as its fixed-grid solver)
                    s_t = torch.tensor([-t_h[i], -t_h[i - 1]], dtype=t.dtype)
                    grid = (fixed_grid(s_t, float(step)) if step is not None else s_t).tolist()
                    for sa, sb in zip(grid[:-1], grid[1:]):
                        h = sb - sa
                        if h == 0.0:
                            continue
                        yo = ybuf[0] if ybuf[0] is not y else ybuf[1]
                        ao = abuf[0] if abuf[0] is not a else abuf[1]
                        _fused_step('rk4', func, -sa, -h, -sb, y, ws_y, out=yo)
                        ys = [y, ws_y['a'], ws_y['b'], ws_y['c']]
                        arhs.begin_step(ys, [h / 8.0, 3.0 * h / 8.0, 3.0 * h / 8.0, h / 8.0])
                        _fused_step('rk4', arhs, sa, h, sb, a, ws_a, out=ao)
                        if add_source:  # d beta/ds = <a, x0> at the four stages
                            for c, av in zip((1.0, 3.0, 3.0, 1.0), (a, ws_a['a'], ws_a['b'], ws_a['c'])):
                                gb = gb + (c * h / 8.0) * ops.dot(av, x0)
                        y, a = yo, ao
                    a = a + internal(grad_y[i - 1])
                sig = torch.sigmoid(func.alpha_train.detach()).double()
                ga = ops.sum_f64(drow) * (1.0 - sig)
                if lay is not None:
                    gy = torch.empty_like(a)
                    _to_user(a, gy, lay)
                else:
                    gy = a
            finally:
                func._layout = None
        out = []
        for p in params:
            if p is func.alpha_train:
                out.append(ga.to(p.dtype).reshape(p.shape))
            elif p is func.beta_train and add_source:
                out.append(gb.to(p.dtype).reshape(p.shape))
            else:
                out.append(torch.zeros_like(p))
        return (gy.view(grad_y.shape[1:]), None, None) + tuple(out)


def odeint_adjoint(func, y0, t, rtol=1e-7, atol=1e-9, method=None, options=None, adjoint_rtol=None,
                   adjoint_atol=None, adjoint_method=None, adjoint_options=None, adjoint_params=None):
    """torchdiffeq.odeint_adjoint(func, y0, t, ...) with its defaults: the adjoint
    tolerances / method default to the forward ones, adjoint_options to the
    forward options (without 'norm') when the methods match, adjoint_params to
    func's parameters that require grad.  Gradients reach y0 and adjoint_params
    (as in torchdiffeq, not other tensors the RHS closes over)."""
    method = method or 'dopri5'
    if adjoint_params is None:
        adjoint_params = tuple(p for p in func.parameters() if p.requires_grad)
    adjoint_params = tuple(adjoint_params)
    adjoint_rtol = rtol if adjoint_rtol is None else adjoint_rtol
    adjoint_atol = atol if adjoint_atol is None else adjoint_atol
    adjoint_method = method if adjoint_method is None else adjoint_method
    if adjoint_options is None:
        adjoint_options = {k: v for k, v in (options or {}).items() if k != 'norm'} if adjoint_method == method \
            else {}
    if not isinstance(t, torch.Tensor):
        t = torch.as_tensor(t)
    cfg = (func, rtol, atol, method, options, adjoint_rtol, adjoint_atol, adjoint_method, adjoint_options)
    if _fused_adjoint_ok(func, y0, adjoint_method, adjoint_params):
        return _LaplacianAdjointFn.apply(y0, t, cfg, *adjoint_params)
    return _OdeintAdjoint.apply(y0, t, cfg, *adjoint_params)


__all__ = ['odeint', 'odeint_adjoint', 'fixed_grid', 'FIXED_METHODS', 'ADAPTIVE_METHODS', 'math']
