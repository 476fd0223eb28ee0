"""The dense output of a one-output-time Krylov dopri5 solve folded into the steps'
last launch (ABI 8 gnpde_stage_epilogue_t.dense_out, integrator.DENSE_FOLD; reference
anchor src/block_constant.py:46-51 — ODEblock.forward integrates to its one output
time self.t[1] and torchdiffeq interpolates there).  The launch that writes y1, f1 and
the error rows also writes torchdiffeq's 4th-order interpolant at the output time
straight into sol[1] (in the caller's numbering) when the device time the controller
advances says the step crosses it.

Checked against the separate dense-output pass (GNPDE_DENSE_FOLD=0): the same step
sequence, values within fp32 rounding of it (the coefficients are formed in fp64 on
the device instead of the host, then rounded to fp32); against the oracle's float64
restatement of torchdiffeq's loop with its step count; replayed solves bit-equal to
the first; rejected steps (and discarded steps ahead) never leave their interpolant."""
import numpy as np
import pytest
import torch

import gnpde_oracle as O
from gnpde import integrator as gi, ops

from test_gpu_adaptive import DEV, RTOL, T, _graph, _laplacian, rel

pytestmark = pytest.mark.gpu


def _solve(func, x, ts, rtol, atol, opts=None):
    tt = torch.tensor(ts, dtype=torch.float64, device=DEV)
    with torch.no_grad():
        z = gi.odeint(func, T(x), tt, rtol=rtol, atol=atol, method='dopri5', options=opts or {})
    torch.cuda.synchronize()
    return z.clone(), gi.odeint.last_n_steps, gi.odeint.last_dense_fold, gi.odeint.last_path


@pytest.mark.parametrize("layout", [False, True])
@pytest.mark.parametrize("add_source", [False, True])
@pytest.mark.parametrize("rtol,T1", [(1e-3, 1.7), (1e-5, 2.3), (3e-2, 4.0)])
def test_dense_fold_vs_pass_and_oracle(monkeypatch, layout, add_source, rtol, T1):
    N, E, C = 4000, 40000, 64
    eo, wo, rng = _graph(N, E, 41)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    x0 = rng.standard_normal((1, N, C)).astype(np.float32)
    if layout:
        monkeypatch.setattr(ops, "LAYOUT_MIN_ROWS", 1)
        monkeypatch.setattr(ops, "LAYOUT_MIN_BYTES", 1)
    ts = [0.0, T1]
    res = {}
    for fold in (False, True):
        monkeypatch.setattr(gi, "DENSE_FOLD", fold)
        func = _laplacian(C, eo, wo, alpha=0.3, add_source=add_source, x0=T(x0) if add_source else None)
        if layout:
            assert func.node_layout(T(x)) is not None
        runs = [_solve(func, x, ts, rtol, rtol * 0.1) for _ in range(3)]  # eager, captured, replayed
        for z, n, f, path in runs:
            assert path == 'fused_krylov' and f == fold
        assert all(torch.equal(runs[0][0], r[0]) and runs[0][1] == r[1] for r in runs[1:])
        res[fold] = runs[0]
    (zp, npass, _, _), (zf, nfold, _, _) = res[False], res[True]
    assert nfold == npass
    assert torch.equal(zf[0], zp[0])
    assert rel(zf[1], zp[1]) <= 1e-6
    f = lambda t, y: O.laplacian_rhs(eo, y, x0, 0.3, 0.4, edge_weight=wo, add_source=add_source)  # noqa: E731
    want, n_want = O.odeint_adaptive(f, x, ts, 'dopri5', rtol, rtol * 0.1)
    assert nfold == n_want
    assert rel(zf, want) <= RTOL


def test_dense_fold_rejections_and_steps_ahead(monkeypatch):
    """A large first step (options first_step) forces rejections right away, with the
    steps-ahead loop discarding a step already enqueued: the fold's output equals the
    pass's, and the device time restored on each rejection keeps later crossings right."""
    N, E, C = 3000, 30000, 32
    eo, wo, rng = _graph(N, E, 43)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    out = {}
    for fold in (False, True):
        monkeypatch.setattr(gi, "DENSE_FOLD", fold)
        func = _laplacian(C, eo, wo, alpha=2.0)
        runs = [_solve(func, x, [0.0, 3.0], 1e-6, 1e-7, {'first_step': 2.5}) for _ in range(2)]
        assert runs[1][2] == fold and torch.equal(runs[0][0], runs[1][0])
        out[fold] = runs[1]
    assert out[True][1] == out[False][1] and out[True][1] > 3
    assert rel(out[True][0][1], out[False][0][1]) <= 1e-6
    f = lambda t, y: O.laplacian_rhs(eo, y, None, 2.0, 0.0, edge_weight=wo)  # noqa: E731
    want, n_want = O.odeint_adaptive(f, x, [0.0, 3.0], 'dopri5', 1e-6, 1e-7, first_step=2.5)
    assert out[True][1] == n_want
    assert rel(out[True][0], want) <= RTOL


def test_dense_fold_only_for_one_output_time(monkeypatch):
    """Several output times keep the dense-output pass (the device predicate knows one
    output time); the fold is on by default for one."""
    N, E, C = 2000, 16000, 32
    eo, wo, rng = _graph(N, E, 47)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    func = _laplacian(C, eo, wo)
    _, _, f2, _ = _solve(func, x, [0.0, 0.4, 1.0], 1e-4, 1e-5)
    _, _, f1, _ = _solve(func, x, [0.0, 1.0], 1e-4, 1e-5)
    assert not f2 and f1


@pytest.mark.parametrize("path", ["rows", "lin"])
@pytest.mark.parametrize("add_source", [False, True])
@pytest.mark.parametrize("rtol", [1e-3, 1e-6])
def test_initial_step_from_launch_rows(monkeypatch, path, add_source, rtol):
    """The first step of an affine solve from the row sums of the f0 launch (err rows of f0
    and scale_rows of y0, tol = atol + rtol |y0|) and of the probe launch over L f0
    (integrator.INIT_ROWS, gnpde_initial_step_rows) against torchdiffeq's
    _select_initial_step restated in fp64 on the oracle's RHS (src/block_constant.py:46-51
    solves with the solver's default first step): within 1e-6 relative — the fp32 path
    (GNPDE_INIT_ROWS=0) forms (f1 - f0) / h0 in fp32, the rows path L f0 itself.  path 'lin'
    (integrator.LIN_INIT, the default): phase 0 beside the probe v = L f0 on a second stream,
    d2 = rms(v / scale) (gnpde_initial_step_lin_f32)."""
    N, E, C = 3000, 30000, 48
    eo, wo, rng = _graph(N, E, 53)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    x0 = rng.standard_normal((1, N, C)).astype(np.float32)
    func = _laplacian(C, eo, wo, alpha=0.7, add_source=add_source, x0=T(x0) if add_source else None)
    atol = rtol * 0.1
    monkeypatch.setattr(gi, "INIT_ROWS", path == "rows")
    monkeypatch.setattr(gi, "LIN_INIT", path == "lin")
    seen = {}
    orig = gi._RKAdaptiveFused._initial_step_device

    def spy(self, st, t0):
        read = orig(self, st, t0)
        seen['h'] = st.h.clone()
        seen['path'] = 'rows' if self.init_rows else ('lin' if self.lin_init else None)
        return read
    monkeypatch.setattr(gi._RKAdaptiveFused, "_initial_step_device", spy)
    _solve(func, x, [0.0, 0.5], rtol, atol)
    assert seen['path'] == path
    h = seen['h'].cpu().numpy()
    f = lambda y: O.laplacian_rhs(eo, y, x0, 0.7, 0.4, edge_weight=wo, add_source=add_source)  # noqa: E731
    y = x.astype(np.float64)
    f0 = f(y)
    sc = atol + np.abs(y) * rtol
    rms = lambda v: np.sqrt(np.mean(np.square(v)))  # noqa: E731
    d0, d1 = rms(y / sc), rms(f0 / sc)
    h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else 0.01 * d0 / d1
    d2 = rms((f(y + h0 * f0) - f0) / sc) / h0
    h1 = max(1e-6, h0 * 1e-3) if (d1 <= 1e-15 and d2 <= 1e-15) else (0.01 / max(d1, d2)) ** (1.0 / 5)
    want = min(100 * h0, h1)
    assert abs(h[0] - h0) <= 1e-6 * h0 and abs(h[1] - d1) <= 1e-6 * d1
    assert abs(h[2] - want) <= 1e-6 * want


@pytest.mark.parametrize("add_source", [False, True])
def test_lin_init_first_step_vs_probe_path(monkeypatch, add_source):
    """The first step after the lin_init probe (u_1 = dt v scaled in place, v = L f0 from
    the probe) against the probe path (GNPDE_LIN_INIT=0: probe f0 + h0 L f0, first step
    like the others): the same step count and NFE (the reused evaluation is counted, as
    torchdiffeq evaluates it), values within 1e-6 (the first step sizes differ by the
    fp32 cancellation the probe path carries), both within RTOL of the oracle; replayed
    solves bit-equal."""
    N, E, C = 4000, 40000, 64
    eo, wo, rng = _graph(N, E, 59)
    x = rng.standard_normal((1, N, C)).astype(np.float32)
    x0 = rng.standard_normal((1, N, C)).astype(np.float32)
    res = {}
    for lin in (False, True):
        monkeypatch.setattr(gi, "LIN_INIT", lin)
        func = _laplacian(C, eo, wo, alpha=0.3, add_source=add_source, x0=T(x0) if add_source else None)
        runs = []
        for _ in range(3):
            n0 = func.nfe
            z, n, _, path = _solve(func, x, [0.0, 2.0], 1e-4, 1e-5)
            runs.append((z, n, func.nfe - n0))
        assert torch.equal(runs[1][0], runs[2][0]) and runs[1][1:] == runs[2][1:]
        res[lin] = runs[2]
    assert res[True][1] == res[False][1] and res[True][2] == res[False][2]
    assert rel(res[True][0], res[False][0]) <= 1e-6
    f = lambda t, y: O.laplacian_rhs(eo, y, x0, 0.3, 0.4, edge_weight=wo, add_source=add_source)  # noqa: E731
    want, n_want = O.odeint_adaptive(f, x, [0.0, 2.0], 'dopri5', 1e-4, 1e-5)
    assert res[True][1] == n_want
    assert rel(res[True][0], want) <= RTOL
