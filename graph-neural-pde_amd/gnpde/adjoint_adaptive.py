"""Fused adaptive adjoint of the Laplacian RHS.

Three of the reference's best_params train with an ADAPTIVE adjoint method
(src/best_params.py:3-5: Pubmed adaptive_heun — the reference's default
adjoint_method, src/run_GNN.py:334 —, CoauthorCS and Computers dopri5;
src/base_classes.py:45-49 and src/block_constant.py:34-44 pass adjoint_method,
adjoint_atol / adjoint_rtol from tol_scale_adjoint).  torchdiffeq's
odeint_adjoint (0.2.x OdeintAdjointMethod, not installed here: restated, parity
with it unpinned) integrates the augmented state [y | a | theta] from t[-1] back
to t[0] in s = -t with the same adaptive solver as the forward and the mixed norm
(the max over the components of their RMS norms).  For the Laplacian
f(y) = sigma(alpha)(A y - y) [+ beta x0] (src/function_laplacian_diffusion.py)
the augmented RHS is, with L = sigma(alpha)(A - I):

    dy/ds     = -f(y)                        K1 over the CSR with alpha -> -sigma(alpha), beta -> -beta
    da/ds     = L^T a                        K1 over the CSC
    dalpha/ds = (1 - sigma(alpha)) <L^T a, y>  the CSC launch's dot rows (ABI 7: beside its error rows)
    dbeta/ds  = <a, x0>                      (add_source) one fp64 dot per stage

and every other parameter's component has derivative 0 (so its value and error
stay 0).  integrator._OdeintAdjoint runs that as torchdiffeq does — a packed
[y | a | params] vector, torch stage combinations, per-component norms — at
~0.64 ms per augmented evaluation on G-arxiv, 0.45 of it solver glue.

This module runs the same loop (integrator._RKAdaptive: the tableau, the initial
step selection, the controller, the dense output) with the y and a halves kept in
one packed device state [2, B, N, C] and every stage combination in the K1
epilogues (integrator._AdaptivePlan: launch i of a step evaluates both halves at
stage input X_i and writes X_{i+1} and the error rows of its half; the CSC launch
adds the alpha integrand's rows <L^T a_i, y_i>).  The scalar components (alpha,
beta) are integrated on the host in fp64 from the per-stage sums: one segment-sum
launch per step reduces the two halves' error rows and the stages' alpha rows, and
the host reads that record once per step (accept / reject and the next dt, as
torchdiffeq's loop).  Step arithmetic: fp32 state, fp64 error norms and scalar
components (the restated loop runs every component in fp32).
"""
import math

import numpy as np
import torch

from . import ops
from .utils import MaxNFEException


def _f32(v):
    return float(np.float32(v))


class AdaptiveAdjoint(object):
    """The backward of odeint_adjoint for a LaplacianODEFunc with an adaptive
    adjoint method: ``run(t_h, ans, grad_y)`` -> (grad of y0, {id(param): grad})."""

    def __init__(self, func, params, method, rtol, atol, options=None):
        from . import integrator as gi
        self.gi = gi
        self.func, self.params = func, tuple(params)
        self.method = method
        self.plan = gi._adaptive_plan(method)
        self.order = float(self.plan.order)
        self.rtol, self.atol = float(rtol), float(atol)
        opts = dict(options or {})
        self.first_step = opts.get('first_step')
        self.max_num_steps = opts.get('max_num_steps', 2 ** 31 - 1)
        self.safety, self.ifactor, self.dfactor = 0.9, 10.0, 0.2
        self.n_steps = 0
        self.add_source = bool(func.opt.get('add_source', False))

    # ------------------------------------------------------------------ setup
    def _setup(self, y_like):
        gi, P, func = self.gi, self.plan, self.func
        C = y_like.shape[-1]
        packed = torch.empty((2,) + tuple(y_like.shape), dtype=torch.float32, device=y_like.device)
        st = gi._AdaptiveState(P, packed, False)
        self.bufs = st.bufs
        self.scale = st.scale
        R = y_like.numel() // C
        self.R, self.C, self.ny = R, C, y_like.numel()
        ns = P.ns
        # row channels: 0 / 1 the y / a error rows, 2 + j the alpha rows of stage derivative j
        self.rows = torch.zeros((3 + ns, R), dtype=torch.float64, device=y_like.device)
        # the step's record: the segment sums (3 + ns), the beta stage dots (ns + 1), the initial
        # step's squared sums (4: y / a halves, two each)
        self.nrec = 3 + ns + (ns + 1) + 4
        self.rec = torch.zeros(self.nrec, dtype=torch.float64, device=y_like.device)
        self.rec_host = torch.empty(self.nrec, dtype=torch.float64, pin_memory=True)
        g = func.graph_for(y_like)
        w, tag = func._weights_tensor()
        self.g = g
        self.w_csr = func.csr_weights(g, w, tag)
        self.w_csc = func.csr_weights(g, w, tag, transpose=True)
        self.x0 = func.stable_x0(y_like) if self.add_source else None
        alpha = func.alpha_train.detach()
        self.alpha = alpha.float().reshape(()).contiguous()
        # y-half: -f(y) = (-sigma(alpha))(A y - y) + (-beta) x0 from the same K1 (alpha taken as given)
        self.neg_sig = (-torch.sigmoid(alpha.float())).reshape(()).contiguous()
        self.neg_beta = (-func.beta_train.detach().float()).reshape(()).contiguous()
        self.one_minus_sig = 1.0 - 1.0 / (1.0 + math.exp(-float(alpha)))

    def _read(self):
        self.rec_host.copy_(self.rec, non_blocking=True)
        torch.cuda.current_stream(self.rec.device).synchronize()
        return self.rec_host.tolist()

    # ------------------------------------------------------------------ RHS launches
    def _count(self, n=1):
        f = self.func
        if f.nfe > f.opt["max_nfe"]:
            raise MaxNFEException
        f.nfe += n

    def _rhs(self, x, stage_y, stage_a, dot_row, beta_slot):
        """One augmented evaluation at the packed stage input x: the y-half over the
        CSR, the a-half over the CSC with the alpha rows <L^T a, y> into rows[dot_row],
        and (add_source) <a, x0> into rec[beta_slot]."""
        self._count()
        ops.spmm_rhs(self.g, self.w_csr, x[0], x0=self.x0, alpha=self.neg_sig, beta=self.neg_beta, rhs=True,
                     alpha_sigmoid=False, add_source=self.add_source, stage=stage_y)
        stage_a.dot = (x[0], self.rows[dot_row], 1.0, False)
        ops.spmm_rhs(self.g, self.w_csc, x[1], alpha=self.alpha, rhs=True, alpha_sigmoid=True, transpose=True,
                     stage=stage_a)
        if self.add_source:
            ops.dot(x[1], self.x0, out=self.rec[beta_slot:beta_slot + 1])

    def _beta_slot(self, j):
        return 3 + self.plan.ns + j

    def _combo(self, spec, h, x):
        b = self.bufs
        base, terms, cfc = spec
        bt = {'Y': b['Y'], 'X': x, 'E': b.get('E'), None: None}[base]
        bt = bt[h] if bt is not None else None
        return bt, (1.0 if bt is not None else 0.0), cfc, [(b[k][h], c) for k, c in terms]

    def _launch(self, i, mid):
        P, b = self.plan, self.bufs
        L = P.launches[i]
        x = b['X%d' % i]
        j = i + 1
        stages = []
        for h in (0, 1):
            outs = []
            for key, dst in (('next', 'X%d' % (i + 1)), ('y1', 'Y1'), ('epart', 'E')):
                if L[key] is not None:
                    bt, cb, cf, ks = self._combo(L[key], h, x)
                    outs.append((b[dst][h], bt, cb, cf, ks))
            err = None
            if L['err'] is not None:
                bt, cb, cf, ks = self._combo(L['err'], h, x)
                err = (self.rows[h], (bt, cb, cf, ks), b['Y'][h], 0 if L['y1'] is not None else -1, self.atol,
                       self.rtol)
            f_out = b['K%d' % j][h] if (j in P.store or (mid and j in P.store_mid)) else None
            stages.append(ops.Stage(f_out=f_out, outs=outs, err=err, scale=self.scale))
        self._rhs(x, stages[0], stages[1], 2 + j, self._beta_slot(j))

    def _step(self, mid):
        """Enqueue one step: the first stage input X0 = Y + dt b00 K0 (one pass over the
        packed state), the ns launches of each half, one segment-sum launch."""
        P, b = self.plan, self.bufs
        ops.stage_apply(ops.Stage(outs=[(b['X0'], b['Y'], 1.0, 0.0, [(b['K0'], P.beta[0][0])])], scale=self.scale),
                        None, None, b['Y'])
        for i in range(P.ns):
            self._launch(i, mid)
        ops.segment_sums(self.rows, self.rec[:3 + P.ns])

    # ------------------------------------------------------------------ scalar components
    def _ratio(self, e2y, e2a, s0, s1, k, dt):
        """torchdiffeq's mixed error norm: max of the halves' RMS error ratios and the
        scalar components' |e| / tol; s1 = the scalars at the step's end."""
        P = self.plan
        r = max(math.sqrt(e2y / self.ny), math.sqrt(e2a / self.ny))
        for c in range(len(s0)):
            e = dt * sum(P.c_err[j] * k[c][j] for j in range(P.ns + 1) if P.c_err[j] != 0.0)
            tol = self.atol + self.rtol * max(abs(s0[c]), abs(s1[c]))
            r = max(r, abs(e) / tol)
        return r

    def _initial_step(self, s0, k0):
        """_select_initial_step over the mixed norm: the halves' squared sums on the
        device (gnpde_scaled_sq_sums_f32), the scalar components on the host; the probe
        z0 + h0 f0 is one stage pass and one augmented evaluation.  h0 and the result
        are rounded to fp32 as torch computes them on an fp32 state."""
        b, n = self.bufs, float(self.ny)
        off = 3 + self.plan.ns + self.plan.ns + 1
        ops.scaled_sq_sums(b['Y'][0], b['K0'][0], None, self.atol, self.rtol, self.rec[off:off + 2])
        ops.scaled_sq_sums(b['Y'][1], b['K0'][1], None, self.atol, self.rtol, self.rec[off + 2:off + 4])
        r = self._read()
        sc = [self.atol + abs(v) * self.rtol for v in s0]
        d0 = max([math.sqrt(r[off] / n), math.sqrt(r[off + 2] / n)] + [abs(v) / s for v, s in zip(s0, sc)])
        d1 = max([math.sqrt(r[off + 1] / n), math.sqrt(r[off + 3] / n)] + [abs(v) / s for v, s in zip(k0, sc)])
        h0 = 1e-6 if (d0 < 1e-5 or d1 < 1e-5) else _f32(0.01 * d0 / d1)
        # probe f(z0 + h0 f0): stage input in X0, its derivative in Y1 (both free before the first step)
        self.scale.fill_(h0)
        ops.stage_apply(ops.Stage(outs=[(b['X0'], b['Y'], 1.0, 0.0, [(b['K0'], 1.0)])], scale=self.scale), None,
                        None, b['Y'])
        slot = 2 + self.plan.ns  # the last stage's alpha rows: free before the first step
        self._rhs(b['X0'], ops.Stage(f_out=b['Y1'][0]), ops.Stage(f_out=b['Y1'][1]), slot, self._beta_slot(self.plan.ns))
        ops.segment_sums(self.rows[slot:slot + 1], self.rec[slot:slot + 1])
        ops.scaled_sq_sums(b['Y'][0], b['K0'][0], b['Y1'][0], self.atol, self.rtol, self.rec[off:off + 2])
        ops.scaled_sq_sums(b['Y'][1], b['K0'][1], b['Y1'][1], self.atol, self.rtol, self.rec[off + 2:off + 4])
        r = self._read()
        k1 = [self.one_minus_sig * r[slot]]
        if self.add_source:
            k1.append(r[self._beta_slot(self.plan.ns)])
        d2 = max([math.sqrt(r[off] / n), math.sqrt(r[off + 2] / n)] +
                 [abs(a - c) / s for a, c, s in zip(k1, k0, sc)]) / h0
        if d1 <= 1e-15 and d2 <= 1e-15:
            h1 = max(1e-6, h0 * 1e-3)
        else:
            h1 = (0.01 / max(d1, d2)) ** (1.0 / self.order)
        return _f32(min(100.0 * h0, h1))

    # ------------------------------------------------------------------ one interval
    def _interval(self, t0, t1, s0):
        """Integrate the packed state in bufs['Y'] (y | a) and the scalars s0 from
        s = t0 to t1 > t0; returns (the a-half at t1, the scalars at t1)."""
        P, b = self.plan, self.bufs
        ns = P.ns
        # f0 = f(z0): K0 and the scalars' derivatives
        self._rhs(b['Y'], ops.Stage(f_out=b['K0'][0]), ops.Stage(f_out=b['K0'][1]), 2, self._beta_slot(0))
        ops.segment_sums(self.rows[2:3], self.rec[2:3])
        if self.first_step is None:
            r = self._read()
            k0 = [self.one_minus_sig * r[2]] + ([r[self._beta_slot(0)]] if self.add_source else [])
            dt = self._initial_step(s0, k0)
        else:
            dt = float(self.first_step)
            r = self._read()
            k0 = [self.one_minus_sig * r[2]] + ([r[self._beta_slot(0)]] if self.add_source else [])
        t_cur = t0
        last = None
        while t1 > t_cur:
            if not (t_cur + dt > t_cur):
                raise AssertionError('underflow in dt {}'.format(dt))
            if self.n_steps >= self.max_num_steps:
                raise AssertionError('max_num_steps exceeded ({}>={})'.format(self.n_steps, self.max_num_steps))
            mid = t_cur + dt >= t1
            self.scale.fill_(dt)
            self._step(mid)
            r = self._read()
            ks = [k0[0]] + [self.one_minus_sig * r[2 + j] for j in range(1, ns + 1)]
            kk = [ks]
            if self.add_source:
                kk.append([k0[1]] + [r[self._beta_slot(j)] for j in range(1, ns + 1)])
            s1 = [s0[c] + dt * sum(P.c_sol[j] * kk[c][j] for j in range(ns + 1) if P.c_sol[j] != 0.0)
                  for c in range(len(s0))]
            ratio = self._ratio(r[0], r[1], s0, s1, kk, dt)
            if ratio <= 1:
                last = (t_cur, dt, dict(b), list(s0), list(s1), [list(v) for v in kk])
                t_cur = t_cur + dt
                s0 = s1
                k0 = [v[ns] for v in kk]
                self._rotate()
            if ratio == 0:
                dt = dt * self.ifactor
            else:
                df = 1.0 if ratio < 1 else self.dfactor
                dt = dt * min(self.ifactor, max(self.safety / ratio ** (1.0 / self.order), df))
            self.n_steps += 1
        if last is None or t1 == t_cur:
            return self.bufs['Y'][1], s0
        return self._interp(last, t1, t_cur)

    def _rotate(self):
        b, kn = self.bufs, 'K%d' % self.plan.ns
        b['Y'], b['Y1'] = b['Y1'], b['Y']
        b['K0'], b[kn] = b[kn], b['K0']
        if self.plan.fsal:
            b['X%d' % (self.plan.ns - 1)] = b['Y1']

    def _interp(self, last, t, t1):
        """torchdiffeq's 4th-order dense output of the last accepted step (integrator.
        _RKAdaptive._interp) for the a-half (one stage pass) and the scalars."""
        P = self.plan
        t0, dt, d, s0, s1, kk = last
        x = (t - t0) / (t1 - t0)
        x2, x3, x4 = x * x, x * x * x, x * x * x * x
        cy0 = 1.0 - 11.0 * x2 + 18.0 * x3 - 8.0 * x4
        cy1 = -5.0 * x2 + 14.0 * x3 - 8.0 * x4
        cym = 16.0 * x2 - 32.0 * x3 + 16.0 * x4
        cf0 = dt * (x - 4.0 * x2 + 5.0 * x3 - 2.0 * x4)
        cf1 = dt * (x2 - 3.0 * x3 + 2.0 * x4)
        ns = P.ns
        h = 1
        y0, y1, f0, f1 = d['Y'][h], d['Y1'][h], d['K0'][h], d['K%d' % ns][h]
        coef = {}
        order = []

        def add(tn, c):
            if c == 0.0:
                return
            if id(tn) not in coef:
                coef[id(tn)] = [tn, 0.0]
                order.append(id(tn))
            coef[id(tn)][1] += c
        add(y1, cy1)
        for j in range(ns + 1):
            if P.c_mid[j] != 0.0:
                add(d['K%d' % j][h] if j < ns else f1, cym * dt * P.c_mid[j])
        add(f0, cf0)
        cf_f1 = coef.pop(id(f1))[1] + cf1 if id(f1) in coef else cf1
        terms = [tuple(coef[k]) for k in order if k in coef]
        out = torch.empty_like(y0)
        ops.stage_apply(ops.Stage(outs=[(out, y0, cy0 + cym, cf_f1, terms)]), f1, y0, y0)
        sv = []
        for c in range(len(s0)):
            k = kk[c]
            ymid = s0[c] + dt * sum(P.c_mid[j] * k[j] for j in range(ns + 1))
            sv.append(cy0 * s0[c] + cy1 * s1[c] + cym * ymid + cf0 * k[0] + cf1 * k[ns])
        return out, sv

    # ------------------------------------------------------------------ the backward
    def run(self, t_h, ans, grad_y):
        gi, func = self.gi, self.func
        lay = gi._node_layout(func, ans[0])
        if lay is not None:
            func._layout = lay
        try:
            self._setup(ans[0])
            b = self.bufs

            def load(dst, src):
                if lay is None:
                    dst.copy_(src)
                elif (self.C * 4) % 16 == 0:
                    ops.rows_copy(src.contiguous(), dst, order=lay.order)
                else:
                    torch.index_select(src.reshape(-1, self.C), 0, lay.order, out=dst.view(-1, self.C))
            load(b['Y'][1], grad_y[-1])
            s = [0.0] + ([0.0] if self.add_source else [])
            for i in range(len(t_h) - 1, 0, -1):
                load(b['Y'][0], ans[i])
                if i < len(t_h) - 1:
                    load(b['Y'][1], a_user)
                a_end, s = self._interval(-t_h[i], -t_h[i - 1], s)
                a_user = torch.empty_like(grad_y[i - 1])
                gi._to_user(a_end, a_user, lay)
                a_user += grad_y[i - 1]
        finally:
            func._layout = None
        grads = {id(func.alpha_train): s[0]}
        if self.add_source:
            grads[id(func.beta_train)] = s[1]
        return a_user, grads
