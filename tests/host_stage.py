"""CPU evaluation of the fused stage epilogue (include/gnpde.h gnpde_stage_epilogue_t,
gnpde.ops.Stage) — TEST INFRASTRUCTURE: lets the integrator's fused solver logic
(fixed-grid and adaptive plans) run on CPU with an injected RHS, so its control
flow and combination algebra are checked without a GPU.  The product path applies
stages only in HIP."""
import torch


def _combo(base, cb, cf, terms, f, sc=1.0):
    r = torch.zeros_like(f) if base is None else cb * base
    for k, c in terms:
        r = r + (c * sc) * k
    return r + (cf * sc) * f


def apply_stage(stage, f, x):
    """Every store of ``stage`` for RHS value f (None: 0) and RHS input x."""
    if f is None:
        like = stage.outs[0][0] if stage.outs else stage.err[2]
        f = torch.zeros_like(like)
    sc = float(stage.scale) if stage.scale is not None else 1.0
    if getattr(stage, 'f_lin', 0.0):
        f = x + (sc * stage.f_lin) * f
    if stage.f_out is not None:
        stage.f_out.copy_(f)
    vals = []
    unscaled = getattr(stage, 'unscaled', ())
    for i, (out, base, cb, cf, terms) in enumerate(stage.outs):
        v = _combo(base, cb, cf, terms, f, 1.0 if i in unscaled else sc)
        vals.append(v)
        out.copy_(v)
    if stage.err is not None:
        rows, (base, cb, cf, terms), y0, y1_out, atol, rtol = stage.err
        e = _combo(base, cb, cf, terms, f, sc).double()
        y1 = x if y1_out < 0 else vals[y1_out]
        tol = atol + rtol * torch.maximum(y0.abs(), y1.abs()).double()
        C = f.shape[-1]
        rows.copy_(((e / tol) ** 2).reshape(-1, C).sum(-1))


class HostLinearRHS(object):
    """f(y) = y @ A^T over rows [R, C] (A [C, C]) on CPU, with the integrator's
    host-stage hooks."""

    host_stages = True

    def __init__(self, A):
        self.A = A
        self.nfe = 0
        self.n_stage = 0  # RHS calls that carried a stage epilogue

    def __call__(self, t, y):
        self.nfe += 1
        return y @ self.A.T

    affine = True  # f(y) = A y: its own linear part

    def rhs_stage(self, t, x, stage, linear=False):
        self.nfe += 1
        self.n_stage += 1
        apply_stage(stage, x @ self.A.T, x)

    def host_stage_apply(self, stage, f, x, like):
        apply_stage(stage, f, x)
