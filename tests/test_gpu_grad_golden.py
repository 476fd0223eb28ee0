"""GPU: gradients of the RHS through the HIP backward against the REFERENCE's
own fp64 autograd (tests/golden/grad_*.npz, written by
tests/golden/gen_golden.py grads from src/function_laplacian_diffusion.py and
src/function_transformer_attention.py).

d <gout, f> / d (x, alpha_train, beta_train, the block's edge weights or the
attention's Q / K parameters [, output_var, lengthscale]), for the Laplacian
RHS (constant / attention-mean / mixed weights, add_source, no_alpha_sigmoid)
and the transformer RHS (the fork's scaled_dot under norm_idx 0 and 1,
exp_kernel, cosine_sim, pearson).

Tolerance: max |g - g_ref| <= max(1e-4 * max |g_ref|, 1e-6 * S) per gradient,
S = the largest reference gradient of the case (fp32 backward against fp64
autograd; the chains are 3-6 sums deep).  The second term covers gradients
that vanish analytically and that the reference leaves at fp64 rounding
level: the fork's scaled_dot under source-grouped softmax cannot move the
attention, and under destination-grouped softmax d/d bq =
S/sqrt(dk) * sum_e g_s[e], where every softmax group's g_s sums to
(1 - sum att) * ... ~ 0 — fp32 gives the cancellation's rounding instead."""
import glob
import json
import os

import numpy as np
import pytest
import torch

import gnpde
from conftest import GOLDEN
from test_gpu_parity import DEV, OPT, T

pytestmark = pytest.mark.gpu
GRAD_RTOL = 1e-4
FIX = sorted(glob.glob(os.path.join(GOLDEN, "grad_*.npz")))


def _load(path):
    d = np.load(path, allow_pickle=False)
    return d, json.loads(str(d["meta"]))


def _case_scale(d):
    return max(float(np.abs(d[k]).max()) for k in d.files if k.startswith("g_") and d[k].size)


def _check(name, got, want, scale):
    got = np.zeros_like(want) if got is None else got.detach().double().cpu().numpy().reshape(want.shape)
    err = np.abs(got - want).max() if want.size else 0.0
    tol = max(GRAD_RTOL * (np.abs(want).max() if want.size else 0.0), 1e-6 * scale)
    assert err <= tol, "%s: max err %.3e, tolerance %.3e" % (name, err, tol)


@pytest.mark.parametrize("path", [p for p in FIX if os.path.basename(p).startswith("grad_lap_")],
                         ids=os.path.basename)
def test_laplacian_grad_golden(path):
    d, m = _load(path)
    C = m["C"]
    opt = dict(OPT, hidden_dim=C, block=m["block"], add_source=m["add_source"], no_alpha_sigmoid=m["no_alpha_sigmoid"],
               heads=m["heads"])
    func = gnpde.LaplacianODEFunc(C, C, opt, DEV).to(DEV)
    with torch.no_grad():
        func.alpha_train.fill_(float(d["alpha_train"]))
        func.beta_train.fill_(float(d["beta_train"]))
    func.edge_index = T(d["edge_index"])
    w = T(d["weights"]).requires_grad_(True)
    if m["block"] == "constant":
        func.edge_weight = w
    else:
        func.attention_weights = w
    func.x0 = T(d["x0"])
    x = T(d["x"]).requires_grad_(True)
    f = func(torch.tensor(0.0), x)
    (f * T(d["gout"])).sum().backward()
    scale = _case_scale(d)
    _check("x", x.grad, d["g_x"], scale)
    _check("alpha_train", func.alpha_train.grad, d["g_alpha_train"], scale)
    _check("beta_train", func.beta_train.grad, d["g_beta_train"], scale)
    _check("weights", w.grad, d["g_weights"], scale)


@pytest.mark.parametrize("path", [p for p in FIX if os.path.basename(p).startswith("grad_att_")],
                         ids=os.path.basename)
def test_transformer_grad_golden(path):
    d, m = _load(path)
    C = m["C"]
    opt = dict(OPT, hidden_dim=C, heads=m["heads"], attention_dim=m["attention_dim"],
               attention_norm_idx=m["attention_norm_idx"], attention_type=m["attention_type"],
               add_source=m["add_source"], no_alpha_sigmoid=m["no_alpha_sigmoid"], function='transformer')
    func = gnpde.ODEFuncTransformerAtt(C, C, opt, DEV).to(DEV)
    lay = func.multihead_att_layer
    with torch.no_grad():
        func.alpha_train.fill_(float(d["alpha_train"]))
        func.beta_train.fill_(float(d["beta_train"]))
        lay.Q.weight.copy_(T(d["Wq"]))
        lay.Q.bias.copy_(T(d["bq"]))
        lay.K.weight.copy_(T(d["Wk"]))
        lay.K.bias.copy_(T(d["bk"]))
        if m["attention_type"] == "exp_kernel":
            lay.output_var.fill_(m["output_var"])
            lay.lengthscale.fill_(m["lengthscale"])
    func.edge_index = T(d["edge_index"])
    func.x0 = T(d["x0"])
    x = T(d["x"]).requires_grad_(True)
    f = func(torch.tensor(0.0), x)
    (f * T(d["gout"])).sum().backward()
    scale = _case_scale(d)
    _check("x", x.grad, d["g_x"], scale)
    _check("alpha_train", func.alpha_train.grad, d["g_alpha_train"], scale)
    _check("beta_train", func.beta_train.grad, d["g_beta_train"], scale)
    for name, p in (("Wq", lay.Q.weight), ("bq", lay.Q.bias), ("Wk", lay.K.weight), ("bk", lay.K.bias)):
        _check(name, p.grad, d["g_" + name], scale)
    if m["attention_type"] == "exp_kernel":
        _check("output_var", lay.output_var.grad, d["g_output_var"], scale)
        _check("lengthscale", lay.lengthscale.grad, d["g_lengthscale"], scale)
