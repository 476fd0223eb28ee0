#!/usr/bin/env python
"""Golden-vector generator for the GRAND/BLEND ODE right-hand side.

RUNS ONLY IN THE BUILD CONTAINER (it imports the read-only reference tree at
/root/reference/src).  It is committed so the fixtures can be regenerated and
audited; nothing under tests/ imports it, and the GPU box never runs it.

What it does
------------
Imports the reference's own RHS modules

  * src/function_laplacian_diffusion.py  (LaplacianODEFunc, :15-77)
  * src/function_transformer_attention.py (ODEFuncTransformerAtt :9-62,
                                           SpGraphTransAttentionLayer :65-270)
  * src/utils.py                          (softmax :116-127)

and runs them on small seeded inputs in float64, writing inputs + outputs to
``tests/golden/*.npz``.  Inputs are generated in float32 and up-cast, so the
float32 inputs stored in the fixture are exactly the values the float64 run
saw.  A float32 run of the same reference code is stored beside it (``f_ref32``)
to show the reference's own fp32 rounding.

Three third-party modules the reference imports are absent from this image
(SURVEY.md §8(c)); in-process stand-ins are injected into ``sys.modules``:

  * ``torch_scatter`` (pinned 2.0.5, environment.yml:89, pyG_install.sh:4):
    ``scatter_add`` / ``scatter_max`` restated from their published semantics
    (index broadcast over trailing dims; out-of-group slots 0).  Only the
    per-group max/sum inside ``utils.softmax`` uses them; the softmax value does
    not depend on which shift is subtracted, so this only affects rounding.
  * ``torch_geometric.nn.conv.MessagePassing`` -> ``torch.nn.Module`` (used only
    as a base class, src/base_classes.py:3,193,214).
  * ``data_multi`` -> empty module (import-only, function_transformer_attention.py:4).

No reference source or bytecode is written anywhere (sys.dont_write_bytecode).
"""
import json
import os
import sys
import types

sys.dont_write_bytecode = True

import numpy as np
import torch

REF_SRC = "/root/reference/src"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- stand-ins
def _install_standins():
    ts = types.ModuleType("torch_scatter")

    def _bcast(index, src):
        idx = index
        while idx.dim() < src.dim():
            idx = idx.unsqueeze(-1)
        return idx.expand_as(src)

    def scatter_add(src, index, dim=-1, out=None, dim_size=None):
        idx = _bcast(index, src)
        shape = list(src.shape)
        shape[dim] = dim_size if dim_size is not None else int(index.max()) + 1
        return torch.zeros(shape, dtype=src.dtype).scatter_add_(dim, idx, src)

    def scatter_max(src, index, dim=-1, out=None, dim_size=None):
        idx = _bcast(index, src)
        shape = list(src.shape)
        shape[dim] = dim_size if dim_size is not None else int(index.max()) + 1
        out = torch.zeros(shape, dtype=src.dtype).scatter_reduce_(dim, idx, src, "amax", include_self=False)
        return out, None

    ts.scatter_add = scatter_add
    ts.scatter_max = scatter_max
    ts.scatter = None
    sys.modules["torch_scatter"] = ts

    pyg = types.ModuleType("torch_geometric")
    pyg_nn = types.ModuleType("torch_geometric.nn")
    pyg_conv = types.ModuleType("torch_geometric.nn.conv")
    pyg_conv.MessagePassing = torch.nn.Module
    sys.modules["torch_geometric"] = pyg
    sys.modules["torch_geometric.nn"] = pyg_nn
    sys.modules["torch_geometric.nn.conv"] = pyg_conv

    dm = types.ModuleType("data_multi")
    dm.get_dataset = None
    sys.modules["data_multi"] = dm


_install_standins()
sys.path.insert(0, REF_SRC)
import function_laplacian_diffusion as ref_lap  # noqa: E402
import function_transformer_attention as ref_att  # noqa: E402
import utils as ref_utils  # noqa: E402
import block_mixed as ref_mixed  # noqa: E402  (module import only; the block's __init__ needs torchdiffeq)

# test/test_params.py:5-16 (the reference tests' shared OPT dict), restated as data.
BASE_OPT = {
    'self_loop_weight': 1, 'leaky_relu_slope': 0.2, 'heads': 2, 'attention_norm_idx': 0, 'add_source': False,
    'hidden_dim': 6, 'block': 'constant', 'function': 'laplacian', 'augment': False, 'adjoint': False,
    'tol_scale': 1, 'time': 1, 'method': 'euler', 'no_alpha_sigmoid': False, 'reweight_attention': False,
    'step_size': 1, 'beltrami': False, 'attention_type': 'scaled_dot', 'square_plus': False,
    'max_nfe': 1000, 'data_norm': 'rw', 'max_iters': 1000, 'multi_modal': False, 'mix_features': False,
    'attention_dim': 16, 'feat_hidden_dim': 16, 'pos_enc_hidden_dim': 8,
}


# --------------------------------------------------------------------------- graphs
def random_graph(rng, B, N, E, dup_frac=0.05, n_isolated=2, self_loop_frac=0.1):
    """[B,2,E] int64 edge_index with duplicates, self loops and isolated nodes."""
    ei = np.zeros((B, 2, E), dtype=np.int64)
    for b in range(B):
        iso = rng.choice(N, size=n_isolated, replace=False) if n_isolated else np.array([], np.int64)
        live = np.setdiff1d(np.arange(N), iso)
        src = rng.choice(live, size=E)
        dst = rng.choice(live, size=E)
        nl = int(self_loop_frac * E)
        dst[:nl] = src[:nl]
        nd = int(dup_frac * E)
        if nd:
            pick = rng.choice(E - nd, size=nd)
            src[E - nd:] = src[pick]
            dst[E - nd:] = dst[pick]
        perm = rng.permutation(E)
        ei[b, 0] = src[perm]
        ei[b, 1] = dst[perm]
    return ei


def f32(a):
    return np.asarray(a, dtype=np.float32)


# --------------------------------------------------------------------------- laplacian
def run_laplacian(name, rng, B, N, E, C, block='constant', heads=4, add_source=False,
                  no_alpha_sigmoid=False, alpha=0.3, beta=0.7, **gkw):
    opt = dict(BASE_OPT, hidden_dim=C, block=block, add_source=add_source, no_alpha_sigmoid=no_alpha_sigmoid,
               heads=heads)
    ei = random_graph(rng, B, N, E, **gkw)
    x = f32(rng.standard_normal((B, N, C)))
    x0 = f32(rng.standard_normal((B, N, C)))
    if block == 'attention':
        w = f32(rng.uniform(0.05, 1.0, (B, E, heads)))
    else:
        w = f32(rng.uniform(0.05, 1.0, (B, E)))
    alpha, beta = float(np.float32(alpha)), float(np.float32(beta))  # exactly representable in fp32
    out = {}
    for dt, tag in ((torch.float64, 'f'), (torch.float32, 'f_ref32')):
        func = ref_lap.LaplacianODEFunc(C, C, opt, 'cpu').to(dt)
        with torch.no_grad():
            func.alpha_train.fill_(alpha)
            func.beta_train.fill_(beta)
        func.edge_index = torch.from_numpy(ei)
        if block in ('attention', 'mixed', 'hard_attention'):
            func.attention_weights = torch.from_numpy(w).to(dt)
        else:
            func.edge_weight = torch.from_numpy(w).to(dt)
        func.x0 = torch.from_numpy(x0).to(dt)
        with torch.no_grad():
            f = func(torch.tensor(0.0), torch.from_numpy(x).to(dt))
        out[tag] = f.numpy()
    meta = dict(kind='laplacian', B=B, N=N, E=E, C=C, block=block, heads=heads, add_source=add_source,
                no_alpha_sigmoid=no_alpha_sigmoid)
    np.savez_compressed(os.path.join(OUT_DIR, name + '.npz'), meta=json.dumps(meta), edge_index=ei, x=x, x0=x0,
                        weights=w, alpha_train=f32(alpha), beta_train=f32(beta), f=out['f'], f_ref32=out['f_ref32'])
    return name


# --------------------------------------------------------------------------- transformer
def run_transformer(name, rng, B, N, E, C, heads, att_dim, norm_idx, attention_type='scaled_dot',
                    add_source=False, no_alpha_sigmoid=False, alpha=0.2, beta=0.5, wstd=0.1, x=None,
                    ei=None, weights=None, **gkw):
    opt = dict(BASE_OPT, hidden_dim=C, heads=heads, attention_dim=att_dim, attention_norm_idx=norm_idx,
               attention_type=attention_type, add_source=add_source, no_alpha_sigmoid=no_alpha_sigmoid,
               function='transformer')
    if ei is None:
        ei = random_graph(rng, B, N, E, **gkw)
    if x is None:
        x = f32(rng.standard_normal((B, N, C)))
    x0 = f32(rng.standard_normal((B, N, C)))
    if weights is None:
        Wq = f32(rng.standard_normal((att_dim, C)) * wstd)
        bq = f32(rng.standard_normal((att_dim,)) * wstd)
        Wk = f32(rng.standard_normal((att_dim, C)) * wstd)
        bk = f32(rng.standard_normal((att_dim,)) * wstd)
    else:
        Wq, bq, Wk, bk = weights
    alpha, beta = float(np.float32(alpha)), float(np.float32(beta))  # exactly representable in fp32
    out = {}
    for dt, tag in ((torch.float64, ''), (torch.float32, '_ref32')):
        func = ref_att.ODEFuncTransformerAtt(C, C, opt, 'cpu').to(dt)
        lay = func.multihead_att_layer
        with torch.no_grad():
            func.alpha_train.fill_(alpha)
            func.beta_train.fill_(beta)
            lay.Q.weight.copy_(torch.from_numpy(Wq))
            lay.Q.bias.copy_(torch.from_numpy(bq))
            lay.K.weight.copy_(torch.from_numpy(Wk))
            lay.K.bias.copy_(torch.from_numpy(bk))
            if attention_type == 'exp_kernel':
                lay.output_var.fill_(float(np.float32(1.3)))
                lay.lengthscale.fill_(float(np.float32(0.8)))
        func.edge_index = torch.from_numpy(ei)
        func.x0 = torch.from_numpy(x0).to(dt)
        func.y = None
        xt = torch.from_numpy(x).to(dt)
        with torch.no_grad():
            att, (_, prods) = lay(xt, func.edge_index, None)
            f = func(torch.tensor(0.0), xt)
        out['f' + tag] = f.numpy()
        out['attention' + tag] = att.numpy()
        out['prods' + tag] = prods.numpy()
    meta = dict(kind='transformer', B=B, N=int(x.shape[1]), E=int(ei.shape[2]), C=C, heads=heads,
                attention_dim=att_dim, attention_norm_idx=norm_idx, attention_type=attention_type,
                add_source=add_source, no_alpha_sigmoid=no_alpha_sigmoid,
                output_var=float(np.float32(1.3)) if attention_type == 'exp_kernel' else None,
                lengthscale=float(np.float32(0.8)) if attention_type == 'exp_kernel' else None)
    np.savez_compressed(os.path.join(OUT_DIR, name + '.npz'), meta=json.dumps(meta), edge_index=ei, x=x, x0=x0,
                        Wq=Wq, bq=bq, Wk=Wk, bk=bk, alpha_train=f32(alpha), beta_train=f32(beta),
                        f=out['f'], attention=out['attention'], prods=out['prods'],
                        f_ref32=out['f_ref32'], attention_ref32=out['attention_ref32'])
    return name


# --------------------------------------------------------------------------- softmax
def run_softmax(name, rng, B, E, H, n_nodes):
    src = f32(rng.standard_normal((B, E, H)) * 3)
    index = rng.integers(0, n_nodes, size=(B, E)).astype(np.int64)
    out = ref_utils.softmax(torch.from_numpy(src).double(), torch.from_numpy(index)).numpy()
    np.savez_compressed(os.path.join(OUT_DIR, name + '.npz'), meta=json.dumps(dict(kind='softmax')),
                        src=src, index=index, out=out)
    return name


# --------------------------------------------------------------------------- mixed block weights
def run_mixed(name, rng, B, E, H, gamma):
    """MixedODEblock.get_mixed_attention (src/block_mixed.py:29-33), called
    unbound on a namespace holding exactly the attributes it reads (the block
    itself cannot be constructed: its __init__ imports torchdiffeq)."""
    att = f32(rng.uniform(0.0, 1.0, (B, E, H)))
    ew = f32(rng.uniform(0.0, 1.0, (B, E)))
    gamma = float(np.float32(gamma))
    out = {}
    for dt, tag in ((torch.float64, 'w'), (torch.float32, 'w_ref32')):
        att_t = torch.from_numpy(att).to(dt)
        ns = types.SimpleNamespace(gamma=torch.tensor([gamma], dtype=dt),
                                   odefunc=types.SimpleNamespace(edge_weight=torch.from_numpy(ew).to(dt)),
                                   get_attention_weights=lambda x, a=att_t: a)
        with torch.no_grad():
            out[tag] = ref_mixed.MixedODEblock.get_mixed_attention(ns, None).numpy()
    meta = dict(kind='mixed', B=B, E=E, H=H)
    np.savez_compressed(os.path.join(OUT_DIR, name + '.npz'), meta=json.dumps(meta), attention=att, edge_weight=ew,
                        gamma=f32(gamma), w=out['w'], w_ref32=out['w_ref32'])
    return name


def main_blocks():
    """Fixtures of the mixed block's weight producer (separate seed, so the
    fixtures of main() are untouched)."""
    rng = np.random.default_rng(20250118)
    made = [run_mixed('mixed_w_b1_h1', rng, 1, 500, 1, 0.0), run_mixed('mixed_w_b2_h4', rng, 2, 700, 4, -0.7),
            run_mixed('mixed_w_b1_h8', rng, 1, 300, 8, 1.3)]
    path = os.path.join(OUT_DIR, 'MANIFEST.json')
    have = json.load(open(path))
    with open(path, 'w') as fh:
        json.dump(sorted(set(have) | set(made)), fh, indent=1)
    print('wrote', len(made), 'fixtures to', OUT_DIR)


# --------------------------------------------------------------------------- gradients (torch autograd, fp64)
def _grads(loss_fn, named):
    """fp64 autograd gradients of loss_fn() w.r.t. the named leaf tensors."""
    loss = loss_fn()
    gs = torch.autograd.grad(loss, [t for _, t in named], allow_unused=True)
    return {'g_' + n: (np.zeros(tuple(t.shape)) if g is None else g.detach().numpy()) for (n, t), g in zip(named, gs)}


def grad_laplacian(name, rng, B, N, E, C, block='constant', heads=4, add_source=False, no_alpha_sigmoid=False,
                   alpha=0.3, beta=0.7, **gkw):
    """Gradients of <gout, f> through the reference LaplacianODEFunc.forward
    (src/function_laplacian_diffusion.py:39-77; the COO -> to_dense -> matmul
    chain differentiates to the edge weights) w.r.t. x, alpha_train, beta_train
    and the weights the block hands over (edge_weight [B,E] or attention [B,E,h])."""
    opt = dict(BASE_OPT, hidden_dim=C, block=block, add_source=add_source, no_alpha_sigmoid=no_alpha_sigmoid,
               heads=heads)
    ei = random_graph(rng, B, N, E, **gkw)
    x = f32(rng.standard_normal((B, N, C)))
    x0 = f32(rng.standard_normal((B, N, C)))
    w = f32(rng.uniform(0.05, 1.0, (B, E, heads) if block == 'attention' else (B, E)))
    gout = f32(rng.standard_normal((B, N, C)))
    alpha, beta = float(np.float32(alpha)), float(np.float32(beta))
    func = ref_lap.LaplacianODEFunc(C, C, opt, 'cpu').double()
    with torch.no_grad():
        func.alpha_train.fill_(alpha)
        func.beta_train.fill_(beta)
    func.edge_index = torch.from_numpy(ei)
    wt = torch.from_numpy(w).double().requires_grad_(True)
    if block in ('attention', 'mixed', 'hard_attention'):
        func.attention_weights = wt
    else:
        func.edge_weight = wt
    func.x0 = torch.from_numpy(x0).double()
    xt = torch.from_numpy(x).double().requires_grad_(True)
    go = torch.from_numpy(gout).double()
    g = _grads(lambda: (func(torch.tensor(0.0), xt) * go).sum(),
               [('x', xt), ('alpha_train', func.alpha_train), ('beta_train', func.beta_train), ('weights', wt)])
    meta = dict(kind='laplacian_grad', B=B, N=N, E=E, C=C, block=block, heads=heads, add_source=add_source,
                no_alpha_sigmoid=no_alpha_sigmoid)
    np.savez_compressed(os.path.join(OUT_DIR, name + '.npz'), meta=json.dumps(meta), edge_index=ei, x=x, x0=x0,
                        weights=w, alpha_train=f32(alpha), beta_train=f32(beta), gout=gout, **g)
    return name


def grad_transformer(name, rng, B, N, E, C, heads, att_dim, norm_idx, attention_type='scaled_dot', add_source=False,
                     no_alpha_sigmoid=False, alpha=0.2, beta=0.5, wstd=0.1, **gkw):
    """Gradients of <gout, f> through the reference ODEFuncTransformerAtt.forward
    (src/function_transformer_attention.py:44-59, 218-267: Q/K projections,
    the score, utils.softmax, the head-mean aggregation) w.r.t. x, alpha_train,
    beta_train, Q.weight, Q.bias, K.weight, K.bias (+ output_var, lengthscale
    for exp_kernel)."""
    opt = dict(BASE_OPT, hidden_dim=C, heads=heads, attention_dim=att_dim, attention_norm_idx=norm_idx,
               attention_type=attention_type, add_source=add_source, no_alpha_sigmoid=no_alpha_sigmoid,
               function='transformer')
    ei = random_graph(rng, B, N, E, **gkw)
    x = f32(rng.standard_normal((B, N, C)))
    x0 = f32(rng.standard_normal((B, N, C)))
    Wq = f32(rng.standard_normal((att_dim, C)) * wstd)
    bq = f32(rng.standard_normal((att_dim,)) * wstd)
    Wk = f32(rng.standard_normal((att_dim, C)) * wstd)
    bk = f32(rng.standard_normal((att_dim,)) * wstd)
    gout = f32(rng.standard_normal((B, N, C)))
    alpha, beta = float(np.float32(alpha)), float(np.float32(beta))
    func = ref_att.ODEFuncTransformerAtt(C, C, opt, 'cpu').double()
    lay = func.multihead_att_layer
    with torch.no_grad():
        func.alpha_train.fill_(alpha)
        func.beta_train.fill_(beta)
        lay.Q.weight.copy_(torch.from_numpy(Wq))
        lay.Q.bias.copy_(torch.from_numpy(bq))
        lay.K.weight.copy_(torch.from_numpy(Wk))
        lay.K.bias.copy_(torch.from_numpy(bk))
        if attention_type == 'exp_kernel':
            lay.output_var.fill_(float(np.float32(1.3)))
            lay.lengthscale.fill_(float(np.float32(0.8)))
    func.edge_index = torch.from_numpy(ei)
    func.x0 = torch.from_numpy(x0).double()
    func.y = None
    xt = torch.from_numpy(x).double().requires_grad_(True)
    go = torch.from_numpy(gout).double()
    named = [('x', xt), ('alpha_train', func.alpha_train), ('beta_train', func.beta_train), ('Wq', lay.Q.weight),
             ('bq', lay.Q.bias), ('Wk', lay.K.weight), ('bk', lay.K.bias)]
    if attention_type == 'exp_kernel':
        named += [('output_var', lay.output_var), ('lengthscale', lay.lengthscale)]
    g = _grads(lambda: (func(torch.tensor(0.0), xt) * go).sum(), named)
    meta = dict(kind='transformer_grad', B=B, N=N, E=E, C=C, heads=heads, attention_dim=att_dim,
                attention_norm_idx=norm_idx, attention_type=attention_type, add_source=add_source,
                no_alpha_sigmoid=no_alpha_sigmoid,
                output_var=float(np.float32(1.3)) if attention_type == 'exp_kernel' else None,
                lengthscale=float(np.float32(0.8)) if attention_type == 'exp_kernel' else None)
    np.savez_compressed(os.path.join(OUT_DIR, name + '.npz'), meta=json.dumps(meta), edge_index=ei, x=x, x0=x0,
                        Wq=Wq, bq=bq, Wk=Wk, bk=bk, alpha_train=f32(alpha), beta_train=f32(beta), gout=gout, **g)
    return name


def main_grads():
    """Reference autograd gradient fixtures (separate seed: earlier fixtures untouched)."""
    rng = np.random.default_rng(20250119)
    made = [grad_laplacian('grad_lap_const_b1', rng, 1, 60, 300, 8),
            grad_laplacian('grad_lap_const_b2_src', rng, 2, 40, 160, 6, add_source=True, no_alpha_sigmoid=True,
                           alpha=-0.4, beta=0.9),
            grad_laplacian('grad_lap_attn_mean_b2', rng, 2, 50, 260, 16, block='attention', heads=4),
            grad_laplacian('grad_lap_mixed_b1', rng, 1, 80, 420, 12, block='mixed')]
    made += [grad_transformer('grad_att_sd_n1_h2', rng, 1, 60, 320, 12, 2, 16, 1),
             grad_transformer('grad_att_sd_n0_h2', rng, 1, 60, 320, 12, 2, 16, 0),
             grad_transformer('grad_att_sd_n1_h8_b2', rng, 2, 40, 200, 16, 8, 32, 1, wstd=0.1),
             grad_transformer('grad_att_sd_n1_src', rng, 1, 50, 260, 10, 2, 8, 1, add_source=True,
                              no_alpha_sigmoid=True, alpha=0.8, beta=-0.3)]
    for st in ('exp_kernel', 'cosine_sim', 'pearson'):
        for ni in (0, 1):
            made.append(grad_transformer('grad_att_%s_n%d' % (st, ni), rng, 2, 40, 200, 10, 2, 8, ni,
                                         attention_type=st, wstd=0.3))
    path = os.path.join(OUT_DIR, 'MANIFEST.json')
    have = json.load(open(path))
    with open(path, 'w') as fh:
        json.dump(sorted(set(have) | set(made)), fh, indent=1)
    print('wrote', len(made), 'fixtures to', OUT_DIR)


def main():
    rng = np.random.default_rng(20250117)
    made = []
    # ---- Laplacian RHS (function_laplacian_diffusion.py:39-77)
    made.append(run_laplacian('lap_const_b1', rng, 1, 60, 300, 8))
    made.append(run_laplacian('lap_const_b3_src', rng, 3, 40, 150, 5, add_source=True, no_alpha_sigmoid=True,
                              alpha=-0.4, beta=0.9))
    made.append(run_laplacian('lap_attn_mean_b2', rng, 2, 50, 260, 16, block='attention', heads=4))
    made.append(run_laplacian('lap_hard_b1', rng, 1, 70, 400, 12, block='hard_attention'))
    made.append(run_laplacian('lap_mixed_b2_c80', rng, 2, 120, 700, 80, block='mixed', add_source=True))
    made.append(run_laplacian('lap_const_c128', rng, 1, 300, 2400, 128, dup_frac=0.1, n_isolated=5))
    made.append(run_laplacian('lap_const_c162', rng, 1, 200, 1400, 162))
    made.append(run_laplacian('lap_const_c256', rng, 1, 150, 1200, 256))
    # ---- Transformer RHS, fork scaled_dot (function_transformer_attention.py:218-267)
    made.append(run_transformer('att_sd_n0_h2', rng, 1, 60, 320, 12, 2, 16, 0))
    made.append(run_transformer('att_sd_n1_h2', rng, 1, 60, 320, 12, 2, 16, 1))
    made.append(run_transformer('att_sd_n1_h8_b2', rng, 2, 50, 240, 20, 8, 32, 1))
    made.append(run_transformer('att_sd_n1_h1', rng, 1, 40, 200, 7, 1, 8, 1))
    made.append(run_transformer('att_sd_n0_h1_b3', rng, 3, 30, 100, 9, 1, 4, 0))
    made.append(run_transformer('att_sd_n1_src', rng, 1, 70, 350, 16, 4, 16, 1, add_source=True,
                                no_alpha_sigmoid=True, alpha=0.8, beta=-0.3))
    made.append(run_transformer('att_sd_n1_c128', rng, 1, 400, 2400, 128, 2, 32, 1, wstd=0.05))
    made.append(run_transformer('att_sd_n1_c80_h8', rng, 1, 300, 1800, 80, 8, 128, 1, wstd=0.03))
    made.append(run_transformer('att_sd_n0_c162', rng, 1, 150, 900, 162, 2, 32, 0, wstd=0.05))
    made.append(run_transformer('att_sd_n1_c162', rng, 1, 150, 900, 162, 2, 32, 1, wstd=0.05))
    # ---- other score types (per-edge; §8(f) next-4)
    for st in ('exp_kernel', 'cosine_sim', 'pearson'):
        for ni in (0, 1):
            made.append(run_transformer('att_%s_n%d' % (st, ni), rng, 2, 40, 200, 10, 2, 8, ni, attention_type=st,
                                        wstd=0.3))
    # ---- KAT: test/test_transformer_attention.py:98-106 (x = ones, complete 3-graph -> attention 0.5)
    ei_sym = np.array([[[0, 0, 1, 1, 2, 2], [1, 2, 0, 2, 0, 1]]], dtype=np.int64)
    one = np.full((32, 2), 1e-5, np.float32)
    made.append(run_transformer('att_kat_symmetric', rng, 1, 3, 6, 2, 2, 32, 0, x=np.ones((1, 3, 2), np.float32),
                                ei=ei_sym, weights=(one, np.zeros(32, np.float32), one, np.zeros(32, np.float32))))
    # ---- edge softmax (utils.py:116-127)
    made.append(run_softmax('softmax_b2', rng, 2, 500, 3, 40))
    made.append(run_softmax('softmax_b1_h8', rng, 1, 2000, 8, 300))
    with open(os.path.join(OUT_DIR, 'MANIFEST.json'), 'w') as fh:
        json.dump(sorted(made), fh, indent=1)
    print('wrote', len(made), 'fixtures to', OUT_DIR)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'blocks':
        main_blocks()
    elif len(sys.argv) > 1 and sys.argv[1] == 'grads':
        main_grads()
    else:
        main()
