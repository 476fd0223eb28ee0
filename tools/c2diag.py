import sys, numpy as np, torch
sys.path.insert(0,'graph-neural-pde_amd'); sys.path.insert(0,'oracle'); sys.path.insert(0,'tests')
import gnpde, gnpde_oracle as O
DEV='cuda'
T=lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
from test_gpu_parity import OPT, _set_qk, _prep_oracle, rel
N, E, C, h, att = 2708, 10556, 80, 8, 128
rng = np.random.default_rng(90)
ei = rng.integers(0, N, size=(1, 2, E))
x = rng.standard_normal((1, N, C)).astype(np.float32)
for method, tol, step in (('dopri5', 1.0, None), ('dopri5', 0.01, None), ('rk4', 1.0, 0.02)):
    opt = dict(OPT, hidden_dim=C, heads=h, attention_dim=att, function='transformer', attention_norm_idx=1,
               method=method, tol_scale=tol, step_size=step)
    blk = gnpde.ConstantODEblock(gnpde.ODEFuncTransformerAtt, [], opt, DEV, t=torch.tensor([0, 1])).to(DEV).eval()
    r2 = np.random.default_rng(90); r2.integers(0, N, size=(1, 2, E)); r2.standard_normal((1, N, C))
    Wq, bq, Wk, bk = _set_qk(blk.odefunc.multihead_att_layer, r2, C, att, scale=0.03)
    with torch.no_grad(): blk.odefunc.alpha_train.fill_(0.5)
    data = gnpde.GraphData(); data.new_graph(T(ei), N)
    with torch.no_grad(): z = blk(T(x), data)
    eo, _ = _prep_oracle(ei, N)
    f = lambda t, y: O.transformer_rhs(eo, y, None, Wq, bq, Wk, bk, h, 1, 0.5, 0.0)
    want = O.odeint_fixed(f, x, 0.0, 1.0, 'rk4', 0.02)
    print(method, tol, 'rel', rel(z, want), 'nfe', blk.odefunc.nfe, flush=True)
