"""Diagnostic: one fused rk4-stage evaluation of the transformer RHS against the
RHS and a torch combination (fork scaled_dot norm_idx 1 and per-edge)."""
import sys
sys.path.insert(0, '/root/repo/graph-neural-pde_amd')
import torch, gnpde
from gnpde import ops, synthetic
DEV = 'cuda'
N, E, C, h, att = 60000, 450000, 128, 2, 32
ei, _ = synthetic.rw_graph(N, E, seed=32, device=DEV)
x = synthetic.features(1, N, C, seed=8, device=DEV)
y0 = synthetic.features(1, N, C, seed=9, device=DEV)
def rel(a, b): return float((a.double() - b.double()).abs().max() / b.double().abs().max())
for mode, heads in (('reference', 2), ('reference', 4), ('per_edge', 2)):
    opt = {'hidden_dim': C, 'heads': heads, 'attention_dim': att, 'attention_norm_idx': 1, 'attention_type': 'scaled_dot',
           'attention_score_mode': mode, 'function': 'transformer', 'add_source': False, 'no_alpha_sigmoid': False,
           'max_nfe': 10 ** 9, 'multi_modal': False, 'mix_features': False, 'square_plus': False, 'beltrami': False}
    func = gnpde.ODEFuncTransformerAtt(C, C, opt, DEV).to(DEV).eval()
    gen = torch.Generator(device=DEV); gen.manual_seed(9)
    with torch.no_grad():
        for lin in (func.multihead_att_layer.Q, func.multihead_att_layer.K):
            lin.weight.copy_(torch.randn(att, C, generator=gen, device=DEV) * 0.1)
            lin.bias.copy_(torch.randn(att, generator=gen, device=DEV) * 0.1)
        func.alpha_train.fill_(0.3)
    func.edge_index = ei
    with torch.no_grad():
        f = func(None, x)
        f_again = func(None, x)
        out = torch.empty_like(x)
        func.rhs_stage(0.0, x, ops.Stage(outs=[(out, x, -1.0, 0.25, [(y0, 2.0)])]))
        want = -x + 0.25 * f + 2.0 * y0
        fo = torch.empty_like(x)
        func.rhs_stage(0.0, x, ops.Stage(f_out=fo, outs=[(torch.empty_like(x), x, 0.0, 0.0, [])]))
    print(mode, heads, "f repeat", rel(f_again, f), "stage out vs f-combination", rel(out, want), "f_out vs f", rel(fo, f))
