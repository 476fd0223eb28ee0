#!/usr/bin/env python
"""Pieces of the reference-mode attention RHS (fork scaled_dot, norm_idx 1) on
G-arxiv (C=128, h=2, att=32), each timed alone with HIP events (us), plus the
whole RHS of ODEFuncTransformerAtt replayed from a captured graph.  One JSON
line.  Run under `rocprofv3 --kernel-trace --stats` for per-kernel times."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

from gnpde import ops, synthetic  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps * 1e3, 1)


def graph_us(fn, reps):
    fn()
    torch.cuda.synchronize()
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        fn()
    return timeit(cg.replay, reps)


def main():
    import gnpde
    N, E = synthetic.ARXIV_N, synthetic.ARXIV_E
    C = int(os.environ.get("ATT_C", 128))
    H, att = int(os.environ.get("ATT_H", 2)), int(os.environ.get("ATT_DIM", 32))
    reps = int(os.environ.get("ATT_REPS", 50))
    dev = torch.device("cuda", 0)
    ei, _ = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    Wq, Wk = [torch.randn(att, C, generator=gen, device=dev) * 0.1 for _ in range(2)]
    bq, bk = [torch.randn(att, generator=gen, device=dev) * 0.1 for _ in range(2)]
    g = ops.GraphCSR(ei, N)
    alpha = torch.tensor(0.0, device=dev)
    r = {"N": N, "E": E, "C": C, "H": H, "att": att}
    with torch.no_grad():
        ns = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'reference')
        m, rl = ops.softmax_stats(g, ns, 1)
        r["scores_us"] = timeit(lambda: ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'reference'), reps)
        r["stats_seg_us"] = timeit(lambda: ops.softmax_stats(g, ns, 1, seg=True), reps)
        r["stats_group_us"] = timeit(lambda: ops.softmax_stats(g, ns, 1, seg=False), reps)
        r["k1_fused_us"] = timeit(lambda: ops.attn_rhs(g, ns, m, rl, 1, x, alpha=alpha), reps)
        _, _, mr = ops.softmax_stats(g, ns, 1, packed=True)
        r["stats_packed_us"] = timeit(lambda: ops.softmax_stats(g, ns, 1, packed=True), reps)
        r["k1_records_us"] = timeit(lambda: ops.attn_rhs(g, ns, None, None, 1, x, alpha=alpha, mr=mr), reps)
        r["weights_us"] = timeit(lambda: ops.attn_weights(g, ns, m, rl, 1, seg=False), reps)
        w = ops.attn_weights(g, ns, m, rl, 1, seg=False)
        r["k1_plain_us"] = timeit(lambda: ops.spmm_rhs(g, w, x, alpha=alpha), reps)
        f1 = ops.attn_rhs(g, ns, m, rl, 1, x, alpha=alpha)
        f2 = ops.attn_rhs(g, ns, m, rl, 1, x, alpha=alpha, fuse=False, seg=False)
        r["fused_vs_unfused_bitequal"] = bool(torch.equal(f1, f2))
        opt = {'hidden_dim': C, 'heads': H, 'attention_dim': att, 'attention_norm_idx': 1,
               'attention_type': 'scaled_dot', 'attention_score_mode': 'reference', 'function': 'transformer',
               'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False,
               'mix_features': False, 'square_plus': False, 'beltrami': False}
        func = gnpde.ODEFuncTransformerAtt(C, C, opt, dev).to(dev).eval()
        lay = func.multihead_att_layer
        lay.Q.weight.copy_(Wq)
        lay.Q.bias.copy_(bq)
        lay.K.weight.copy_(Wk)
        lay.K.bias.copy_(bk)
        func.edge_index = ei
        func.graph_for(x)
        r["rhs_graph_us"] = graph_us(lambda: func(None, x), reps)
        r["rhs_eager_us"] = timeit(lambda: func(None, x), reps)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
