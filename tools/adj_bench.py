#!/usr/bin/env python
"""Where the adjoint launches of a training step spend their time: K1 over the
CSC (A^T) against K1 over the CSR, plain and with the adjoint's stage epilogues
(one output + the fp64 dot term, the two-output launch), on G-arxiv in the
solve's node numbering.  Prints one JSON line of microseconds per launch."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        for _ in range(reps):
            fn()
    cg.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    cg.replay()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps * 1e3, 2)


def main():
    import bench
    import gnpde
    from gnpde import ops, synthetic
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    out = {}
    with torch.no_grad():
        lay = func.node_layout(x)
        func._layout = lay
        xs = lay.to_internal(x) if lay is not None else x
        gr = lay.graph if lay is not None else func.graph_for(xs)
        wt, _ = func._weights_tensor()
        w_csr = func.csr_weights(gr, wt, 'w')
        w_csc = gr.gather_weights(wt.detach(), transpose=True)
        one = torch.ones((), dtype=torch.float32, device=dev)
        T = dict(alpha=one, rhs=True, alpha_sigmoid=False)
        e = [torch.randn_like(xs) * 0.1 for _ in range(6)]
        g, v, gk, x4, o1, o2 = e
        drow = torch.zeros(N, dtype=torch.float64, device=dev)
        f = torch.empty_like(xs)
        out["csr_plain"] = timeit(lambda: ops.spmm_rhs(gr, w_csr, g, out=f.view(-1, C), **T))
        out["csc_plain"] = timeit(lambda: ops.spmm_rhs(gr, w_csc, g, out=f.view(-1, C), transpose=True, **T))
        out["csr_stage1"] = timeit(lambda: ops.spmm_rhs(gr, w_csr, g, stage=ops.Stage(
            outs=[(o1, g, 1.0, 0.1, [(v, 0.2)])]), **T))
        out["csc_stage1"] = timeit(lambda: ops.spmm_rhs(gr, w_csc, g, transpose=True, stage=ops.Stage(
            outs=[(o1, g, 1.0, 0.1, [(v, 0.2)])]), **T))
        out["csc_stage3"] = timeit(lambda: ops.spmm_rhs(gr, w_csc, g, transpose=True, stage=ops.Stage(
            f_out=v, outs=[(o1, g, 0.3, 0.1, [])], dot=(x4, drow, 0.1, True)), **T))
        out["csc_stage3_nodot"] = timeit(lambda: ops.spmm_rhs(gr, w_csc, g, transpose=True, stage=ops.Stage(
            f_out=v, outs=[(o1, g, 0.3, 0.1, [])]), **T))
        out["csc_stage2"] = timeit(lambda: ops.spmm_rhs(gr, w_csc, gk, transpose=True, stage=ops.Stage(
            outs=[(o1, g, 0.1, 0.1, [(v, 0.1), (x4, -0.1)]), (o2, x4, 0.2, 0.2, [(v, 0.2)])],
            dot=(x4, drow, 1.0, True)), **T))
        func._layout = None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
