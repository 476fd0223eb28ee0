#!/usr/bin/env python
"""Where does the fused-stage K1 lose time against the plain RHS?  Times K1 on
G-arxiv (C=128) for: the plain RHS on a fixed input, the plain RHS on inputs
rotating through 5 state buffers (the rk4 working set), the stage-epilogue
variants of one rk4 step on a fixed input, and the STG kernel storing f only.
One JSON line (microseconds per launch)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

import gnpde  # noqa: E402
from gnpde import integrator as gi, ops, synthetic  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(reps):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps * 1e3, 2)


def main():
    N = int(os.environ.get("K1_N", synthetic.ARXIV_N))
    E = int(os.environ.get("K1_E", synthetic.ARXIV_E))
    C = int(os.environ.get("K1_C", 128))
    reps = int(os.environ.get("K1_REPS", 40))
    dev = torch.device("cuda", 0)
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, device=dev)
    opt = {'hidden_dim': C, 'block': 'constant', 'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9,
           'multi_modal': False}
    if os.environ.get("K1_CHUNK"):
        opt['gnpde_chunk'] = int(os.environ["K1_CHUNK"])  # hub-splitting threshold (default 256)
    func = gnpde.LaplacianODEFunc(C, C, opt, dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    r = {"N": N, "E": E, "C": C, "chunk": opt.get('gnpde_chunk', 256)}
    with torch.no_grad():
        g = func.graph_for(x)
        wc = func.csr_weights(g, w, 'w')
        a = func.alpha_train.detach()
        bufs = [x.clone() for _ in range(5)]
        out = torch.empty_like(x)
        y0, x3 = x.clone(), x.clone()
        dt = 0.25

        def k1(xin, o=None, stage=None):
            return ops.spmm_rhs(g, wc, xin, alpha=a, out=None if o is None else o.view(-1, C), stage=stage)

        r["hub_inlaunch"] = os.environ.get("GNPDE_HUB_FIXUP") != "1"
        r["plain_fixed"] = timeit(lambda i: k1(x, out), reps)
        r["plain_rotating"] = timeit(lambda i: k1(bufs[i % 5], bufs[(i + 1) % 5]), reps)
        r["stg_f_only"] = timeit(lambda i: k1(x, stage=ops.Stage(f_out=out)), reps)
        r["stage1_fixed"] = timeit(lambda i: k1(x, stage=ops.Stage(outs=[(out, x, 1.0, dt / 3, [])])), reps)
        r["stage1_rotating"] = timeit(
            lambda i: k1(bufs[i % 5], stage=ops.Stage(outs=[(bufs[(i + 1) % 5], bufs[i % 5], 1.0, dt / 3, [])])), reps)
        r["stage2_fixed"] = timeit(lambda i: k1(x, stage=ops.Stage(outs=[(out, x, -1.0, dt, [(y0, 2.0)])])), reps)
        r["stage4_fixed"] = timeit(
            lambda i: k1(x, stage=ops.Stage(outs=[(out, x, 0.375, dt / 8, [(x3, 0.75), (y0, -0.125)])])), reps)
        ws = gi._Workspace()
        pp = [x.clone(), x.clone()]
        r["rk4_step_per_rhs"] = round(timeit(lambda i: gi._fused_step('rk4', func, 0.0, dt, dt, pp[i % 2], ws,
                                                                     out=pp[(i + 1) % 2]), reps) / 4, 2)
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
