"""The transformer attention RHS inside G-arxiv dopri5 solves (ogbn-arxiv best_params T /
tol_scale; bench.attention_func's shapes): median wall time per solve and per RHS under the
process's settings (run it once per GNPDE_WIDE_PRECOMPUTE=0/1: captured step graphs do not
change with the module switch).   python tools/attn_dopri5_ab.py [reps]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    import gnpde
    from gnpde import ops, synthetic
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, _ = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    T, ts = bench.ARXIV_DOPRI5
    t = torch.tensor([0.0, T], dtype=torch.float32, device=dev)
    kw = dict(method='dopri5', rtol=1e-9 * ts, atol=1e-7 * ts)
    for mode, norm_idx in bench.ATTN_MODES:
        func = bench.attention_func(mode, norm_idx, C, dev)
        func.edge_index = ei
        with torch.no_grad():
            for _ in range(2):
                gnpde.odeint(func, x, t, **kw)
            torch.cuda.synchronize()
            tm = []
            for _ in range(reps):
                n0 = func.nfe
                t0 = time.perf_counter()
                gnpde.odeint(func, x, t, **kw)
                torch.cuda.synchronize()
                tm.append(time.perf_counter() - t0)
                nfe = func.nfe - n0
        med = statistics.median(tm)
        print("%s_norm%d precompute=%d: %.3f ms/solve, %d RHS, %.4f ms/RHS" %
              (mode, norm_idx, ops.WIDE_PRECOMPUTE, med * 1e3, nfe, med * 1e3 / nfe))


if __name__ == "__main__":
    main()
