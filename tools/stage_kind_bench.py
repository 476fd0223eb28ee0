"""Launch time of the G-arxiv Laplacian K1 (C = 128) under several stage epilogues (the
f0 / probe launches of the adaptive initial step): HIP events over 20 launches each.
  python tools/stage_kind_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402


def main():
    import gnpde
    from gnpde import ops, synthetic
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    func = gnpde.LaplacianODEFunc(C, C, {'hidden_dim': C, 'block': 'constant', 'add_source': False,
                                        'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False},
                                  dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    y = x.clone()
    k = torch.empty_like(x)
    o2 = torch.empty_like(x)
    rows = torch.empty(N, dtype=torch.float64, device=dev)
    rows2 = torch.empty(N, dtype=torch.float64, device=dev)
    t0 = torch.tensor(0.0)
    cases = {
        "stg1 f_out": (y, dict(f_out=k), False),
        "stg1 out": (y, dict(outs=[(o2, y, 1.0, 0.5, [])]), False),
        "stg4 f_out+err(y0=x)": (y, dict(f_out=k, err=(rows, (None, 0.0, 1.0, []), y, -2, 1e-4, 1e-6)), False),
        "stg4 f_out+err+scale": (y, dict(f_out=k, err=(rows, (None, 0.0, 1.0, []), y, -2, 1e-4, 1e-6),
                                        scale_rows=rows2), False),
        "stg4 err(y0=x)": (y, dict(err=(rows, (None, 0.0, 1.0, []), y, -2, 1e-4, 1e-6)), True),
        "stg4 err(y0 other)": (k, dict(err=(rows, (None, 0.0, 1.0, []), y, -2, 1e-4, 1e-6)), True),
        "stg4 f_out only (3 ops)": (y, dict(outs=[(o2, y, 1.0, 0.5, [(k, 0.1), (x, 0.2), (rows2.new_empty(0)
                                                                                          if False else o2, 0.0)])]),
                                    False),
    }
    with torch.no_grad():
        func(t0, y)  # graph build
        for name, (inp, kw, lin) in cases.items():
            if name.endswith("(3 ops)"):
                continue
            st = ops.Stage(**kw)
            for _ in range(3):
                func.rhs_stage(t0, inp, st, linear=lin)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                func.rhs_stage(t0, inp, st, linear=lin)
            b.record()
            torch.cuda.synchronize()
            print("%-28s %.1f us" % (name, a.elapsed_time(b) / 20 * 1e3))


if __name__ == "__main__":
    main()
