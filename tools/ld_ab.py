#!/usr/bin/env python
"""Row stride of a bf16 state (BLEND C = 168 after padding): plain K1 with the rows
at 336 B (ld 168) against whole 128-byte lines (ld 192) — one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    import gnpde
    from gnpde import _lib, ops, synthetic
    from gnpde.ops import _ptr, _stream, _partials, _flags
    dev = torch.device("cuda", 0)
    N, E = synthetic.ARXIV_N, synthetic.ARXIV_E
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    func = gnpde.LaplacianODEFunc(128, 128, dict(bench.LAP_OPT, hidden_dim=128), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    C = 168
    out = {}
    a = torch.tensor(0.5, device=dev)
    for dt in (torch.bfloat16, torch.float32):
        for ld in (168, 192, 176):
            xb = torch.randn(N, ld, device=dev).to(dt)
            with torch.no_grad():
                g = func.graph_for(xb[:, :128].contiguous().float().unsqueeze(0))
            plan = g.csr.plan
            wt, tag = func._weights_tensor()
            wc = func.csr_weights(g, wt, tag)
            f = torch.empty(N, ld, device=dev, dtype=dt)
            part = _partials(plan, C, dev)
            plan.order_launch(dev)
            name = "gnpde_spmm_rhs_bf16" if dt == torch.bfloat16 else "gnpde_spmm_rhs_f32"

            def run():
                _lib.call(name, _ptr(plan.items), plan.n_items, _ptr(plan.heavy), plan.n_heavy, _ptr(g.csr.col),
                          _ptr(wc), C, _ptr(xb), ld, None, C, _ptr(a), None, _flags(True, True, False), _ptr(f), ld,
                          _ptr(part), plan.n_slots, None, _stream(dev))
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(50):
                run()
            e.record()
            torch.cuda.synchronize()
            out["%s_ld%d" % (str(dt)[6:], ld)] = round(s.elapsed_time(e) / 50 * 1e3, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
