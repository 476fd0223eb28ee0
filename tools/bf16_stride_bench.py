#!/usr/bin/env python
"""Hypothesis check: bf16 rows of 168 columns (BLEND, 336 B) gathered from a
state whose row STRIDE is 192 columns (384 B = three whole 128-byte lines)
instead of 168 (rows straddle 3-4 lines).  Plain K1 through the C ABI directly
(gnpde_spmm_rhs_bf16 with ldx = ldf = stride), G-arxiv graph."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

from gnpde import _lib, ops, synthetic  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 168
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    g = ops.GraphCSR(ei, N)
    lay = g.node_layout
    for name, gg in (("user", g), ("degree", lay.graph)):
        wc = gg.gather_weights(w)
        plan = gg.csr.plan
        alpha = torch.zeros((), device=dev)
        for ld in (168, 176, 192):
            xs = torch.randn(N, ld, device=dev).to(torch.bfloat16)
            fs = torch.empty_like(xs)
            parts = ops._partials(plan, C, dev)
            st = ops._stream(dev)

            def run():
                _lib.call("gnpde_spmm_rhs_bf16", ops._ptr(plan.items), plan.n_items, ops._ptr(plan.heavy),
                          plan.n_heavy, ops._ptr(gg.csr.col), ops._ptr(wc), C, ops._ptr(xs), ld, ctypes.c_void_p(0), ld,
                          ops._ptr(alpha), ctypes.c_void_p(0), ops._flags(True, True, False), ops._ptr(fs), ld,
                          ops._ptr(parts), None, st)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(50):
                run()
            e.record()
            torch.cuda.synchronize()
            print(json.dumps({"numbering": name, "C": C, "ld": ld, "rhs_us": round(s.elapsed_time(e) / 50 * 1e3, 2)}),
                  flush=True)


if __name__ == "__main__":
    main()
