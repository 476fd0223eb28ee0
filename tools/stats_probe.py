#!/usr/bin/env python
"""Where the reference statistics kernel spends its time: the G-arxiv CSC
statistics (norm_idx 1, packed records) launched whole and over each item class
alone (hub chunks, long wavefronts, short items), HIP events over a hipGraph of
REPS launches each (no host launch cost in the time).  Prints one JSON line."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

REPS = 50


def main():
    import bench
    from gnpde import _lib, ops, synthetic
    dev = torch.device("cuda", 0)
    ei, _ = synthetic.rw_graph(synthetic.ARXIV_N, synthetic.ARXIV_E, seed=0, device=dev)
    x = synthetic.features(1, synthetic.ARXIV_N, 128, seed=1, device=dev)
    func = bench.attention_func("reference", 1, 128, dev)
    func.edge_index = ei
    g = func.graph_for(x)
    lay = func.multihead_att_layer
    with torch.no_grad():
        ns = lay.node_scores(g, x)
        ops.softmax_stats(g, ns, 1, packed=True)
    grouped = g.csc
    plan = grouped.seg_plan(_lib.fn("gnpde_seg_block_edges")(ns.mode, ns.heads, ns.dk), True)
    mr = torch.empty(g.R, ops.stats_record_floats(ns.heads), dtype=torch.float32, device=dev)
    partials = torch.empty(max(plan.n_slots, 1) * 2 * ns.heads, dtype=torch.float64, device=dev)

    def launch(off, n, nh, nl):
        s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        it = ctypes.c_void_p(plan.items.data_ptr() + 16 * off)
        _lib.call("gnpde_seg_softmax_f32", it, n, nh, nl, ops._ptr(plan.chunk_items), 0, ops._ptr(plan.heavy),
                  plan.n_heavy, ops._ptr(grouped.rowptr), ops._ptr(grouped.rowidx), ops._ptr(grouped.col), 1, 1,
                  ns.mode, ns.heads, ns.dk, ops._ptr(ns.cs), None, None, 1, 1.0, 1.0, None, None, None, ops._ptr(mr),
                  ops._ptr(partials), s)

    def timed(*a):
        for _ in range(3):
            launch(*a)
        torch.cuda.synchronize()
        cg = torch.cuda.CUDAGraph()
        with torch.cuda.graph(cg):
            for _ in range(REPS):
                launch(*a)
        cg.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        cg.replay()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / REPS * 1e3, 2)

    nh, nl, n = plan.n_hub, plan.n_long, plan.n_items
    it = plan.items.view(-1, 4)[:n].cpu()
    ln = (it[:, 1] - it[:, 0]).long()
    out = {"n_hub": nh, "n_long": nl, "n_short": n - nh - nl, "hub_edges": int(ln[:nh].sum()),
           "long_edges": int(ln[nh:nh + nl].sum()), "short_edges": int(ln[nh + nl:].sum()),
           "max_hub": int(ln[:nh].max()) if nh else 0,
           "all_us": timed(0, n, nh, nl), "hubs_us": timed(0, nh, nh, 0),
           "longs_us": timed(nh, nl, 0, nl), "shorts_us": timed(nh + nl, n - nh - nl, 0, 0)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
