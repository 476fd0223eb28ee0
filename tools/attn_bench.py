#!/usr/bin/env python
"""Micro-benchmark of the attention RHS on G-arxiv (C=128, h=2, att=32 unless
overridden by ATT_C / ATT_H / ATT_DIM): per mode, the fused RHS and the
two-kernel path (weights + K1), plus the pieces.  One JSON line per mode.
Run under `rocprofv3 --kernel-trace --stats` for per-kernel times."""
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
    return round(s.elapsed_time(e) / reps * 1e3, 1)  # us


def main():
    N = int(os.environ.get("ATT_N", synthetic.ARXIV_N))
    E = int(os.environ.get("ATT_E", synthetic.ARXIV_E))
    C = int(os.environ.get("ATT_C", 128))
    H = int(os.environ.get("ATT_H", 2))
    att = int(os.environ.get("ATT_DIM", 32))
    reps = int(os.environ.get("ATT_REPS", 20))
    modes = os.environ.get("ATT_MODES", "per_edge:0,per_edge:1,reference:1").split(",")
    dev = torch.device("cuda", 0)
    ei, _ = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    Wq, Wk = [torch.randn(att, C, generator=gen, device=dev) * 0.1 for _ in range(2)]
    bq, bk = [torch.randn(att, generator=gen, device=dev) * 0.1 for _ in range(2)]
    g = ops.GraphCSR(ei, N)
    alpha = torch.tensor(0.0, device=dev)
    with torch.no_grad():
        for spec in modes:
            mode, norm_idx = spec.split(":")
            norm_idx = int(norm_idx)
            ns = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', mode)
            m, rl = ops.softmax_stats(g, ns, norm_idx)
            r = {"mode": mode, "norm_idx": norm_idx, "N": N, "E": E, "C": C, "H": H, "att": att}
            r["scores_us"] = timeit(lambda: ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', mode), reps)
            r["pergroup_stats_us"] = timeit(lambda: ops.softmax_stats(g, ns, norm_idx, seg=False), reps)
            r["seg_rhs_us"] = timeit(lambda: ops.attn_rhs(g, ns, m if norm_idx else None, rl, norm_idx, x, alpha=alpha), reps)
            r["seg_w_us"] = timeit(lambda: ops.attn_weights(g, ns, m, rl, norm_idx), reps)
            r["seg_stats_us"] = timeit(lambda: ops.softmax_stats(g, ns, norm_idx), reps)
            r["pergroup_rhs_us"] = timeit(lambda: ops.attn_rhs(g, ns, m, rl, norm_idx, x, alpha=alpha, seg=False), reps)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
