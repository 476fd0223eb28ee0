"""Implied per-rank RHS times of the sharded attention and Laplacian RHS at N ranks,
from one-GPU timings of EVERY rank's share (the slowest rank counts), for DESIGN.md §7
(not a scaling measurement — the 8-GPU runs are the driver's).

Column stripes (gnpde.dist.ColumnShardedTransformer / ColumnShardedLaplacian) on G-arxiv
(C = 128, heads 2, attention_dim 32), user numbering: a rank's share of one RHS is
  * reference scaled_dot, norm_idx 1: its stripe's key-sum and node-score shares, the
    statistics of its block of destination rows (partitioned, all-gathered), K1 over its
    columns with the full scores;
  * per-edge scaled_dot, norm_idx 0: its stripe's q|k projection share, the one-pass
    per-edge K1 over its columns with the full q|k;
  * reference scaled_dot, norm_idx 1, edge-sharded weights (ColumnShardedTransformer
    edge_weights, the default at world > 1): the score shares and statistics block as
    above, the head-mean weights of its block of E / N edges, the plain-weight K1 over its
    columns with the gathered weights;
  * per-edge scaled_dot, norm_idx 0, edge-sharded weights: the q|k share, its CSR rows'
    source statistics (row-range K2) and their edges' weights, the plain-weight K1;
  * Laplacian: the plain K1 over its columns.
Each share's launches are captured in one hipGraph and replayed (median of 3 x 20
replays).  The collectives are listed with their payloads; their time is not modelled
here.  Prints one JSON line per workload.
  python tools/mgpu_implied.py [--worlds 1,2,4,8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def replay_ms(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return sorted(ts)[1]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--worlds", default="1,2,4,8")
    a = p.parse_args()
    worlds = [int(v) for v in a.worlds.split(",")]
    import bench
    from gnpde import dist as gd, ops, synthetic
    dev = torch.device("cuda", 0)
    N, E, C, H, ATT = synthetic.ARXIV_N, synthetic.ARXIV_E, 128, bench.ATTN_HEADS, bench.ATTN_DIM
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    g = ops.GraphCSR(ei, N)
    wc = g.gather_weights(w)
    gen = torch.Generator(device=dev)
    gen.manual_seed(2)
    Wq, Wk = [torch.randn(ATT, C, generator=gen, device=dev) * 0.1 for _ in range(2)]
    bq, bk = [torch.randn(ATT, generator=gen, device=dev) * 0.1 for _ in range(2)]
    Wc, bc = torch.cat([Wq, Wk], 0), torch.cat([bq, bk], 0)
    a0 = torch.tensor(0.3, device=dev)
    with torch.no_grad():
        ns_full = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'reference')
        qk_full = ops.linear(x, Wc, bc)[0]
        ns_dot = gd._qk_scores(qk_full, H, ATT)
        _, _, mr_full = ops.softmax_stats(g, ns_full, 1, packed=True)
        m_full, rl_full = ops.softmax_stats(g, ns_full, 1)
        w_full = ops.attn_weights(g, ns_full, m_full, rl_full, 1)
        m0, rl0 = ops.softmax_stats(g, ns_dot, 0)
        w_dot0 = ops.attn_weights(g, ns_dot, m0, rl0, 0)
        loc = gd._HipAttentionLocal(g)
        for wl in ("reference_norm1", "reference_norm1_edges", "per_edge_norm0", "per_edge_norm0_edges",
                   "laplacian"):
            res = {"workload": wl, "graph": "G-arxiv N=%d E'=%d C=%d" % (N, E, C), "ranks": {}}
            for world in worlds:
                cols = gd.col_blocks(C, world)
                dblocks, _ = gd._dst_blocks(ei, N, world, g)
                per_rank = []
                for p, (c0, c1) in enumerate(cols):
                    xs = x[..., c0:c1].contiguous()
                    first = p == 0
                    if wl == "reference_norm1":
                        Wks, Wqs = Wk[:, c0:c1].contiguous(), Wq[:, c0:c1].contiguous()
                        bks = bk if first else torch.zeros_like(bk)
                        bqs = bq if first else torch.zeros_like(bq)
                        d0, d1 = dblocks[p]

                        def share():
                            S = ops.ref_keysum(g, xs, Wks, bks)
                            ops.ref_scores_from_keysum(g, xs, S, Wqs, bqs, H)
                            ops.softmax_stats(g, ns_full, 1, packed=True, rows=(d0, d1))
                            ops.attn_rhs(g, ns_full, None, None, 1, xs, alpha=a0, mr=mr_full)
                    elif wl == "reference_norm1_edges":
                        Wks, Wqs = Wk[:, c0:c1].contiguous(), Wq[:, c0:c1].contiguous()
                        bks = bk if first else torch.zeros_like(bk)
                        bqs = bq if first else torch.zeros_like(bq)
                        d0, d1 = dblocks[p]
                        ne = g.nnz
                        eb = (ne * p // world, ne * (p + 1) // world)

                        def share():
                            S = ops.ref_keysum(g, xs, Wks, bks)
                            ops.ref_scores_from_keysum(g, xs, S, Wqs, bqs, H)
                            ops.softmax_stats(g, ns_full, 1, packed=False, rows=(d0, d1))
                            ops.attn_weights(g, ns_full, m_full, rl_full, 1, edges=eb)
                            ops.spmm_rhs(g, w_full, xs, alpha=a0)
                    elif wl == "per_edge_norm0_edges":
                        Wcs = Wc[:, c0:c1].contiguous()
                        bcs = bc if first else torch.zeros_like(bc)
                        (eb,), (rb,) = [v[p:p + 1] for v in loc.edge_blocks(world)]

                        def share():
                            ops.linear(xs, Wcs, bcs)
                            ms, rls = loc.src_stats(ns_dot, *rb)
                            ops.attn_weights(g, ns_dot, ms, rls, 0, edges=eb)
                            ops.spmm_rhs(g, w_dot0, xs, alpha=a0)
                    elif wl == "per_edge_norm0":
                        Wcs = Wc[:, c0:c1].contiguous()
                        bcs = bc if first else torch.zeros_like(bc)

                        def share():
                            ops.linear(xs, Wcs, bcs)
                            ops.attn_rhs(g, ns_dot, None, None, 0, xs, alpha=a0)
                    else:
                        def share():
                            ops.spmm_rhs(g, wc, xs, alpha=a0)
                    per_rank.append(replay_ms(share))
                coll = {"reference_norm1": {"all_reduce S": 8 * ATT, "all_reduce cs": 8 * N * H,
                                            "all_gather stats records": 4 * ops.stats_record_floats(H) * N},
                        "reference_norm1_edges": {"all_reduce S": 8 * ATT, "all_reduce cs": 8 * N * H,
                                                  "all_gather stats m, rl": 12 * H * N,
                                                  "all_gather weights": 4 * g.nnz},
                        "per_edge_norm0": {"all_reduce q|k": 4 * N * 2 * ATT},
                        "per_edge_norm0_edges": {"all_reduce q|k": 4 * N * 2 * ATT, "all_gather weights": 4 * g.nnz},
                        "laplacian": {}}[wl]
                res["ranks"][world] = {"rank_ms": [round(v, 4) for v in per_rank], "max_ms": round(max(per_rank), 4),
                                       "collective_bytes": coll if world > 1 else {}}
            base = res["ranks"][worlds[0]]["max_ms"] if worlds[0] == 1 else None
            if base:
                for world in worlds:
                    r = res["ranks"][world]
                    r["implied_speedup_compute_only"] = round(base / r["max_ms"], 2)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
