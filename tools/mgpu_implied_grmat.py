"""Implied per-rank times of configs[4] (G-rmat: RMAT N = 2M, E = 20M, C = 256) at N ranks, both
multi-GPU layouts of gnpde.dist, from one-GPU timings of EVERY rank's share (the slowest rank
counts), plus the per-RHS collective each layout needs modelled from its payload at an assumed
RCCL bus bandwidth (not a scaling measurement — 8-GPU runs are the driver's).

* column stripes (ColumnShardedLaplacian, the default for N > 1): rank p integrates C/N columns
  of the state over the shared graph; a fixed-grid step needs NO collective (the columns are
  independent; the solution is all-gathered once per solve).  Share = one rk4 step of the
  stripe, the production path (in-degree numbering, fused STG1 K1, replayed step graphs).
* row partition (RowShardedLaplacian, the north star's literal edge partition): rank p owns an
  nnz-balanced block of rows and all-gathers the whole state (R x C x 4 bytes) before every
  RHS.  Share = 4 K1 launches over the rank's rows (an rk4 step) + 4 all-gathers.

Collective model: ring all-gather / all-reduce at BUS_GBS (default 300 GB/s per GPU, the
order of RCCL's measured bus bandwidth on an 8-GPU xGMI node — MI355X_MICROARCH.md gives
7 links x ~153 GB/s peak per GPU); all-gather time = (N-1)/N x total bytes / BUS_GBS.
  python tools/mgpu_implied_grmat.py [--worlds 1,2,4,8] [--bus-gbs 300]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def replay_ms(fn, reps=10):
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
    p.add_argument("--bus-gbs", type=float, default=300.0)
    p.add_argument("--steps", type=int, default=8)
    p.add_argument("--row-weights", default="0", help="balanced_row_blocks row_weight values to try (rows layout)")
    p.add_argument("--rows-only", action="store_true")
    a = p.parse_args()
    worlds = [int(v) for v in a.worlds.split(",")]
    import bench
    import gnpde
    from gnpde import dist as gd, ops, synthetic
    dev = torch.device("cuda", 0)
    N, E, C, h = 2_000_000, 20_000_000, 256, 0.25
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    a0 = torch.tensor(0.3, device=dev)
    out = {"graph": "G-rmat N=%d E=%d C=%d (configs[4])" % (N, E, C), "bus_gbs_assumed": a.bus_gbs, "cols": {},
           "rows": {}}
    # column stripes: one rk4 step of each stripe's solve (a stripe is an independent LaplacianODEFunc of C/N
    # columns on the shared graph: exactly the work ColumnShardedLaplacian gives a rank, no collective per RHS)
    for world in ([] if a.rows_only else worlds):
        per = []
        for (c0, c1) in gd.col_blocks(C, world)[:1] if world > 1 else [(0, C)]:
            xs = x[..., c0:c1].contiguous()
            func = gnpde.LaplacianODEFunc(c1 - c0, c1 - c0, dict(bench.LAP_OPT, hidden_dim=c1 - c0), dev).to(dev)
            func.edge_index, func.edge_weight = ei, w
            el, _ = bench.timed_solve(func, xs, a.steps, 1, h, dev, 1)
            per.append(el * 1e3 / a.steps)
            del func, xs
            torch.cuda.empty_cache()
        gather = (world - 1) / world * N * C * 4 / (a.bus_gbs * 1e9) * 1e3 if world > 1 else 0.0
        out["cols"][world] = {"rk4_step_ms_per_rank": round(max(per), 4),
                              "per_rhs_collective": "none (columns independent)",
                              "per_solve_all_gather_ms_modelled": round(gather, 3)}
        print(json.dumps({"cols": world, **out["cols"][world]}), flush=True)
    # row partition: K1 over each rank's nnz-balanced row block (in the in-degree numbering, as the solve)
    func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    lay = func.node_layout(x)
    g = lay.graph if lay is not None else func.graph_for(x)
    xi = lay.to_internal(x) if lay is not None else x
    wc = g.gather_weights(w)
    rws = [float(v) for v in a.row_weights.split(",")]
    for rw, world in [(r, n) for r in rws for n in worlds]:
        blocks = gd.balanced_row_blocks(g.csr.rowptr.cpu().numpy(), world, row_weight=rw)
        per = []
        for (r0, r1) in blocks:
            plan = gd._local_plan(g.csr, r0, r1, g.chunk)
            if plan is None:
                per.append(0.0)
                continue
            xr = xi.view(-1, C)[r0:r1].contiguous()

            def share():
                ops.spmm_rhs_rows(g, plan, wc, xi.view(-1, C), xr, r0, alpha=a0)
            per.append(4 * replay_ms(share))
        gather = 4 * (world - 1) / world * N * C * 4 / (a.bus_gbs * 1e9) * 1e3 if world > 1 else 0.0
        ent = {"row_weight": rw, "rk4_step_compute_ms_per_rank": round(max(per), 4),
               "per_rk4_step_all_gathers_ms_modelled": round(gather, 3),
               "rk4_step_ms_implied": round(max(per) + gather, 4), "rank_compute_ms": [round(v, 4) for v in per]}
        if rw == rws[0]:
            out["rows"][world] = ent
        else:
            out.setdefault("rows_row_weight", {}).setdefault(str(rw), {})[world] = ent
        print(json.dumps({"rows": world, **{k: v for k, v in ent.items() if k != "rank_compute_ms"}}), flush=True)
    b1 = out["cols"][worlds[0]]["rk4_step_ms_per_rank"] if (worlds[0] == 1 and out["cols"]) else None
    if b1:
        for world in worlds:
            c = out["cols"][world]
            c["implied_speedup"] = round(b1 / c["rk4_step_ms_per_rank"], 2)
            r = out["rows"][world]
            r["implied_speedup_compute_only"] = round(b1 / r["rk4_step_compute_ms_per_rank"], 2)
            r["implied_speedup_with_all_gathers"] = round(b1 / r["rk4_step_ms_implied"], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
