#!/usr/bin/env python
"""Benchmark: ODE RHS evals/s at |E|≈1.2M, d=128 (BASELINE.json `metric`).

Workload (BASELINE.json configs[2], the config the metric is quoted on):
G-arxiv synthetic graph — N = 169,343 nodes, E' = 1,200,000 edges (RMAT +
self loops, rw-normalised), C = 128 fp32 features — integrated with rk4
(torchdiffeq rk4_alt_step_func, 4 RHS evaluations per step) through the drop-in
LaplacianODEFunc (function='laplacian', block='constant', add_source=False:
src/best_params.py:7 for ogbn-arxiv) and gnpde.odeint.  A "step" is one rk4
step: 4 RHS evaluations (K1, gnpde_spmm_rhs_f32) whose epilogues also emit the
Runge-Kutta stage combinations.

value = RHS evaluations per second over the whole job, inputs resident in HBM.

Multi-GPU (one process per GPU, RCCL): by default ONE shared graph, strong
scaling.  The headline is G-arxiv in feature-column stripes
(gnpde.dist.ColumnShardedLaplacian: replicated CSR, C/N columns per rank, no
per-RHS collective); every line also carries the configs[4] graph (G-rmat:
N = 2M, E = 20M, C = 256) in column stripes and in the north star's literal
row partition (nnz-balanced blocks + an RCCL all-gather of the state before
every RHS), each with the same graph timed unsharded on one GPU of the same
job ("speedup_vs_1gpu").  --mode replicas keeps the old independent-graph
weak-scaling layout.

Extra objects on the JSON line:
  roofline      K1: measured HBM bytes per launch (PMC 2*FETCH_SIZE + WRITE_SIZE,
                profiles/k1_traffic.json) over the mean launch time from HIP
                events on the launch stream, vs 8 TB/s; the SURVEY §8(d)
                algorithmic byte count over the same time is kept as
                algorithmic_achieved / algorithmic_frac;
  cpu_baseline  torch sparse CSR A@x on the host cores (the reference's CPU
                path restated with torch.sparse), bounded sample, rank 0, N=1;
  attention     the transformer RHS (config C4 shape: C=128, h=2, att=32) in
                reference (fork scaled_dot) and per_edge modes;
  blend_c162    configs[3] shape (C = 162) rk4 steps, fp32 and bf16 state;
  grmat         configs[4] graph (see above).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def graph_name(N, E):
    if (N, E) == (169343, 1200000):
        return "G-arxiv"
    if (N, E) == (2000000, 20000000):
        return "G-rmat (configs[4] graph)"
    return "RMAT N=%d E=%d" % (N, E)


def lap_bytes(N, E, C, add_source=False):
    """Algorithmic HBM bytes of one Laplacian RHS:
    gathered x rows 4EC + x_i read & f write 8NC + col/weight 8E + rowptr 4(N+1)."""
    return 4 * E * C + 8 * N * C + 8 * E + 4 * (N + 1) + (4 * N * C if add_source else 0)


def rk4_fused_step_bytes(N, E, C):
    """Algorithmic bytes of one rk4 step with the stage combinations fused into
    the four K1 epilogues (gnpde.integrator._fused_step): 4 x (gathers 4EC +
    indices 8E + rowptr 4(N+1) + input row 4NC) + 8 state passes of 4NC
    (stage 1 writes x2; stage 2 reads y, writes x3; stage 3 reads x2, writes
    x4; stage 4 reads x3 and y, writes y1)."""
    return 4 * (4 * E * C + 8 * E + 4 * (N + 1) + 4 * N * C) + 8 * 4 * N * C


def attn_bytes(N, E, C, att, mode):
    """Algorithmic bytes of one attention RHS.  per_edge: projection
    4NC + 8N*att, stats+aggregation 4N*att + 4E*att + 4EC + 8NC + 4E + 4(N+1);
    reference: the k gather is replaced by the key-sum pass 4N*att + 4N; uniform: see below."""
    if mode == "uniform":
        # fork scaled_dot with norm_idx=0: weights 1/outdeg are graph-only and cached, so one RHS is the
        # aggregation alone (CSR 4(N+1) + 4E, weights 4E, gathers 4EC, own row 4NC, f 4NC)
        return 4 * (N + 1) + 8 * E + 4 * E * C + 8 * N * C
    base = 4 * N * C + 8 * N * att + 4 * N * att + 4 * E * C + 8 * N * C + 4 * E + 4 * (N + 1)
    return base + (4 * E * att if mode == "per_edge" else 4 * N * att + 4 * N)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--nodes", type=int, default=169343)
    p.add_argument("--edges", type=int, default=1200000)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--step-size", type=float, default=0.25)
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-baseline sample")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-attention", action="store_true")
    p.add_argument("--no-train", action="store_true", help="skip the training-step (forward + backward) measurement")
    p.add_argument("--no-grmat", action="store_true", help="skip the configs[4] graph (G-rmat) measurements")
    p.add_argument("--grmat-steps", type=int, default=10, help="timed rk4 steps on G-rmat")
    p.add_argument("--rhs-only", action="store_true", help="time K plain RHS calls instead of rk4 steps")
    p.add_argument("--rhs-plain-reps", type=int, default=20, help="plain-RHS launches timed after the steps")
    p.add_argument("--mode", choices=("auto", "replicas", "rows", "cols"), default="auto",
                   help="multi-GPU layout of the headline: auto = cols for N > 1; cols / rows = one shared graph "
                        "(column stripes / row partition + all-gather per RHS, strong scaling); replicas = an "
                        "independent graph per rank (weak scaling)")
    return p.parse_args()


LAP_OPT = {'block': 'constant', 'function': 'laplacian', 'add_source': False, 'no_alpha_sigmoid': False,
           'max_nfe': 10 ** 9, 'multi_modal': False}


def sync_all(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(v, world, dev):
    if world > 1:
        t = torch.tensor([v], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        v = float(t)
    return v


_T = {}


def rk4_solve(func, y0, n, h, dev):
    """Exactly n rk4 steps through the drop-in integrator (stage combinations
    fused into the RHS epilogues, steps replayed from captured hipGraphs).  The
    time tensor is made once per (n, h) and reused, as ODEblock keeps its
    ``self.t`` (src/base_classes.py): the integrator then reads its values once."""
    import gnpde
    key = (n, h, str(dev))
    if key not in _T:
        _T[key] = torch.tensor([0.0, n * h], dtype=torch.float32, device=dev)
    return gnpde.odeint(func, y0, _T[key], method='rk4', options={'step_size': h})[1]


def timed_solve(func, y0, steps, warmup, h, dev, world, sync_world=None):
    """W warm-up steps, then the one-time capture of the step / block graphs the
    timed call replays (a warm-up shorter than GRAPH_MIN_STEPS captures nothing),
    then EXACTLY `steps` rk4 steps between barriers; max over ranks."""
    import gnpde.integrator as integ
    sw = world if sync_world is None else sync_world
    with torch.no_grad():
        if warmup > 0:
            rk4_solve(func, y0, warmup, h, dev)
        if getattr(func, 'graph_capturable', True) and steps >= integ.GRAPH_MIN_STEPS:
            # one-time setup: capture the block graphs a solve of `steps` steps replays
            # (the first solve of a module runs its first step eagerly, the second
            # captures the block sizes of the whole run)
            for _ in range(2):
                rk4_solve(func, y0, steps, h, dev)
        sync_all(sw)
        t0 = time.perf_counter()
        y = rk4_solve(func, y0, steps, h, dev)
        sync_all(sw)
        el = time.perf_counter() - t0
    assert torch.isfinite(y).all()
    return max_over_ranks(el, sw, dev), y


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    mode = args.mode if args.mode != "auto" else ("replicas" if world == 1 else "cols")
    if world > 1 or (mode != "replicas" and "MASTER_ADDR" in os.environ):
        # one process per GPU under torch.distributed.run: RCCL through env:// (a
        # world of one too, so a one-GPU rehearsal takes the N > 1 code path)
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if mode == "replicas":
        result = bench_single(args, world, rank, dev)
    else:
        result = bench_sharded(args, world, rank, dev, mode)
    if not args.no_grmat:
        result["grmat"] = bench_grmat(args, world, rank, dev)
    if rank == 0:
        print(json.dumps(result))
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def bench_single(args, world, rank, dev):
    """The configs[2] headline: G-arxiv rk4 on one GPU (with N > 1 in replicas
    mode: an independent graph per rank, weak scaling)."""
    import gnpde
    from gnpde import ops, synthetic

    N, E, C = args.nodes, args.edges, args.dim
    ei, w = synthetic.rw_graph(N, E, seed=rank, device=dev)
    x = synthetic.features(1, N, C, seed=1 + rank, device=dev)
    func = gnpde.LaplacianODEFunc(C, C, dict(LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    h = args.step_size

    # instrument the K1 launches with HIP events on the launch (current) stream
    events = []
    orig_spmm = ops.spmm_rhs

    def timed_spmm(*a, **k):
        if torch.cuda.is_current_stream_capturing():  # launches recorded into a hipGraph: timed at replay
            return orig_spmm(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = orig_spmm(*a, **k)
        e.record()
        events.append((s, e))
        return out

    def run_steps(n, y):
        if args.rhs_only:
            for _ in range(n):
                y = func(None, y)
            return y
        return rk4_solve(func, y, n, h, dev)

    import gnpde.function_laplacian_diffusion as fld
    import gnpde.integrator as integ
    with torch.no_grad():
        g = func.graph_for(x)  # once per graph: CSR + plan (outside the timed region)
        if args.warmup > 0:
            run_steps(args.warmup, x)
        if not args.rhs_only and args.steps >= integ.GRAPH_MIN_STEPS:
            # one-time setup outside the timed region whatever W is: capture the block
            # hipGraphs a solve of --steps steps replays from the integrator's cache
            for _ in range(2):
                run_steps(args.steps, x)
        sync_all(world)
        ops.spmm_rhs = fld.ops.spmm_rhs = timed_spmm
        replays = []
        integ.replay_events = replays  # hipGraph replays: events around each replayed rk4 step
        t0 = time.perf_counter()
        y = run_steps(args.steps, x)
        sync_all(world)
        elapsed = time.perf_counter() - t0
        ops.spmm_rhs = fld.ops.spmm_rhs = orig_spmm
        integ.replay_events = None
    assert torch.isfinite(y).all()
    # per-RHS launch time: eager launches are bracketed one by one; a replayed
    # step (4 K1 launches, hub rows combined inside them, nothing else) is bracketed whole
    t_ev = sum(s.elapsed_time(e) for s, e in events) + sum(s.elapsed_time(e) for s, e, _ in replays)
    n_ev = len(events) + sum(n for _, _, n in replays)
    k1_ms = t_ev / max(n_ev, 1)
    elapsed = max_over_ranks(elapsed, world, dev)
    rhs_per_step = 1 if args.rhs_only else 4
    total_rhs = world * args.steps * rhs_per_step
    value = total_rhs / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    if args.rhs_only:
        nbytes = lap_bytes(N, E, C)
        kname = "agg_kernel<4,32,1,4,2,0,PlainWeights,float> (two rows per wavefront; hub rows combined in-launch)"
    else:
        nbytes = rk4_fused_step_bytes(N, E, C) / 4.0
        kname = "agg_kernel<4,32,1,4,2,1,PlainWeights,float>: K1 with fused rk4 stage, two rows per wavefront " \
                "(hub rows combined in-launch)"

    # the plain RHS (no fused stage) on the same graph, for the per-RHS roofline
    plain = None
    if args.rhs_plain_reps > 0:
        with torch.no_grad():
            # on the numbering the solve ran in (the integrator's NodeLayout, when it used one)
            lay = func.node_layout(x)
            gp, xp = (lay.graph, lay.to_internal(x)) if lay is not None else (g, x)
            wc = func.csr_weights(gp, w, 'w')
            out = torch.empty_like(x).view(-1, C)
            for _ in range(3):
                orig_spmm(gp, wc, xp, alpha=func.alpha_train.detach(), out=out)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.rhs_plain_reps):
                orig_spmm(gp, wc, xp, alpha=func.alpha_train.detach(), out=out)
            e.record()
            torch.cuda.synchronize()
        pms = s.elapsed_time(e) / args.rhs_plain_reps
        plain = roofline(pms, lap_bytes(N, E, C), kernel_traffic("lap", PLAIN_K1),
                         "agg_kernel<4,32,1,4,2,0,PlainWeights,float> (hub rows combined in-launch)",
                         lap_compulsory(N, E, C, 1))
        plain["rhs_ms"] = round(pms, 4)

    rl = roofline(k1_ms, nbytes, kernel_traffic("lap", PLAIN_K1 if args.rhs_only else FUSED_K1) if
                  (N, E, C) == (169343, 1200000, 128) else None, kname,
                  lap_compulsory(N, E, C, 1 if args.rhs_only else 2))
    rl.update({"launch_ms": round(k1_ms, 4), "launches": n_ev, "graph_replays": len(replays)})
    result = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "RHS evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded RMAT graph per rank, N(0,1) features)",
        "config": {"workload": "%s laplacian RHS, rk4%s" % (graph_name(N, E), " (configs[2])" if C == 128 else ""),
                   "nodes": N, "edges": E, "dim": C,
                   "method": "rk4", "step_size": h, "rhs_per_step": rhs_per_step, "global_batch": world,
                   "parallelism": "replicas%d" % world, "chunk": g.chunk,
                   "node_order": "none" if args.rhs_only or func.node_layout(x) is None else ops.NODE_ORDER,
                   "hub_rows": g.csr.plan.n_heavy},
        "rhs_ms": round(k1_ms, 4),
        "roofline": rl,
        "rhs_plain": plain,
        "solve_overhead_ms": round(elapsed * 1e3 - args.steps * rhs_per_step * k1_ms, 4),
        "traffic_source": traffic_source(),
    }

    progress("headline: %.1f RHS evals/s" % value)
    if not args.no_attention and rank == 0:
        result["attention"] = bench_attention(g, x, dev, ops)
        progress("attention done")
        result["blend_c162"] = bench_blend(g, dev)
        progress("blend done")
    if not args.no_attention and rank == 0:
        result["dopri5"] = bench_dopri5(ei, w, x, dev, k1_ms, plain["rhs_ms"] if plain else None)
    if not args.no_train and rank == 0 and world == 1:
        result["block_forward"] = bench_block(ei, x, h, dev)
        result["train_rk4"] = bench_train(ei, w, x, h, dev)
        fwd = result.get("dopri5", {}).get("garxiv_laplacian", {}).get("ms_per_solve")
        result["train_adjoint"] = bench_train_adjoint(ei, w, x, dev, fwd)
        result["hard_attention_train"] = bench_hard_attention_train(ei, x, dev)
        result["train_cora"] = bench_train_cora(dev)
        progress("block / train done")

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(ei, w, x, N, E, C, args.cpu_seconds)
    return result


METRIC = "ODE RHS evals/s (and ms/step) at |E|≈1.2M, d=128; achieved HBM GB/s vs roofline"
FUSED_K1 = "agg_kernel<4, 32, 1, 4, 2, 1, PlainWeights, float>"
PLAIN_K1 = "agg_kernel<4, 32, 1, 4, 2, 0, PlainWeights, float>"
GRMAT_K1 = "agg_kernel<4, 64, 1, 4, 1, 1, PlainWeights, float>"


TRAFFIC_FILE = os.path.join("profiles", "traffic.json")
_TRAFFIC = None


def traffic():
    """profiles/traffic.json (tools/prof_r03.sh -> tools/pmc_reduce.py): PMC bytes
    (2*FETCH_SIZE + WRITE_SIZE, the gfx950 corrections of MI355X_MICROARCH.md
    §HBM) per dispatch of every kernel of each bench workload, measured in
    separate rocprofv3 --pmc passes of tools/pmc_run.py."""
    global _TRAFFIC
    if _TRAFFIC is None:
        _TRAFFIC = {}
        path = os.path.join(ROOT, TRAFFIC_FILE)
        if os.path.exists(path):
            with open(path) as fh:
                _TRAFFIC = json.load(fh)
    return _TRAFFIC


def traffic_source():
    """Where the counter bytes come from, and whether they were measured on the
    library that is running (build id = hash of csrc/)."""
    tj = traffic()
    src = {"file": TRAFFIC_FILE, "tag": tj.get("tag"), "build_id": tj.get("build_id")}
    try:
        from gnpde import _lib
        src["fresh"] = tj.get("build_id") == _lib.build_id()
    except Exception:  # noqa: BLE001
        src["fresh"] = None
    return src


def kernel_traffic(workload, kernel_prefix):
    """Mean PMC bytes per dispatch of the kernel whose name starts with
    kernel_prefix in `workload`, or None."""
    w = traffic().get("workloads", {}).get(workload)
    if not w:
        return None
    best = None
    for k in w["kernels"]:
        if k["kernel"].startswith(kernel_prefix) and (best is None or k["count"] > best["count"]):
            best = k
    return best["bytes"] if best else None


def step_traffic(workload):
    """PMC bytes of one replayed adaptive step of a workload (tools/pmc_run.py dopri5)."""
    w = traffic().get("workloads", {}).get(workload)
    return w.get("per_step_bytes") if w else None


def rhs_traffic(workload):
    """PMC bytes of one RHS evaluation of an attention workload (every kernel it dispatches)."""
    w = traffic().get("workloads", {}).get(workload)
    return w.get("per_rhs_bytes") if w else None


def roofline(launch_ms, algorithmic, traffic_b, kernel, compulsory=None):
    """frac = PMC bytes per launch / launch time / 8 TB/s: the HBM (fabric)
    fraction — FETCH_SIZE counts Infinity-Cache hits too, so it bounds HBM
    traffic from above.  Beside it: the §8(d) algorithmic bytes (every gathered
    x row charged; x is re-read from L2 and the Infinity Cache, so that rate can
    pass 8 TB/s: not a roofline fraction) and the compulsory bytes (x read once,
    the CSR, the launch's state passes): traffic / compulsory is the re-fetch
    ratio."""
    t = launch_ms * 1e-3
    alg = algorithmic / t / 1e9
    out = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": kernel,
           "algorithmic_bytes_per_launch": int(algorithmic), "algorithmic_achieved": round(alg, 1),
           "algorithmic_frac": round(alg / HBM_PEAK_GBS, 4)}
    if compulsory:
        out.update({"compulsory_bytes": int(compulsory),
                    "compulsory_frac": round(compulsory / t / 1e9 / HBM_PEAK_GBS, 4)})
    if traffic_b:
        ach = traffic_b / t / 1e9
        out.update({"achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": int(traffic_b),
                    "basis": "PMC bytes per launch (%s, 2*FETCH_SIZE+WRITE_SIZE; the counters include Infinity-Cache "
                             "hits, so frac bounds HBM traffic from above) / HIP-event launch time" %
                             TRAFFIC_FILE})
        if compulsory:
            out["refetch_ratio"] = round(traffic_b / compulsory, 3)
    else:
        out.update({"achieved": None, "frac": None, "traffic": None,
                    "basis": "no PMC traffic for this shape in %s" % TRAFFIC_FILE})
    return out


def lap_compulsory(N, E, C, state_passes):
    """Compulsory bytes of one K1 launch: x read once (its own rows and every
    gathered row), the CSR (col + weight 8E, rowptr), and `state_passes` more
    full passes over [N, C] (f written: 1; a fused rk4 stage: 2 on average —
    its stage output plus the average 1 extra stage operand)."""
    return 4 * N * C * (1 + state_passes) + 8 * E + 4 * (N + 1)


def bench_sharded(args, world, rank, dev, mode):
    """The headline on ONE graph shared by all ranks (strong scaling): 'cols' =
    feature-column stripes (no per-RHS collective), 'rows' = nnz-balanced row
    partition + RCCL all-gather of the state per RHS.  Also times the same graph
    unsharded on each rank's GPU first (speedup_vs_1gpu)."""
    N, E, C, h = args.nodes, args.edges, args.dim, args.step_size
    if not dist.is_initialized():  # single process: a world of one
        import random
        dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % random.randint(20000, 40000), rank=0,
                                world_size=1, device_id=dev)
    r = sharded_point(N, E, C, h, args.steps, args.warmup, world, dev, mode)
    return {
        "metric": METRIC, "value": r["value"], "unit": "RHS evals/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": r["ms_per_step"], "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "data": "synthetic (seeded RMAT graph, N(0,1) features)",
        "config": {"workload": "%s laplacian RHS, rk4, one graph sharded over %d GPUs (%s)%s" % (
            graph_name(N, E), world, mode, " (configs[2])" if C == 128 else ""),
            "nodes": N, "edges": E, "dim": C, "method": "rk4", "step_size": h, "rhs_per_step": 4,
            "global_batch": 1, "parallelism": "%s%d" % (mode, world)},
        "speedup_vs_1gpu": r["speedup_vs_1gpu"], "one_gpu_value": r["one_gpu_value"],
        "shard": r.get("shard"),
        "attention_sharded": None if args.no_attention else bench_attention_sharded(args, world, dev, mode),
    }


def progress(*a):
    """One line to stderr per bench phase (long sharded / G-rmat phases stay visibly alive)."""
    print("[bench %.1fs]" % (time.perf_counter() - T_START), *a, file=sys.stderr, flush=True)


T_START = time.perf_counter()


def sharded_point(N, E, C, h, steps, warmup, world, dev, mode, seed=0):
    """RHS evals/s of one graph in `mode` over the job's ranks, and the same graph
    integrated unsharded on one GPU (every rank at once, max over ranks)."""
    import gnpde
    from gnpde import dist as gd, synthetic
    progress("sharded point: N=%d E=%d C=%d mode=%s world=%d" % (N, E, C, mode, world))
    ei, w = synthetic.rw_graph(N, E, seed=seed, device=dev)
    x = synthetic.features(1, N, C, seed=1 + seed, device=dev)
    # the 1-GPU point of the curve: the whole graph on this rank's GPU
    func = gnpde.LaplacianODEFunc(C, C, dict(LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    el1, _ = timed_solve(func, x, steps, warmup, h, dev, world)
    progress("unsharded 1-GPU point: %.3f ms per step" % (el1 * 1e3 / steps))
    del func
    torch.cuda.empty_cache()
    alpha = torch.zeros((), device=dev)
    if mode == "rows":
        sh = gd.RowShardedLaplacian(ei, w, N, alpha)
        y0 = sh.scatter(x.view(-1, C))
        info = {"blocks_nnz": None, "nbmax": sh.nb}
    else:
        sh = gd.ColumnShardedLaplacian(ei, w, N, C, alpha)
        y0 = sh.split(x)
        info = {"columns_per_rank": sh.c1 - sh.c0}
    el, y = timed_solve(sh, y0, steps, warmup, h, dev, world)
    progress("%s: %.3f ms per step" % (mode, el * 1e3 / steps))
    if mode == "rows":
        rp = sh.g.csr.rowptr.cpu()
        info["blocks_nnz"] = [int(rp[b] - rp[a]) for a, b in sh.blocks]
    v1 = steps * 4 / el1
    v = steps * 4 / el
    out = {"value": round(v, 2), "ms_per_step": round(el * 1e3 / steps, 4), "one_gpu_value": round(v1, 2),
           "one_gpu_ms_per_step": round(el1 * 1e3 / steps, 4), "speedup_vs_1gpu": round(v / v1, 3),
           "shard": info}
    del sh, y, y0, x, ei, w
    torch.cuda.empty_cache()
    return out


def bench_attention_sharded(args, world, dev, mode, steps=8):
    """The transformer RHS on G-arxiv (configs[3]'s attention shape: heads 2,
    attention_dim 32, C = 128) sharded in `mode` (gnpde.dist.ColumnShardedTransformer
    / RowShardedTransformer) for the fork's scaled_dot (norm_idx 1)
    and upstream GRAND's per-edge scaled_dot (norm_idx 0): rk4 steps through the
    fused stages, against the unsharded ODEFuncTransformerAtt on each rank's GPU."""
    import gnpde
    from gnpde import dist as gd, synthetic
    N, E, C, h = args.nodes, args.edges, args.dim, args.step_size
    ei, _ = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    out = {"config": "ODEFuncTransformerAtt on %s (heads %d, attention_dim %d, C=%d), rk4 %d steps, %s over %d GPUs"
                     % (graph_name(N, E), ATTN_HEADS, ATTN_DIM, C, steps, mode, world)}
    for smode, norm_idx in (("reference", 1), ("per_edge", 0)):
        func = attention_func(smode, norm_idx, C, dev)
        func.edge_index = ei
        el1, _ = timed_solve(func, x, steps, 2, h, dev, world)
        lay = func.multihead_att_layer
        a = torch.full((), 0.0, device=dev)
        args_ = (ei, N, C, lay.Q.weight.detach(), lay.Q.bias.detach(), lay.K.weight.detach(), lay.K.bias.detach(),
                 ATTN_HEADS, norm_idx, a)
        if mode == "rows":
            sh = gd.RowShardedTransformer(*args_, score_mode=smode)
            y0 = sh.scatter(x)
        else:
            sh = gd.ColumnShardedTransformer(*args_, score_mode=smode)
            y0 = sh.split(x)
        el, _ = timed_solve(sh, y0, steps, 2, h, dev, world)
        out["%s_norm%d" % (smode, norm_idx)] = {
            "ms_per_step": round(el * 1e3 / steps, 4), "rhs_evals_per_s": round(4 * steps / el, 1),
            "one_gpu_ms_per_step": round(el1 * 1e3 / steps, 4), "speedup_vs_1gpu": round(el1 / el, 3),
            "collective_bytes_per_rhs": sh.bytes_per_rhs}
        progress("attention %s %s_norm%d: %.3f ms per step" % (mode, smode, norm_idx, el * 1e3 / steps))
        del sh, y0, func
        torch.cuda.empty_cache()
    return out


def bench_grmat(args, world, rank, dev):
    """configs[4]: G-rmat (N = 2M, E = 20M, C = 256) — one GPU at N = 1 (the first
    point of the curve); at N > 1 column stripes and the row partition +
    all-gather, each with its own unsharded 1-GPU time on the same job."""
    N, E, C, h = 2_000_000, 20_000_000, 256, args.step_size
    out = {"config": "configs[4] graph: RMAT N=%d E=%d C=%d, rk4 %d timed steps (step %.3g)" % (
        N, E, C, args.grmat_steps, h)}
    progress("configs[4] graph (G-rmat)")
    if world == 1:
        import gnpde
        from gnpde import synthetic
        ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
        x = synthetic.features(1, N, C, seed=1, device=dev)
        func = gnpde.LaplacianODEFunc(C, C, dict(LAP_OPT, hidden_dim=C), dev).to(dev)
        func.edge_index, func.edge_weight = ei, w
        el, _ = timed_solve(func, x, args.grmat_steps, 1, h, dev, world)
        launch_ms = el * 1e3 / args.grmat_steps / 4  # a replayed step is its 4 K1 launches back to back
        rl = roofline(launch_ms, rk4_fused_step_bytes(N, E, C) / 4.0, kernel_traffic("grmat", GRMAT_K1),
                      "agg_kernel<4,64,1,4,1,1,PlainWeights,float>: K1 with fused rk4 stage, one row per wavefront "
                      "(launch time = the replayed solve's time / its launches)", lap_compulsory(N, E, C, 2))
        rl["launch_ms"] = round(launch_ms, 4)
        out["one_gpu"] = {"value": round(args.grmat_steps * 4 / el, 2), "unit": "RHS evals/s",
                          "ms_per_step": round(el * 1e3 / args.grmat_steps, 4), "roofline": rl}
        del func, x, ei, w
        torch.cuda.empty_cache()
        return out
    for mode in ("cols", "rows"):
        out[mode] = sharded_point(N, E, C, h, args.grmat_steps, 1, world, dev, mode)
    return out


ATTN_HEADS, ATTN_DIM = 2, 32
ATTN_MODES = (("reference", 1), ("reference", 0), ("per_edge", 0), ("per_edge", 1))


def attention_func(mode, norm_idx, C, dev):
    """The drop-in ODEFuncTransformerAtt of the attention lines (configs[3] shape
    h = 2, att = 32), Q/K weights N(0, 0.1^2) drawn from one seed per mode."""
    import gnpde
    gen = torch.Generator(device=dev)
    gen.manual_seed(2 + 10 * ATTN_MODES.index((mode, norm_idx)))
    opt = {'hidden_dim': C, 'heads': ATTN_HEADS, 'attention_dim': ATTN_DIM, 'attention_norm_idx': norm_idx,
           'attention_type': 'scaled_dot', 'attention_score_mode': mode, 'function': 'transformer',
           'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9, 'multi_modal': False,
           'mix_features': False, 'square_plus': False, 'beltrami': False}
    func = gnpde.ODEFuncTransformerAtt(C, C, opt, dev).to(dev).eval()
    with torch.no_grad():
        for lin in (func.multihead_att_layer.Q, func.multihead_att_layer.K):
            lin.weight.copy_(torch.randn(ATTN_DIM, C, generator=gen, device=dev) * 0.1)
            lin.bias.copy_(torch.randn(ATTN_DIM, generator=gen, device=dev) * 0.1)
    return func


def blend_func(dev):
    """configs[3] shape: the BLEND transformer RHS (fork scaled_dot, norm_idx 0), C = 162."""
    import gnpde
    C = BLEND_C
    opt = {'hidden_dim': C, 'heads': 2, 'attention_dim': 32, 'attention_norm_idx': 0, 'attention_type': 'scaled_dot',
           'function': 'transformer', 'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9,
           'multi_modal': False, 'mix_features': False, 'square_plus': False, 'beltrami': False}
    return gnpde.ODEFuncTransformerAtt(C, C, opt, dev).to(dev).eval()


BLEND_C = 162
BLEND_K1 = {"fp32": "agg_kernel<4, 64, 1, 4, 1, 1, PlainWeights, float>",
            "bf16": "agg_kernel<8, 21, 1, 4, 3, 1, PlainWeights, bf16>"}


def solve_numbering(func, x):
    """(state, layout): the numbering a fixed-grid solve of ``func`` runs in
    (gnpde.ops.NodeLayout, the graph's in-degree order) and x in it; (x, None)
    when the module keeps the user numbering."""
    lay = func.node_layout(x)
    return (x, None) if lay is None else (lay.to_internal(x), lay)


def _time_rhs(func, x, lay, reps):
    """(eager ms, graph-replayed ms: the median of three windows of ``reps``
    replays) of one RHS evaluation of ``func`` at x in the numbering ``lay``
    (None: the user numbering)."""
    func._layout = lay
    try:
        with torch.no_grad():
            for _ in range(3):
                func(None, x)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                func(None, x)
            e.record()
            torch.cuda.synchronize()
            ms_eager = s.elapsed_time(e) / reps
            # the same RHS replayed from a captured hipGraph, as the fixed-grid integrator
            # runs it (gnpde.integrator._StepGraphs): device time without the eager path's
            # per-launch host cost
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg):
                func(None, x)
            for _ in range(3):
                cg.replay()
            torch.cuda.synchronize()
            wins = []
            for _ in range(3):  # the median of three windows of `reps` replays
                s.record()
                for _ in range(reps):
                    cg.replay()
                e.record()
                torch.cuda.synchronize()
                wins.append(s.elapsed_time(e) / reps)
            ms = sorted(wins)[1]
            del cg
    finally:
        func._layout = None
    return ms_eager, ms


def bench_attention(g, x, dev, ops, reps=50):
    """The transformer RHS through the drop-in ODEFuncTransformerAtt (config C4 shape),
    in the node numbering a fixed-grid solve runs it in (the graph's in-degree order,
    gnpde.ops.NodeLayout: VERDICT r3 item 4); the user-numbering time beside it."""
    C = x.shape[-1]
    heads, att = ATTN_HEADS, ATTN_DIM
    out = {"config": "ODEFuncTransformerAtt, C=%d heads=%d attention_dim=%d (configs[3] shape, fp32), one RHS in "
                     "the solve's node numbering" % (C, heads, att)}
    for mode, norm_idx in ATTN_MODES:
        func = attention_func(mode, norm_idx, C, dev)
        func.edge_index = g.edge_index
        func.graph_for(x)  # builds this function's CSR/CSC + plans once (outside the timed loop)
        xs, lay = solve_numbering(func, x)
        ms_eager, ms = _time_rhs(func, xs, lay, reps)
        ms_user = _time_rhs(func, x, None, reps)[1] if lay is not None else ms
        kind = "uniform" if (mode, norm_idx) == ("reference", 0) else mode
        nb = attn_bytes(g.N, g.nnz, C, att, kind)
        cb = attn_compulsory(g.N, g.nnz, C, att, kind)
        tb = rhs_traffic("attn:%s_norm%d" % (mode, norm_idx))
        t = ms * 1e-3
        ent = {"rhs_ms": round(ms, 4), "rhs_ms_eager": round(ms_eager, 4), "rhs_ms_user_numbering": round(ms_user, 4),
               "node_order": "degree" if lay is not None else "none",
               "algorithmic_bytes": nb, "algorithmic_frac": round(nb / t / 1e9 / HBM_PEAK_GBS, 4),
               "compulsory_bytes": cb, "compulsory_frac": round(cb / t / 1e9 / HBM_PEAK_GBS, 4)}
        if tb:
            ent.update({"traffic": int(tb), "achieved_GBs": round(tb / t / 1e9, 1),
                        "frac": round(tb / t / 1e9 / HBM_PEAK_GBS, 4),
                        "basis": "PMC bytes of every kernel of one RHS (%s workload attn:%s_norm%d, same numbering; "
                                 "counters include Infinity-Cache hits: an upper bound of HBM bytes) / "
                                 "replayed RHS time" % (TRAFFIC_FILE, mode, norm_idx)})
        else:
            ent.update({"traffic": None, "frac": None, "basis": "no PMC traffic in %s" % TRAFFIC_FILE})
        # the RHS inside the adaptive solve the reference runs (dopri5 at ogbn-arxiv's best_params
        # T / tol_scale): the fused step's stage pass and error reduction included
        T, ts = ARXIV_DOPRI5
        func.nfe = 0
        el, steps, nfe = _timed_dopri5(func, x, T, ts, dev, 3)
        ent["dopri5"] = {"ms_per_solve": round(el * 1e3, 4), "steps": steps, "rhs_evals": nfe,
                         "dopri5_ms_per_step": round(el * 1e3 / max(steps, 1), 4),
                         "ms_per_rhs_in_solve": round(el * 1e3 / max(nfe, 1), 4),
                         "config": "dopri5 over [0, %.3f] at tol_scale %.1f (ogbn-arxiv best_params)" % (T, ts)}
        out["%s_norm%d" % (mode, norm_idx)] = ent
    return out


def attn_compulsory(N, E, C, att, mode):
    """Compulsory bytes of one attention RHS: x read once and f written (8NC), the
    aggregation CSR (col 4E, rowptr 4(N+1)); the softmax groups' CSC (4E +
    4(N+1)) when the weights depend on x (not 'uniform', whose 1/outdeg weights
    are cached: + 4E); per_edge: + q, k written and read once (4 * 2N*att * 2)."""
    base = 8 * N * C + 4 * E + 4 * (N + 1)
    if mode == "uniform":
        return base + 4 * E
    if mode == "per_edge":
        return base + 4 * E + 4 * (N + 1) + 16 * N * att
    return base + 4 * E + 4 * (N + 1)


def bench_blend(g, dev, reps=50):
    """configs[3] shape: the BLEND transformer RHS (fork scaled_dot under
    source-grouped softmax -> cached 1/outdeg weights), C = 162 (64 features +
    98 positional), one rk4 step per 4 RHS, fp32 and bf16 state storage.
    Checked on the spot: one bf16 RHS against the fp32 RHS of the same state
    (SURVEY §8(d) bf16 gate 2e-2), and the RHS of a constant state is 0 (the
    1/outdeg weights are row-stochastic: A 1 = 1); the fp64 oracle check at full
    size is tests/test_gpu_blend.py."""
    import gnpde
    from gnpde import synthetic
    C = BLEND_C
    out = {"config": "BLEND transformer RHS, fork scaled_dot norm_idx 0 (uniform weights), C=162, rk4 steps "
                     "(configs[3] shape on the G-arxiv graph)"}
    x32 = synthetic.features(1, g.N, C, seed=3, device=dev)
    res = {}
    for name, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        func = blend_func(dev)
        func.edge_index = g.edge_index
        x = x32.to(dt)
        with torch.no_grad():
            t = torch.tensor([0.0, 0.25 * reps], device=dev)
            gnpde.odeint(func, x, t, method='rk4', options={'step_size': 0.25})  # warm-up: same call
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            gnpde.odeint(func, x, t, method='rk4', options={'step_size': 0.25})
            e.record()
            torch.cuda.synchronize()
            # one RHS of the same (bf16-representable) state in both storages
            res[name] = func(None, x32.to(torch.bfloat16).to(dt))
            if name == "fp32":
                const_rhs = float(func(None, torch.ones_like(x)).abs().max())
        ms = s.elapsed_time(e) / reps
        es = 2 if dt == torch.bfloat16 else 4
        Cp = 168 if dt == torch.bfloat16 else 164  # the zero-padded width the fused integrator runs
        # per step: 4 x (gathers es*EC + CSR/weights 8E + 4(N+1) + own row es*NC) + 8 state passes es*NC
        nb = 4 * (es * g.nnz * Cp + 8 * g.nnz + 4 * (g.N + 1) + es * g.N * Cp) + 8 * es * g.N * Cp
        gbs = nb / (ms * 1e-3) / 1e9
        ent = {"ms_per_step": round(ms, 4), "rhs_per_s": round(4e3 / ms, 1), "algorithmic_GBs": round(gbs, 1),
               "algorithmic_frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_step": nb}
        kb = kernel_traffic("blend_%s" % name, BLEND_K1[name])
        if kb:
            # K1 launches at ~the step's time / 4: the counter bytes of the four over the step time
            ent.update({"k1": BLEND_K1[name], "traffic_per_step": int(4 * kb),
                        "frac": round(4 * kb / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                        "basis": "PMC bytes of the 4 K1 launches of a step (%s workload blend_%s; counters include "
                                 "Infinity-Cache hits: an upper bound of HBM bytes) / step time" %
                                 (TRAFFIC_FILE, name)})
        out[name] = ent
    a, b = res["fp32"].double(), res["bf16"].double()
    rel = float((a - b).abs().max() / a.abs().max())
    out["check"] = {"bf16_vs_fp32_rel": round(rel, 6), "constant_state_rhs_max": const_rhs,
                    "ok": bool(rel <= 2e-2 and const_rhs <= 1e-5)}
    return out


# src/best_params.py: every dataset integrates with dopri5; ogbn-arxiv (:7) over T = 3.676 at
# tol_scale 11353.6, Cora (:1, configs[1]) over T = 18.29 at tol_scale 822.0 (atol = 1e-7 tol_scale,
# rtol = 1e-9 tol_scale, src/base_classes.py set_tol)
ARXIV_DOPRI5 = (3.6760155951687636, 11353.558848254957)
CORA_DOPRI5 = (18.294754260552843, 821.9773048827274)


def _timed_dopri5(func, x, T, tol_scale, dev, reps):
    """Two warm-up solves, then `reps` solves of dopri5 over [0, T], each timed from its
    call to a device sync after it (the steps' host reads inside); the median solve
    (a box's occasional slow solve — host preemption — does not move it)."""
    import gnpde
    import gnpde.integrator as integ
    t = torch.tensor([0.0, T], dtype=torch.float32, device=dev)
    kw = dict(method='dopri5', rtol=1e-9 * tol_scale, atol=1e-7 * tol_scale)
    with torch.no_grad():
        for _ in range(2):  # warm-up: the step graphs of every binding a solve meets are captured
            z = gnpde.odeint(func, x, t, **kw)[1]
        torch.cuda.synchronize()
        nfe0 = func.nfe
        els = []
        for _ in range(reps):
            t0 = time.perf_counter()
            z = gnpde.odeint(func, x, t, **kw)[1]
            torch.cuda.synchronize()
            els.append(time.perf_counter() - t0)
        el = sorted(els)[len(els) // 2]
    assert torch.isfinite(z).all()
    steps = integ.odeint.last_n_steps
    nfe = (func.nfe - nfe0) // reps
    return el, steps, nfe


def bench_dopri5(ei, w, x, dev, k1_stage_ms, k1_plain_ms, reps=9):
    """dopri5 as the reference runs it (src/best_params.py): the fused adaptive step
    (gnpde.integrator._RKAdaptiveFused: stage combinations and error rows in the RHS
    epilogues, one fixed-order norm reduction and one host read per step).
    G-arxiv Laplacian at ogbn-arxiv's T / tol_scale, and configs[1]'s shape (a
    Cora-sized graph, transformer RHS: fork scaled_dot, heads 8, attention_dim 128,
    norm_idx 1, C = 80) at Cora's."""
    import gnpde
    import gnpde.integrator as integ
    from gnpde import synthetic
    out = {}
    C = x.shape[-1]
    func = gnpde.LaplacianODEFunc(C, C, dict(LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    T, ts = ARXIV_DOPRI5
    el, steps, nfe = _timed_dopri5(func, x, T, ts, dev, reps)
    plan = integ._adaptive_plan('dopri5')
    ms_step = el * 1e3 / max(steps, 1)
    r, wr = plan.state_passes()
    affine = bool(getattr(func, 'affine', False)) and integ.AFFINE_STAGE
    krylov = affine and integ.KRYLOV_STEP
    if krylov:  # the Krylov step (integrator._KrylovPlan): only the last launch reads / writes more
        r, wr = integ._KrylovPlan(plan).state_passes()
    elif affine:  # no first stage-input pass (y0 and k0 read, X0 written): launch 0 reads k0 as its input
        r, wr = r - 2, wr - 1
    # device time of one step: a captured step (6 RHS launches, the error reduction and the device
    # controller) replayed back to back between HIP events on the launch stream
    dev_ms = None
    g = integ.adaptive_step_graph(func)
    if g is not None:
        for _ in range(3):
            g.replay()
        torch.cuda.synchronize()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record()
        for _ in range(20):
            g.replay()
        s1.record()
        torch.cuda.synchronize()
        dev_ms = s0.elapsed_time(s1) / 20
    N, E = x.shape[1], ei.shape[2]
    # algorithmic bytes of one step: 6 x (gathers 4EC + CSR 8E + rowptr 4(N+1) + own row 4NC) + the plan's
    # further state passes (reads + writes of 4NC each)
    alg = 6 * (4 * E * C + 8 * E + 4 * (N + 1) + 4 * N * C) + (r + wr) * 4 * N * C
    tb = step_traffic("dopri5")
    rl = None
    if dev_ms:
        t = dev_ms * 1e-3
        kern = ("5 STG1 + 1 STG5 agg_kernel launches (Krylov step; STG5: STG4 + the folded dense output)"
                if krylov else
                "2 STG1 + 4 STG4 agg_kernel launches")
        rl = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": "one replayed dopri5 step (%s, "
              "sum_partial_kernel, adaptive_control_kernel)" % kern, "step_ms": round(dev_ms, 4),
              "algorithmic_bytes_per_step": int(alg), "algorithmic_frac": round(alg / t / 1e9 / HBM_PEAK_GBS, 4)}
        if tb:
            rl.update({"traffic": int(tb), "achieved": round(tb / t / 1e9, 1),
                       "frac": round(tb / t / 1e9 / HBM_PEAK_GBS, 4),
                       "basis": "PMC bytes of one replayed step (%s workload dopri5; counters include Infinity-Cache "
                                "hits) / HIP-event step time" % TRAFFIC_FILE})
        else:
            rl.update({"traffic": None, "achieved": None, "frac": None,
                       "basis": "no PMC traffic for workload dopri5 in %s" % TRAFFIC_FILE})
    out["garxiv_laplacian"] = {
        "config": "G-arxiv laplacian (C=128), dopri5 over [0, %.3f], tol_scale %.1f (ogbn-arxiv best_params)" % (T, ts),
        "ms_per_solve": round(el * 1e3, 4), "steps": steps, "rhs_evals": nfe, "ms_per_step": round(ms_step, 4),
        "rhs_evals_per_s": round(nfe / el, 1),
        "ms_per_step_over_6_rhs_stage": round(ms_step / (6 * k1_stage_ms), 4),
        "ms_per_step_over_6_rhs_plain": round(ms_step / (6 * k1_plain_ms), 4) if k1_plain_ms else None,
        "step_ms_device": round(dev_ms, 4) if dev_ms else None,
        "state_passes_per_step": {"reads": r, "writes": wr},
        "affine_first_stage": affine,
        "krylov_step": krylov,
        "roofline": rl,
        "basis": "ms_per_step = whole solve (entry copy, initial-step selection, steps, dense output) / steps; "
                 "per step: 6 RHS launches (Krylov step, f affine: u_{p+1} = dt L u_p, the last launch forming y1, "
                 "f1, the error rows and — in the step crossing the output time — the dense output, from "
                 "u_0..u_5) + the error reduction with the device step-size controller, one host read; the "
                 "initial step's probe v = L f0 is the first step's u_1 / dt; rhs_stage_ms = the rk4 fused-stage "
                 "K1 launch time"}
    progress("dopri5 G-arxiv: %.3f ms/step, %d steps" % (ms_step, steps))
    # configs[1] shape
    N, E, Cc, h, att = 2708, 13264, 80, 8, 128  # Cora: 10,556 edges + 2,708 self loops
    gei, _ = synthetic.rw_graph(N, E, seed=5, device=dev)
    xc = synthetic.features(1, N, Cc, seed=6, device=dev)
    opt = {'hidden_dim': Cc, 'heads': h, 'attention_dim': att, 'attention_norm_idx': 1, 'attention_type': 'scaled_dot',
           'function': 'transformer', 'add_source': False, 'no_alpha_sigmoid': False, 'max_nfe': 10 ** 9,
           'multi_modal': False, 'mix_features': False, 'square_plus': False, 'beltrami': False}
    tf = gnpde.ODEFuncTransformerAtt(Cc, Cc, opt, dev).to(dev).eval()
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    with torch.no_grad():
        for lin in (tf.multihead_att_layer.Q, tf.multihead_att_layer.K):
            lin.weight.copy_(torch.randn(att, Cc, generator=gen, device=dev) * 0.03)
            lin.bias.copy_(torch.randn(att, generator=gen, device=dev) * 0.03)
    tf.edge_index = gei
    T, ts = CORA_DOPRI5
    el, steps, nfe = _timed_dopri5(tf, xc, T, ts, dev, reps)
    out["c2_transformer"] = {
        "config": "configs[1] shape: N=2708 E'=%d (RMAT + self loops), transformer RHS (fork scaled_dot, heads 8, "
                  "attention_dim 128, norm_idx 1), C=80, dopri5 over [0, %.2f], tol_scale %.1f (Cora best_params)"
                  % (E, T, ts),
        "ms_per_solve": round(el * 1e3, 4), "steps": steps, "rhs_evals": nfe,
        "ms_per_step": round(el * 1e3 / max(steps, 1), 4), "rhs_evals_per_s": round(nfe / el, 1)}
    progress("dopri5 C2: %.3f ms/step, %d steps" % (el * 1e3 / max(steps, 1), steps))
    return out


def bench_block(ei, x, h, dev, T=4.0, reps=5):
    """The drop-in block as GRAND's forward calls it (src/GNN.py:17 ->
    ConstantODEblock.forward, src/block_constant.py:22-59): reset_graph_data
    (self loops + rw normalisation, cached per graph), set_x0, rk4 over [0, T]
    through gnpde.odeint (in-degree numbering, captured steps), eval mode.  The
    raw RMAT edge list goes in (the block adds its own self loops)."""
    import gnpde
    C = x.shape[-1]
    N = x.shape[1]
    opt = dict(LAP_OPT, hidden_dim=C, method='rk4', step_size=h, self_loop_weight=1.0, data_norm='rw',
               tol_scale=1.0, adjoint=False, augment=False)
    blk = gnpde.ConstantODEblock(gnpde.LaplacianODEFunc, [], opt, dev,
                                 t=torch.tensor([0.0, T], device=dev)).to(dev).eval()
    data = gnpde.GraphData()
    raw = ei[:, :, :ei.shape[2] - N]  # synthetic.rw_graph appended N self loops; the block adds its own
    data.new_graph(raw, N)
    with torch.no_grad():
        for _ in range(2):
            blk.set_x0(x)
            blk(x, data)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            blk.set_x0(x)
            z = blk(x, data)
        e.record()
        torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    steps = int(round(T / h))
    assert torch.isfinite(z).all()
    return {"config": "ConstantODEblock.forward (eval), G-arxiv raw edges + block self loops, rk4 over [0, %g], "
                      "step %g" % (T, h),
            "ms_per_forward": round(ms, 4), "rk4_steps": steps, "rhs_evals_per_s": round(4 * steps / ms * 1e3, 1),
            "nfe": blk.odefunc.nfe}


def bench_train(ei, w, x, h, dev, steps=4, reps=5):
    """one training step of the drop-in path on G-arxiv —
    `steps` rk4 steps with autograd through every RHS (the eager path: K1
    forward, K1 over the CSC for d/dx, the alpha reduction), a linear loss, and
    backward to x and alpha_train.  Timed with events around the whole step."""
    import gnpde
    C = x.shape[-1]
    func = gnpde.LaplacianODEFunc(C, C, dict(LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    gout = torch.randn(x.shape, generator=gen, device=dev)
    t = torch.tensor([0.0, steps * h], dtype=torch.float32, device=dev)

    def one():
        xi = x.detach().requires_grad_(True)  # a fresh leaf on x's storage (no copy: not the step's work)
        func.alpha_train.grad = None
        y = gnpde.odeint(func, xi, t, method='rk4', options={'step_size': h})[1]
        (y * gout).sum().backward()
        return xi.grad

    for _ in range(2):
        one()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        gx = one()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    assert torch.isfinite(gx).all() and func.alpha_train.grad is not None
    return {"config": "G-arxiv laplacian, %d rk4 steps forward with autograd + backward to x and alpha_train "
                      "(eager drop-in path)" % steps,
            "ms_per_train_step": round(ms, 4), "ms_per_rk4_step_fwd_bwd": round(ms / steps, 4),
            "forward_rhs": 4 * steps}


def bench_train_adjoint(ei, w, x, dev, fwd_ms=None, reps=3):
    """SURVEY §8(f) next-1 as the reference trains ogbn-arxiv (src/best_params.py:7, src/base_classes.py:45-49,
    src/block_constant.py:34-44): odeint_adjoint with method dopri5 over [0, 3.676] at tol_scale 11353.6 and
    adjoint_method rk4 with adjoint_step_size 1 — forward the fused no-grad dopri5 solve, backward the fused
    continuous adjoint (gnpde.integrator._LaplacianAdjointFn: y and a integrated back over s = -t, eight K1
    launches per rk4 step, the alpha gradient's row terms in the CSC epilogues).  A linear loss, backward to x
    and alpha_train; HIP events around the whole training step."""
    import gnpde
    import gnpde.integrator as integ
    C = x.shape[-1]
    func = gnpde.LaplacianODEFunc(C, C, dict(LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    T, ts = ARXIV_DOPRI5
    t = torch.tensor([0.0, T], dtype=torch.float32, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(9)
    gout = torch.randn(x.shape, generator=gen, device=dev)

    def one():
        xi = x.detach().requires_grad_(True)
        func.alpha_train.grad = None
        y = integ.odeint_adjoint(func, xi, t, rtol=1e-9 * ts, atol=1e-7 * ts, method='dopri5',
                                 adjoint_method='rk4', adjoint_options={'step_size': 1.0},
                                 adjoint_rtol=1e-9, adjoint_atol=1e-7)[1]
        (y * gout).sum().backward()
        return xi.grad

    for _ in range(2):
        one()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    nfe0 = func.nfe
    s.record()
    for _ in range(reps):
        gx = one()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    assert torch.isfinite(gx).all() and func.alpha_train.grad is not None
    out = {"config": "G-arxiv laplacian (C=128), ogbn-arxiv best_params training: odeint_adjoint, dopri5 forward "
                     "over [0, %.3f] at tol_scale %.1f, adjoint_method rk4, adjoint_step_size 1" % (T, ts),
           "fused": integ._fused_adjoint_ok(func, x, 'rk4', tuple(p for p in func.parameters() if p.requires_grad)),
           "ms_per_train_step": round(ms, 4), "forward_ms_per_solve": fwd_ms,
           "train_over_forward": round(ms / fwd_ms, 3) if fwd_ms else None,
           "rhs_evals_per_train_step": (func.nfe - nfe0) // reps}
    out["adaptive_adjoint"] = _train_adaptive_adjoint(ei, x, gout, dev, reps)
    return out


# best_params of the attention-block datasets trained with an ADAPTIVE adjoint (src/best_params.py:3-4;
# src/base_classes.py set_tol: rtol = 1e-9 tol_scale, atol = 1e-7 tol_scale, the adjoint's from tol_scale_adjoint)
COAUTHOR_ADJ = (3.126400580172773, 9348.983916372074, 6599.1250595331385)
PUBMED_ADJ = (12.942327880200853, 1991.0688305523001, 16324.368093998313)
ADJ_BLOCKS = {
    # CoauthorCS (:4): block attention, scaled_dot heads 4 / attention_dim 8, norm_idx 1, dopri5 adjoint
    "coauthorcs": (COAUTHOR_ADJ, dict(heads=4, attention_dim=8, attention_norm_idx=1, attention_type='scaled_dot',
                                      leaky_relu_slope=0.7181389780997276, adjoint_method='dopri5', add_source=False)),
    # Pubmed (:3): block attention, cosine_sim heads 1 / attention_dim 16, norm_idx 0, adaptive_heun adjoint, add_source
    "pubmed": (PUBMED_ADJ, dict(heads=1, attention_dim=16, attention_norm_idx=0, attention_type='cosine_sim',
                                leaky_relu_slope=0.2, adjoint_method='adaptive_heun', add_source=True)),
}


def _adjoint_block(case, x, ei, dev):
    import gnpde
    C, N = x.shape[-1], x.shape[1]
    (T, ts, tsa), extra = ADJ_BLOCKS[case]
    opt = dict(LAP_OPT, hidden_dim=C, block='attention', function='laplacian', method='dopri5', adjoint=True,
               tol_scale=ts, tol_scale_adjoint=tsa, self_loop_weight=1.0, data_norm='rw', reweight_attention=False,
               square_plus=False, mix_features=False, beltrami=False, augment=False, max_iters=100, step_size=1,
               adjoint_step_size=1, **extra)
    torch.manual_seed(17)
    blk = gnpde.AttODEblock(gnpde.LaplacianODEFunc, [], opt, dev, t=torch.tensor([0.0, T], device=dev)).to(dev).train()
    data = gnpde.GraphData()
    data.new_graph(ei[:, :, :ei.shape[2] - N], N)  # synthetic.rw_graph appended N self loops; the block adds its own
    return blk, data, opt


def _train_adaptive_adjoint(ei, x, gout, dev, reps):
    """AttODEblock training steps as best_params runs them with an adaptive adjoint (src/best_params.py:3-4,
    src/block_transformer_attention.py:40-50, src/base_classes.py:45-49) on the G-arxiv graph (C = 128): the block
    attention, the dopri5 forward under no_grad, odeint_adjoint's backward with the attention weights a constant
    of it (torchdiffeq's semantics).  Backward paths: 'fused' (gnpde.adjoint_adaptive: stage combinations, error
    rows and the alpha integrand in the K1 epilogues), 'direct' (the restated torchdiffeq loop with the augmented
    RHS by K1 launches, GNPDE_FUSED_ADAPTIVE_ADJOINT=0), 'autograd' (that loop with autograd VJPs)."""
    import gnpde.integrator as integ
    res = {}
    saved = (integ.FUSED_ADJOINT, integ.FUSED_ADAPTIVE_ADJOINT)
    try:
        for case in ("coauthorcs", "pubmed"):
            blk, data, opt = _adjoint_block(case, x, ei, dev)
            (T, ts, tsa), _ = ADJ_BLOCKS[case]
            ent = {"config": "AttODEblock (%s best_params: heads %d, attention_dim %d, %s, norm_idx %d, add_source %s) "
                             "on G-arxiv, dopri5 over [0, %.3f] at tol_scale %.1f, adjoint %s at tol_scale_adjoint %.1f"
                             % (case, opt['heads'], opt['attention_dim'], opt['attention_type'],
                                opt['attention_norm_idx'], opt['add_source'], T, ts, opt['adjoint_method'], tsa)}

            def one():
                xi = x.detach().requires_grad_(True)
                blk.odefunc.alpha_train.grad = None
                blk.set_x0(xi)
                z = blk(xi, data)
                (z * gout).sum().backward()
                return xi.grad
            modes = (("fused", True, True), ("direct", True, False)) + \
                ((("autograd", False, False),) if case == "coauthorcs" else ())
            for name, fa, faa in modes:
                integ.FUSED_ADJOINT, integ.FUSED_ADAPTIVE_ADJOINT = fa, faa
                one()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                nfe0 = blk.odefunc.nfe
                s.record()
                for _ in range(reps):
                    gx = one()
                e.record()
                torch.cuda.synchronize()
                assert torch.isfinite(gx).all()
                ent[name] = {"ms_per_train_step": round(s.elapsed_time(e) / reps, 4),
                             "rhs_evals_per_train_step": (blk.odefunc.nfe - nfe0) // reps,
                             "backward_path": integ._OdeintAdjoint.last_path}
                progress("adaptive adjoint %s %s: %.3f ms" % (case, name, ent[name]["ms_per_train_step"]))
            res[case] = ent
    finally:
        integ.FUSED_ADJOINT, integ.FUSED_ADAPTIVE_ADJOINT = saved
    return res


# HardAttODEblock best_params (src/best_params.py:5,7): ogbn-arxiv (heads 2, attention_dim 32, att_samp_pct 0.81,
# adjoint rk4 step 1) and Computers (heads 4, attention_dim 64, att_samp_pct 0.573, adjoint dopri5)
HARD_BLOCKS = {
    "arxiv": dict(T=ARXIV_DOPRI5[0], tol_scale=ARXIV_DOPRI5[1], heads=2, attention_dim=32,
                  att_samp_pct=0.8105268910037231, adjoint_method='rk4', tol_scale_adjoint=1.0),
    "computers": dict(T=3.249016177876166, tol_scale=127.46369887079446, heads=4, attention_dim=64,
                      att_samp_pct=0.572918052062338, adjoint_method='dopri5', tol_scale_adjoint=443.81436775321754),
}


def bench_hard_attention_train(ei, x, dev, reps=3):
    """HardAttODEblock in training mode as best_params runs it (src/block_transformer_hard_attention.py:37-99) on
    G-arxiv (C = 128) at ogbn-arxiv's and Computers' parameters: one training forward — block attention, quantile
    threshold, sampling mask, group renormalisation, the dopri5 solve — and the training step with its adjoint
    backward.  The sampled graph reuses the full graph's CSR and plans: K1 gathers the retained edges only,
    compacted inside the plan's items on the device (gnpde_compact_items_f32, ops.CompactWeights); the forward is
    also timed over the masked full graph (GNPDE_COMPACT_SAMPLED=0) for comparison."""
    import contextlib
    import io

    import gnpde
    import gnpde.base_classes as bc
    C = x.shape[-1]
    N = x.shape[1]
    raw = ei[:, :, :ei.shape[2] - N]  # synthetic.rw_graph appended N self loops; the block adds its own
    data = gnpde.GraphData()
    data.new_graph(raw, N)
    gen = torch.Generator(device=dev)
    gen.manual_seed(13)
    gout = torch.randn(x.shape, generator=gen, device=dev)
    out = {}
    for case, prm in HARD_BLOCKS.items():
        T = prm['T']
        opt = dict(LAP_OPT, hidden_dim=C, block='hard_attention', function='laplacian', heads=prm['heads'],
                   attention_dim=prm['attention_dim'], attention_norm_idx=0, attention_type='scaled_dot',
                   att_samp_pct=prm['att_samp_pct'], method='dopri5', step_size=1, tol_scale=prm['tol_scale'],
                   adjoint=True, adjoint_method=prm['adjoint_method'], adjoint_step_size=1,
                   tol_scale_adjoint=prm['tol_scale_adjoint'], max_iters=100, self_loop_weight=1.0, data_norm='rw',
                   leaky_relu_slope=0.2, reweight_attention=False, square_plus=False, mix_features=False,
                   beltrami=False, use_flux=False, augment=False)
        torch.manual_seed(19)
        blk = gnpde.HardAttODEblock(gnpde.LaplacianODEFunc, [], opt, dev,
                                    t=torch.tensor([0.0, T], device=dev)).to(dev).train()

        def fwd():
            blk.set_x0(x)
            with contextlib.redirect_stdout(io.StringIO()):  # the reference's 'retaining ...' line per forward
                return blk(x, data)

        def sample():
            with contextlib.redirect_stdout(io.StringIO()):
                blk.sample_edges(x)

        def step():
            xi = x.detach().requires_grad_(True)
            blk.set_x0(xi)
            with contextlib.redirect_stdout(io.StringIO()):
                z = blk(xi, data)
            (z * gout).sum().backward()
            return xi.grad

        def timed(fn, with_grad):
            for _ in range(2):
                if with_grad:
                    fn()
                else:
                    with torch.no_grad():
                        fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                if with_grad:
                    fn()
                else:
                    with torch.no_grad():
                        fn()
            e.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e) / reps

        ms_fwd = timed(fwd, False)
        ms_sample = timed(sample, False)
        ms_step = timed(step, True)
        saved = bc.COMPACT_SAMPLED
        try:
            bc.COMPACT_SAMPLED = False
            ms_fwd_masked = timed(fwd, False)
        finally:
            bc.COMPACT_SAMPLED = saved
        out[case] = {"config": "HardAttODEblock.forward (training), %s best_params on G-arxiv (C=128): heads %d, "
                               "attention_dim %d, att_samp_pct %.3f, dopri5 over [0, %.3f] at tol_scale %.1f, adjoint %s"
                               % (case, prm['heads'], prm['attention_dim'], prm['att_samp_pct'], T, prm['tol_scale'],
                                  prm['adjoint_method']),
                     "ms_per_forward": round(ms_fwd, 4), "ms_per_forward_masked_full_graph": round(ms_fwd_masked, 4),
                     "ms_sampling": round(ms_sample, 4), "sampling_share": round(ms_sample / ms_fwd, 4),
                     "graph_rebuild_ms": 0.0, "retained_edges": int(blk.retained), "edges": int(raw.shape[2] + N),
                     "ms_per_train_step": round(ms_step, 4)}
        progress("hard attention %s: forward %.3f (masked %.3f) ms, step %.3f ms" % (case, ms_fwd, ms_fwd_masked,
                                                                                    ms_step))
    out["basis"] = ("sampling = block attention + head mean + quantile + threshold mask + group renormalisation (one "
                    "host read for the reference's 'retaining' line); the sampled graph reuses the full graph's CSR / "
                    "plans, its retained edges compacted inside the plan's items on the device (no rebuild)")
    return out


# Cora best_params (src/best_params.py:1): block attention over the Laplacian, heads 8, attention_dim 128,
# attention_norm_idx 1, scaled_dot, add_source, dopri5 over [0, 18.29] at tol_scale 822, direct backprop
# (adjoint False), hidden_dim 80, max_nfe 2000
CORA_TRAIN = dict(heads=8, attention_dim=128, attention_norm_idx=1, attention_type='scaled_dot', add_source=True,
                  leaky_relu_slope=0.2, max_nfe=2000)


def bench_train_cora(dev, reps=5):
    """One AttODEblock training step at Cora's best_params on a Cora-sized synthetic graph
    (2,708 nodes, 10,556 edges; the block adds self loops, rw normalisation; C = 80): the block attention
    (autograd-tracked), the dopri5 solve with autograd through every RHS (backprop, as Cora trains), a linear
    loss and the backward to x, alpha / beta and Q / K.  The dataset is absent (no network): synthetic data, so
    Cora's accuracy stays unpinned."""
    import gnpde
    import gnpde.integrator as integ
    from gnpde import synthetic
    N, E, C = 2708, 10556, 80
    T, ts = CORA_DOPRI5
    ei, _ = synthetic.rw_graph(N, E + N, seed=5, device=dev)
    raw = ei[:, :, :E]
    x = synthetic.features(1, N, C, seed=6, device=dev)
    opt = dict(LAP_OPT, hidden_dim=C, block='attention', function='laplacian', method='dopri5', step_size=1,
               tol_scale=ts, adjoint=False, self_loop_weight=1.0, data_norm='rw', reweight_attention=False,
               square_plus=False, mix_features=False, beltrami=False, augment=False, max_iters=100, **CORA_TRAIN)
    torch.manual_seed(23)
    blk = gnpde.AttODEblock(gnpde.LaplacianODEFunc, [], opt, dev, t=torch.tensor([0.0, T], device=dev)).to(dev).train()
    gen = torch.Generator(device=dev)
    gen.manual_seed(24)
    with torch.no_grad():
        for lin in (blk.multihead_att_layer.Q, blk.multihead_att_layer.K):
            lin.weight.copy_(torch.randn(lin.weight.shape, generator=gen, device=dev) * 0.03)
    data = gnpde.GraphData()
    data.new_graph(raw, N)
    gout = torch.randn(x.shape, generator=gen, device=dev)

    def fwd():
        blk.set_x0(x)
        return blk(x, data)

    def step():
        xi = x.detach().requires_grad_(True)
        blk.zero_grad(set_to_none=True)
        blk.set_x0(xi)
        z = blk(xi, data)
        (z * gout).sum().backward()
        return xi.grad

    def timed(fn, grad):
        with torch.set_grad_enabled(grad):
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            nfe0 = blk.odefunc.nfe
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                out = fn()
            e.record()
            torch.cuda.synchronize()
        assert torch.isfinite(out).all()
        return s.elapsed_time(e) / reps, (blk.odefunc.nfe - nfe0) // reps
    ms_step, nfe_step = timed(step, True)
    steps_train = integ.odeint.last_n_steps
    train_path = integ.odeint.last_path
    ms_fwd_grad, _ = timed(fwd, True)
    ms_eval, nfe_eval = timed(fwd, False)
    out = {"config": "AttODEblock training step, Cora best_params (heads 8, attention_dim 128, norm_idx 1, scaled_dot, "
                     "add_source, dopri5 over [0, %.2f] at tol_scale %.1f, backprop) on a Cora-sized synthetic graph "
                     "(N=%d, E=%d + self loops, C=%d)" % (T, ts, N, E, C),
           "ms_per_train_step": round(ms_step, 4), "rhs_evals_per_train_step": nfe_step, "steps": steps_train,
           "ms_forward_with_grad": round(ms_fwd_grad, 4), "ms_forward_no_grad": round(ms_eval, 4),
           "rhs_evals_no_grad": nfe_eval, "train_path": train_path, "eval_path": integ.odeint.last_path,
           "basis": "train_path 'fused_backprop': the solve and its discrete adjoint as one autograd node "
                    "(gnpde.adaptive_backprop); 'restated': autograd through every RHS (GNPDE_ADAPTIVE_BACKPROP=0)",
           "accuracy": "unpinned (the Cora dataset is absent: no network)"}
    progress("train cora: %.3f ms per step (%d RHS), no-grad forward %.3f ms" % (ms_step, nfe_step, ms_eval))
    return out


def cpu_baseline(ei, w, x, N, E, C, budget_s):
    """The reference's CPU path restated with torch.sparse: f = sigma(a)(A x - x)
    with A a torch CSR tensor (fp32), on the host cores of the GPU box, on a
    bounded sample of the same workload (as many full G-arxiv RHS evaluations as
    fit in ~budget_s seconds).  The literal reference densifies A ([N,N] = 114.7 GB
    at G-arxiv) and cannot run at this size.  The oracle's OpenMP C
    restatement is reported beside it (secondary)."""
    import numpy as np
    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = cgroup_cpus()
    # the job's CPU share: the cgroup quota when one is set (the GPU box gives each GPU's job
    # 16 CPUs of a 256-CPU host and exports OMP_NUM_THREADS=16 to match), else every visible CPU
    threads = int(os.environ.get("OMP_NUM_THREADS", quota or cpus))
    model = "unknown CPU"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass

    def timed(fn, budget):
        fn()  # warm
        n, t0 = 0, time.perf_counter()
        while True:
            y = fn()
            n += 1
            el = time.perf_counter() - t0
            if (el > budget and n >= 3) or n >= 2000:
                return n, el, y

    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        ec, wcpu = ei[0].cpu(), w[0].cpu()
        A = torch.sparse_coo_tensor(ec, wcpu, (N, N)).coalesce().to_sparse_csr()
        xc = x.view(N, C).cpu()
        a = torch.sigmoid(torch.tensor(0.0))
        n, el, y = timed(lambda: a * (A @ xc - xc), budget_s / 2)
        assert torch.isfinite(y).all()
    finally:
        torch.set_num_threads(prev)
    out = {"value": round(n / el, 3), "unit": "RHS evals/s", "cores": threads, "kind": "port",
           "sample": "%d full G-arxiv Laplacian RHS evaluations (N=%d, E'=%d, C=%d) in %.1f s: torch sparse CSR "
                     "A@x, fp32, torch %s, %d threads of %d visible host CPUs (%s)" % (
                         n, N, E, C, el, torch.__version__, threads, cpus, model),
           "cpu_model": model, "visible_cpus": cpus, "cgroup_cpu_quota": quota}
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        out["attention"] = cpu_attention_baseline(ei, x, N, C, budget_s / 3, threads, timed)
    finally:
        torch.set_num_threads(prev)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import gnpde_oracle as O
        ein, wn, xn = ei.cpu().numpy(), w.cpu().numpy(), x.cpu().numpy()
        co = O.COracle()
        csr = co.csr(ein, wn, N)
        n2, el2, y2 = timed(lambda: co.laplacian_rhs(csr, xn, 0.0, nthreads=threads), budget_s / 6)
        assert np.isfinite(y2).all()
        out["oracle_c_openmp"] = {"value": round(n2 / el2, 3), "unit": "RHS evals/s", "cores": threads,
                                  "sample": "%d RHS evaluations in %.1f s; oracle C restatement (fp32 CSR, OpenMP)" %
                                            (n2, el2)}
    except OSError as exc:  # liboracle.so not built
        out["oracle_c_openmp"] = {"error": "oracle/build/liboracle.so unavailable: %s" % exc}
    return out


def cgroup_cpus():
    """CPUs the job's cgroup may use (cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as fh:
                q, p = fh.read().split()[:2]
            if q != "max":
                return max(1, int(round(int(q) / int(p))))
        except (OSError, ValueError):
            pass
    return None


def cpu_attention_baseline(ei, x, N, C, budget, threads, timed):
    """The attention RHS of the bench's reference_norm1 line (fork scaled_dot,
    destination-grouped softmax, head mean, aggregation; src/function_transformer_
    attention.py:218-267, src/utils.py:116-127) restated with torch CPU ops in
    fp32 at O(E*d) — the fork's literal [h, E, E] score matmul is 2.9 TB at
    G-arxiv and cannot run.  Same weights as the GPU line (bench.attention_func)."""
    gen = torch.Generator(device=x.device)
    gen.manual_seed(2)  # attention_func's seed for ("reference", 1)
    Wq = (torch.randn(ATTN_DIM, C, generator=gen, device=x.device) * 0.1).cpu()
    bq = (torch.randn(ATTN_DIM, generator=gen, device=x.device) * 0.1).cpu()
    Wk = (torch.randn(ATTN_DIM, C, generator=gen, device=x.device) * 0.1).cpu()
    bk = (torch.randn(ATTN_DIM, generator=gen, device=x.device) * 0.1).cpu()
    src, dst = ei[0, 0].cpu(), ei[0, 1].cpu()
    xc = x.view(N, C).cpu()
    H, dk = ATTN_HEADS, ATTN_DIM // ATTN_HEADS
    a = torch.sigmoid(torch.tensor(0.0))

    def rhs():
        q = xc @ Wq.t() + bq
        k = xc @ Wk.t() + bk
        S = k.index_select(0, dst).sum(0)                            # the fork's sum over edges of k_dst
        cs = (q.view(N, H, dk) * S.view(1, H, dk)).sum(-1) / dk ** 0.5  # [N, H]
        s = cs.index_select(0, src)                                   # [E, H]
        m = torch.full((N, H), -float("inf")).index_reduce_(0, dst, s, "amax")
        e = torch.exp(s - m.index_select(0, dst))
        den = torch.zeros(N, H).index_add_(0, dst, e)
        att = e / (den.index_select(0, dst) + 1e-16)
        wm = att.mean(1)
        ax = torch.zeros(N, C).index_add_(0, src, wm[:, None] * xc.index_select(0, dst))
        return a * (ax - xc)

    n, el, y = timed(rhs, budget)
    assert torch.isfinite(y).all()
    out = {"value": round(n / el, 3), "unit": "RHS evals/s", "cores": threads, "kind": "port",
           "sample": "%d attention RHS evaluations (reference scaled_dot, norm_idx 1, h=%d, att=%d, G-arxiv) in "
                     "%.1f s: torch CPU fp32 index ops" % (n, H, ATTN_DIM, el)}
    if x.is_cuda:  # the restatement computes what the GPU line computes
        func = attention_func("reference", 1, C, x.device)
        func.edge_index = ei
        with torch.no_grad():
            fg = func(None, x).view(N, C).cpu()
        out["vs_gpu_rel"] = float((fg - y).abs().max() / y.abs().max())
    return out


if __name__ == "__main__":
    main()
