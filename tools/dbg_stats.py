"""Per-block destination statistics (gnpde.dist partitioned statistics, per-edge
scaled_dot on G-arxiv) against the whole-CSC launch: rows that differ, their degree
and values, at 2 / 4 / 8 blocks (tests/test_gpu_attn_sharded.py's bar).
  python tools/dbg_stats.py"""
import sys, os, torch
sys.path.insert(0, "graph-neural-pde_amd"); sys.path.insert(0, ".")
from gnpde import ops, synthetic, dist as gd
dev = "cuda"
N, E, C, H, ATT = 169343, 1200000, 128, 2, 32
ei, _ = synthetic.rw_graph(N, E, seed=0, device=dev)
g = ops.GraphCSR(ei, N)
x = synthetic.features(1, N, C, seed=1, device=dev)
gen = torch.Generator(device=dev); gen.manual_seed(2)
Wq, Wk = [torch.randn(ATT, C, generator=gen, device=dev) * 0.1 for _ in range(2)]
bq, bk = [torch.randn(ATT, generator=gen, device=dev) * 0.1 for _ in range(2)]
ns = ops.node_scores(g, x, Wq, bq, Wk, bk, H, 'scaled_dot', 'per_edge', wcat=(torch.cat([Wq, Wk]), torch.cat([bq, bk])))
_, _, mr = ops.softmax_stats(g, ns, 1, packed=True)
nz = torch.diff(g.csc.rowptr) > 0
deg = torch.diff(g.csc.rowptr)
for world in (2, 4, 8):
    blocks, nb = gd._dst_blocks(ei, N, world, g)
    got = torch.full_like(mr, float('nan'))
    for r0, r1 in blocks:
        part = gd._hip_stats_rows(g, ns, r0, r1)
        got[r0:r1] = part[0][r0:r1]
    bad = (got != mr).any(1) & nz
    idx = bad.nonzero().flatten()
    print(world, "bad rows", int(bad.sum()), "nan", int(torch.isnan(got[nz]).any(1).sum()), "first", idx[:5].tolist(),
          "deg", deg[idx[:5]].tolist(), "blocks", blocks[:3])
    if len(idx):
        i = int(idx[0]); print(" got", got[i].tolist(), "want", mr[i].tolist())
