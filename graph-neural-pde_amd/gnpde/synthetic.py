"""Seeded synthetic graphs for measurement and parity tests.

No datasets are reachable (no network); the benchmark graphs are RMAT graphs of
the reference configs' sizes:

* G-arxiv: N = 169,343 nodes, E' = 1,200,000 edges = 1,030,657 RMAT edges
  (a,b,c,d = 0.57,0.19,0.19,0.05; duplicates kept and summed) + N self loops,
  random-walk normalised (w_e = 1/indeg(dst(e)), utils.get_rw_adj norm_dim=1).
* G-cora: N = 2,708, E' = 13,264; G-rmat: N = 2,000,000, E = 20,000,000.

Generated on the device with torch (once, outside every timed region).
"""
import math

import torch

ARXIV_N = 169343
ARXIV_E = 1200000
CORA_N = 2708
CORA_E = 13264


def rmat_edges(num_nodes, num_edges, a=0.57, b=0.19, c=0.19, seed=0, device='cuda'):
    """[2, num_edges] int64 RMAT edges folded into [0, num_nodes) by modulo."""
    scale = max(1, int(math.ceil(math.log2(max(num_nodes, 2)))))
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    src = torch.zeros(num_edges, dtype=torch.int64, device=device)
    dst = torch.zeros(num_edges, dtype=torch.int64, device=device)
    ab, abc = a + b, a + b + c
    for _ in range(scale):
        r = torch.rand(num_edges, generator=gen, device=device)
        sbit = (r > ab).long()
        dbit = (((r > a) & (r <= ab)) | (r > abc)).long()
        src = src * 2 + sbit
        dst = dst * 2 + dbit
    return torch.stack([src % num_nodes, dst % num_nodes], 0)


def rw_graph(num_nodes, num_edges_total, seed=0, device='cuda', batch=1, self_loops=True):
    """[B,2,E'] edge_index (RMAT + self loops) and rw-normalised weights [B,E']."""
    n_rmat = num_edges_total - (num_nodes if self_loops else 0)
    eis = []
    for b in range(batch):
        e = rmat_edges(num_nodes, n_rmat, seed=seed + 7919 * b, device=device)
        if self_loops:
            ar = torch.arange(num_nodes, device=device)
            e = torch.cat([e, torch.stack([ar, ar])], 1)
        eis.append(e)
    ei = torch.stack(eis, 0)
    w = torch.ones(ei.shape[0], ei.shape[2], dtype=torch.float32, device=device)
    deg = torch.zeros(ei.shape[0], num_nodes, dtype=torch.float32, device=device).scatter_add_(1, ei[:, 1], w)
    w = w / torch.gather(deg, 1, ei[:, 1])
    return ei, w


def features(batch, num_nodes, dim, seed=1, device='cuda'):
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    return torch.randn(batch, num_nodes, dim, generator=gen, device=device, dtype=torch.float32)
