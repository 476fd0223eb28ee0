"""Team-mode vs lane-mode attention kernels on one small graph (diagnostics):
prints max |diff| of m, rl and the COO attention against the oracle.  Run with
GNPDE_TEAM=0 and =1."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import gnpde_oracle as O  # noqa: E402
from gnpde import ops  # noqa: E402
from test_gpu_parity import hub_graph  # noqa: E402

DEV = torch.device("cuda", 0)
T = lambda a: torch.as_tensor(a, device=DEV)  # noqa: E731
for mode in ["scaled_dot", "exp_kernel", "cosine_sim", "pearson"]:
    for norm_idx in (0, 1):
        N, E, C, h, att = 2000, 30000, 48, 4, 32
        ei = hub_graph(N, E, seed=norm_idx + 5)
        rng = np.random.default_rng(9)
        x = rng.standard_normal((1, N, C)).astype(np.float32)
        Wq, Wk = [(rng.standard_normal((att, C)) * 0.1).astype(np.float32) for _ in range(2)]
        bq, bk = [(rng.standard_normal(att) * 0.1).astype(np.float32) for _ in range(2)]
        g = ops.GraphCSR(T(ei), N)
        ns = ops.node_scores(g, T(x), T(Wq), T(bq), T(Wk), T(bk), h, mode, 'per_edge', 1.3, 0.8)
        m, rl = ops.softmax_stats(g, ns, norm_idx)
        a = ops.edge_attention(g, ns, m, rl, norm_idx)
        wa = O.transformer_attention(x, ei, Wq, bq, Wk, bk, h, norm_idx, mode, 'per_edge', output_var=1.3,
                                     lengthscale=0.8)
        d = np.abs(a.double().cpu().numpy() - wa)
        print(os.environ.get("GNPDE_TEAM", "1"), mode, norm_idx, "att maxdiff %.3g" % d.max(),
              "m finite %d/%d" % (int(torch.isfinite(m).sum()), m.numel()), "nan att %d" % int(torch.isnan(a).sum()))
