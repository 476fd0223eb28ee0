"""One part of bench.py on its own (G-arxiv, C = 128): python tools/bench_part.py PART [reps]
PART: adaptive_adjoint | hard_attention | dopri5 | train_adjoint | train_cora | train_rk4 | blend -> one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from gnpde import synthetic  # noqa: E402


def main():
    part = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    if part == "adaptive_adjoint":
        gen = torch.Generator(device=dev)
        gen.manual_seed(9)
        gout = torch.randn(x.shape, generator=gen, device=dev)
        res = bench._train_adaptive_adjoint(ei, x, gout, dev, reps)
    elif part == "hard_attention":
        res = bench.bench_hard_attention_train(ei, x, dev, reps)
    elif part == "dopri5":
        res = bench.bench_dopri5(ei, w, x, dev, 0.0888, 0.0760, reps)
    elif part == "train_adjoint":
        res = bench.bench_train_adjoint(ei, w, x, dev, None, reps)
    elif part == "train_cora":
        res = bench.bench_train_cora(dev, reps)
    elif part == "train_rk4":
        res = bench.bench_train(ei, w, x, 0.25, dev)
    elif part == "blend":
        import gnpde
        func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
        func.edge_index, func.edge_weight = ei, w
        with torch.no_grad():
            g = func.graph_for(x)
        res = bench.bench_blend(g, dev)
    else:
        raise SystemExit("unknown part %r" % part)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
