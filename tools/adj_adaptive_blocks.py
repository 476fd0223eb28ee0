"""The adaptive-adjoint training steps of bench.py (AttODEblock at CoauthorCS / Pubmed best_params on
G-arxiv) on their own: python tools/adj_adaptive_blocks.py [reps] -> one JSON line."""
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(9)
    gout = torch.randn(x.shape, generator=gen, device=dev)
    print(json.dumps(bench._train_adaptive_adjoint(ei, x, gout, dev, reps)), flush=True)


if __name__ == "__main__":
    main()
