#!/usr/bin/env python
"""bench.bench_train on G-arxiv (4 rk4 steps forward + backward), run under
rocprofv3 --kernel-trace to see one training step's kernel timeline
(tools/timeline.py reads the trace).  Markers: a fill kernel of 7 elements
before and after the last step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    from gnpde import synthetic
    dev = torch.device("cuda", 0)
    N, E = synthetic.ARXIV_N, synthetic.ARXIV_E
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, 128, seed=1, device=dev)
    r = bench.bench_train(ei, w, x, 0.25, dev, reps=3)
    print(r)


if __name__ == "__main__":
    main()
