#!/usr/bin/env python
"""bench.bench_train on G-arxiv (4 rk4 steps forward + backward), run under
rocprofv3 --kernel-trace to see one training step's kernel timeline
(tools/timeline.py reads the trace).  After the bench's own reps, one more
training step runs between two markers (gnpde_dot_f64 launches: dot_final_kernel,
used nowhere else in the step): the timeline's window starts at the first."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    import gnpde
    from gnpde import ops, synthetic
    dev = torch.device("cuda", 0)
    N, E = synthetic.ARXIV_N, synthetic.ARXIV_E
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, 128, seed=1, device=dev)
    r = bench.bench_train(ei, w, x, 0.25, dev, reps=3)
    print(r)
    # one more step between markers, as bench_train's one()
    C = x.shape[-1]
    func = gnpde.LaplacianODEFunc(C, C, dict(bench.LAP_OPT, hidden_dim=C), dev).to(dev)
    func.edge_index, func.edge_weight = ei, w
    gout = torch.randn(x.shape, device=dev)
    t = torch.tensor([0.0, 1.0], dtype=torch.float32, device=dev)
    mk = torch.ones(64, device=dev)

    def one():
        xi = x.detach().requires_grad_(True)
        func.alpha_train.grad = None
        y = gnpde.odeint(func, xi, t, method='rk4', options={'step_size': 0.25})[1]
        (y * gout).sum().backward()
        return xi.grad
    for _ in range(2):
        one()
    torch.cuda.synchronize()
    ops.dot(mk, mk)
    one()
    ops.dot(mk, mk)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
