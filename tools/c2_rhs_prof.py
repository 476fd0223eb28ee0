"""configs[1]'s transformer RHS (Cora-sized graph, 8 heads, norm_idx 1) evaluated
`reps` times between two marker kernels, for per-kernel timings of one RHS under
rocprofv3 --kernel-trace (tools/timeline.py --summary): kernel probes that change
the results (experiment builds) can be timed here, outside an adaptive solve.
  python tools/c2_rhs_prof.py [--reps 50]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dopri5_prof  # noqa: E402  (sets sys.path)
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=50)
    a = p.parse_args()
    from gnpde import ops
    func, x, t, kw = dopri5_prof.problem(True)
    mk = torch.ones(64, device=x.device)
    with torch.no_grad():
        for _ in range(3):
            func(None, x)
        torch.cuda.synchronize()
        ops.dot(mk, mk)
        for _ in range(a.reps):
            func(None, x)
        ops.dot(mk, mk)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
