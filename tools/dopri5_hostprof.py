"""Host-side cost of a fused dopri5 solve (G-arxiv, or --c2): cProfile of warm
solves, sorted by own time, to find the Python work between the device launches.
  python tools/dopri5_hostprof.py [--c2] [--reps 20]"""
import argparse
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dopri5_prof  # noqa: E402  (sets sys.path)
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--c2", action="store_true")
    a = p.parse_args()
    func, x, t, kw = dopri5_prof.problem(a.c2)
    import gnpde
    with torch.no_grad():
        for _ in range(3):
            gnpde.odeint(func, x, t, **kw)
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(a.reps):
            gnpde.odeint(func, x, t, **kw)
        torch.cuda.synchronize()
        pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
