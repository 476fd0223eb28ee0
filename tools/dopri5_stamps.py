"""Host time of the pieces of a warm fused dopri5 solve (G-arxiv, ogbn-arxiv best_params):
every integrator / ops entry of the solve's path wrapped with a perf_counter timer
(inclusive host time per solve, launches are asynchronous), beside the solve's wall time.
  python tools/dopri5_stamps.py [--reps 20]"""
import argparse
import collections
import functools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dopri5_prof  # noqa: E402  (sets sys.path)
import torch  # noqa: E402

ACC = collections.defaultdict(float)
CNT = collections.defaultdict(int)


def wrap(obj, name, label=None):
    fn = getattr(obj, name)
    label = label or "%s.%s" % (getattr(obj, '__name__', type(obj).__name__), name)

    @functools.wraps(fn)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            ACC[label] += time.perf_counter() - t0
            CNT[label] += 1
    setattr(obj, name, w)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    a = p.parse_args()
    func, x, t, kw = dopri5_prof.problem(False)
    import gnpde
    from gnpde import integrator as gi, ops
    R = gi._RKAdaptiveFused
    for n in ("_state", "_initial_step_device", "_run_step", "_rec_reader", "_krylov_launches", "_integrate",
              "integrate", "_interp_into", "_step"):
        wrap(R, n, "RKAdaptiveFused." + n)
    for n in ("_capture_state", "_graph_cache_key", "_node_layout", "_host_times", "_entry_copy", "_to_user",
              "_fused_adaptive_ok"):
        wrap(gi, n)
    for n in ("spmm_rhs", "initial_step", "adaptive_control", "stage_apply", "rows_copy"):
        if hasattr(ops, n):
            wrap(ops, n)
    wrap(type(func), "rhs_stage", "func.rhs_stage")
    with torch.no_grad():
        for _ in range(3):
            gnpde.odeint(func, x, t, **kw)
        torch.cuda.synchronize()
        ACC.clear()
        CNT.clear()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            gnpde.odeint(func, x, t, **kw)
            torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.reps
    print("wall per solve %.1f us" % (wall * 1e6))
    for k, v in sorted(ACC.items(), key=lambda kv: -kv[1]):
        print("%9.1f us  %6.1f calls  %s" % (v / a.reps * 1e6, CNT[k] / a.reps, k))


if __name__ == "__main__":
    main()
