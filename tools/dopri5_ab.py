"""In-process A/B of the G-arxiv dopri5 solve (ogbn-arxiv best_params) over integrator
switches, alternating configurations, median wall time per solve (host sync after each):
  python tools/dopri5_ab.py [reps]"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dopri5_prof  # noqa: E402
import torch  # noqa: E402

CONFIGS = {
    "default": dict(DENSE_FOLD=True, INIT_ROWS=False, GRAPH_RECORD_COPY=True, LIN_INIT=True, PROLOGUE_GRAPH=True),
    "no-pro": dict(DENSE_FOLD=True, INIT_ROWS=False, GRAPH_RECORD_COPY=True, LIN_INIT=True, PROLOGUE_GRAPH=False),
    "no-lin": dict(DENSE_FOLD=True, INIT_ROWS=False, GRAPH_RECORD_COPY=True, LIN_INIT=False, PROLOGUE_GRAPH=False),
    "round5": dict(DENSE_FOLD=False, INIT_ROWS=False, GRAPH_RECORD_COPY=False, LIN_INIT=False, PROLOGUE_GRAPH=False),
}


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    func, x, t, kw = dopri5_prof.problem(False)
    import gnpde
    from gnpde import integrator as gi
    times = {k: [] for k in CONFIGS}
    steps = {}
    with torch.no_grad():
        for k, cfg in CONFIGS.items():  # warm every variant (graphs captured)
            for n, v in cfg.items():
                setattr(gi, n, v)
            for _ in range(3):
                gnpde.odeint(func, x, t, **kw)
        torch.cuda.synchronize()
        for _ in range(reps):
            for k, cfg in CONFIGS.items():
                for n, v in cfg.items():
                    setattr(gi, n, v)
                t0 = time.perf_counter()
                z = gnpde.odeint(func, x, t, **kw)
                torch.cuda.synchronize()
                times[k].append(time.perf_counter() - t0)
                steps[k] = gi.odeint.last_n_steps
    for k, v in times.items():
        print("%-10s median %.1f us  min %.1f us  steps %d" % (k, statistics.median(v) * 1e6, min(v) * 1e6, steps[k]))


if __name__ == "__main__":
    main()
