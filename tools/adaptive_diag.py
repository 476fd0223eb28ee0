"""Per-step error ratios of the fused dopri5 solve and of the unfused tableau loop
on tests/test_gpu_adaptive.py::test_fused_adaptive_vs_unfused_loop's problem, and
the fp64 oracle's step count: where a step count differs, whether a ratio sits at 1.
  python tools/adaptive_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import test_gpu_adaptive as TA
    from gnpde import integrator as gi
    import gnpde_oracle as O
    N, E, C = 5000, 60000, 64
    eo, wo, rng = TA._graph(N, E, 32)
    x = TA.T(rng.standard_normal((1, N, C)).astype(np.float32))
    x0 = TA.T(rng.standard_normal((1, N, C)).astype(np.float32))
    func = TA._laplacian(C, eo, wo, add_source=True, x0=x0)
    t = torch.tensor([0.0, 0.7, 1.5], dtype=torch.float64, device="cuda")
    fused = []
    orig = gi._RKAdaptiveFused._rec_reader

    def rec(self, st, r, slot=None):
        rd = orig(self, st, r, slot)
        if slot is None:
            def read():
                v = rd()
                fused.append(v[0])
                return v
            return read
        return rd
    gi._RKAdaptiveFused._rec_reader = rec
    with torch.no_grad():
        gi.odeint(func, x, t, rtol=1e-5, atol=1e-6, method='dopri5')
        nf = gi.odeint.last_n_steps
        loop = []
        on = gi._rms_norm

        def norm(v):
            r = on(v)
            loop.append(float(r))
            return r
        gi._rms_norm = norm
        os.environ["GNPDE_FUSED_ADAPTIVE"] = "0"
        gi.odeint(func, x, t, rtol=1e-5, atol=1e-6, method='dopri5')
        nl = gi.odeint.last_n_steps
    print("fused steps", nf, "ratios", ["%.9f" % r for r in fused])
    print("loop  steps", nl, "norms", ["%.9f" % r for r in loop])
    f = lambda tt, y: O.laplacian_rhs(TA._oracle_graph(eo) if hasattr(TA, '_oracle_graph') else eo, y, None, 0.0, 0.0)  # noqa
    del f


if __name__ == "__main__":
    main()
