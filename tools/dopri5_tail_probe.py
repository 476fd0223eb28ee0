import os, sys, time
ROOT = "/root/repo"
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dopri5_prof
import torch
func, x, t, kw = dopri5_prof.problem(False)
import gnpde
from gnpde import integrator as gi
R = gi._RKAdaptiveFused
orig = R._rec_reader
stamps = []
def rr(self, st, rec, slot=None):
    read = orig(self, st, rec, slot)
    def r2():
        a = time.perf_counter(); v = read(); b = time.perf_counter()
        stamps.append((a, b)); return v
    return r2
R._rec_reader = rr
with torch.no_grad():
    for _ in range(3): gnpde.odeint(func, x, t, **kw)
    torch.cuda.synchronize()
    res = []
    for _ in range(10):
        stamps.clear()
        t0 = time.perf_counter()
        gnpde.odeint(func, x, t, **kw)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res.append((t1 - t0, t2 - t1, t1 - stamps[-1][1], [b - a for a, b in stamps], stamps[0][0] - t0))
for r in res:
    print("solve host %.1f us, sync after %.1f, after last read %.1f us, first read at %.1f; waits %s" % (
        r[0]*1e6, r[1]*1e6, r[2]*1e6, r[4]*1e6, ["%.0f" % (w*1e6) for w in r[3]]))
