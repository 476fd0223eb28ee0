#!/usr/bin/env python
"""Micro-benchmark of the MFMA projection (gnpde_linear_f32) at the attention
shape: R = 169,343 rows, K = C = 128, Nout = 2 * att = 64 (Q | K)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

from gnpde import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    R, K, Nout = int(os.environ.get("LIN_R", 169343)), int(os.environ.get("LIN_K", 128)), int(os.environ.get("LIN_N", 64))
    x = torch.randn(R, K, device=dev)
    W = torch.randn(Nout, K, device=dev) * 0.1
    b = torch.randn(Nout, device=dev) * 0.1
    for _ in range(3):
        ops.linear(x, W, b, split=Nout // 2)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 50
    s.record()
    for _ in range(reps):
        ops.linear(x, W, b, split=Nout // 2)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / reps * 1e3
    qa, kb = ops.linear(x, W, b, split=Nout // 2)
    ref = (x.double() @ W.double().t() + b.double())
    err = float((torch.cat([qa, kb], 1).double() - ref).abs().max() / ref.abs().max())
    print(json.dumps({"R": R, "K": K, "Nout": Nout, "us": round(us, 2), "waves": os.environ.get("GNPDE_LIN_WAVES", "2048"),
                      "variant": os.environ.get("GNPDE_LINEAR", "0"), "TFLOPs": round(2 * R * K * Nout / us / 1e6, 1),
                      "GBs": round((4 * R * K + 4 * R * Nout) / us / 1e3, 1), "rel_err": err}))


if __name__ == "__main__":
    main()
