#!/usr/bin/env python
"""One attention RHS of the bench's shape (G-arxiv, C=128, h=2, att=32) replayed
from a captured graph, for the library GNPDE_LIB points at (A/B of variant
builds, make -C graph-neural-pde_amd variant ...): prints one JSON line.
ATT_MODES: comma list of mode:norm_idx (default per_edge:0)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    from gnpde import _lib, synthetic
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, _ = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    out = {"lib": os.path.basename(os.environ.get("GNPDE_LIB", _lib.LIB_PATH))}
    ref = None
    for spec in os.environ.get("ATT_MODES", "per_edge:0").split(","):
        mode, norm = spec.split(":")
        func = bench.attention_func(mode, int(norm), C, dev)
        func.edge_index = ei
        func.graph_for(x)
        with torch.no_grad():
            f = func(None, x)
            cg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(cg):
                func(None, x)
            for _ in range(3):
                cg.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(50):
                cg.replay()
            e.record()
            torch.cuda.synchronize()
        out[spec] = round(s.elapsed_time(e) / 50 * 1e3, 1)
        if spec == "per_edge:0":
            ref = f
    if ref is not None:
        out["sum"] = float(ref.double().abs().sum())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
