#!/usr/bin/env python
"""The bench's training-step measurement alone (bench.bench_train), for profiling."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from gnpde import synthetic  # noqa: E402

dev = torch.device("cuda", 0)
ei, w = synthetic.rw_graph(synthetic.ARXIV_N, synthetic.ARXIV_E, seed=0, device=dev)
x = synthetic.features(1, synthetic.ARXIV_N, 128, seed=1, device=dev)
print(json.dumps(dict(lib=os.path.basename(os.environ.get("GNPDE_LIB", "libgnpde.so")),
                      **bench.bench_train(ei, w, x, 0.25, dev))))
