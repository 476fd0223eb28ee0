set -u
for a in 16 128 64; do
  GNPDE_PAD_ALIGN_BF16=$a timeout -k 10 300 python - <<'PY' || exit 1
import os, sys, json, torch
sys.path.insert(0, "graph-neural-pde_amd"); sys.path.insert(0, ".")
import bench
from gnpde import ops, synthetic
dev = torch.device("cuda", 0)
ei, w = synthetic.rw_graph(synthetic.ARXIV_N, synthetic.ARXIV_E, seed=0, device=dev)
g = ops.GraphCSR(ei, synthetic.ARXIV_N)
r = bench.bench_blend(g, dev)
print(os.environ["GNPDE_PAD_ALIGN_BF16"], r["fp32"]["ms_per_step"], r["bf16"]["ms_per_step"], r["check"]["ok"])
PY
done
