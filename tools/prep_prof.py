"""Graph preprocessing and hard-attention sampling kernels on G-arxiv, for rocprofv3
--kernel-trace --stats (VERDICT r4 item 3's per-kernel bars): self loops +
row-normalised weights (gnpde.utils.get_rw_adj), the threshold mask of the sampled
attention, the in-degree.  Each repeated `reps` times.
  python tools/prep_prof.py [--reps 5]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    from gnpde import ops, synthetic, utils
    dev = torch.device("cuda", 0)
    N, E = synthetic.ARXIV_N, synthetic.ARXIV_E
    ei = synthetic.rmat_edges(N, E - N, seed=0, device=dev)[None]
    v = torch.rand(ei.shape[-1], device=dev)
    thr = torch.quantile(v, 0.19).reshape(())
    for _ in range(a.reps):
        utils.get_rw_adj(ei, None, norm_dim=1, fill_value=1.0, num_nodes=N)
        ops.threshold_mask(v, thr)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
