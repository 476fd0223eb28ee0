"""Profile target: HardAttODEblock training forwards at ogbn-arxiv's best_params on G-arxiv (no grad), N reps."""
import contextlib
import io
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "graph-neural-pde_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import gnpde  # noqa: E402
from gnpde import synthetic  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    case = sys.argv[2] if len(sys.argv) > 2 else "arxiv"
    dev = torch.device("cuda", 0)
    N, E, C = synthetic.ARXIV_N, synthetic.ARXIV_E, 128
    ei, w = synthetic.rw_graph(N, E, seed=0, device=dev)
    x = synthetic.features(1, N, C, seed=1, device=dev)
    prm = bench.HARD_BLOCKS[case]
    opt = dict(bench.LAP_OPT, hidden_dim=C, block='hard_attention', function='laplacian', heads=prm['heads'],
               attention_dim=prm['attention_dim'], attention_norm_idx=0, attention_type='scaled_dot',
               att_samp_pct=prm['att_samp_pct'], method='dopri5', step_size=1, tol_scale=prm['tol_scale'],
               adjoint=True, adjoint_method=prm['adjoint_method'], adjoint_step_size=1,
               tol_scale_adjoint=prm['tol_scale_adjoint'], max_iters=100, self_loop_weight=1.0, data_norm='rw',
               leaky_relu_slope=0.2, reweight_attention=False, square_plus=False, mix_features=False,
               beltrami=False, use_flux=False, augment=False)
    blk = gnpde.HardAttODEblock(gnpde.LaplacianODEFunc, [], opt, dev,
                                t=torch.tensor([0.0, prm['T']], device=dev)).to(dev).train()
    data = gnpde.GraphData()
    data.new_graph(ei[:, :, :E - N], N)
    with torch.no_grad(), contextlib.redirect_stdout(io.StringIO()):
        for _ in range(reps):
            blk.set_x0(x)
            blk(x, data)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
