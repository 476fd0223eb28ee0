#!/bin/bash
# BLEND (configs[3] shape) fp32 vs bf16 rk4 step time under K1 lane-geometry knobs.
# BLEND_CFGS="vec:variant ..." (GNPDE_BF16_VEC : GNPDE_AGG_VARIANT)
for cfg in ${BLEND_CFGS:-8:0 4:0 8:1 8:3 4:3}; do set -- ${cfg/:/ }
GNPDE_BF16_VEC=$1 GNPDE_AGG_VARIANT=$2 timeout -k 10 200 python -c "
import sys, torch, json; sys.path.insert(0,'graph-neural-pde_amd'); sys.path.insert(0,'.')
import bench
from gnpde import ops, synthetic
dev=torch.device('cuda',0)
ei,w=synthetic.rw_graph(169343,1200000,seed=0,device=dev)
g=ops.GraphCSR(ei,169343)
d=bench.bench_blend(g, dev)
print('vec $1 variant $2 fp32 %.4f %.3f bf16 %.4f %.3f' % (d['fp32']['ms_per_step'], d['fp32']['frac'], d['bf16']['ms_per_step'], d['bf16']['frac']))
" || exit 1; done
