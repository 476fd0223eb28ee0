#!/bin/bash
# One-GPU rehearsal of the N > 1 code paths under torch.distributed.run (RCCL,
# env://), round 4: the sharded transformer attention RHS (G-arxiv, configs[3]
# attention shape) in column stripes and in the row partition (bench.py --mode
# cols / rows: the Laplacian headline line plus "attention_sharded"), the G-rmat
# Laplacian in both layouts, and the dopri5 column solve (fused adaptive step,
# global error norm through one all-reduce per step).  JSON lines -> $OUT.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-mgpu4}
mkdir -p $OUT
cd $R
run() {  # name, port, args...
  local name=$1 port=$2; shift 2
  timeout -k 10 420 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -h '^{' $OUT/$name.log | cut -c1-1500
  [ $rc = 0 ] || exit $rc
}
run attn_cols 29527 bench.py --gpus 1 --mode cols --steps 10 --warmup 2 --no-grmat --no-cpu-baseline --no-train
run attn_rows 29528 bench.py --gpus 1 --mode rows --steps 10 --warmup 2 --no-grmat --no-cpu-baseline --no-train
run grmat_cols 29529 bench.py --gpus 1 --mode cols --nodes 2000000 --edges 20000000 --dim 256 --steps 10 --warmup 2 \
  --no-grmat --no-cpu-baseline --no-attention --no-train
run grmat_rows 29530 bench.py --gpus 1 --mode rows --nodes 2000000 --edges 20000000 --dim 256 --steps 10 --warmup 2 \
  --no-grmat --no-cpu-baseline --no-attention --no-train
run dopri5 29531 tools/mgpu_dopri5.py
