#!/bin/bash
# One-GPU rehearsal of the N > 1 code paths under torch.distributed.run (RCCL,
# env://): the bench's sharded modes on the configs[4] graph (G-rmat) in column
# stripes and in the row partition + per-RHS all-gather, and a dopri5 column
# solve through the all-reduce of its global error norm.  JSON lines -> $OUT.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-mgpu}
mkdir -p $OUT
cd $R
run() {  # name, port, args...
  local name=$1 port=$2; shift 2
  timeout -k 10 420 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port "$@" > $OUT/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc"; grep -h '^{' $OUT/$name.log | cut -c1-1200
  [ $rc = 0 ] || exit $rc
}
run cols 29517 bench.py --gpus 1 --mode cols --nodes 2000000 --edges 20000000 --dim 256 --steps 10 --warmup 2 \
  --no-grmat --no-cpu-baseline --no-attention --no-train
run rows 29518 bench.py --gpus 1 --mode rows --nodes 2000000 --edges 20000000 --dim 256 --steps 10 --warmup 2 \
  --no-grmat --no-cpu-baseline --no-attention --no-train
run dopri5 29519 tools/mgpu_dopri5.py
