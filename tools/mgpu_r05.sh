#!/bin/bash
# One-GPU record of the N > 1 code paths under torch.distributed.run (RCCL, env://),
# round 5: the sharded transformer attention RHS (bench.py --mode cols / rows, the
# "attention_sharded" object; step graphs now capture the RCCL collectives at a world
# of one, partitioned destination statistics) and the row-partitioned Laplacian.
# JSON lines -> $OUT/*.log
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-mgpu5}
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
