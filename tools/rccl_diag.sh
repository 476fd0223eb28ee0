set -u
mkdir -p gpurun_out
export NCCL_DEBUG=WARN
timeout -k 10 120 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
  tools/rccl_diag.py > gpurun_out/rccl_diag.log 2>&1; rc=$?
echo "diag rc=$rc"; grep -v amdgpu.ids gpurun_out/rccl_diag.log | tail -15
