set -u
mkdir -p gpurun_out
for m in cols rows; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 1 --mode $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/mgpu_$m.log 2>&1; rc=$?
  echo "$m rc=$rc"; grep '^{' gpurun_out/mgpu_$m.log | cut -c1-900
  case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 600 python bench.py --no-cpu-baseline --no-grmat > gpurun_out/bench_train.log 2>&1; rc=$?
echo "bench rc=$rc"; python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bench_train.log') if l.startswith('{\"metric\"')][-1]; print(d['value'], json.dumps(d.get('train_rk4')))"
