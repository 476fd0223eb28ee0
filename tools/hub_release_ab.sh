set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_layout.py -q --timeout 200 --timeout-method thread > gpurun_out/layout_tests.log 2>&1; rc=$?
echo "layout tests rc=$rc"; tail -3 gpurun_out/layout_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
GNPDE_LIB=$PWD/graph-neural-pde_amd/gnpde/variants/libgnpde_rel.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > gpurun_out/rel_tests.log 2>&1; rc=$?
echo "release-variant parity rc=$rc"; tail -2 gpurun_out/rel_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2; do
  for v in default rel; do
    if [ $v = rel ]; then export GNPDE_LIB=$PWD/graph-neural-pde_amd/gnpde/variants/libgnpde_rel.so; else unset GNPDE_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-attention --no-grmat > gpurun_out/b_$v.log 2>&1 || exit 1
    python -c "import json; d=[json.loads(l) for l in open('gpurun_out/b_$v.log') if l.startswith('{\"metric\"')][-1]; print('$v', d['value'], d['ms_per_step'], d['rhs_plain']['rhs_ms'])"
    timeout -k 10 300 python tools/k1_bench.py || exit 1
  done
done
