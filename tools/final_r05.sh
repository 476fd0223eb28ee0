#!/bin/bash
# Round-5 closing checks on one MI355X: the GPU test suite, smoke(), and the
# preprocessing kernel trace of the final library.  Stops after a crash or time limit.
OUT=gpurun_out/r05g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc2=$?
tail -3 $OUT/smoke.log
case $rc2 in 124|137|134|139) exit $rc2;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o prep -- \
  python3 $GRAFT_REPO_ROOT/tools/prep_prof.py > $GRAFT_REPO_ROOT/$OUT/pp.log 2>&1
echo "pytest rc=$rc smoke rc=$rc2"
