#!/bin/bash
# r12o (round-6 final build 4077bdf): full GPU suite, smoke, the driver bench line
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r12o_tests.log 2>&1; rc=$?; tail -3 $O/r12o_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r12o_smoke.log 2>&1; rc=$?; tail -1 $O/r12o_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/r12o_bench.log 2>&1; rc=$?; tail -1 $O/r12o_bench.log; [ $rc -ne 0 ] && exit $rc
