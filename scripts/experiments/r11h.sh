#!/bin/bash
# r11h: full GPU suite + the driver's bench line (N = 1, all secondaries) on the current build
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/r11h_tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $O/r11h_tests.log | tail -15
[ $rc -gt 1 ] && exit $rc
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/r11h_bench.log 2>&1 || { tail -5 $O/r11h_bench.log; exit 1; }
grep '"value"' $O/r11h_bench.log | tee $O/r11h_bench.json
