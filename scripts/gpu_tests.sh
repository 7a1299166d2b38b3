#!/bin/bash
# GPU test suite + one 1-GPU bench line. Stops on crash/timeout (rc > 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 500 python -m pytest tests -q -m gpu -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|Error|error" $O/tests.log | tail -15
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep '"value"' $O/bench.log
exit $rc
