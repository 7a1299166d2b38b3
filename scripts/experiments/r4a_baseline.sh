#!/bin/bash
# round-2 re-entry baseline: GPU suite, 70B mb64 bench, 8B mb1 bench
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/r4a_tests.log 2>&1; rc=$?
tail -3 $O/r4a_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/r4a_b70.log 2>&1 || { tail -5 $O/r4a_b70.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r4a_b70.log
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 --warmup 5 > $O/r4a_b8.log 2>&1 || { tail -5 $O/r4a_b8.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r4a_b8.log
exit $rc
