#!/bin/bash
# paged KV + argmax hand-off: full GPU suite, headline bench, single stream
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r2l_tests.log 2>&1 || { tail -40 $O/r2l_tests.log; exit 1; }
tail -2 $O/r2l_tests.log
timeout -k 10 200 python bench.py > $O/r2l_bench70b_mb64.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 > $O/r2l_bench8b_mb1.log 2>&1 || exit 1
