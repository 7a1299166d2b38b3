#!/bin/bash
# full GPU suite + headline benches
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r2y_tests.log 2>&1; rc=$?; tail -3 $O/r2y_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 bench.py > $O/r2y_b70.log 2>&1 || { tail -5 $O/r2y_b70.log; exit 1; }; tail -1 $O/r2y_b70.log
timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 > $O/r2y_b8.log 2>&1 || { tail -5 $O/r2y_b8.log; exit 1; }; tail -1 $O/r2y_b8.log
timeout -k 10 300 python3 bench.py --mb-size 1 > $O/r2y_b70m1.log 2>&1 || { tail -5 $O/r2y_b70m1.log; exit 1; }; tail -1 $O/r2y_b70m1.log
