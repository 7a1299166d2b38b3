#!/bin/bash
# GEMV kernel tests + micro-benchmark sweep + 70B bench (quick perf iteration)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider -k gemv > $O/kt.log 2>&1; rc=$?; tail -2 $O/kt.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/gemv_bench.py --types Q4_K,Q6_K --M 1,16 --tpw ${TPW:-1,2,4} > $O/gemv_sweep.log 2>&1 || { tail -5 $O/gemv_sweep.log; exit 1; }
grep shape $O/gemv_sweep.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 2>&1 | grep '"value"' | cut -c1-200
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | cut -c1-200
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 30 --warmup 3 --mb-size 1 2>&1 | grep '"value"' | cut -c1-200
