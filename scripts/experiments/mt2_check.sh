#!/bin/bash
# GEMV row-group (M <= 32) check: kernel + engine tests, then a micro-batch sweep
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/mt2_tests.log 2>&1 || { tail -30 $O/mt2_tests.log; exit 1; }
tail -2 $O/mt2_tests.log
bash scripts/experiments/mb_sweep.sh "--mb-size 16" "--mb-size 32" "--mb-size 48" "--mb-size 64" "--mb-size 64 --model llama3-8b --ftype Q4_K_M" "--mb-size 64 --model mixtral-8x7b --ftype Q4_K_M" "--mb-size 16 --model mixtral-8x7b --ftype Q4_K_M"
