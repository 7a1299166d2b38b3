#!/bin/bash
# deterministic mode + dequant code-gen change: GPU tests, mode cost, headline
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_deterministic_gpu.py tests/test_kernels_gpu.py tests/test_gemv_fused_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r2k_tests.log 2>&1 || { tail -40 $O/r2k_tests.log; exit 1; }
tail -2 $O/r2k_tests.log
timeout -k 10 200 python bench.py > $O/r2k_bench70b_mb64.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --set deterministic=true > $O/r2k_bench70b_mb64_det.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mb-size 1 --steps 20 > $O/r2k_bench70b_mb1.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mb-size 1 --steps 20 --set deterministic=true > $O/r2k_bench70b_mb1_det.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 > $O/r2k_bench8b_mb1.log 2>&1 || exit 1
