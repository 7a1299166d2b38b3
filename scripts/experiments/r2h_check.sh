#!/bin/bash
# deferred-norm check: kernel/engine GPU tests, 8B mb1 profile, single-stream + headline benches
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gemv_fused_gpu.py tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $O/r2h_tests.log 2>&1 || { tail -40 $O/r2h_tests.log; exit 1; }
tail -2 $O/r2h_tests.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p8h -o run --output-format csv -- python3 $R/bench.py --model llama3-8b --ftype Q4_K_M --steps 10 --warmup 2 --mb-size 1 > $O/p8h.log 2>&1 || { tail -5 $O/p8h.log; exit 1; }
python3 $R/tools/prof_summary.py $O/p8h > $O/r2h_prof_8b_mb1.txt || exit 1
cd $R
timeout -k 10 200 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 > $O/r2h_bench8b.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mb-size 1 --steps 20 > $O/r2h_bench70b_mb1.log 2>&1 || exit 1
