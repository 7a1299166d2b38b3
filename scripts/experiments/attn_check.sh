#!/bin/bash
# attention kernel tests, then 70B mb16 + 8B mb1 benches and a kernel-stats profile of 70B mb16
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/attn_tests.log 2>&1 || { tail -30 $O/attn_tests.log; exit 1; }
tail -3 $O/attn_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/b70.log 2>&1 || { tail -5 $O/b70.log; exit 1; }
grep '"value"' $O/b70.log
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --steps 30 --warmup 3 --mb-size 1 > $O/b8.log 2>&1 || { tail -5 $O/b8.log; exit 1; }
grep '"value"' $O/b8.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 $R/tools/prof_summary.py $O/prof > $O/prof_70b_mb16.txt && head -14 $O/prof_70b_mb16.txt
