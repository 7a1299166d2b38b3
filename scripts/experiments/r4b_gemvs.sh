#!/bin/bash
# gemvs: kernel tests, engine tests, 8B / 70B single-stream bench, kernel profile of 8B mb1
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemvs_gpu.py tests/test_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/r4b_tests.log 2>&1; rc=$?
tail -5 $O/r4b_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 50 --warmup 5 > $O/r4b_b8.log 2>&1 || { tail -5 $O/r4b_b8.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r4b_b8.log
timeout -k 10 300 python bench.py --model llama3-70b --ftype Q4_K --mb-size 1 --steps 20 --warmup 3 > $O/r4b_b70.log 2>&1 || { tail -5 $O/r4b_b70.log; exit 1; }
grep -o '"value": [0-9.]*' $O/r4b_b70.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r4b_prof -o run -- python3 bench.py --model llama3-8b --ftype Q4_K_M --mb-size 1 --steps 10 --warmup 2 > $O/r4b_prof.log 2>&1 || { tail -5 $O/r4b_prof.log; exit 1; }
echo done
