#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "speculative" > $O/spec_tests.log 2>&1 || { tail -30 $O/spec_tests.log; exit 1; }
tail -1 $O/spec_tests.log
timeout -k 10 300 python tools/spec_bench.py --model llama3-8b > $O/spec_8b.log 2>&1 || { tail -5 $O/spec_8b.log; exit 1; }
grep same_output $O/spec_8b.log
timeout -k 10 300 python tools/spec_bench.py --model llama3-8b --repeat-prompt > $O/spec_8b_r.log 2>&1 || { tail -5 $O/spec_8b_r.log; exit 1; }
grep same_output $O/spec_8b_r.log
timeout -k 10 300 python tools/spec_bench.py --model llama3-70b --ftype Q4_K --n 32 > $O/spec_70b.log 2>&1 || { tail -5 $O/spec_70b.log; exit 1; }
grep same_output $O/spec_70b.log
