#!/bin/bash
# decode-attention restructure: GPU tests, then A/B old vs new lib (70B mb64 headline, 8B mb1 long context)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
cd $R && timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_paged_kv.py tests/test_kernels_gpu.py tests/test_deterministic_gpu.py > $O/r2r_tests.log 2>&1; rc=$?; tail -3 $O/r2r_tests.log; [ $rc = 0 ] || exit 1
for L in libold.so libmipipe.so; do
  MIPIPE_LIB=$L timeout -k 10 300 python3 $R/bench.py --model llama3-8b --mb-size 1 --prompt-len 8192 --steps 30 > $O/r2r_long_$L.log 2>&1 || { tail -5 $O/r2r_long_$L.log; exit 1; }
  echo "8B mb1 8K $L: $(grep -o '"value": [0-9.]*' $O/r2r_long_$L.log)"
  MIPIPE_LIB=$L timeout -k 10 300 python3 $R/bench.py --model llama3-8b --mb-size 64 --prompt-len 1024 --steps 10 --warmup 3 > $O/r2r_m64_$L.log 2>&1 || { tail -5 $O/r2r_m64_$L.log; exit 1; }
  echo "8B mb64 1K $L: $(grep -o '"value": [0-9.]*' $O/r2r_m64_$L.log)"
done
cd /tmp && bash $R/scripts/experiments/ab_lib.sh libold.so libmipipe.so --steps 20 --warmup 5
