#!/bin/bash
# fp8 KV cache: GPU tests (fp8 + full engine suite), then f16 vs fp8 decode benches
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py -k fp8 > $O/r3e_fp8_tests.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" $O/r3e_fp8_tests.log | head -20; [ $rc = 0 ] || exit 1
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/r3e_tests.log 2>&1; rc=$?; tail -2 $O/r3e_tests.log; [ $rc = 0 ] || exit 1
for KV in f16 fp8; do
  timeout -k 10 300 python3 bench.py --set kv_dtype=$KV > $O/r3e_70b_$KV.log 2>&1 || { tail -5 $O/r3e_70b_$KV.log; exit 1; }
  echo "70B mb64 kv=$KV $(grep -o '"value": [0-9.]*' $O/r3e_70b_$KV.log)"
  for cfg in "32768 1" "32768 8" "8192 64"; do
    set -- $cfg
    timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --prompt-len $1 --mb-size $2 --steps 20 --warmup 2 --set kv_dtype=$KV > $O/r3e_8b_$KV_$1_$2.log 2>&1 || { tail -5 $O/r3e_8b_$KV_$1_$2.log; exit 1; }
    grep '"value"' $O/r3e_8b_$KV_$1_$2.log > $O/r3e_8b_${KV}_$1_$2.json
    echo "8B prompt $1 mb $2 kv=$KV $(grep -o '"value": [0-9.]*' $O/r3e_8b_$KV_$1_$2.log)"
  done
done
