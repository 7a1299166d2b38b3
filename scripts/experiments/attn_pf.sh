#!/bin/bash
# decode attention chunk prefetch: tests + short/long context benches (compare with profiles r1g_*)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "attn or attention or long_context or engine_matches or pipeline" > $O/apf_tests.log 2>&1 || { tail -30 $O/apf_tests.log; exit 1; }
tail -1 $O/apf_tests.log
for cfg in "llama3-8b Q4_K_M 32768 1" "llama3-8b Q4_K_M 8192 1" "llama3-8b Q4_K_M 32768 8" "llama3-8b Q4_K_M 128 1" "llama3-70b Q4_K 128 64" "llama3-70b Q4_K 128 1"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --model $1 --ftype $2 --prompt-len $3 --mb-size $4 --steps 20 --warmup 2 > $O/apf.log 2>&1 || { tail -5 $O/apf.log; exit 1; }
  echo "$1 prompt $3 mb $4: $(grep -o '"value": [0-9.]*' $O/apf.log)"
done
