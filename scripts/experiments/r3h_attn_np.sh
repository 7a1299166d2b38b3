#!/bin/bash
# decode attention: no-prefetch occupancy-3 variant for many-split contexts; tests + long-context benches
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_paged_kv.py tests/test_kernels_gpu.py > $O/r3h_tests.log 2>&1; rc=$?; tail -2 $O/r3h_tests.log; [ $rc = 0 ] || exit 1
for KV in f16 fp8; do
  for cfg in "32768 1" "32768 8" "8192 1"; do
    set -- $cfg
    timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --prompt-len $1 --mb-size $2 --steps 20 --warmup 2 --set kv_dtype=$KV > $O/r3h.log 2>&1 || { tail -5 $O/r3h.log; exit 1; }
    grep '"value"' $O/r3h.log > $O/r3h_8b_${KV}_$1_$2.json
    echo "8B prompt $1 mb $2 kv=$KV $(grep -o '"value": [0-9.]*' $O/r3h.log)"
  done
done
