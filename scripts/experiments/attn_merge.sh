#!/bin/bash
# parallel split merge in the fused decode attention: tests, then long-context 8B benches per split target
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "attn or attention or long_context or engine_matches or pipeline or spec or checkpoint or prefix" > $O/am_tests.log 2>&1 || { tail -30 $O/am_tests.log; exit 1; }
tail -1 $O/am_tests.log
for t in 256 1024; do
for cfg in "32768 1" "8192 1" "32768 8" "128 1" "128 64"; do
  set -- $cfg
  MIPIPE_ATTN_WG_TARGET=$t timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --prompt-len $1 --mb-size $2 --steps 20 --warmup 2 > $O/at.log 2>&1 || { tail -5 $O/at.log; exit 1; }
  grep '"value"' $O/at.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('target $t: 8B prompt', $1, 'mb', $2, '->', d['value'], 'tok/s')"
done; done
