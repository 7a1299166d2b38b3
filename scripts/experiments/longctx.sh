#!/bin/bash
# long-context decode: Llama-3-8B Q4_K_M with 8K / 32K-token prompts (chunked prefill, flash-decoding splits)
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_engine_gpu.py -k long_context > $O/lc_test.log 2>&1 || { tail -20 $O/lc_test.log; exit 1; }
tail -1 $O/lc_test.log
for cfg in "8192 1" "32768 1" "32768 8" "8192 64"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --prompt-len $1 --mb-size $2 --steps 20 --warmup 2 > $O/lc.log 2>&1 || { tail -5 $O/lc.log; exit 1; }
  grep '"value"' $O/lc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('8B prompt', $1, 'mb', $2, '->', d['value'], 'tok/s', d['ms_per_step'], 'ms/step')"
  grep '"value"' $O/lc.log > $O/lc_$1_$2.json
done
