#!/bin/bash
# decode-attention split heuristic: workgroup target 256 (default) vs 1024 at long contexts
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
for t in 256 1024 2048; do
for cfg in "32768 1" "8192 1" "32768 8" "128 1"; do
  set -- $cfg
  MIPIPE_ATTN_WG_TARGET=$t timeout -k 10 300 python3 bench.py --model llama3-8b --ftype Q4_K_M --prompt-len $1 --mb-size $2 --steps 20 --warmup 2 > $O/at.log 2>&1 || { tail -5 $O/at.log; exit 1; }
  grep '"value"' $O/at.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('target $t: 8B prompt', $1, 'mb', $2, '->', d['value'], 'tok/s')"
done; done
