#!/bin/bash
# decode attention time vs context at mb64 (8B: same 8 kv heads x 128 as 70B)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for P in 16 128 1024; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/actx_$P -o run --output-format csv -- python3 $R/bench.py --model llama3-8b --mb-size 64 --prompt-len $P --steps 10 --warmup 3 > $O/actx_$P.log 2>&1 || { tail -5 $O/actx_$P.log; exit 1; }
  echo "== prompt $P $(grep -o '"value": [0-9.]*' $O/actx_$P.log)"
  python3 $R/tools/prof_summary.py $O/actx_$P > $O/actx_$P.txt && grep -E 'attn|rmsnorm' $O/actx_$P.txt | head -6
done
