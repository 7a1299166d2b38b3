#!/bin/bash
# decode attention split length at mb64 (auto = one split for ctx <= 192 vs 128-key splits) and unfused path
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for s in "" "--set attn_split_len=128" "--set fused_attn=false"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/as_prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 $s > $O/as.log 2>&1 || { tail -5 $O/as.log; exit 1; }
  echo "== [$s] $(grep -o '"value": [0-9.]*' $O/as.log)"
  python3 $R/tools/prof_summary.py $O/as_prof | sed -n '/last 5 decode/,$p' | grep -i "attn\|rope\|last 5"
  rm -rf $O/as_prof
done
