#!/bin/bash
# kernel profile of the wide decode micro-batches (70B mb256, 8B mb128 / mb256)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for cfg in "70b 256 llama3-70b Q4_K" "8b 128 llama3-8b Q4_K_M" "8b 256 llama3-8b Q4_K_M"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$1_$2 -o run --output-format csv -- python3 $R/bench.py --model $3 --ftype $4 --mb-size $2 --steps 6 --warmup 2 > $O/prof_$1_$2.log 2>&1 || { tail -5 $O/prof_$1_$2.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/prof_$1_$2 > $O/r5b_prof_$1_mb$2.txt && sed -n '/last 5/,$p' $O/r5b_prof_$1_mb$2.txt | head -14
done
