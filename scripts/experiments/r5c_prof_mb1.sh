#!/bin/bash
# kernel profile of single-stream decode (gemvs path): 8B Q4_K_M and 70B Q4_K, mb1
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for cfg in "8b llama3-8b Q4_K_M" "70b llama3-70b Q4_K"; do
  set -- $cfg
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1_$1 -o run --output-format csv -- python3 $R/bench.py --model $2 --ftype $3 --mb-size 1 --steps 10 --warmup 2 > $O/prof1_$1.log 2>&1 || { tail -5 $O/prof1_$1.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/prof1_$1 > $O/r5c_prof_$1_mb1.txt && sed -n '/last 5/,$p' $O/r5c_prof_$1_mb1.txt | head -14
done
