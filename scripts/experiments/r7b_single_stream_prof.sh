#!/bin/bash
# Single-stream kernel profile (8B Q4_K_M mb1, 70B Q4_K mb1): per-round breakdown + one layer in dispatch order
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
for cfg in "llama3-8b Q4_K_M" "llama3-70b Q4_K"; do
  set -- $cfg
  tag=${1#llama3-}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$tag -o run --output-format csv -- \
    python3 $R/bench.py --model $1 --ftype $2 --mb-size 1 --steps 30 --warmup 3 --no-secondary > $O/prof_$tag.log 2>&1 \
    || { echo "prof $tag failed"; tail -5 $O/prof_$tag.log; exit 1; }
  grep '"value"' $O/prof_$tag.log | cut -c1-200
  PROF_SEQ=16 python3 $R/tools/prof_summary.py $O/prof_$tag > $O/prof_${tag}_mb1.txt && tail -36 $O/prof_${tag}_mb1.txt
  rm -rf $O/prof_$tag
done
