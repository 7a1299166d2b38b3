#!/bin/bash
# r9k: Mixtral 8x7B Q4_K_M, 256 vs 64 sequences on the final build, interleaved in one call (the
# review's MoE scaling ratio)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
BB="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-secondary --model mixtral-8x7b --ftype Q4_K_M"
for rep in 1 2; do for mb in 256 64; do
  $BB --mb-size $mb > $O/r9k.log 2>&1 || { tail -3 $O/r9k.log; exit 1; }
  echo "rep $rep mixtral mb$mb $(grep -o '"value": [0-9.]*' $O/r9k.log)"
done; done
